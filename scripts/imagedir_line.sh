#!/bin/bash
set -e
mkdir -p gpurun_out
python - <<'PY'
import os, numpy as np
from PIL import Image
rng = np.random.RandomState(0)
for c in range(4):
    d = f"/tmp/imgs/c{c}"; os.makedirs(d, exist_ok=True)
    for k in range(96):
        Image.fromarray(rng.randint(0, 256, (256, 320, 3), dtype=np.uint8)).save(f"{d}/{k}.jpg", quality=90)
PY
timeout -k 10 300 python -u apps/train.py alexnet -b 256 --iterations 20 --warmup 2 --graph --image-dir /tmp/imgs > gpurun_out/alexnet_imagedir.log 2>&1
