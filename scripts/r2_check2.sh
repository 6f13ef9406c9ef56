#!/bin/bash
# fp32 kernel tests, full GPU suite, headline bench, image-folder AlexNet, rocprof of the bench
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_fp32.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench_n1.jsonl 2> gpurun_out/bench_n1.err
python - <<'PY'
import os, numpy as np
from PIL import Image
rng = np.random.RandomState(0)
for c in range(4):
    d = f"/tmp/imgs/c{c}"; os.makedirs(d, exist_ok=True)
    for k in range(96):
        Image.fromarray(rng.randint(0, 256, (256, 320, 3), dtype=np.uint8)).save(f"{d}/{k}.jpg", quality=90)
PY
timeout -k 10 300 python -u apps/train.py alexnet -b 256 --iterations 10 --warmup 2 --graph --image-dir /tmp/imgs > gpurun_out/alexnet_imagedir.log 2>&1
bash scripts/prof_bench.sh prof_r2b_fp32
python tools/prof_summary.py gpurun_out/prof_r2b_fp32/*/run_results.db 20 > gpurun_out/prof_r2b_fp32_kernels.txt 2>&1 || python tools/prof_summary.py $(ls gpurun_out/prof_r2b_fp32/*results.db gpurun_out/prof_r2b_fp32/*/*results.db 2>/dev/null | head -1) 20 > gpurun_out/prof_r2b_fp32_kernels.txt
