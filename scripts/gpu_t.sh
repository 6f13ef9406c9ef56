#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -m pytest tests/test_gpu_fp32_split.py tests/test_gpu_fp32.py -q -x --timeout 120 \
  --timeout-method thread -k "nonfinite or smallk" > gpurun_out/p10_pre.log 2>&1 || { tail -30 gpurun_out/p10_pre.log; exit 1; }
tail -1 gpurun_out/p10_pre.log
bash scripts/gpu_tune.sh
