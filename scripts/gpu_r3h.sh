#!/bin/bash
# side-stream split-K reduce: GPU numerics (GEMM / Linear / DLRM tests), bench A/B, step profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py tests/test_gpu_kernels.py tests/test_pipeline.py tests/test_gpu_models.py > $O/r3h_tests.log 2>&1 || exit $?
bash scripts/gpu_ab_bench.sh r3h - FM_GEMM_ASYNC_REDUCE=0 - FM_GEMM_ASYNC_REDUCE=0 || exit $?
bash scripts/gpu_profile_step.sh r3h_async || exit $?
exit 0
