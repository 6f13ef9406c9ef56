#!/bin/bash
# fp32 dW through hipBLASLt (FM_DW_LIB): numerics (fp32 GPU tests) and bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py tests/test_pipeline.py > $O/r3j_tests.log 2>&1 || exit $?
bash scripts/gpu_ab_bench.sh r3j - FM_DW_LIB=0 - FM_DW_LIB=0 || exit $?
exit 0
