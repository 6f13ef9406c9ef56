#!/bin/bash
# claim ratio 0.2 as the default: DLRM / embedding GPU tests, bench (fp32 + bf16)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py tests/test_gpu_kernels.py tests/test_gpu_models.py -k "dlrm or overlap or embedding or sparse" > $O/r5cr2_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py > $O/r5cr2_bench.log 2>&1 || exit $?
bash scripts/gpu_r5tr.sh || exit $?
exit 0
