#!/bin/bash
# r5e: thin-input fp32 Linear kernels (gemm_small.hip): float64-oracle tests, bench A/B
# (FM_SMALLK=0 vs 1), then a kernel trace of the default bench with the step timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 240 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py -k "smallk or skinny or linear" > $O/r5e_tests.log 2>&1 || exit $?
FM_SMALLK=0 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > $O/r5e_bench_smallk0.log 2>&1 || exit $?
FM_SMALLK=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > $O/r5e_bench_smallk1.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r5e || exit $?
exit 0
