#!/bin/bash
# r5j: new defaults (split policy 3, de-phased x3 schedule, batched split-K reduces): the whole
# GPU suite, the bench (fp32 + bf16 secondary), the step trace; register-split x3 form A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r5j_gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > $O/r5j_bench_default.log 2>&1 || exit $?
FM_X3_MODE=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py -k "split2 or orientations" > $O/r5j_split_tests_m1.log 2>&1 || exit $?
FM_X3_MODE=1 timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 > $O/r5j_lab_m1.jsonl 2> $O/r5j_lab_m1.err || exit $?
bash scripts/gpu_profile_step.sh r5j --no-secondary || exit $?
exit 0
