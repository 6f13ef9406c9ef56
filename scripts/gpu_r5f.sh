#!/bin/bash
# r5f: small-K kernels v2 (LDS-staged x, batched loads) standalone + tests, identity colsum
# without the y reads, bench A/B, the step trace; then the second split-bf16 fp32 GEMM form
# (gemm_x3.hip): float64-oracle tests and the DLRM-shape lab against native / hipBLASLt
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 240 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py tests/test_gpu_kernels.py -k "smallk or skinny or linear or act or bias" > $O/r5f_tests.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/bench_smallk.py > $O/r5f_smallk.jsonl 2> $O/r5f_smallk.err || exit $?
FM_SMALLK=0 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5f_bench_smallk0.log 2>&1 || exit $?
FM_SMALLK=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5f_bench_smallk1.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r5f --no-secondary || exit $?
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py > $O/r5f_split_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/gemm_f32_lab.py 0,-2 > $O/r5f_lab.jsonl 2> $O/r5f_lab.err || exit $?
FM_F32_SPLIT=2 FM_DW_LIB=0 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5f_bench_split2.log 2>&1 || exit $?
exit 0
