#!/bin/bash
# r5w: big-tile bf16 GEMM (gemm_x1.hip) tests + lab A/B; embedding tests + overlap equivalence
# (late join); fp32 step A/B of the late join and the backward grid cap; bf16 step with / without x1
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "x1" > $O/r5w_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py -k "overlap" >> $O/r5w_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/gemm_variant_ab.py 0,1024 > $O/r5w_x1_ab.jsonl 2> $O/r5w_x1_ab.err || exit $?
for rep in 1 2; do
  for cfg in "1 0" "0 0" "1 256"; do
    set -- $cfg
    FM_EMB_LATE_JOIN=$1 FM_EMB_BWD_BLOCKS=$2 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5w_bench_l$1_c$2_$rep.log 2>&1 || exit $?
  done
done
for x1 in 1 0; do
  FM_GEMM_X1=$x1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > $O/r5w_bench_x1_$x1.log 2>&1 || exit $?
done
exit 0
