#!/bin/bash
# r5v: embedding tests (atomic and row-block paths) + overlap equivalence (late join); A/B of the
# dense update's late join and of the backward grid cap beside the bottom MLP
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k "embedding" > $O/r5v_tests.log 2>&1 || exit $?
for rep in 1 2; do
  for cfg in "1 0" "0 0" "1 256" "1 512"; do
    set -- $cfg
    FM_EMB_LATE_JOIN=$1 FM_EMB_BWD_BLOCKS=$2 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5v_bench_l$1_c$2_$rep.log 2>&1 || exit $?
  done
done
bash scripts/gpu_profile_step.sh r5v --no-secondary || exit $?
exit 0
