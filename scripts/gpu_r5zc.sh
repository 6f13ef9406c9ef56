#!/bin/bash
# r5zc: embedding forward sample unroll (SU) on / off x grid cap, interleaved in one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for rep in 1 2; do
  for cfg in "0 256" "1 256" "1 128"; do
    set -- $cfg
    FM_EMB_FWD_SU=$1 FM_EMB_FWD_BLOCKS=$2 timeout -k 10 300 python3 -u bench.py --steps 40 --warmup 5 --no-secondary > $O/r5zc_bench_su$1_c$2_$rep.log 2>&1 || exit $?
  done
done
exit 0
