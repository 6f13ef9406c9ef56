#!/bin/bash
# stream priority A/B: main (MLP) stream high priority vs both default
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for rep in 1 2; do
  for p in 0 1; do
    FM_STREAM_PRIO=$p timeout -k 10 300 python3 -u bench.py --steps 40 --warmup 5 --no-secondary > $O/r5p_bench_prio${p}_$rep.log 2>&1 || exit $?
  done
done
FM_STREAM_PRIO=1 bash scripts/gpu_profile_step.sh r5prio --no-secondary || exit $?
exit 0
