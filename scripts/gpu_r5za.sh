#!/bin/bash
# r5za: embedding-forward fork delay (the first bottom-MLP layer alone before the gather), A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for rep in 1 2; do
  for dl in 0 1 2; do
    FM_EMB_FWD_DELAY=$dl timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5za_bench_d${dl}_$rep.log 2>&1 || exit $?
  done
done
FM_EMB_FWD_DELAY=1 bash scripts/gpu_profile_step.sh r5za --no-secondary || exit $?
exit 0
