#!/bin/bash
# claim (owner-computes) path for mid-size tables: FM_EMB_CLAIM_RATIO 1 (rows > lookups) vs 0.5 / 0.2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for rep in 1 2; do
  for cr in 1 0.5 0.2; do
    FM_EMB_CLAIM_RATIO=$cr timeout -k 10 300 python3 -u bench.py --steps 40 --warmup 5 --no-secondary > $O/r5cr_bench_cr${cr}_$rep.log 2>&1 || exit $?
  done
done
exit 0
