#!/bin/bash
# claim ratio 0.2 (default) vs 0.1 (the 976- and 1543-row tables join the owner-computes path)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for rep in 1 2; do
  for cr in 0.2 0.1; do
    FM_EMB_CLAIM_RATIO=$cr timeout -k 10 300 python3 -u bench.py --steps 40 --warmup 5 --no-secondary > $O/r5cr3_bench_cr${cr}_$rep.log 2>&1 || exit $?
  done
done
exit 0
