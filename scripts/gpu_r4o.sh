#!/bin/bash
# MLPerf headline A/B: this tree vs the pre-session build (worktree _old at 6aa9cb7), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
L=$O/r4o_ab.jsonl
: > $L
for arm in new old new old; do
  echo "# $arm" >> $L
  if [ $arm = old ]; then D=$R/_old; else D=$R; fi
  (cd $D && timeout -k 10 300 python3 bench.py --steps 60 --warmup 10 --no-dp >> $L 2>> $O/r4o_bench.err) || exit $?
done
exit 0
