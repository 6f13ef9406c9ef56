#!/bin/bash
# r5t: isolate the row-block embedding backward: whole small-table set and subsets, on / off
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for rb in 0 1; do
  for set in "" "7420,7120,2208,1543" "976" "155,108,63,36" "14,10,4,3"; do
    FM_EMB_ROWBLOCK=$rb timeout -k 10 120 python3 -u tools/bench_emb_bwd.py "$set" >> $O/r5t_emb.jsonl 2>> $O/r5t_emb.err || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/r5t_prof -o run -- python3 $R/tools/bench_emb_bwd.py "" 8192 5 > $O/r5t_prof.log 2>&1 || exit $?
exit 0
