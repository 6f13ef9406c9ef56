#!/bin/bash
# One GPU session: plain bench line, then a rocprofv3 kernel trace of the same bench, summarised
# on the box (per-kernel totals + the fp32 and bf16 step timelines).
# usage: scripts/gpu_profile_step.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 "$@" > $O/${TAG}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${TAG}_prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 "$@" > $O/${TAG}_prof.log 2>&1 || exit $?
DB=$(find $O/${TAG}_prof -name "*results.db" | head -1)
cd $R
python3 tools/prof_summary.py $DB 27 > $O/${TAG}_kernels.txt 2>&1
python3 tools/prof_step.py $DB "fm_emb_fwd_multi<float|fm_emb_fwd_split<float" > $O/${TAG}_step_fp32.txt 2>&1
python3 tools/prof_step.py $DB "fm_emb_fwd_multi<unsigned short|fm_emb_fwd_split<unsigned short" > $O/${TAG}_step_bf16.txt 2>&1
rm -f $DB
exit 0
