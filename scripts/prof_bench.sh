#!/bin/bash
# rocprofv3 kernel trace of bench.py (N=1) into gpurun_out/<tag>; extra env passed through.
# usage: scripts/prof_bench.sh TAG [bench args...]
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 "$@" > $GRAFT_REPO_ROOT/gpurun_out/$TAG.log 2>&1
