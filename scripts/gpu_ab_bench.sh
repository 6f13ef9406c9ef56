#!/bin/bash
# A/B of environment knobs on the N=1 bench: each arm is one full bench.py run (fp32 + bf16)
# usage: scripts/gpu_ab_bench.sh TAG "ENV=.. ENV2=.." "ENV=.." ...   (use "-" for the default arm)
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
: > $O/${TAG}_ab.txt
i=0
for arm in "$@"; do
  i=$((i+1))
  envs=""
  [ "$arm" != "-" ] && envs="$arm"
  echo "== arm $i: ${envs:-default}" >> $O/${TAG}_ab.txt
  env $envs timeout -k 10 240 python3 $R/bench.py --steps 50 --warmup 10 > $O/${TAG}_arm$i.log 2>&1 || exit $?
  grep '^{' $O/${TAG}_arm$i.log >> $O/${TAG}_ab.txt
done
exit 0
