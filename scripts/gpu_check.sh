#!/bin/bash
# One GPU session after a change: GPU test suite, smoke, then an A/B of one environment knob on the
# default bench (two runs per arm, alternating), each step under its own time limit.
# usage: scripts/gpu_check.sh TAG [KNOB "v1 v2"]   e.g. scripts/gpu_check.sh p5 FM_GEMM_DMA "0 1"
set -o pipefail
TAG=$1
KNOB=$2
VALS=$3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/${TAG}_tests.log 2>&1 || { tail -30 $O/${TAG}_tests.log; exit 1; }
tail -2 $O/${TAG}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit $?
if [ -n "$KNOB" ]; then
  for rep in 1 2; do
    for v in $VALS; do
      echo "== $KNOB=$v rep $rep" >> $O/${TAG}_ab.txt
      env $KNOB=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 >> $O/${TAG}_ab.txt 2>&1 || exit $?
    done
  done
  grep -o '^== .*\|"ms_per_step": [0-9.]*' $O/${TAG}_ab.txt
fi
exit 0
