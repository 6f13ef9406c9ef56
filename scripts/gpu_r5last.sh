#!/bin/bash
# last check of the committed tree (tiny-table threshold 64, claim ratio 0.2): full GPU suite,
# smoke, default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r5last_gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r5last_smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py > $O/r5last_bench.log 2>&1 || exit $?
exit 0
