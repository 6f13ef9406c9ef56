#!/bin/bash
# end-of-session validation: full GPU suite, smoke, default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/r4j_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r4j_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/r4j_bench.jsonl 2> $O/r4j_bench.err || exit $?
exit 0
