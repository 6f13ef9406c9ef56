#!/bin/bash
# chunked DLRM tail on MI355X (eager + captured, fp32 + bf16) and the headline bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_pipeline.py > $O/r3g_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 30 --warmup 10 > $O/r3g_bench.txt 2>&1 || exit $?
exit 0
