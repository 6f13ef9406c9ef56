#!/bin/bash
# Re-entry baseline: full GPU suite, smoke, bench (N=1, fp32 + bf16)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r3k_gpu_suite.log 2>&1 || exit $?
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/r3k_smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 > $O/r3k_bench.log 2>&1 || exit $?
exit 0
