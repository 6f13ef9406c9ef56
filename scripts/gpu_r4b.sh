#!/bin/bash
# checkpoint: full GPU suite, smoke, bench (N=1), DLRM step profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r4b_gpu_suite.log 2>&1 || exit $?
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/r4b_smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 > $O/r4b_bench.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r4b_dlrm || exit $?
exit 0
