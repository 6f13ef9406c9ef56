#!/bin/bash
# round-4 final check on the committed tree: full GPU suite, smoke, the driver's default bench
# invocation and a 30-step run, step traces (fp32 + bf16)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r5f_gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r5f_smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py > $O/r5f_bench_default.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > $O/r5f_bench.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r5f || exit $?
exit 0
