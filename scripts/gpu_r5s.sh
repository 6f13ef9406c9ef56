#!/bin/bash
# r5s: row-block ownership embedding backward (no global atomics for the 3..8192-row tables):
# embedding tests, bench A/B against the atomic / tiny kernels (interleaved), step trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "embedding" > $O/r5s_tests.log 2>&1 || exit $?
for rb in 0 1 0 1; do
  FM_EMB_ROWBLOCK=$rb timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary >> $O/r5s_bench_rb$rb.log 2>&1 || exit $?
done
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > $O/r5s_bench_both.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r5s --no-secondary || exit $?
exit 0
