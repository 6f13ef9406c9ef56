#!/bin/bash
# r5v: embedding tests (atomic and row-block paths); backward grid cap beside the bottom MLP (A/B)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "embedding" > $O/r5v_tests.log 2>&1 || exit $?
for rep in 1 2; do
  for cap in 0 128 256 512; do
    FM_EMB_BWD_BLOCKS=$cap timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5v_bench_c${cap}_$rep.log 2>&1 || exit $?
  done
done
exit 0
