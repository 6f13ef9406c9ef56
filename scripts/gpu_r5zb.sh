#!/bin/bash
# r5zb: embedding forward with 4 samples' loads in flight per lane (bag 1): tests, then the step
# A/B over the per-table grid cap (smaller grids leave CU slots to the bottom MLP beside it)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k "embedding" > $O/r5zb_tests.log 2>&1 || exit $?
for rep in 1 2; do
  for cap in 256 128 64; do
    FM_EMB_FWD_BLOCKS=$cap timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5zb_bench_c${cap}_$rep.log 2>&1 || exit $?
  done
done
FM_EMB_FWD_BLOCKS=128 bash scripts/gpu_profile_step.sh r5zb --no-secondary || exit $?
exit 0
