#!/bin/bash
# r5x: big-tile bf16 GEMM with 64-deep stages (tests + lab A/B vs the register-staged kernel);
# embedding backward grid cap with the regular join (fp32 step A/B)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "x1" > $O/r5x_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/gemm_variant_ab.py 0,1024 > $O/r5x_x1_ab.jsonl 2> $O/r5x_x1_ab.err || exit $?
for rep in 1 2; do
  for cap in 0 256 512; do
    FM_EMB_BWD_BLOCKS=$cap timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5x_bench_c${cap}_$rep.log 2>&1 || exit $?
  done
done
exit 0
