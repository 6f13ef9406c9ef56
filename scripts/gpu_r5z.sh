#!/bin/bash
# r5z: max-pool parity-phase scatter (tests + AlexNet A/B); fp32 step with the split-MFMA
# interaction forward by default; smoke
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pool_negpad.py tests/test_gpu_fp32.py -k "pool or dot" > $O/r5z_tests.log 2>&1 || exit $?
for ph in 0 1 0 1; do
  FM_POOL_SCATTER_PHASES=$ph timeout -k 10 300 python3 -u apps/train.py alexnet -b 256 --iterations 20 --warmup 3 --graph --dtype bf16 >> $O/r5z_alexnet_ph$ph.log 2>&1 || exit $?
done
for rep in 1 2; do
  for dl in 0 1 2; do
    FM_EMB_FWD_DELAY=$dl timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5z_bench_d${dl}_$rep.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r5z_smoke.log 2>&1 || exit $?
exit 0
