#!/bin/bash
# r5c: MFMA probe (register staging vs LDS-DMA, HBM vs L2 sources); embedding-into-interaction
# gather kernels + model equivalence; DLRM bench A/B with the fusion on/off
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/bin/mfma_probe 4000 > $O/r5c_probe.jsonl 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py -k "dot_interaction or gather or overlap" > $O/r5c_tests.log 2>&1 || exit $?
for arm in 1 0 1 0; do
  echo "== FM_EMB_GATHER=$arm" >> $O/r5c_bench.txt
  FM_EMB_GATHER=$arm timeout -k 10 200 python3 -u bench.py --steps 30 --warmup 5 --no-secondary >> $O/r5c_bench.txt 2>&1 || exit $?
done
exit 0
