#!/bin/bash
# r5u: row-block embedding backward with wave-owned rows (no LDS float atomics): tests, isolated
# table sets on / off, then the step A/B if the isolated numbers win
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "embedding" > $O/r5u_tests.log 2>&1 || exit $?
for rb in 0 1; do
  for set in "" "7420,7120,2208,1543" "976" "155,108,63,36" "14,10,4,3"; do
    FM_EMB_ROWBLOCK=$rb timeout -k 10 120 python3 -u tools/bench_emb_bwd.py "$set" >> $O/r5u_emb.jsonl 2>> $O/r5u_emb.err || exit $?
  done
done
for rb in 0 1 0 1; do
  FM_EMB_ROWBLOCK=$rb timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary >> $O/r5u_bench_rb$rb.log 2>&1 || exit $?
done
exit 0
