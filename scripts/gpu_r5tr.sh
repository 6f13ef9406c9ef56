#!/bin/bash
# wave-private LDS backward for small tables up to FM_EMB_TINY_ROWS rows (16 / 40 / 64): embedding
# tests at 64, isolated small-table bench, MLPerf fp32 step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
FM_EMB_TINY_ROWS=64 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "embedding" > $O/r5tr_tests.log 2>&1 || exit $?
for tr in 16 40 64; do
  FM_EMB_TINY_ROWS=$tr timeout -k 10 120 python3 -u tools/bench_emb_bwd.py "155,108,63,36,14,10,4,3" >> $O/r5tr_emb.jsonl 2>> $O/r5tr_emb.err || exit $?
done
for rep in 1 2; do
  for tr in 16 40 64; do
    FM_EMB_TINY_ROWS=$tr timeout -k 10 300 python3 -u bench.py --steps 40 --warmup 5 --no-secondary > $O/r5tr_bench_t${tr}_$rep.log 2>&1 || exit $?
  done
done
exit 0
