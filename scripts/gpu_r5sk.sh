#!/bin/bash
# smallk dW rows per partial block (64 / 128 / 256): tests, kernel lab, step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for rw in 64 128 256; do
  FM_SK_DW_ROWS=$rw timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py -k "smallk" >> $O/r5sk_tests.log 2>&1 || exit $?
  FM_SK_DW_ROWS=$rw timeout -k 10 200 python3 -u tools/bench_smallk.py "8192,16,512" >> $O/r5sk_lab_$rw.jsonl 2>> $O/r5sk_lab.err || exit $?
done
for rep in 1 2; do
  for rw in 64 128 256; do
    FM_SK_DW_ROWS=$rw timeout -k 10 300 python3 -u bench.py --steps 40 --warmup 5 --no-secondary > $O/r5sk_bench_r${rw}_$rep.log 2>&1 || exit $?
  done
done
exit 0
