#!/bin/bash
# GEMM tuner: forced-configuration numerics first, then measure the table for the bench configs,
# then A/B the table against the heuristics on the default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm_tune.py -x -q --timeout 120 --timeout-method thread \
  > $O/tune_tests.log 2>&1 || { tail -30 $O/tune_tests.log; exit 1; }
tail -1 $O/tune_tests.log
timeout -k 10 600 python3 -u tools/tune_gemm.py --configs "${TUNE_CONFIGS:-mlperf:8192}" --out $O/gemm_mi355x.json \
  --log $O/tune_cands.jsonl > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
tail -3 $O/tune.log
for rep in 1 2; do
  for v in 0 $O/gemm_mi355x.json; do
    echo "== FM_GEMM_TUNE=$v rep $rep" >> $O/tune_ab.txt
    FM_GEMM_TUNE=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 >> $O/tune_ab.txt 2>&1 || exit $?
  done
done
grep -o '^== .*\|"ms_per_step": [0-9.]*' $O/tune_ab.txt
