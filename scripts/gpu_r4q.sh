#!/bin/bash
# batched W loads in the LDS-staged fused-SGD epilogue: numerics + summit_large lines
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_sgd.py tests/test_gpu_models.py > $O/r4q_tests.log 2>&1 || exit $?
L=$O/r4q_lines.jsonl
: > $L
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config summit_large --batch-per-gpu 256 --steps 40 --warmup 5 --no-dp >> $L 2>> $O/r4q_bench.err || exit $?
done
exit 0
