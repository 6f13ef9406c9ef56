#!/bin/bash
# fused SGD compiled into its own GEMM instantiations: numerics + MLPerf A/B vs the pre-session
# build (worktree _old at 6aa9cb7) + summit_large line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_sgd.py tests/test_gpu_fp32.py > $O/r4p_tests.log 2>&1 || exit $?
L=$O/r4p_ab.jsonl
: > $L
for arm in new old new old; do
  echo "# $arm" >> $L
  if [ $arm = old ]; then D=$R/_old; else D=$R; fi
  (cd $D && timeout -k 10 300 python3 bench.py --steps 60 --warmup 10 --no-dp >> $L 2>> $O/r4p_bench.err) || exit $?
done
echo "# summit_large new" >> $L
timeout -k 10 300 python3 bench.py --config summit_large --batch-per-gpu 256 --steps 40 --warmup 5 --no-dp >> $L 2>> $O/r4p_bench.err || exit $?
exit 0
