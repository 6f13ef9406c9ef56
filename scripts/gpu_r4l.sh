#!/bin/bash
# fused SGD after the vector segmented update: tests, mlperf A/B (alternating arms), mlperf step timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_sgd.py tests/test_gpu_pool_negpad.py > $O/r4l_tests.log 2>&1 || exit $?
L=$O/r4l_ab.jsonl
: > $L
for arm in 1 0 1 0; do
  echo "# mlperf FM_FUSED_SGD=$arm" >> $L
  FM_FUSED_SGD=$arm timeout -k 10 300 python3 bench.py --steps 60 --warmup 10 --no-dp >> $L 2>> $O/r4l_bench.err || exit $?
done
bash scripts/gpu_profile_step.sh r4l_ml --no-dp || exit $?
exit 0
