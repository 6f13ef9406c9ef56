#!/bin/bash
# bag-split embedding forward: numerics, summit_large A/B, step timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_models.py > $O/r4n_tests.log 2>&1 || exit $?
L=$O/r4n_ab.jsonl
: > $L
for arm in 1 0 1 0; do
  echo "# summit_large FM_EMB_FWD_SPLIT=$arm" >> $L
  FM_EMB_FWD_SPLIT=$arm timeout -k 10 300 python3 bench.py --config summit_large --batch-per-gpu 256 --steps 40 --warmup 5 --no-dp >> $L 2>> $O/r4n_bench.err || exit $?
done
bash scripts/gpu_profile_step.sh r4n_sl --config summit_large --batch-per-gpu 256 --no-dp || exit $?
exit 0
