#!/bin/bash
# fused dW-GEMM + SGD: numerics, model tests, summit_large / mlperf lines with the fusion on/off,
# summit_large step timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_sgd.py tests/test_gpu_models.py tests/test_gpu_fp32.py > $O/r4i_tests.log 2>&1 || exit $?
L=$O/r4i_lines.jsonl
: > $L
for cfg in summit_large:256 mlperf:8192; do
  for f in 1 0; do
    echo "# $cfg FM_FUSED_SGD=$f" >> $L
    FM_FUSED_SGD=$f timeout -k 10 300 python3 bench.py --config ${cfg%%:*} --batch-per-gpu ${cfg##*:} --steps 30 --warmup 5 --no-dp >> $L 2>> $O/r4i_bench.err || exit $?
  done
done
for f in 1 0; do
  echo "== alexnet -b 256 FM_FUSED_SGD=$f" >> $O/r4i_cnn.txt
  FM_FUSED_SGD=$f timeout -k 10 240 python3 apps/train.py alexnet -b 256 --iterations 20 --graph --dtype bf16 >> $O/r4i_cnn.txt 2>&1 || exit $?
done
bash scripts/gpu_profile_step.sh r4i_sl --config summit_large --batch-per-gpu 256 --no-dp || exit $?
exit 0
