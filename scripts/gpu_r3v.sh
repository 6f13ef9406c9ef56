#!/bin/bash
# conv tile A/B: 8-wave vs 4-wave 128x128 blocks (bench_conv op path), ResNet-50 b64 line each
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for arm in 0 1; do
  FM_CONV_NHWC_4WAVE=$arm timeout -k 10 200 python3 tools/bench_conv.py --net all --path op --reps 20 > $O/r3v_conv_4wave$arm.txt 2>&1 || exit $?
  FM_CONV_NHWC_4WAVE=$arm timeout -k 10 200 python3 apps/train.py resnet50 -b 64 --iterations 20 --graph --dtype bf16 > $O/r3v_resnet_4wave$arm.txt 2>&1 || exit $?
done
# summit_large (small-M GEMMs) and run_random lines after the fused-epilogue 64x64 tiles
for c in summit_large:256 run_random:256; do
  timeout -k 10 300 python3 bench.py --config ${c%%:*} --batch-per-gpu ${c##*:} --steps 20 --warmup 5 >> $O/r3v_ref_lines.jsonl 2>> $O/r3v_ref_lines.err || exit $?
done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py > $O/r3v_fp32_tests.log 2>&1 || exit $?
exit 0
