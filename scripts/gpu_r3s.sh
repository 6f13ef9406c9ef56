#!/bin/bash
# NHWC conv: numerics, op timings, CNN model lines (bf16, hipGraph)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_nhwc.py tests/test_gpu_conv.py tests/test_gpu_conv_phase.py > $O/r3s_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/bench_conv.py --net all --path op --reps 20 > $O/r3s_conv_op_nhwc.txt 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_models.py tests/test_gpu_kernels.py > $O/r3s_models.log 2>&1 || exit $?
L=$O/r3s_cnn.txt
: > $L
for spec in "alexnet -b 256" "resnet50 -b 64" "resnet50 -b 256" "inception_v3 -b 64" "inception_v3 -b 256"; do
  echo "== $spec --graph bf16" >> $L
  timeout -k 10 240 python3 apps/train.py $spec --iterations 20 --graph --dtype bf16 >> $L 2>&1 || exit $?
done
exit 0
