#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k "conv or pool" > gpurun_out/conv_tests.log 2>&1
rm -f gpurun_out/cnn_lines.log
for m in "alexnet -b 256" "resnet50 -b 64" "inception_v3 -b 64"; do
  timeout -k 10 300 python -u apps/train.py $m --iterations 10 --warmup 3 --graph --dtype bf16 >> gpurun_out/cnn_lines.log 2>&1
done
timeout -k 10 300 python -u apps/train.py alexnet -b 256 --iterations 10 --warmup 3 --graph --dtype fp32 >> gpurun_out/cnn_lines.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_alex -o alex -- python apps/train.py alexnet -b 256 --iterations 5 --warmup 2 --dtype bf16 > gpurun_out/prof_alex.log 2>&1
