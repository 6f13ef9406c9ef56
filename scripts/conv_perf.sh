#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k "conv or pool" > gpurun_out/conv_tests.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py -k "alexnet or resnet or inception or cnn or zoo" > gpurun_out/cnn_model_tests.log 2>&1
timeout -k 10 300 python -u apps/train.py alexnet -b 256 --iterations 10 --warmup 3 --graph --dtype bf16 > gpurun_out/alex_line.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_alex -o alex -- python apps/train.py alexnet -b 256 --iterations 5 --warmup 2 --dtype bf16 > gpurun_out/prof_alex.log 2>&1
