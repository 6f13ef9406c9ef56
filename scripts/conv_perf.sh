#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k "conv or pool" > gpurun_out/conv_tests.log 2>&1
timeout -k 10 200 python -u tools/bench_conv.py --net all --dtype bf16 > gpurun_out/bench_conv_bf16.txt 2>&1
timeout -k 10 300 python -u apps/train.py alexnet -b 256 --iterations 10 --warmup 3 --graph --dtype bf16 > gpurun_out/alex_line.log 2>&1
bash scripts/pmc_conv.sh conv2 fwd c2f > gpurun_out/pmc_c2f.log 2>&1
