#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/cnn_lines.log
for dt in bf16 fp32; do
  for m in "alexnet -b 256" "resnet50 -b 64" "inception_v3 -b 64"; do
    echo "== $m $dt" >> gpurun_out/cnn_lines.log
    timeout -k 10 300 python -u apps/train.py $m --iterations 10 --warmup 3 --graph --dtype $dt >> gpurun_out/cnn_lines.log 2>&1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn50 -o rn -- python apps/train.py resnet50 -b 64 --iterations 5 --warmup 2 --dtype bf16 > gpurun_out/prof_rn50.log 2>&1
