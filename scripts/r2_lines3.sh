#!/bin/bash
# reference-config bench lines + NMT + CNN lines with the current kernels (8-wave GEMMs)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ref_lines3.jsonl gpurun_out/nmt_ref3.log gpurun_out/cnn_lines3.log
for c in summit:512 summit_large:256 kaggle_day1:128 criteo_kaggle:256 run_random:256; do
  timeout -k 10 300 python -u bench.py --config ${c%%:*} --batch-per-gpu ${c##*:} --steps 20 --warmup 5 >> gpurun_out/ref_lines3.jsonl 2>> gpurun_out/ref_lines3.err
done
for dt in fp32 bf16; do
  timeout -k 10 240 python -u apps/train.py nmt -b 64 --iterations 20 --warmup 3 --graph --dtype $dt >> gpurun_out/nmt_ref3.log 2>&1
done
for dt in bf16 fp32; do
  for m in "alexnet -b 256" "resnet50 -b 64" "inception_v3 -b 64"; do
    echo "== $m $dt" >> gpurun_out/cnn_lines3.log
    timeout -k 10 300 python -u apps/train.py $m --iterations 10 --warmup 3 --graph --dtype $dt >> gpurun_out/cnn_lines3.log 2>&1
  done
done
