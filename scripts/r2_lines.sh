#!/bin/bash
# Round-2 measurement batch: embedding-group calibration (fp32 + bf16 DBs), NMT reference config
# and the Summit / Kaggle-day-1 DLRM bench lines.  Every GPU step has its own time limit.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
cp flexmi/parallel/costdb/mi355x_fp32.json gpurun_out/mi355x_fp32.json
cp flexmi/parallel/costdb/mi355x.json gpurun_out/mi355x_bf16.json
timeout -k 10 300 python -u tools/calibrate_costs.py --dtype fp32 --gpus 1 --out gpurun_out/mi355x_fp32.json > gpurun_out/cal_fp32.log 2>&1
timeout -k 10 300 python -u tools/calibrate_costs.py --dtype bf16 --gpus 1 --out gpurun_out/mi355x_bf16.json > gpurun_out/cal_bf16.log 2>&1
for dt in fp32 bf16; do
  timeout -k 10 240 python -u apps/train.py nmt -b 64 --iterations 20 --warmup 3 --graph --dtype $dt >> gpurun_out/nmt_ref.log 2>&1
done
for c in summit:512 summit_large:256 kaggle_day1:128 criteo_kaggle:256 run_random:256; do
  timeout -k 10 300 python -u bench.py --config ${c%%:*} --batch-per-gpu ${c##*:} --steps 20 --warmup 5 >> gpurun_out/ref_lines.jsonl 2>> gpurun_out/ref_lines.err
done
