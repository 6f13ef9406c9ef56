#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
cp flexmi/parallel/costdb/mi355x_fp32.json gpurun_out/mi355x_fp32_nmt.json
timeout -k 10 700 python -u tools/calibrate_costs.py --model nmt --dtype fp32 --gpus 1,2,4 --batch-per-gpu 64 --time-budget 600 --reps 5 --out gpurun_out/mi355x_fp32_nmt.json > gpurun_out/cal_nmt.log 2>&1
