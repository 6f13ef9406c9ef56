#!/bin/bash
# refresh the fp32 cost DB's DLRM GEMM / interaction entries after kernel changes
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
cp flexmi/parallel/costdb/mi355x_fp32.json gpurun_out/mi355x_fp32_refresh.json
timeout -k 10 800 python -u tools/calibrate_costs.py --model dlrm-mlperf --dtype fp32 --gpus 1,2,4,8 --refresh OP_LINEAR,OP_DOT_INTERACTION --reps 5 --time-budget 600 --out gpurun_out/mi355x_fp32_refresh.json > gpurun_out/cal_dlrm_fp32.log 2>&1
