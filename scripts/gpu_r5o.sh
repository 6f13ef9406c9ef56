#!/bin/bash
# r5o: new defaults (split sched 3, embedding forward cap): whole GPU suite, bench (fp32 + bf16),
# step trace; refresh the fp32 cost DB's DLRM entries (the search prices plans with it)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r5o_gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > $O/r5o_bench_default.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r5o || exit $?
cp flexmi/parallel/costdb/mi355x_fp32.json $O/mi355x_fp32_refresh.json
timeout -k 10 600 python3 -u tools/calibrate_costs.py --model dlrm-mlperf --dtype fp32 --gpus 1,2,4,8 --refresh OP_LINEAR,OP_DOT_INTERACTION,OP_EMBEDDING --reps 5 --time-budget 420 --out $O/mi355x_fp32_refresh.json > $O/r5o_cal_dlrm_fp32.log 2>&1 || exit $?
exit 0
