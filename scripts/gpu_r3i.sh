#!/bin/bash
# per-layer conv timings (current kernels) + refresh of the fp32 cost DB's DLRM entries
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python3 tools/bench_conv.py --net all --dtype bf16 > $O/r3i_conv_bf16.txt 2>&1 || exit $?
cp flexmi/parallel/costdb/mi355x_fp32.json $O/mi355x_fp32_r3i.json
timeout -k 10 600 python3 -u tools/calibrate_costs.py --dtype fp32 --gpus 1,2,4,8 --refresh OP_LINEAR,OP_DOT_INTERACTION,OP_EMBEDDING --time-budget 420 --out $O/mi355x_fp32_r3i.json > $O/r3i_calib.log 2>&1 || exit $?
exit 0
