#!/bin/bash
# r5d: persistent ring fp32 GEMM configs (LDS-DMA / register-staged) vs the default kernel and
# hipBLASLt; native DLRM on the HIP engine; CNN cost-DB calibration (InceptionV3 shard shapes)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 420 python3 -u tools/gemm_f32_lab.py 0,20000,20001,20002,20003,20004,20005,20006,20007 > $O/r5d_lab.jsonl 2> $O/r5d_lab.err || exit $?
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_native_model.py > $O/r5d_native.log 2>&1 || exit $?
cp flexmi/parallel/costdb/mi355x.json $O/costdb_bf16.json
timeout -k 10 300 python3 -u tools/calibrate_costs.py --model inception_v3 --gpus 1 --batch-per-gpu 64 --dtype bf16 --reps 10 --time-budget 240 --out $O/costdb_bf16.json > $O/r5d_cal1.log 2>&1 || exit $?
timeout -k 10 420 python3 -u tools/calibrate_costs.py --model inception_v3 --gpus 2,4,8 --batch-per-gpu 64 --dtype bf16 --reps 10 --time-budget 360 --out $O/costdb_bf16.json > $O/r5d_cal2.log 2>&1 || exit $?
exit 0
