#!/bin/bash
# fp32 split-bf16 GEMM: numerics vs float64 / native, timings vs native + hipBLASLt, DLRM step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py > $O/r4c_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_f32_split.py > $O/r4c_gemm.jsonl 2>&1 || exit $?
bash scripts/gpu_ab_bench.sh r4c - FM_F32_SPLIT=1 - FM_F32_SPLIT=1 || exit $?
exit 0
