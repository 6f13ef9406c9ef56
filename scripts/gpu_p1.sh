#!/bin/bash
# p1: plane GEMM (gemm_pl.hip) lab vs the in-kernel split kernel and hipBLASLt; fp32 split tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/gemm_pl_lab.py > $O/p1_lab.jsonl 2> $O/p1_lab.err || exit $?
timeout -k 10 300 python3 -u tools/gemm_pl_lab.py "8192,1024,1024" --emit > $O/p1_lab_emit.jsonl 2>> $O/p1_lab.err || exit $?
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py tests/test_gpu_fp32.py > $O/p1_tests.log 2>&1 || exit $?
exit 0
