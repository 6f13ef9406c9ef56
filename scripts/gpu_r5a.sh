#!/bin/bash
# r5a: ring fp32 GEMM (LDS-DMA NS-stage ring) configs vs the default kernel and hipBLASLt, DLRM shapes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u tools/gemm_f32_lab.py 0,20000,20001,20002,20003,20004,20005,20006,20007 > $O/r5a_lab.jsonl 2> $O/r5a_lab.err || exit $?
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > $O/r5a_bench.log 2>&1 || exit $?
exit 0
