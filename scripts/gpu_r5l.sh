#!/bin/bash
# r5l: split GEMM with row x k-octet MN staging (no LDS write conflicts): tests, lab (256x128 vs
# 128x128 tiles), PMC bank conflicts of the dW, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py tests/test_gpu_fp32.py > $O/r5l_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 > $O/r5l_lab256.jsonl 2> $O/r5l_lab256.err || exit $?
FM_X3_BM=128 timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 > $O/r5l_lab128.jsonl 2> $O/r5l_lab128.err || exit $?
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5l_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT -d $O/r5l_pmc_dw -o run --output-format csv -- python3 $R/tools/gemm_one.py 8192 1024 1024 dw 20 fp32 > $O/r5l_pmc_dw.log 2>&1 || exit $?
cd $R
python3 tools/pmc_summary.py $(find $O -path "*r5l_pmc_dw*" -name "*counter_collection.csv") --kernel x3v2 > $O/r5l_pmc_dw.txt 2>&1
exit 0
