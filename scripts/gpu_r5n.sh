#!/bin/bash
# r5n: split GEMM with row x k-octet MN staging + schedule 3 (loads two steps ahead): tests, lab
# (sched 2 vs 3, 128x128 tiles), dW PMC; embedding-forward grid cap beside the bottom MLP; bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
FM_X3_SCHED=3 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py tests/test_gpu_fp32.py > $O/r5n_tests.log 2>&1 || exit $?
for sc in 2 3; do
  FM_X3_SCHED=$sc timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 > $O/r5n_lab_s$sc.jsonl 2> $O/r5n_lab_s$sc.err || exit $?
done
FM_X3_BM=128 timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 > $O/r5n_lab128.jsonl 2> $O/r5n_lab128.err || exit $?
for cfg in "2 2048" "3 2048" "3 256" "3 64"; do
  set -- $cfg
  FM_X3_SCHED=$1 FM_EMB_FWD_BLOCKS=$2 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5n_bench_s$1_e$2.log 2>&1 || exit $?
done
FM_X3_SCHED=3 FM_FUSED_SGD_MIN=1 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5n_bench_s3_fusedsgd_all.log 2>&1 || exit $?
FM_X3_SCHED=3 FM_FUSED_SGD_MIN=262144 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5n_bench_s3_fusedsgd_256k.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT -d $O/r5n_pmc_dw -o run --output-format csv -- python3 $R/tools/gemm_one.py 8192 1024 1024 dw 20 fp32 > $O/r5n_pmc_dw.log 2>&1 || exit $?
cd $R
python3 tools/pmc_summary.py $(find $O -path "*r5n_pmc_dw*" -name "*counter_collection.csv") --kernel x3v2 > $O/r5n_pmc_dw.txt 2>&1
exit 0
