#!/bin/bash
# r5g: count / update embedding backward (tests + bench A/B), split-bf16 form 2: 256x128 default
# vs FM_X3_BM=128, schedule A/B (FM_X3_SCHED=1: all fragment reads ahead of the staging pass) on
# the DLRM shapes, bench combos, then the step trace of split 2 + count
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 240 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "embedding" > $O/r5g_emb_tests.log 2>&1 || exit $?
FM_X3_SCHED=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py -k "split2 or orientations" > $O/r5g_split_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/gemm_f32_lab.py 0,-2 > $O/r5g_lab256.jsonl 2> $O/r5g_lab256.err || exit $?
FM_X3_SCHED=1 timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 > $O/r5g_lab256s1.jsonl 2> $O/r5g_lab256s1.err || exit $?
FM_X3_BM=128 FM_X3_SCHED=1 timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 > $O/r5g_lab128s1.jsonl 2> $O/r5g_lab128s1.err || exit $?
for cfg in "0 claim" "0 count" "2 count"; do
  set -- $cfg
  FM_F32_SPLIT=$1 FM_EMB_BWD=$2 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5g_bench_s$1_$2.log 2>&1 || exit $?
done
FM_F32_SPLIT=2 FM_EMB_BWD=count bash scripts/gpu_profile_step.sh r5g --no-secondary || exit $?
exit 0
