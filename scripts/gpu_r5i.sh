#!/bin/bash
# r5i: split-bf16 form 2 without the staging selects (loads wait at their use a step later):
# float64-oracle tests, schedule A/B (FM_X3_SCHED 0 / 1 / 2) on the DLRM shapes; count / update
# embedding backward tests; bench combos; step trace of split 2 + count
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
FM_X3_SCHED=2 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py > $O/r5i_split_tests.log 2>&1 || exit $?
for sc in 0 1 2; do
  FM_X3_SCHED=$sc timeout -k 10 300 python3 -u tools/gemm_f32_lab.py 0,-2 > $O/r5i_lab_s$sc.jsonl 2> $O/r5i_lab_s$sc.err || exit $?
done
FM_X3_MODE=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py -k "split2 or orientations" > $O/r5i_split_tests_m1.log 2>&1 || exit $?
FM_X3_MODE=1 timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 > $O/r5i_lab_m1.jsonl 2> $O/r5i_lab_m1.err || exit $?
timeout -k 10 240 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "embedding or skinny" > $O/r5i_emb_tests.log 2>&1 || exit $?
for cfg in "0 claim 0" "0 count 0" "2 count 2" "3 count 2" "3 count 0"; do
  set -- $cfg
  FM_F32_SPLIT=$1 FM_EMB_BWD=$2 FM_X3_SCHED=$3 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5i_bench_s$1_$2_x$3.log 2>&1 || exit $?
done
FM_F32_SPLIT=3 FM_EMB_BWD=count FM_X3_SCHED=2 bash scripts/gpu_profile_step.sh r5i --no-secondary || exit $?
exit 0
