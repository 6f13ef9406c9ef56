#!/bin/bash
# r5h: split-bf16 form 2 without the staging selects (loads wait at their use a step later):
# float64-oracle tests, schedule A/B (FM_X3_SCHED 0 / 1 / 2) on the DLRM shapes, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
FM_X3_SCHED=2 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py > $O/r5h_split_tests.log 2>&1 || exit $?
for sc in 0 1 2; do
  FM_X3_SCHED=$sc timeout -k 10 300 python3 -u tools/gemm_f32_lab.py 0,-2 > $O/r5h_lab_s$sc.jsonl 2> $O/r5h_lab_s$sc.err || exit $?
done
for sc in 0 2; do
  FM_F32_SPLIT=2 FM_X3_SCHED=$sc timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5h_bench_s$sc.log 2>&1 || exit $?
done
exit 0
