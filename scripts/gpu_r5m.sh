#!/bin/bash
# r5m: split GEMM schedule 3 (loads two steps ahead) vs 2; embedding-forward grid cap beside the
# bottom MLP; bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
FM_X3_SCHED=3 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32_split.py > $O/r5m_tests.log 2>&1 || exit $?
for sc in 2 3; do
  FM_X3_SCHED=$sc timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 > $O/r5m_lab_s$sc.jsonl 2> $O/r5m_lab_s$sc.err || exit $?
done
for cfg in "2 2048" "3 2048" "3 256" "3 128" "3 64"; do
  set -- $cfg
  FM_X3_SCHED=$1 FM_EMB_FWD_BLOCKS=$2 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5m_bench_s$1_e$2.log 2>&1 || exit $?
done
exit 0
