#!/bin/bash
# fp16 two-plane split (FM_F32_SPLIT=4) vs the bf16 three-plane split (3): split-GEMM numerics, then
# the DLRM step A/B (30 steps, alternating) and a kernel trace of the F16 step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fp32_split.py -x -q --timeout 120 --timeout-method thread > $O/split_tests.log 2>&1 || { tail -30 $O/split_tests.log; exit 1; }
tail -1 $O/split_tests.log
timeout -k 10 300 python3 -u tools/f16x3_lab.py > $O/f16lab3.jsonl 2>&1 || exit $?
for rep in 1 2; do
  for v in 3 4; do
    echo "== FM_F32_SPLIT=$v rep $rep" >> $O/ab_f16b.txt
    FM_F32_SPLIT=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary >> $O/ab_f16b.txt 2>&1 || exit $?
  done
done
grep -o '^== .*\|"ms_per_step": [0-9.]*' $O/ab_f16b.txt
FM_F32_SPLIT=4 bash scripts/gpu_profile_step.sh r7c --no-secondary
