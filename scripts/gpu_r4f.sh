#!/bin/bash
# fused-epilogue split-K: numerics + summit_large lines (fp32 headline + bf16) + fp32 GEMM tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py tests/test_gpu_kernels.py tests/test_gpu_models.py > $O/r4f_tests.log 2>&1 || exit $?
for c in summit_large:256 summit:512; do
  timeout -k 10 300 python3 bench.py --config ${c%%:*} --batch-per-gpu ${c##*:} --steps 20 --warmup 5 >> $O/r4f_ref_lines.jsonl 2>> $O/r4f_ref_lines.err || exit $?
done
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 > $O/r4f_bench.log 2>&1 || exit $?
exit 0
