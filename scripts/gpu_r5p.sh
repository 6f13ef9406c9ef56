#!/bin/bash
# r5p: 64-way split-K for tiny-tile fp32 dW, 16-deep slab sums, 8-deep skinny backward batches:
# tests, bench, step trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py tests/test_gpu_kernels.py tests/test_gpu_fused_sgd.py tests/test_gpu_models.py > $O/r5p_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/gemm_f32_lab.py 0 "8192,256,128;8192,512,256" > $O/r5p_lab.jsonl 2> $O/r5p_lab.err || exit $?
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5p_bench.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r5p --no-secondary || exit $?
exit 0
