#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp32.py -k skinny > gpurun_out/skinny_tests.log 2>&1
for c in summit_large:256 kaggle_day1:128 criteo_kaggle:256 run_random:256; do
  timeout -k 10 300 python -u bench.py --config ${c%%:*} --batch-per-gpu ${c##*:} --steps 20 --warmup 5 >> gpurun_out/ref_lines.jsonl 2>> gpurun_out/ref_lines.err
done
