#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench_n1.jsonl 2> gpurun_out/bench_n1.err
