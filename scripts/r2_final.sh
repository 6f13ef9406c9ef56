#!/bin/bash
# end-of-session validation: smoke(), full GPU suite, headline bench, rocprof of the fp32 step
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench_n1.jsonl 2> gpurun_out/bench_n1.err
bash scripts/prof_bench.sh prof_r2c
python tools/prof_summary.py $(ls gpurun_out/prof_r2c/*results.db gpurun_out/prof_r2c/*/*results.db 2>/dev/null | head -1) 27 > gpurun_out/prof_r2c_kernels.txt
