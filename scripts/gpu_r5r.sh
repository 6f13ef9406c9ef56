#!/bin/bash
# r5r: after removing the spilling ablation knob: GPU suite, lab, bench x2 (fp32 + bf16), trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r5r_gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/gemm_f32_lab.py 0,-2 > $O/r5r_lab.jsonl 2> $O/r5r_lab.err || exit $?
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > $O/r5r_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5r_bench2.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r5r --no-secondary || exit $?
exit 0
