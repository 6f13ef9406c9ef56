#!/bin/bash
# NHWC-staged conv: numerics (new + existing conv tests), per-layer timings raw NCHW vs op path
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_nhwc.py > $O/r3m_nhwc_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_conv_phase.py tests/test_gpu_pool_negpad.py > $O/r3m_conv_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/bench_conv.py --net all --path op --reps 20 > $O/r3m_conv_op_nhwc.txt 2>&1 || exit $?
FM_CONV_NHWC=0 timeout -k 10 200 python3 tools/bench_conv.py --net all --path op --reps 20 > $O/r3m_conv_op_nchw.txt 2>&1 || exit $?
exit 0
