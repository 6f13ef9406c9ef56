#!/bin/bash
# NHWC conv after the origin table + fused G staging: numerics, op timings, kernel breakdown
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_nhwc.py tests/test_gpu_conv.py tests/test_gpu_conv_phase.py > $O/r3p_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/bench_conv.py --net all --path op --reps 20 > $O/r3p_conv_op_nhwc.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for L in r2_3x3 r2_1x1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/r3p_$L -o run -- python3 $R/tools/bench_conv.py --net all --layer $L --path op --reps 10 > $O/r3p_$L.log 2>&1 || exit $?
  DB=$(find $O/r3p_$L -name "*results.db" | head -1)
  (cd $R && python3 tools/prof_summary.py $DB 11 > $O/r3p_${L}_kernels.txt 2>&1)
  rm -rf $O/r3p_$L
done
exit 0
