#!/bin/bash
# per-layer measured conv forms: numerics, then CNN throughput with FM_CONV_TUNE 0 / 1 (alternating)
# and the AlexNet kernel summary with the tuner on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv_tune.py tests/test_gpu_conv_nhwc.py tests/test_gpu_conv.py tests/test_gpu_conv_phase.py -x -q --timeout 120 --timeout-method thread > $O/conv_tests.log 2>&1 || { tail -30 $O/conv_tests.log; exit 1; }
tail -1 $O/conv_tests.log
L=$O/ab_conv_tune.txt
: > $L
for rep in 1 2; do
  for v in 0 1; do
    for m in "alexnet -b 256" "resnet50 -b 64"; do
      echo "== FM_CONV_TUNE=$v $m rep $rep" >> $L
      FM_CONV_TUNE=$v timeout -k 10 300 python3 apps/train.py $m --iterations 20 --graph --dtype bf16 >> $L 2>&1 || exit $?
    done
  done
done
grep -o '^== .*\|THROUGHPUT = [0-9.]*' $L
grep "conv-tune" $L | sort | uniq | head -40
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/ct_prof -o run -- python3 $R/apps/train.py alexnet -b 256 --iterations 10 --warmup 2 --graph --dtype bf16 > $R/$O/ct_prof.log 2>&1 || exit $?
DB=$(find $R/$O/ct_prof -name "*results.db" | head -1)
(cd $R && python3 tools/prof_summary.py $DB 14 > $O/r7_alexnet_b256_kernels.txt 2>&1)
rm -rf $R/$O/ct_prof
exit 0
