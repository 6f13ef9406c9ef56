#!/bin/bash
# multi-plane band pooling: numerics + CNN lines + Inception kernel summary
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pool_negpad.py tests/test_gpu_conv_nhwc.py tests/test_gpu_conv.py tests/test_gpu_models.py tests/test_gpu_kernels.py > $O/r4a_tests.log 2>&1 || exit $?
L=$O/r4a_cnn.txt
: > $L
for spec in "alexnet -b 256" "resnet50 -b 64" "resnet50 -b 256" "inception_v3 -b 64" "inception_v3 -b 256"; do
  echo "== $spec --graph bf16" >> $L
  timeout -k 10 240 python3 apps/train.py $spec --iterations 20 --graph --dtype bf16 >> $L 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
for m in inception_v3:64 alexnet:256; do
  name=${m%%:*}; b=${m##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/r4a_prof_$name -o run -- python3 $R/apps/train.py $name -b $b --iterations 10 --warmup 2 --graph --dtype bf16 > $O/r4a_prof_$name.log 2>&1 || exit $?
  DB=$(find $O/r4a_prof_$name -name "*results.db" | head -1)
  (cd $R && python3 tools/prof_summary.py $DB 12 > $O/r4a_${name}_b${b}_kernels.txt 2>&1)
  rm -rf $O/r4a_prof_$name
done
exit 0
