#!/bin/bash
# conflict-free staging tiles: numerics + CNN lines + stage kernel times
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_nhwc.py tests/test_gpu_conv.py tests/test_gpu_models.py > $O/r4h_tests.log 2>&1 || exit $?
L=$O/r4h_cnn.txt
: > $L
for spec in "alexnet -b 256" "resnet50 -b 64" "resnet50 -b 256" "inception_v3 -b 64" "inception_v3 -b 256"; do
  echo "== $spec --graph bf16" >> $L
  timeout -k 10 240 python3 apps/train.py $spec --iterations 20 --graph --dtype bf16 >> $L 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/r4h_prof -o run -- python3 $R/apps/train.py resnet50 -b 64 --iterations 10 --warmup 2 --graph --dtype bf16 > $O/r4h_prof.log 2>&1 || exit $?
DB=$(find $O/r4h_prof -name "*results.db" | head -1)
(cd $R && python3 tools/prof_summary.py $DB 12 > $O/r4h_resnet50_b64_kernels.txt 2>&1)
rm -rf $O/r4h_prof
exit 0
