#!/bin/bash
# numerics after batched-load pooling / staging; A/B of staging width threshold and wgrad split target
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pool_negpad.py tests/test_gpu_conv_nhwc.py tests/test_gpu_conv.py tests/test_gpu_models.py > $O/r3y_tests.log 2>&1 || exit $?
L=$O/r3y_ab.txt
: > $L
for arm in "-" "FM_STAGE_FLAT_BELOW=64" "FM_STAGE_FLAT_BELOW=128" "FM_CONV_WGRAD_BLOCKS=256" "FM_CONV_WGRAD_BLOCKS=1024"; do
  envs=""; [ "$arm" != "-" ] && envs="$arm"
  for spec in "inception_v3 -b 64" "resnet50 -b 64"; do
    echo "== ${envs:-default} $spec" >> $L
    env $envs timeout -k 10 240 python3 apps/train.py $spec --iterations 20 --graph --dtype bf16 2>&1 | grep THROUGHPUT >> $L || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for m in resnet50:64 inception_v3:64; do
  name=${m%%:*}; b=${m##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/r3y_prof_$name -o run -- python3 $R/apps/train.py $name -b $b --iterations 10 --warmup 2 --graph --dtype bf16 > $O/r3y_prof_$name.log 2>&1 || exit $?
  DB=$(find $O/r3y_prof_$name -name "*results.db" | head -1)
  (cd $R && python3 tools/prof_summary.py $DB 12 > $O/r3y_${name}_b${b}_kernels.txt 2>&1)
  rm -rf $O/r3y_prof_$name
done
exit 0
