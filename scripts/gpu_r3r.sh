#!/bin/bash
# CNN model kernel summaries after the NHWC conv path (bf16, hipGraph)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in resnet50:64 inception_v3:64 alexnet:256; do
  name=${m%%:*}; b=${m##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/r3r_prof_$name -o run -- python3 $R/apps/train.py $name -b $b --iterations 10 --warmup 2 --graph --dtype bf16 > $O/r3r_prof_$name.log 2>&1 || exit $?
  DB=$(find $O/r3r_prof_$name -name "*results.db" | head -1)
  (cd $R && python3 tools/prof_summary.py $DB 12 > $O/r3r_${name}_b${b}_kernels.txt 2>&1)
  rm -rf $O/r3r_prof_$name
done
exit 0
