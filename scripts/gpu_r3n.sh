#!/bin/bash
# kernel breakdown of the op-level conv path (NHWC staging) on the ResNet layers
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in r2_3x3 r2_1x1 r5_3x3; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/r3n_$L -o run -- python3 $R/tools/bench_conv.py --net all --layer $L --path op --reps 10 > $O/r3n_$L.log 2>&1 || exit $?
  DB=$(find $O/r3n_$L -name "*results.db" | head -1)
  (cd $R && python3 tools/prof_summary.py $DB 21 > $O/r3n_${L}_kernels.txt 2>&1)
  rm -rf $O/r3n_$L
done
exit 0
