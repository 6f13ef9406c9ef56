#!/bin/bash
# CNN throughput lines (bf16, hipGraph replay and eager) + rocprofv3 kernel summaries.
# usage: scripts/gpu_cnn.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
L=$O/${TAG}_cnn.txt
: > $L
run() {   # label, args...
  echo "== $*" >> $L
  timeout -k 10 240 python3 $R/apps/train.py "$@" --dtype bf16 >> $L 2>&1
}
run alexnet -b 256 --iterations 20 --graph || exit $?
run alexnet -b 256 --iterations 20 || exit $?
run resnet50 -b 64 --iterations 20 --graph || exit $?
run resnet50 -b 64 --iterations 20 || exit $?
run resnet50 -b 256 --iterations 10 --graph || exit $?
run inception_v3 -b 64 --iterations 20 --graph || exit $?
run inception_v3 -b 256 --iterations 10 --graph || exit $?
cd /tmp && export TMPDIR=/tmp
for m in alexnet:256 resnet50:64 inception_v3:64; do
  name=${m%%:*}; b=${m##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${TAG}_prof_$name -o run -- python3 $R/apps/train.py $name -b $b --iterations 10 --warmup 2 --graph --dtype bf16 > $O/${TAG}_prof_$name.log 2>&1 || exit $?
  DB=$(find $O/${TAG}_prof_$name -name "*results.db" | head -1)
  (cd $R && python3 tools/prof_summary.py $DB 12 > $O/${TAG}_${name}_b${b}_kernels.txt 2>&1)
  rm -rf $O/${TAG}_prof_$name
done
exit 0
