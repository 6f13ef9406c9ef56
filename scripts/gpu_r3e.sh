#!/bin/bash
# full GPU test suite, then the dot-forward A/B on the bench, then CNN kernel profiles
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r3e_gputests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_ab_bench.sh r3e - FM_DOT_FWD_STAGED=0 || exit $?
cd /tmp && export TMPDIR=/tmp
for m in alexnet:256 resnet50:64; do
  name=${m%%:*}; b=${m##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/r3e_prof_$name -o run -- python3 $R/apps/train.py $name -b $b --iterations 10 --warmup 2 --graph --dtype bf16 > $R/$O/r3e_prof_$name.log 2>&1 || exit $?
  DB=$(find $R/$O/r3e_prof_$name -name "*results.db" | head -1)
  (cd $R && python3 tools/prof_summary.py $DB 12 > $O/r3e_${name}_b${b}_kernels.txt 2>&1)
  rm -rf $R/$O/r3e_prof_$name
done
exit 0
