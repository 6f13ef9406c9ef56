#!/bin/bash
# end-of-session validation: full GPU suite, smoke, default bench line; CNN lines + AlexNet kernel summary
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/r4j_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r4j_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/r4j_bench.jsonl 2> $O/r4j_bench.err || exit $?
for spec in "alexnet -b 256" "resnet50 -b 64" "inception_v3 -b 64"; do
  echo "== $spec --graph bf16" >> $O/r4j_cnn.txt
  timeout -k 10 240 python3 apps/train.py $spec --iterations 20 --graph --dtype bf16 >> $O/r4j_cnn.txt 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/r4j_prof -o run -- python3 $R/apps/train.py alexnet -b 256 --iterations 10 --warmup 2 --graph --dtype bf16 > $O/r4j_prof.log 2>&1 || exit $?
DB=$(find $O/r4j_prof -name "*results.db" | head -1)
(cd $R && python3 tools/prof_summary.py $DB 12 > $O/r4j_alexnet_b256_kernels.txt 2>&1)
rm -rf $O/r4j_prof
exit 0
