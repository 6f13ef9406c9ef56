#!/bin/bash
# r5y: full GPU suite after the x1 / late-join / 32-entry multi-copy changes; bench A/B of the
# input staging captured into the step graph vs its own graph; step trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r5y_gpu_suite.log 2>&1 || exit $?
for rep in 1 2; do
  for sg in 0 1; do
    FM_BENCH_STAGE_GRAPH=$sg timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5y_bench_sg${sg}_$rep.log 2>&1 || exit $?
  done
done
for x3 in 0 1; do
  FM_DOT_FWD_X3=$x3 timeout -k 10 120 python3 -u tools/bench_interaction.py >> $O/r5y_dot_x3_$x3.txt 2>&1 || exit $?
done
for rep in 1 2; do
  for x3 in 0 1; do
    FM_DOT_FWD_X3=$x3 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5y_bench_dx3_${x3}_$rep.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > $O/r5y_bench_both.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r5y --no-secondary || exit $?
exit 0
