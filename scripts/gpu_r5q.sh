#!/bin/bash
# r5q: split GEMM timing ablations (1 = no staging in the loop, 2 = no MFMAs) on the big DLRM
# shapes; bench after reverting the 16-deep slab sums / 8-deep skinny batches
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
SH="8192,1024,1024;8192,480,1024;8192,1024,512"
for ab in 0 1 2; do
  FM_X3_ABLATE=$ab timeout -k 10 300 python3 -u tools/gemm_f32_lab.py -2 "$SH" > $O/r5q_lab_ab$ab.jsonl 2> $O/r5q_lab_ab$ab.err || true
done
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5q_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5q_bench2.log 2>&1 || exit $?
exit 0
