#!/bin/bash
# conv PMC: MFMA busy / VALU / LDS / waits for the ResNet r2 3x3 fwd+wgrad and the 1x1 fwd
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 200 python3 tools/bench_conv.py --net resnet --reps 20 > $O/r3l_conv_resnet.txt 2>&1 || exit $?
for spec in "r2_3x3 wgrad" "r2_3x3 fwd" "r2_1x1 fwd" "r2_3x3 dgrad"; do
  set -- $spec
  bash scripts/pmc_conv.sh $1 $2 r3l_$1_$2 || exit $?
  (cd $R && python3 tools/pmc_summary.py $(find $O/pmc_r3l_$1_$2_* -name "*counter_collection.csv") --kernel fm_conv_igemm > $O/r3l_pmc_$1_$2.txt 2>&1)
  rm -rf $O/pmc_r3l_$1_$2_*
done
exit 0
