#!/bin/bash
# PMC of the NHWC conv GEMM kernels (op path) on ResNet r2 3x3 and r4 3x3
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in r2_3x3 r4_3x3; do
  i=0
  for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
             "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp -d $O/pmc_r4g_${L}_$i -o run --output-format csv -- python3 $R/tools/bench_conv.py --net all --layer $L --path op --reps 5 > /dev/null 2>&1 || exit 1
  done
  for k in "fm_conv_nhwc<128, 128, 0" "fm_conv_nhwc<64, 128, 0" "fm_conv_nhwc<128, 128, 1" "fm_conv_nhwc<64, 128, 1" "fm_conv_nhwc<128, 128, 2" "fm_conv_nhwc<64, 128, 2" "fm_nhwc_stage"; do
    (cd $R && python3 tools/pmc_summary.py $(find $O/pmc_r4g_${L}_* -name "*counter_collection.csv") --kernel "$k" >> $O/r4g_pmc_$L.txt 2>&1; echo "== $k" >> $O/r4g_pmc_$L.txt)
  done
  rm -rf $O/pmc_r4g_${L}_*
done
exit 0
