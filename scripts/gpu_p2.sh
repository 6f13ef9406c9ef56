#!/bin/bash
# p2: PMC of the plane kernel (fwd / dW 8192x1024x1024) vs the in-kernel split kernel; lab A/B of
# the 128x128 tile and the s_setprio variants
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in 1 2; do
  FM_PL_VAR=$v timeout -k 10 300 python3 -u tools/gemm_pl_lab.py "8192,1024,1024;8192,480,1024" > $O/p2_lab_var$v.jsonl 2>> $O/p2_lab.err || exit $?
done
FM_PL_BM=128 timeout -k 10 300 python3 -u tools/gemm_pl_lab.py "8192,1024,1024;8192,512,256" > $O/p2_lab_bm128.jsonl 2>> $O/p2_lab.err || exit $?
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "planes fwd" "planes dw" "fp32 fwd"; do
  set -- $cfg
  for grp in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" \
             "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp -d $O/p2_pmc_${1}_${2}_$i -o run --output-format csv -- python3 $R/tools/gemm_one.py 8192 1024 1024 $2 20 $1 > $O/p2_pmc_$i.log 2>&1 || exit $?
  done
done
cd $R
for d in $O/p2_pmc_*_*; do
  k=pl3; case $d in *fp32*) k=x3v2;; esac
  echo "== $d" >> $O/p2_pmc.txt
  python3 tools/pmc_summary.py $(find $d -name "*counter_collection.csv") --kernel $k >> $O/p2_pmc.txt 2>&1
done
exit 0
