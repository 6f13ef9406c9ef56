#!/bin/bash
# PMC A/B of one GEMM shape: flexmi (tools/gemm_one.py) vs hipBLASLt (tools/gemm_lib_one.py)
# usage: scripts/pmc_ab.sh M K N orient dtype tag
set -o pipefail
R=$GRAFT_REPO_ROOT
M=$1; K=$2; N=$3; O=$4; DT=$5; TAG=$6
CNT="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS"
cd /tmp && export TMPDIR=/tmp
for who in flexmi lib; do
  prog=$R/tools/gemm_one.py; [ $who = lib ] && prog=$R/tools/gemm_lib_one.py
  timeout -s KILL 90 rocprofv3 --pmc $CNT -d $R/gpurun_out/pmc_${TAG}_$who -o run --output-format csv -- python3 $prog $M $K $N $O 20 $DT > $R/gpurun_out/pmc_${TAG}_$who.log 2>&1 || exit $?
  F=$(find $R/gpurun_out/pmc_${TAG}_$who -name "*counter_collection.csv" | head -1)
  filt=fm_gemm; [ $who = lib ] && filt=Cijk
  python3 $R/tools/pmc_summary.py $F --kernel $filt > $R/gpurun_out/pmc_${TAG}_$who.txt 2>&1
  rm -rf $R/gpurun_out/pmc_${TAG}_$who
done
exit 0
