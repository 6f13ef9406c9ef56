#!/bin/bash
# PMC counters for one flexmi GEMM shape (tools/gemm_one.py) on the gpurun box:
#   scripts/pmc_gemm.sh M K N orient tag
# one rocprofv3 run per counter group (counters only with --kernel-trace-free --pmc runs)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
M=$1; K=$2; N=$3; O=$4; TAG=$5; DT=${6:-bf16}
i=0
for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 $R/tools/gemm_one.py $M $K $N $O 20 $DT || exit 1
done
