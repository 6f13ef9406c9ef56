#!/bin/bash
# PMC counters for one conv layer / pass (tools/bench_conv.py): scripts/pmc_conv.sh layer pass tag [dtype]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=$1; PS=$2; TAG=$3; DT=${4:-bf16}
i=0
for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 $R/tools/bench_conv.py --net all --layer $L --only $PS --reps 5 --dtype $DT || exit 1
done
