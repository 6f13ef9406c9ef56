#!/bin/bash
# r5k: interaction act0 fusion (tests, bench, step trace); PMC counters of the split-bf16 GEMM
# (8192x1024x1024 forward and dW) to see where its non-MFMA cycles go
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp32.py tests/test_gpu_models.py tests/test_gpu_kernels.py > $O/r5k_tests.log 2>&1 || exit $?
FM_DOT_ACT0=0 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5k_bench_act0off.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-secondary > $O/r5k_bench_act0on.log 2>&1 || exit $?
bash scripts/gpu_profile_step.sh r5k --no-secondary || exit $?
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT" \
           "SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for orient in fwd dw; do
    timeout -s KILL 90 rocprofv3 --pmc $grp -d $O/r5k_pmc_${orient}_$i -o run --output-format csv -- python3 $R/tools/gemm_one.py 8192 1024 1024 $orient 20 fp32 > $O/r5k_pmc_${orient}_$i.log 2>&1 || exit $?
  done
done
cd $R
for orient in fwd dw; do
  python3 tools/pmc_summary.py $(find $O -path "*r5k_pmc_${orient}_*" -name "*counter_collection.csv") --kernel x3v2 > $O/r5k_pmc_${orient}.txt 2>&1
done
exit 0
