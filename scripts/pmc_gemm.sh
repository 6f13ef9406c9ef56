cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "SQ_WAIT_ANY SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD"; do
  n=$(echo $grp | tr ' ' '_' | cut -c1-20)
  timeout -k 10 120 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_$n -o run --output-format csv -- python $R/tools/gemm_one.py 8192 1024 1024 fwd 20 || exit 1
done
