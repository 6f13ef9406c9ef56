#!/bin/bash
# r5b: fp32 MFMA pipe probe (tools/mfma_probe.hip): registers-only / + LDS fragments / + barrier / + LDS-DMA
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/bin/mfma_probe 2000 > $O/r5b_probe.jsonl 2>&1 || exit $?
timeout -k 10 120 ./tools/bin/mfma_probe 8000 >> $O/r5b_probe.jsonl 2>&1 || exit $?
exit 0
