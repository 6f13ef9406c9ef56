#!/bin/bash
# summit_large kernel breakdown (fp32 + bf16 steps)
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/gpu_profile_step.sh r4d_summit --config summit_large --batch-per-gpu 256 || exit $?
exit 0
