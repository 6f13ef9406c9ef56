#!/bin/bash
set -o pipefail
bash $GRAFT_REPO_ROOT/scripts/gpu_r3u.sh || exit $?
bash $GRAFT_REPO_ROOT/scripts/gpu_r3v.sh || exit $?
exit 0
