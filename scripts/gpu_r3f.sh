#!/bin/bash
# native C model on the HIP engine; dot-interaction forward A/B (staged LDS kernel vs plain)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_native_model.py tests/test_gpu_pool_negpad.py > $O/r3f_tests.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/bench_interaction.py > $O/r3f_dot_staged.txt 2>&1 || exit $?
FM_DOT_FWD_STAGED=0 timeout -k 10 120 python3 tools/bench_interaction.py > $O/r3f_dot_plain.txt 2>&1 || exit $?
exit 0
