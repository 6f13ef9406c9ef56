#!/bin/bash
# final-tree check: fused SGD + models GPU tests and smoke on the committed build
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_sgd.py tests/test_gpu_kernels.py tests/test_gpu_models.py > $O/r4r_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r4r_smoke.log 2>&1 || exit $?
exit 0
