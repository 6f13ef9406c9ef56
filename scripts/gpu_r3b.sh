#!/bin/bash
# pool / conv negative-pad tests, then the CNN throughput + kernel profiles
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pool_negpad.py tests/test_gpu_kernels.py -k "pool or conv or negpad" > gpurun_out/r3b_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_cnn.sh r3b
