#!/bin/bash
# bisect: pool scatter numerics vs fused SGD on the ResNet BN model test
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
run() {  # test failures (1) are results; anything else (fault, timeout) ends the script
  "$@"; rc=$?
  echo "rc=$rc" >> $O/r4k.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
: > $O/r4k.log
run timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_pool_negpad.py >> $O/r4k.log 2>&1
FM_FUSED_SGD=0 run timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_models.py -k resnet_batchnorm >> $O/r4k.log 2>&1
FM_FUSED_SGD=1 run timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_models.py -k resnet_batchnorm >> $O/r4k.log 2>&1
FM_POOL_BAND=0 run timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_models.py -k resnet_batchnorm >> $O/r4k.log 2>&1
exit 0
