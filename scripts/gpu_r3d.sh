#!/bin/bash
# conv-phase / pool tests, fp32 GEMM big-tile A/B, CNN throughput lines
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_phase.py tests/test_gpu_pool_negpad.py tests/test_gpu_fp32.py -k "phase or pool or negpad or conv" > $O/r3d_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u tools/gemm_f32_lab.py 0,1,3,4096,4104 "8192,480,1024;8192,1024,1024;8192,1024,512" > $O/lab2.jsonl 2>&1 || exit $?
L=$O/r3d_cnn.txt
: > $L
for spec in "alexnet -b 256" "resnet50 -b 64" "resnet50 -b 256" "inception_v3 -b 64"; do
  echo "== $spec --graph bf16" >> $L
  timeout -k 10 240 python3 apps/train.py $spec --iterations 20 --graph --dtype bf16 >> $L 2>&1 || exit $?
done
exit 0
