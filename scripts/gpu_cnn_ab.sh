#!/bin/bash
# CNN throughput A/B of one environment knob: conv tests, then AlexNet b256 / ResNet-50 b64 (bf16,
# captured), two runs per arm, alternating.  usage: scripts/gpu_cnn_ab.sh TAG KNOB "v1 v2"
set -o pipefail
TAG=$1; KNOB=$2; VALS=$3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_nhwc.py tests/test_gpu_conv_phase.py -x -q --timeout 120 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { tail -30 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
for rep in 1 2; do
  for v in $VALS; do
    for m in "alexnet -b 256" "resnet50 -b 64"; do
      echo "== $KNOB=$v $m rep $rep" >> $O/${TAG}_ab.txt
      env $KNOB=$v timeout -k 10 300 python3 apps/train.py $m --iterations 20 --warmup 3 --graph --dtype bf16 >> $O/${TAG}_ab.txt 2>&1 || exit $?
    done
  done
done
grep -o '^== .*\|THROUGHPUT = [0-9.]*' $O/${TAG}_ab.txt
