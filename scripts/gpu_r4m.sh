#!/bin/bash
# LDS-staged fused-SGD epilogue: numerics, summit_large A/B (staged vs direct), AlexNet line + kernel summary
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_sgd.py > $O/r4m_tests.log 2>&1 || exit $?
L=$O/r4m_ab.jsonl
: > $L
for arm in 0 1 0 1; do
  echo "# summit_large FM_SGD_EPI_DIRECT=$arm" >> $L
  FM_SGD_EPI_DIRECT=$arm timeout -k 10 300 python3 bench.py --config summit_large --batch-per-gpu 256 --steps 40 --warmup 5 --no-dp >> $L 2>> $O/r4m_bench.err || exit $?
done
timeout -k 10 240 python3 apps/train.py alexnet -b 256 --iterations 20 --graph --dtype bf16 > $O/r4m_cnn.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/r4m_prof -o run -- python3 $R/apps/train.py alexnet -b 256 --iterations 10 --warmup 2 --graph --dtype bf16 > $O/r4m_prof.log 2>&1 || exit $?
DB=$(find $O/r4m_prof -name "*results.db" | head -1)
(cd $R && python3 tools/prof_summary.py $DB 12 > $O/r4m_alexnet_b256_kernels.txt 2>&1)
rm -rf $O/r4m_prof
exit 0
