#!/bin/bash
# Functional example suite (reference python/test.sh): every example through the flexmi launcher.
#   examples/python/run_all.sh [GPUS]      (GPUS > 1 runs each script SPMD over that many ranks)
# FLEXMI_EXAMPLE_SAMPLES / FLEXMI_EXAMPLE_EPOCHS / FLEXMI_EXAMPLE_MIN_ACC shrink the runs (common.py).
set -e
GPUS=${1:-1}
HERE=$(cd "$(dirname "$0")" && pwd)
RUN="python -m flexmi.run -ll:gpu $GPUS"
export PYTHONPATH="$HERE/../..:$PYTHONPATH"
WORK=$(mktemp -d); cd "$WORK"
for f in seq_mnist_mlp seq_mnist_cnn seq_reuters_mlp seq_cifar10_cnn seq_mnist_mlp_net2net seq_mnist_cnn_net2net \
         seq_mnist_cnn_nested callback unary reshape func_mnist_mlp func_mnist_mlp_concat func_mnist_mlp_concat2 \
         func_mnist_cnn func_mnist_cnn_concat func_cifar10_cnn func_cifar10_cnn_nested func_cifar10_alexnet \
         func_mnist_mlp_net2net func_cifar10_cnn_net2net func_cifar10_cnn_concat func_cifar10_cnn_concat_model \
         func_cifar10_cnn_concat_seq_model; do
  $RUN "$HERE/keras/$f.py"
done
$RUN "$HERE/keras/candle_uno/candle_uno.py"
$RUN "$HERE/native/print_layers.py" --epochs 5
$RUN "$HERE/native/split.py"
$RUN "$HERE/native/alexnet.py" --epochs 1
$RUN "$HERE/native/mnist_mlp.py" --epochs 5
$RUN "$HERE/native/mnist_cnn.py" --epochs 5
$RUN "$HERE/native/cifar10_cnn.py" --epochs 4
$RUN "$HERE/native/cifar10_cnn_attach.py" --epochs 5
$RUN "$HERE/native/mnist_mlp_attach.py" --epochs 5
$RUN "$HERE/native/cifar10_cnn_concat.py" --epochs 4
$RUN "$HERE/native/inception.py"
$RUN "$HERE/native/resnet.py"
$RUN "$HERE/native/tensor_attach.py"
$RUN "$HERE/native/print_input.py"
for f in mnist_mlp cifar10_cnn alexnet resnet; do $RUN "$HERE/onnx/$f.py"; done
for f in mnist_mlp cifar10_cnn; do $RUN "$HERE/pytorch/$f.py"; done
echo "all examples passed"
