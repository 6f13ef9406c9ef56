"""Train the ONNX-imported cifar10_cnn (reference examples/python/onnx/cifar10_cnn.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import common  # noqa: E402
from common import ModelAccuracy  # noqa: E402,F401
from _run import run  # noqa: E402


if __name__ == "__main__":
    print("onnx cifar10_cnn")
    run("cifar10_cnn", (3, 32, 32,), common.cifar10, ModelAccuracy.CIFAR10_CNN)
