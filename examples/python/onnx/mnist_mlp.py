"""Train the ONNX-imported mnist_mlp (reference examples/python/onnx/mnist_mlp.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import common  # noqa: E402
from common import ModelAccuracy  # noqa: E402,F401
from _run import run  # noqa: E402


if __name__ == "__main__":
    print("onnx mnist_mlp")
    run("mnist_mlp", (784,), common.mnist_flat, ModelAccuracy.MNIST_MLP)
