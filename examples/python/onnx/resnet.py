"""Train the ONNX-imported resnet (reference examples/python/onnx/resnet.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import common  # noqa: E402
from common import ModelAccuracy  # noqa: E402,F401
from _run import run  # noqa: E402


if __name__ == "__main__":
    print("onnx resnet")
    run("resnet", (3, 32, 32), common.cifar10, None)
