"""Train the ONNX-imported alexnet (reference examples/python/onnx/alexnet.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import common  # noqa: E402
from common import ModelAccuracy  # noqa: E402,F401
from _run import run  # noqa: E402


def load_upsampled():
    import numpy as np
    x, y = common.cifar10()
    idx = (np.arange(229) * 32) // 229
    return np.ascontiguousarray(x[:, :, idx][:, :, :, idx]), y


if __name__ == "__main__":
    print("onnx alexnet")
    run("alexnet", (3, 229, 229), load_upsampled, None)
