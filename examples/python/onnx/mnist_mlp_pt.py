"""Export the PyTorch MLP to mnist_mlp.onnx (reference examples/python/onnx/mnist_mlp_pt.py), through
flexmi's offline exporter (the onnx package is not installed here)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401

import torch  # noqa: E402
from _models import MLP  # noqa: E402
from flexmi.onnx.export import torch_to_onnx  # noqa: E402


def export(path="mnist_mlp.onnx", batch=64):
    torch.manual_seed(0)
    model = MLP().eval()
    torch_to_onnx(model, [batch, 784], path, input_names=["input.1"])
    return path


if __name__ == "__main__":
    print("wrote", export(sys.argv[1] if len(sys.argv) > 1 else "mnist_mlp.onnx"))
