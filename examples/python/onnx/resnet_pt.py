"""Export the PyTorch ResNet to resnet.onnx (reference examples/python/onnx/resnet_pt.py), through
flexmi's offline exporter (the onnx package is not installed here)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401

import torch  # noqa: E402
from _models import ResNet  # noqa: E402
from flexmi.onnx.export import torch_to_onnx  # noqa: E402


def export(path="resnet.onnx", batch=64):
    torch.manual_seed(0)
    model = ResNet().eval()
    torch_to_onnx(model, [batch, 3, 32, 32], path, input_names=["input.1"])
    return path


if __name__ == "__main__":
    print("wrote", export(sys.argv[1] if len(sys.argv) > 1 else "resnet.onnx"))
