"""Trace the PyTorch CNN with torch.fx and write the FlexFlow text format cnn.ff
(reference examples/python/pytorch/cifar10_cnn_torch.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "onnx"))
import common  # noqa: E402,F401

from _models import CNN  # noqa: E402
from flexmi.torch.fx import torch_to_flexflow  # noqa: E402


def export(path="cnn.ff"):
    torch_to_flexflow(CNN(), path)
    return path


if __name__ == "__main__":
    print("wrote", export(sys.argv[1] if len(sys.argv) > 1 else "cnn.ff"))
