"""Replay cnn.ff (written by cifar10_cnn_torch.py) and train it on CIFAR-10
(reference examples/python/pytorch/cifar10_cnn.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import common  # noqa: E402
from common import ModelAccuracy  # noqa: E402
from mnist_mlp import main  # noqa: E402

if __name__ == "__main__":
    print("pytorch cifar10 cnn")
    main("cnn.ff", (3, 32, 32), common.cifar10, ModelAccuracy.CIFAR10_CNN, "cifar10_cnn_torch")
