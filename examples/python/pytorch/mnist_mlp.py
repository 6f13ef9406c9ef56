"""Replay mlp.ff (written by mnist_mlp_torch.py) onto an FFModel and train it on MNIST
(reference examples/python/pytorch/mnist_mlp.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import common  # noqa: E402
from common import ModelAccuracy, check_accuracy, header, report  # noqa: E402

from flexmi.core import (DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer,  # noqa: E402
                         SingleDataLoader)
from flexmi.torch.model import PyTorchModel  # noqa: E402


def main(ff="mlp.ff", in_shape=(784,), load=common.mnist_flat, acc=ModelAccuracy.MNIST_MLP, exporter="mnist_mlp_torch"):
    cfg = FFConfig()
    cfg.parse_args()
    header(cfg)
    if not os.path.exists(ff):
        __import__(exporter).export(ff)
    model = FFModel(cfg)
    x = model.create_tensor([cfg.get_batch_size()] + list(in_shape), DataType.DT_FLOAT)
    outs = PyTorchModel(ff).apply(model, [x])
    print("output", outs[0].dims if isinstance(outs, (list, tuple)) else outs.dims)
    model.compile(optimizer=SGDOptimizer(model, 0.01), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    xs, ys = load()
    n = len(xs)
    loaders = (SingleDataLoader(model, x, xs, n), SingleDataLoader(model, model.get_label_tensor(), ys, n))
    model.init_layers()
    t0 = cfg.get_current_time()
    model.train(loaders, cfg.get_epochs())
    report(cfg, n, cfg.get_epochs(), t0, cfg.get_current_time())
    check_accuracy(model, acc)


if __name__ == "__main__":
    print("pytorch mnist mlp")
    main()
