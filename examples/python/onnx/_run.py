"""Shared driver of the ONNX examples: export (if needed) -> ONNXModel.apply -> compile -> train
(reference examples/python/onnx/{mnist_mlp,cifar10_cnn,alexnet,resnet}.py)."""
import importlib
import os

from common import check_accuracy, header, report, threshold  # noqa: F401
from flexmi.core import (DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer,  # noqa: E402
                         SingleDataLoader)
from flexmi.onnx import ONNXModel


def run(name, in_shape, load, acc=None):
    cfg = FFConfig()
    cfg.parse_args()
    header(cfg)
    path = f"{name}.onnx"
    if not os.path.exists(path):
        importlib.import_module(f"{name}_pt").export(path)
    model = FFModel(cfg)
    x = model.create_tensor([cfg.get_batch_size()] + list(in_shape), "", DataType.DT_FLOAT)
    onnx_model = ONNXModel(path)
    onnx_model.apply(model, {"input.1": x})
    model.set_sgd_optimizer(SGDOptimizer(model, 0.01))
    model.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    xs, ys = load()
    n = len(xs)
    loaders = (SingleDataLoader(model, x, xs, n), SingleDataLoader(model, model.get_label_tensor(), ys, n))
    model.init_layers()
    onnx_model.copy_weights(model)          # start from the exported PyTorch weights
    t0 = cfg.get_current_time()
    model.train(loaders, cfg.get_epochs())
    report(cfg, n, cfg.get_epochs(), t0, cfg.get_current_time())
    if acc is not None:
        check_accuracy(model, acc)
    return model
