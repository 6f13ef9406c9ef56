"""MNIST MLP through the core API (reference examples/python/native/mnist_mlp.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import ModelAccuracy, check_accuracy, header, mnist_flat, report  # noqa: E402

from flexmi.core import (ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType,  # noqa: E402
                         SGDOptimizer, SingleDataLoader, UniformInitializer)


def main():
    cfg = FFConfig()
    cfg.parse_args()
    header(cfg)
    model = FFModel(cfg)
    x = model.create_tensor([cfg.get_batch_size(), 784], DataType.DT_FLOAT)
    t = model.dense(x, 512, ActiMode.AC_MODE_RELU, kernel_initializer=UniformInitializer(12, -1, 1))
    t = model.dense(t, 512, ActiMode.AC_MODE_RELU)
    t = model.softmax(model.dense(t, 10))
    model.set_sgd_optimizer(SGDOptimizer(model, 0.01))
    model.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    xs, ys = mnist_flat()
    n = len(xs)
    full_x = model.create_tensor([n, 784], DataType.DT_FLOAT)
    full_y = model.create_tensor([n, 1], DataType.DT_INT32)
    full_x.attach_numpy_array(cfg, xs)
    full_y.attach_numpy_array(cfg, ys)
    loaders = (SingleDataLoader(model, x, full_x, n, DataType.DT_FLOAT),
               SingleDataLoader(model, model.get_label_tensor(), full_y, n, DataType.DT_INT32))
    full_x.detach_numpy_array(cfg)
    full_y.detach_numpy_array(cfg)
    model.init_layers()
    t0 = cfg.get_current_time()
    model.train(loaders, cfg.get_epochs())
    t1 = cfg.get_current_time()
    report(cfg, n, cfg.get_epochs(), t0, t1)
    check_accuracy(model, ModelAccuracy.MNIST_MLP)
    model.eval(loaders)
    print("eval accuracy %.2f%%" % model.get_perf_metrics().get_accuracy())


if __name__ == "__main__":
    print("mnist mlp")
    main()
