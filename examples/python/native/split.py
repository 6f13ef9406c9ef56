"""concat -> split round trip inside a CIFAR-10 CNN (reference examples/python/native/split.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import cifar10, header, report  # noqa: E402

from flexmi.core import (ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType,  # noqa: E402
                         SGDOptimizer, SingleDataLoader)


def main():
    cfg = FFConfig()
    cfg.parse_args()
    header(cfg)
    model = FFModel(cfg)
    x = model.create_tensor([cfg.get_batch_size(), 3, 32, 32], DataType.DT_FLOAT)
    towers = [model.conv2d(x, 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU) for _ in range(3)]
    parts = model.split(model.concat(towers, 1), 3, 1)
    assert len(parts) == 3 and all(p.dims[1] == 32 for p in parts)
    t = model.conv2d(parts[1], 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = model.pool2d(t, 2, 2, 2, 2, 0, 0)
    t = model.flat(t)
    t = model.dense(t, 512, ActiMode.AC_MODE_RELU)
    model.softmax(model.dense(t, 10))
    model.compile(optimizer=SGDOptimizer(model, 0.01), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    xs, ys = cifar10()
    n = len(xs)
    loaders = (SingleDataLoader(model, x, xs, n), SingleDataLoader(model, model.get_label_tensor(), ys, n))
    model.init_layers()
    t0 = cfg.get_current_time()
    model.train(loaders, cfg.get_epochs())
    report(cfg, n, cfg.get_epochs(), t0, cfg.get_current_time())


if __name__ == "__main__":
    print("cifar10 cnn split")
    main()
