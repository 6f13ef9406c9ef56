"""Print a loaded input batch (reference examples/python/native/print_input.py): a data loader
fills the input tensor, which is then mapped and read on the host."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import cifar10, header  # noqa: E402

import numpy as np  # noqa: E402
from flexmi.core import (ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType,  # noqa: E402
                         SGDOptimizer, SingleDataLoader)


def main():
    cfg = FFConfig()
    cfg.parse_args()
    header(cfg)
    model = FFModel(cfg)
    b = cfg.get_batch_size()
    x = model.create_tensor([b, 3, 32, 32], DataType.DT_FLOAT)
    t = model.flat(model.pool2d(model.conv2d(x, 8, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU), 2, 2, 2, 2, 0, 0))
    model.softmax(model.dense(t, 10))
    model.compile(optimizer=SGDOptimizer(model, 0.01), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
    xs, ys = cifar10(max(2 * b, 64))
    loader = SingleDataLoader(model, x, xs, len(xs))
    model.init_layers()
    loader.next_batch(model)
    x.inline_map(cfg)
    arr = np.asarray(x.get_array(cfg, DataType.DT_FLOAT))
    x.inline_unmap(cfg)
    assert np.allclose(arr, xs[:b], atol=1e-2), "loaded batch differs from the source rows"
    print(arr.shape, arr.reshape(-1)[:8])


if __name__ == "__main__":
    print("print input")
    main()
