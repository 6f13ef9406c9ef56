"""Layer / parameter introspection (reference examples/python/native/print_layers.py):
get_layer_by_id, get_tensor_by_id, weight / bias tensors, set_weights / get_weights and
in-place edits through inline_map + get_array."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import header  # noqa: E402

import numpy as np  # noqa: E402
from flexmi.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer  # noqa: E402


def main():
    cfg = FFConfig()
    cfg.parse_args()
    header(cfg)
    model = FFModel(cfg)
    b = cfg.get_batch_size()
    img = model.create_tensor([b, 3, 32, 32], DataType.DT_FLOAT)
    vec = model.create_tensor([b, 16], DataType.DT_FLOAT)
    model.conv2d(img, 8, 5, 5, 2, 2, 2, 2)
    model.dense(vec, 8, ActiMode.AC_MODE_RELU)
    model.compile(optimizer=SGDOptimizer(model, 0.01), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY])
    model.init_layers()

    label = model.get_label_tensor()
    label.inline_map(cfg)
    arr = label.get_array(cfg, DataType.DT_INT32)
    arr[...] = 1
    label.inline_unmap(cfg)

    conv_w = model.get_tensor_by_id(0)
    conv_w.set_weights(model, np.full((8, 3, 5, 5), 1.25, np.float32))
    assert np.allclose(conv_w.get_weights(model), 1.25)

    conv = model.get_layer_by_id(0)
    cb = conv.get_bias_tensor()
    cb.set_weights(model, np.full((8,), 2.5, np.float32))
    cb.inline_map(cfg)
    bias = cb.get_array(cfg, DataType.DT_FLOAT)
    bias += 1.0
    cb.inline_unmap(cfg)
    assert np.allclose(cb.get_weights(model), 3.5), cb.get_weights(model)

    cw = conv.get_weight_tensor()
    cw.inline_map(cfg)
    w = cw.get_array(cfg, DataType.DT_FLOAT)
    w[...] = np.arange(w.size, dtype=np.float32).reshape(w.shape)
    cw.inline_unmap(cfg)
    assert cw.get_weights(model).reshape(-1)[7] == 7.0

    dense = model.get_layer_by_id(1)
    db = dense.get_bias_tensor()
    db.inline_map(cfg)
    db.get_array(cfg, DataType.DT_FLOAT)[...] = 0.5
    db.inline_unmap(cfg)
    print("dense bias", db.get_weights(model))
    model.print_layers(0)
    model.print_layers()


if __name__ == "__main__":
    print("print layers")
    main()
