"""CIFAR-10 CNN with a hand-written training loop that writes each batch into the mapped input
and label arrays (reference examples/python/native/cifar10_cnn_attach.py):
inline_map / get_array / inline_unmap, then forward / zero_gradients / backward / update."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import cifar10, header, report, threshold  # noqa: E402

from cifar10_cnn import build  # noqa: E402
from flexmi.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer  # noqa: E402


def write_batch(cfg, tensor, src, dtype):
    tensor.inline_map(cfg)
    arr = tensor.get_array(cfg, dtype)
    arr[...] = src
    tensor.inline_unmap(cfg)


def main():
    cfg = FFConfig()
    cfg.parse_args()
    header(cfg)
    model = FFModel(cfg)
    b = cfg.get_batch_size()
    x = model.create_tensor([b, 3, 32, 32], DataType.DT_FLOAT)
    build(model, x)
    model.compile(optimizer=SGDOptimizer(model, 0.01), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    label = model.get_label_tensor()
    xs, ys = cifar10()
    model.init_layers()
    epochs = cfg.get_epochs()
    t0 = cfg.get_current_time()
    for epoch in range(epochs):
        model.reset_metrics()
        for it in range(len(xs) // b):
            write_batch(cfg, x, xs[it * b:(it + 1) * b], DataType.DT_FLOAT)
            write_batch(cfg, label, ys[it * b:(it + 1) * b], DataType.DT_INT32)
            if epoch > 0:
                cfg.begin_trace(111)
            model.forward()
            model.zero_gradients()
            model.backward()
            model.update()
            if epoch > 0:
                cfg.end_trace(111)
    report(cfg, len(xs), epochs, t0, cfg.get_current_time())
    acc = model.get_perf_metrics().get_accuracy()
    assert acc >= min(30.0, threshold(30.0)), f"accuracy {acc}"
    inp = model.get_layer_by_id(0).get_input_tensor()
    inp.inline_map(cfg)
    print("first layer input", inp.get_flat_array(cfg, DataType.DT_FLOAT).shape)
    inp.inline_unmap(cfg)


if __name__ == "__main__":
    print("cifar10 cnn attach")
    main()
