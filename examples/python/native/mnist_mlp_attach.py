"""MNIST MLP fed batch by batch through ``attach_numpy_array`` on the input tensors themselves
(reference examples/python/native/mnist_mlp_attach.py): the host array is attached, the step runs,
the array is detached -- no data loader."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import ModelAccuracy, check_accuracy, header, mnist_flat, report  # noqa: E402

from flexmi.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer  # noqa: E402


def main():
    cfg = FFConfig()
    cfg.parse_args()
    header(cfg)
    model = FFModel(cfg)
    b = cfg.get_batch_size()
    x = model.create_tensor([b, 784], DataType.DT_FLOAT)
    t = model.dense(x, 512, ActiMode.AC_MODE_RELU)
    t = model.dense(t, 512, ActiMode.AC_MODE_RELU)
    t = model.softmax(model.dense(t, 10))
    model.compile(optimizer=SGDOptimizer(model, 0.01), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                  metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    label = model.get_label_tensor()
    xs, ys = mnist_flat()
    model.init_layers()
    epochs = cfg.get_epochs()
    t0 = cfg.get_current_time()
    for _ in range(epochs):
        model.reset_metrics()
        for it in range(len(xs) // b):
            x.attach_numpy_array(cfg, xs[it * b:(it + 1) * b])
            label.attach_numpy_array(cfg, ys[it * b:(it + 1) * b])
            model.forward()
            model.zero_gradients()
            model.backward()
            model.update()
            x.detach_numpy_array(cfg)
            label.detach_numpy_array(cfg)
    t1 = cfg.get_current_time()
    report(cfg, len(xs), epochs, t0, t1)
    check_accuracy(model, ModelAccuracy.MNIST_MLP)


if __name__ == "__main__":
    print("mnist mlp attach")
    main()
