"""Shared helpers for the example scripts (reference ``examples/python/*/accuracy.py`` + the
per-script dataset boilerplate).

Environment knobs, so the same scripts serve as the functional test suite (``tests/test_examples.py``,
the analogue of the reference's ``python/test.sh``):

* ``FLEXMI_EXAMPLE_SAMPLES`` -- cap on the number of training samples a script loads;
* ``FLEXMI_EXAMPLE_EPOCHS`` -- cap on the epochs of the Keras scripts;
* ``FLEXMI_EXAMPLE_MIN_ACC`` -- overrides every accuracy threshold (percent).

Datasets come from :mod:`flexmi.keras.datasets` (a local ``.npz`` copy when ``FLEXMI_DATASETS`` names
one, otherwise deterministic synthetic data of the real shapes -- there is no network).
"""
import os
import sys
from enum import Enum

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


class ModelAccuracy(Enum):
    """Accuracy thresholds (percent) the reference examples assert."""
    MNIST_MLP = 90
    MNIST_CNN = 90
    REUTERS_MLP = 90
    CIFAR10_CNN = 90
    CIFAR10_ALEXNET = 90


def threshold(acc):
    v = os.environ.get("FLEXMI_EXAMPLE_MIN_ACC")
    base = acc.value if isinstance(acc, ModelAccuracy) else float(acc)
    return float(v) if v is not None else base


def num_samples(default):
    cap = os.environ.get("FLEXMI_EXAMPLE_SAMPLES")
    return min(default, int(cap)) if cap else default


def epochs(default):
    """Epoch count of a Keras example: the script's own value, capped by FLEXMI_EXAMPLE_EPOCHS."""
    cap = os.environ.get("FLEXMI_EXAMPLE_EPOCHS")
    return min(default, int(cap)) if cap else default


def keras_callbacks(acc):
    from flexmi.keras.callbacks import EpochVerifyMetrics, VerifyMetrics
    return [VerifyMetrics(threshold(acc)), EpochVerifyMetrics(threshold(acc))]


def mnist_flat(n=60000):
    from flexmi.keras.datasets import mnist
    n = num_samples(n)
    (x, y), _ = mnist.load_data(n)
    x, y = x[:n], y[:n]
    return (x.reshape(len(x), 784).astype("float32") / 255), y.astype("int32").reshape(-1, 1)


def mnist_images(n=60000):
    x, y = mnist_flat(n)
    return x.reshape(len(x), 1, 28, 28), y


def cifar10(n=10000):
    from flexmi.keras.datasets import cifar10 as c
    n = num_samples(n)
    (x, y), _ = c.load_data(n)
    x, y = x[:n], y[:n]
    return x.astype("float32") / 255, y.astype("int32").reshape(-1, 1)


def reuters(n=8982, words=1000):
    from flexmi.keras.datasets import reuters as r
    n = num_samples(n)
    (x, y), _ = r.load_data(n)
    x, y = x[:n], y[:n]
    return (x.astype("float32") / 255).reshape(len(x), words), y.astype("int32").reshape(-1, 1)


def header(ffconfig):
    print("Python API batchSize(%d) workersPerNodes(%d) numNodes(%d)"
          % (ffconfig.get_batch_size(), ffconfig.get_workers_per_node(), ffconfig.get_num_nodes()))


def report(ffconfig, samples, epochs, ts_start, ts_end):
    run_time = 1e-6 * (ts_end - ts_start)
    print("epochs %d, ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s"
          % (epochs, run_time, samples * epochs / max(run_time, 1e-9)))


def check_accuracy(ffmodel, acc):
    got = ffmodel.get_perf_metrics().get_accuracy()
    need = threshold(acc)
    print(f"accuracy {got:.2f}% (threshold {need:.1f}%)")
    assert got >= need, f"accuracy {got:.2f}% below {need}%"


def fill_synthetic(ffmodel, tensors, seed=0, classes=10):
    """Load a random batch into input tensors and random class ids into the label (the
    reference CNN apps' random-data mode, ``alexnet.cc:151-155``)."""
    from flexmi.core import DataType
    rng = np.random.RandomState(seed)
    ex = ffmodel._ex()
    for t in tensors:
        ex.scatter_from_host(t, rng.rand(*t.dims).astype(np.float32))
    lab = ffmodel.get_label_tensor()
    if lab.data_type == DataType.DT_INT32:
        ex.scatter_from_host(lab, rng.randint(0, classes, lab.dims).astype(np.int32))
