"""Keras datasets (``python/flexflow/keras/datasets``): mnist, cifar10, reuters.

There is no network on the build/GPU hosts, so ``load_data`` reads a local copy when one is
given (``FLEXMI_DATASETS=<dir>`` with ``mnist.npz`` / ``cifar10.npz`` / ``reuters.npz`` holding
``x_train, y_train, x_test, y_test``, loaded with ``allow_pickle=False``) and otherwise returns
deterministic SYNTHETIC data of the real shapes and dtypes: class-dependent means plus noise,
so models can still learn and accuracy-threshold callbacks remain meaningful.
"""
import os

import numpy as np


def _local(name):
    d = os.environ.get("FLEXMI_DATASETS")
    if d and os.path.exists(os.path.join(d, name + ".npz")):
        f = np.load(os.path.join(d, name + ".npz"), allow_pickle=False)
        return (f["x_train"], f["y_train"]), (f["x_test"], f["y_test"])
    return None


def _synthetic(n_train, n_test, shape, classes, seed, dtype=np.uint8, scale=255):
    rng = np.random.RandomState(seed)
    protos = rng.rand(classes, *shape)

    def make(n):
        y = rng.randint(0, classes, n)
        x = 0.6 * protos[y] + 0.4 * rng.rand(n, *shape)
        return (x * scale).astype(dtype), y.astype(np.uint8)
    return make(n_train), make(n_test)


class _DS:
    def __init__(self, name, shape, classes, n_train, n_test, seed):
        self.name, self.shape, self.classes, self.n_train, self.n_test, self.seed = name, shape, classes, n_train, n_test, seed

    def load_data(self, num_samples=None, **kw):
        got = _local(self.name)
        if got is None:
            got = _synthetic(num_samples or self.n_train, min(self.n_test, num_samples or self.n_test), self.shape,
                             self.classes, self.seed)
        return got


mnist = _DS("mnist", (28, 28), 10, 60000, 10000, 1)
cifar10 = _DS("cifar10", (3, 32, 32), 10, 50000, 10000, 2)
reuters = _DS("reuters", (1000,), 46, 8982, 2246, 3)
