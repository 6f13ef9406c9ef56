"""Keras losses (``python/flexflow/keras/losses.py``): each maps to a LossType."""
from flexmi.core.types import LossType


class Loss:
    type = None

    def __init__(self, name=None):
        self.name = name


class CategoricalCrossentropy(Loss):
    type = LossType.LOSS_CATEGORICAL_CROSSENTROPY


class SparseCategoricalCrossentropy(Loss):
    type = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY


class MeanSquaredError(Loss):
    type = LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE


class BinaryCrossentropy(Loss):
    type = LossType.LOSS_BINARY_CROSSENTROPY


_BY_NAME = {"categorical_crossentropy": CategoricalCrossentropy,
            "sparse_categorical_crossentropy": SparseCategoricalCrossentropy,
            "mean_squared_error": MeanSquaredError, "mse": MeanSquaredError,
            "binary_crossentropy": BinaryCrossentropy}


def get(name):
    if name not in _BY_NAME:
        raise ValueError(f"unsupported loss {name!r}")
    return _BY_NAME[name]()
