"""Keras metrics (``python/flexflow/keras/metrics.py``): each maps to a MetricsType."""
from flexmi.core.types import MetricsType


class Metric:
    type = None

    def __init__(self, name=None):
        self.name = name


class Accuracy(Metric):
    type = MetricsType.METRICS_ACCURACY


class CategoricalCrossentropy(Metric):
    type = MetricsType.METRICS_CATEGORICAL_CROSSENTROPY


class SparseCategoricalCrossentropy(Metric):
    type = MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY


class MeanSquaredError(Metric):
    type = MetricsType.METRICS_MEAN_SQUARED_ERROR


class RootMeanSquaredError(Metric):
    type = MetricsType.METRICS_ROOT_MEAN_SQUARED_ERROR


class MeanAbsoluteError(Metric):
    type = MetricsType.METRICS_MEAN_ABSOLUTE_ERROR


_BY_NAME = {"accuracy": Accuracy, "categorical_crossentropy": CategoricalCrossentropy,
            "sparse_categorical_crossentropy": SparseCategoricalCrossentropy, "mean_squared_error": MeanSquaredError,
            "root_mean_squared_error": RootMeanSquaredError, "mean_absolute_error": MeanAbsoluteError}


def get(name):
    if name not in _BY_NAME:
        raise ValueError(f"unsupported metric {name!r}")
    return _BY_NAME[name]()
