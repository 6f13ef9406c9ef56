"""Keras callbacks (``python/flexflow/keras/callbacks.py:21-90``)."""
import numpy as np


class Callback:
    def __init__(self):
        self.model = None
        self.params = None

    def set_params(self, params):
        self.params = params

    def set_model(self, model):
        self.model = model

    def on_epoch_begin(self, epoch, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass

    def on_batch_begin(self, batch, logs=None):
        pass

    def on_batch_end(self, batch, logs=None):
        pass

    def on_train_begin(self, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass


class LearningRateScheduler(Callback):
    def __init__(self, schedule):
        super().__init__()
        self.schedule = schedule

    def on_epoch_begin(self, epoch, logs=None):
        lr = self.schedule(epoch)
        if not isinstance(lr, (float, np.floating)):
            raise ValueError('The output of the "schedule" function should be float.')
        self.model.optimizer.set_learning_rate(float(lr))


def _threshold(a):
    return a.value if hasattr(a, "value") else float(a)


class VerifyMetrics(Callback):
    """Asserts the final accuracy reaches the threshold (a ModelAccuracy member or a float %)."""

    def __init__(self, accuracy):
        super().__init__()
        self.accuracy = _threshold(accuracy)

    def on_train_end(self, logs=None):
        acc = self.model.ffmodel.get_perf_metrics().get_accuracy()
        assert acc >= self.accuracy, f"accuracy {acc:.2f}% < {self.accuracy}%"


class EpochVerifyMetrics(Callback):
    """Early stop once the epoch accuracy exceeds the threshold."""

    def __init__(self, accuracy, early_stop=True):
        super().__init__()
        self.accuracy = _threshold(accuracy)
        self.early_stop = early_stop

    def on_epoch_end(self, epoch, logs=None):
        if not self.early_stop:
            return False
        return self.model.ffmodel.get_perf_metrics().get_accuracy() > self.accuracy
