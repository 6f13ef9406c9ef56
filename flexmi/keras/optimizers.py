"""Keras optimizers (``python/flexflow/keras/optimizers.py``) over flexmi's SGD / Adam."""
from flexmi.core.optimizers import AdamOptimizer, SGDOptimizer


class Optimizer:
    def __init__(self):
        self.ff = None

    def set_learning_rate(self, lr):
        self.lr = float(lr)
        if self.ff is not None:
            self.ff.set_learning_rate(self.lr)


class SGD(Optimizer):
    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, weight_decay=0.0, **kw):
        super().__init__()
        self.lr, self.momentum, self.nesterov, self.weight_decay = float(learning_rate), momentum, nesterov, weight_decay

    def build(self, ffmodel):
        self.ff = SGDOptimizer(ffmodel, self.lr, self.momentum, self.nesterov, self.weight_decay)
        return self.ff


class Adam(Optimizer):
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-8, weight_decay=0.0, **kw):
        super().__init__()
        self.lr, self.b1, self.b2, self.eps, self.weight_decay = float(learning_rate), beta_1, beta_2, epsilon, weight_decay

    def build(self, ffmodel):
        self.ff = AdamOptimizer(ffmodel, self.lr, self.b1, self.b2, self.weight_decay, self.eps)
        return self.ff
