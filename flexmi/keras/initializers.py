"""Keras initializers mapped onto flexmi's counter-based initializers."""
from flexmi.core import initializers as I


class Initializer:
    ff = None


class GlorotUniform(Initializer):
    def __init__(self, seed=0):
        self.ff = I.GlorotUniformInitializer(seed)


class Zeros(Initializer):
    def __init__(self):
        self.ff = I.ZeroInitializer()


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.ff = I.ConstantInitializer(value)


class RandomUniform(Initializer):
    def __init__(self, minval=-0.05, maxval=0.05, seed=0):
        self.ff = I.UniformInitializer(seed, minval, maxval)


class RandomNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05, seed=0):
        self.ff = I.NormInitializer(seed, mean, stddev)
