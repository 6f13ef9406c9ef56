"""Keras-style layers (``python/flexflow/keras/layers/*.py``).

A layer call records a node in a symbolic graph of :class:`KTensor` s (shape without the batch
dim); nothing is built until the model compiles, when every layer is lowered onto the FFModel
builder API (``Layer.build_ff``).  NCHW image layout (``channels_last`` is rejected like the
reference, ``convolutional.py:47-48``).
"""
from __future__ import annotations

import itertools
from typing import List, Sequence

from flexmi.core import initializers as I
from flexmi.core.types import ActiMode, AggrMode, DataType, OperatorType, PoolType

_uid = itertools.count()

_ACT = {None: ActiMode.AC_MODE_NONE, "linear": ActiMode.AC_MODE_NONE, "relu": ActiMode.AC_MODE_RELU,
        "sigmoid": ActiMode.AC_MODE_SIGMOID, "tanh": ActiMode.AC_MODE_TANH}
_DT = {"float32": DataType.DT_FLOAT, "float": DataType.DT_FLOAT, "int32": DataType.DT_INT32,
       "int64": DataType.DT_INT64}


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def _init(x, default=None):
    if x is None or x in ("glorot_uniform", "zeros"):
        return default
    if isinstance(x, I.Initializer):
        return x
    if hasattr(x, "ff"):
        return x.ff
    raise ValueError(f"unknown initializer {x!r}")


class KTensor:
    """Symbolic tensor: ``shape`` excludes the batch dimension."""

    def __init__(self, shape, dtype=DataType.DT_FLOAT, layer=None, index=0):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = dtype
        self.layer = layer
        self.index = index
        self.ff = None        # FFModel tensor after compile

    @property
    def batch_shape(self):
        return (None,) + self.shape

    def __repr__(self):
        return f"KTensor{self.batch_shape}"


class Layer:
    default_name = "layer"

    def __init__(self, name=None, input_shape=None, **kwargs):
        self.name = name or f"{self.default_name}_{next(_uid)}"
        self.input_shape = tuple(input_shape) if input_shape is not None else None
        self.inputs: List[KTensor] = []
        self.outputs: List[KTensor] = []
        self.ff_op = None
        self.prev_layers, self.next_layers = [], []

    # -- symbolic call -----------------------------------------------------------
    def __call__(self, x):
        xs = list(x) if isinstance(x, (list, tuple)) else [x]
        self.inputs = xs
        for t in xs:
            if t.layer is not None:
                t.layer.next_layers.append(self)
                self.prev_layers.append(t.layer)
        shapes = self.compute_output_shape([t.shape for t in xs])
        self.outputs = [KTensor(s, self.out_dtype(xs), self, i) for i, s in enumerate(shapes)]
        return self.outputs[0] if len(self.outputs) == 1 else self.outputs

    def out_dtype(self, xs):
        return DataType.DT_FLOAT

    def compute_output_shape(self, shapes):
        raise NotImplementedError

    def build_ff(self, m, ins):
        raise NotImplementedError

    # -- weights (Keras API; layer_base.py:102-120) --------------------------------
    def get_weights(self, model):
        """(kernel, bias) of the layer; ``model`` is the Keras model or its ``ffmodel``."""
        ff = getattr(model, "ffmodel", model)
        return [w.get_weights(ff) for w in (self.ff_op.weights if self.ff_op else [])]

    def set_weights(self, model, *arrays):
        """``set_weights(ffmodel, kernel, bias)`` (reference ``layer_base.py``) or
        ``set_weights(model, [kernel, bias])``."""
        ff = getattr(model, "ffmodel", model)
        if len(arrays) == 1 and isinstance(arrays[0], (list, tuple)):
            arrays = arrays[0]
        for w, a in zip(self.ff_op.weights, arrays):
            w.set_weights(ff, a)

    def get_summary(self):
        return f"{self.name:24s} {type(self).__name__:20s} {str(self.outputs[0].batch_shape) if self.outputs else ''}\n"

    def __repr__(self):
        return f"{type(self).__name__}({self.name})"


class InputLayer(Layer):
    default_name = "input"

    def __init__(self, shape=None, batch_size=None, dtype="float32", name=None, **kwargs):
        super().__init__(name)
        self.outputs = [KTensor(shape, _DT.get(dtype, dtype) if isinstance(dtype, str) else dtype, self, 0)]


def Input(shape=None, batch_size=None, dtype="float32", name=None, **kwargs):
    return InputLayer(shape, batch_size, dtype, name).outputs[0]


class Dense(Layer):
    default_name = "dense"

    def __init__(self, units, input_shape=None, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", name=None, **kwargs):
        super().__init__(name, input_shape)
        self.units = int(units)
        self.activation = _ACT[activation]
        self.use_bias = use_bias
        self.kinit, self.binit = _init(kernel_initializer), _init(bias_initializer)

    def compute_output_shape(self, shapes):
        return [shapes[0][:-1] + (self.units,)]

    def build_ff(self, m, ins):
        return m.dense(ins[0], self.units, self.activation, self.use_bias, kernel_initializer=self.kinit,
                       bias_initializer=self.binit, name=self.name)


class Conv2D(Layer):
    default_name = "conv2d"

    def __init__(self, filters, input_shape=None, kernel_size=0, strides=(1, 1), padding="valid", data_format=None,
                 dilation_rate=(1, 1), groups=1, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", name=None, **kwargs):
        if data_format == "channels_last":
            raise ValueError("data_format channels_last is not supported (NCHW only)")
        if _pair(dilation_rate) != (1, 1):
            raise ValueError("dilation_rate is not supported")
        super().__init__(name, input_shape)
        self.filters = int(filters)
        self.kernel = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding
        self.groups = groups
        self.activation = _ACT[activation]
        self.use_bias = use_bias
        self.kinit, self.binit = _init(kernel_initializer), _init(bias_initializer)

    def _pads(self):
        if self.padding == "valid":
            return (0, 0)
        if self.padding == "same":
            return ((self.kernel[0] - 1) // 2, (self.kernel[1] - 1) // 2)
        return _pair(self.padding)

    def compute_output_shape(self, shapes):
        c, h, w = shapes[0]
        ph, pw = self._pads()
        return [(self.filters, 1 + (h + 2 * ph - self.kernel[0]) // self.strides[0],
                 1 + (w + 2 * pw - self.kernel[1]) // self.strides[1])]

    def build_ff(self, m, ins):
        ph, pw = self._pads()
        return m.conv2d(ins[0], self.filters, self.kernel[0], self.kernel[1], self.strides[0], self.strides[1], ph, pw,
                        self.activation, self.use_bias, kernel_initializer=self.kinit, bias_initializer=self.binit,
                        name=self.name, groups=self.groups)


class Pooling2D(Layer):
    default_name = "pool2d"
    pool_type = PoolType.POOL_MAX

    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", data_format=None, name=None, **kwargs):
        super().__init__(name)
        self.pool = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool
        self.padding = padding

    def _pads(self):
        if self.padding == "valid":
            return (0, 0)
        if self.padding == "same":
            return ((self.pool[0] - 1) // 2, (self.pool[1] - 1) // 2)
        return _pair(self.padding)

    def compute_output_shape(self, shapes):
        c, h, w = shapes[0]
        ph, pw = self._pads()
        return [(c, 1 + (h + 2 * ph - self.pool[0]) // self.strides[0], 1 + (w + 2 * pw - self.pool[1]) // self.strides[1])]

    def build_ff(self, m, ins):
        ph, pw = self._pads()
        return m.pool2d(ins[0], self.pool[0], self.pool[1], self.strides[0], self.strides[1], ph, pw, self.pool_type,
                        name=self.name)


class MaxPooling2D(Pooling2D):
    default_name = "maxpool2d"
    pool_type = PoolType.POOL_MAX


class AveragePooling2D(Pooling2D):
    default_name = "avgpool2d"
    pool_type = PoolType.POOL_AVG


class Flatten(Layer):
    default_name = "flat"

    def compute_output_shape(self, shapes):
        n = 1
        for d in shapes[0]:
            n *= d
        return [(n,)]

    def build_ff(self, m, ins):
        if len(ins[0].dims) == 2:
            return ins[0]
        return m.flat(ins[0], name=self.name)


class Activation(Layer):
    default_name = "activation"

    def __init__(self, activation=None, name=None, **kwargs):
        super().__init__(name)
        if activation not in ("softmax", "relu", "sigmoid", "tanh", "elu", "exp", None, "linear"):
            raise ValueError(f"unsupported activation {activation!r}")
        self.activation = activation

    def compute_output_shape(self, shapes):
        return [shapes[0]]

    def build_ff(self, m, ins):
        a = self.activation
        if a in (None, "linear"):
            return ins[0]
        return getattr(m, a)(ins[0], name=self.name)


class Dropout(Layer):
    default_name = "dropout"

    def __init__(self, rate, noise_shape=None, seed=None, name=None, **kwargs):
        super().__init__(name)
        self.rate, self.seed = float(rate), seed or 0

    def compute_output_shape(self, shapes):
        return [shapes[0]]

    def build_ff(self, m, ins):
        return m.dropout(ins[0], self.rate, self.seed, name=self.name)


class Reshape(Layer):
    default_name = "reshape"

    def __init__(self, target_shape, input_shape=None, name=None, **kwargs):
        super().__init__(name, input_shape)
        self.target = tuple(target_shape)

    def compute_output_shape(self, shapes):
        return [self.target]

    def build_ff(self, m, ins):
        return m.reshape(ins[0], [ins[0].dims[0]] + list(self.target), name=self.name)


class Embedding(Layer):
    default_name = "embedding"

    def __init__(self, input_dim, output_dim, embeddings_initializer="uniform", input_length=None, name=None, **kwargs):
        super().__init__(name)
        self.input_dim, self.output_dim = int(input_dim), int(output_dim)
        self.init = _init(embeddings_initializer) if embeddings_initializer != "uniform" else None

    def compute_output_shape(self, shapes):
        return [(self.output_dim,)]

    def build_ff(self, m, ins):
        return m.embedding(ins[0], self.input_dim, self.output_dim, AggrMode.AGGR_MODE_SUM,
                           kernel_initializer=self.init, name=self.name)


class BatchNormalization(Layer):
    default_name = "batch_normalization"

    def __init__(self, axis=1, relu=False, name=None, **kwargs):
        super().__init__(name)
        self.relu = relu

    def compute_output_shape(self, shapes):
        return [shapes[0]]

    def build_ff(self, m, ins):
        return m.batch_norm(ins[0], self.relu, name=self.name)


class _Merge(Layer):
    def compute_output_shape(self, shapes):
        return [shapes[0]]


class Concatenate(_Merge):
    default_name = "concatenate"

    def __init__(self, axis=1, name=None, **kwargs):
        super().__init__(name)
        self.axis = axis

    def compute_output_shape(self, shapes):
        ax = self.axis - 1 if self.axis > 0 else len(shapes[0]) + self.axis
        out = list(shapes[0])
        out[ax] = sum(s[ax] for s in shapes)
        return [tuple(out)]

    def build_ff(self, m, ins):
        return m.concat(ins, self.axis, name=self.name)


class Add(_Merge):
    default_name = "add"

    def build_ff(self, m, ins):
        t = ins[0]
        for u in ins[1:]:
            t = m.add(t, u)
        return t


class Subtract(_Merge):
    default_name = "subtract"

    def build_ff(self, m, ins):
        return m.subtract(ins[0], ins[1], name=self.name)


class Multiply(_Merge):
    default_name = "multiply"

    def build_ff(self, m, ins):
        t = ins[0]
        for u in ins[1:]:
            t = m.multiply(t, u)
        return t


def concatenate(tensors, axis=1, **kw):
    return Concatenate(axis, **kw)(tensors)


def add(tensors, **kw):
    return Add(**kw)(tensors)


def subtract(tensors, **kw):
    return Subtract(**kw)(tensors)


def multiply(tensors, **kw):
    return Multiply(**kw)(tensors)
