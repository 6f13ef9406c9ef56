"""Operators (graph semantics + parallel layouts + local compute) and HIP kernel bindings."""
import flexmi.core  # noqa: F401  (initialise core first: core.model imports the ops)
from .base import Op, OpCtx  # noqa
from .linear import Linear  # noqa
from .embedding import Embedding  # noqa
from .elementwise import ElementUnary, ElementBinary  # noqa
from .tensor_ops import Concat, Split, Flat, Reshape, Transpose, Reverse  # noqa
from .nn_ops import Softmax, Dropout, BatchMatmul, DotInteraction  # noqa
from .conv import Conv2D, Pool2D, BatchNorm  # noqa
from .rnn import LSTM  # noqa
