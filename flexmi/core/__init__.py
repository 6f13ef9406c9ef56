"""Reference-compatible core API (``from flexmi.core import *`` mirrors ``from flexflow.core import *``)."""
from .types import *  # noqa
from .config import FFConfig  # noqa
from .tensor import Tensor, Parameter  # noqa
from .initializers import (Initializer, GlorotUniformInitializer, ZeroInitializer, UniformInitializer,  # noqa
                           NormInitializer, NormalInitializer, ConstantInitializer)
from .optimizers import SGDOptimizer, AdamOptimizer, Optimizer  # noqa
from .loss_metrics import PerfMetrics  # noqa
from .dataloader import SingleDataLoader, DataLoader2D, DataLoader4D, NetConfig, PrefetchLoader  # noqa
from .model import FFModel  # noqa
