"""flexmi.keras -- the Keras frontend of the reference (``python/flexflow/keras``): Sequential and
functional models, layers, losses, metrics, optimizers, callbacks, initializers and datasets,
lowered onto flexmi's FFModel (so strategies, search and the MI355X kernels apply unchanged)."""
from . import callbacks, datasets, initializers, layers, losses, metrics, optimizers  # noqa: F401
from .models import Model, Sequential  # noqa: F401
