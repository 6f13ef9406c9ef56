"""flexmi.torch -- PyTorch frontend (``python/flexflow/torch``): torch.fx -> ``.ff`` text format ->
FFModel, plus weight transfer from the torch module."""
from .fx import torch_to_flexflow  # noqa: F401
from .model import PyTorchModel, copy_weights, from_torch  # noqa: F401
