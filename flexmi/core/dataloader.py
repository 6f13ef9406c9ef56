"""Data loaders (``python/flexflow_dataloader.{h,cc,cu}``; DLRM ``examples/cpp/DLRM/dlrm.cc:266-589``).

Reference: the full dataset lives in zero-copy host memory; per shard a GPU task gathers the
shard's sample indices into a pinned buffer and copies H2D (``dlrm.cu:19-122``).  flexmi: the
full array stays in (pinned) host memory or -- for synthetic/benchmark data -- in HBM; every rank
copies ONLY the rows of its own shard of each input (the tensor's home layout, so an embedding
table placed on rank k receives the full batch of its feature on rank k only) with an async copy.
"""
from __future__ import annotations

import numpy as np
import torch

from .types import DataType, to_torch_dtype


def _as_torch(full, pin):
    if hasattr(full, "_attached"):
        full = full._attached
    if isinstance(full, np.ndarray):
        full = torch.from_numpy(np.ascontiguousarray(full))
    if pin and not full.is_cuda and torch.cuda.is_available():
        try:
            full = full.pin_memory()
        except RuntimeError:
            pass
    return full


class SingleDataLoader:
    def __init__(self, ffmodel, input, full_input, num_samples, data_type=None, device_resident=False):
        self.model = ffmodel
        self.input = input
        gpu = ffmodel.config.device == "gpu"
        self.full = _as_torch(full_input, gpu and not device_resident)
        if device_resident and gpu:
            self.full = self.full.to(ffmodel.config.torch_device)
        self.num_samples = int(num_samples)
        self.next_index = 0
        self.batch_size = input.dims[0]

    def set_num_samples(self, samples):
        self.num_samples = int(samples)

    def get_num_samples(self):
        return self.num_samples

    def next_batch(self, ffmodel=None):
        m = ffmodel or self.model
        if self.next_index + self.batch_size > self.num_samples:
            self.next_index = 0
        m._ex().load_batch(self.input, self.full, self.next_index)
        self.next_index += self.batch_size

    def reset(self):
        self.next_index = 0


class DataLoader2D:
    """Input + label pair loader (``flexflow_cbinding.py:1006-1025``)."""

    def __init__(self, ffmodel, input, label, full_input=None, full_label=None, num_samples=0):
        self.a = SingleDataLoader(ffmodel, input, full_input, num_samples)
        self.b = SingleDataLoader(ffmodel, label, full_label, num_samples)

    def set_num_samples(self, samples):
        self.a.set_num_samples(samples)
        self.b.set_num_samples(samples)

    def get_num_samples(self):
        return self.a.get_num_samples()

    def next_batch(self, ffmodel=None):
        self.a.next_batch(ffmodel)
        self.b.next_batch(ffmodel)

    def reset(self):
        self.a.reset()
        self.b.reset()


DataLoader4D = DataLoader2D


class NetConfig:
    def __init__(self):
        self.dataset_path = ""
