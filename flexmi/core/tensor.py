"""Logical tensors and parameters of the model graph.

``struct Tensor`` / ``struct Parameter`` of the reference (``include/model.h:181-231``)
held Legion regions; here a Tensor is a graph handle and the executor owns the per-rank
shard buffers (plain HIP allocations through PyTorch-ROCm).  The host-view API
(``inline_map`` / ``get_array`` / ``attach_numpy_array`` / ``set_weights`` ...) keeps the
reference's semantics: mapping gathers the full logical tensor to
the host, unmapping scatters it back to every shard/replica.
"""
from __future__ import annotations

import itertools

import numpy as np
import torch

from .types import DataType, to_torch_dtype

_guid = itertools.count(1000)


class Tensor:
    def __init__(self, dims, data_type=DataType.DT_FLOAT, owner_op=None, owner_idx=0,
                 create_grad=True, model=None, name=None):
        self.dims = tuple(int(d) for d in dims)
        self.data_type = DataType(data_type)
        self.owner_op = owner_op
        self.owner_idx = owner_idx
        self.create_grad = create_grad
        self.model = model
        self.guid = next(_guid)
        self.name = name or f"tensor_{self.guid}"
        self._mapped = None

    # reference attribute spellings -------------------------------------
    @property
    def num_dims(self):
        return len(self.dims)

    @property
    def adim(self):
        """Reference-internal (reversed) dims, ``src/runtime/model.cc:492-495``."""
        return tuple(reversed(self.dims))

    def volume(self):
        v = 1
        for d in self.dims:
            v *= d
        return v

    @property
    def torch_dtype(self):
        return to_torch_dtype(self.data_type)

    def __repr__(self):
        return f"Tensor({self.name}, dims={list(self.dims)}, {self.data_type.name})"

    # host-view API -----------------------------------------------------
    def _executor(self, ffmodel=None):
        m = ffmodel if ffmodel is not None else self.model
        ex = getattr(m, "executor", None)
        if ex is None and getattr(m, "loss_op", None) is not None:
            # compiled but not initialised: weights exist from compile on in the reference
            # (set_weights between compile and init_layers, keras net2net examples)
            ex = m.init_layers()
        assert ex is not None, "model is not compiled/initialised"
        return ex

    def _live(self):
        """The executor holding this tensor's shards, or None (model not initialised yet, or a
        host-only tensor such as a full dataset that no op consumes)."""
        ex = getattr(self.model, "executor", None)
        if ex is None or self.guid not in ex.home:
            return None
        return ex

    def _host_dtype(self):
        return np.float32 if self.data_type in (DataType.DT_FLOAT, DataType.DT_HALF, DataType.DT_DOUBLE) \
            else torch.empty(0, dtype=self.torch_dtype).numpy().dtype

    def inline_map(self, ffconfig=None):
        """Host view of the whole logical tensor.  Before ``init_layers`` (the reference maps
        input/label regions between compile and init, ``mnist_mlp_attach.py``) the view is a
        host staging array that ``init_layers`` scatters to the shards."""
        ex = self._live()
        if ex is not None:
            self._mapped = ex.gather_to_host(self)
        else:
            pend = getattr(self, "_pending", None)
            if pend is None:
                att = getattr(self, "_attached", None)
                pend = att.numpy().copy() if att is not None else np.zeros(self.dims, self._host_dtype())
            self._mapped = pend
        return self._mapped

    def inline_unmap(self, ffconfig=None):
        if self._mapped is not None:
            ex = self._live()
            if ex is not None:
                ex.scatter_from_host(self, self._mapped)
            else:
                self._pending = self._mapped
        self._mapped = None

    def is_mapped(self):
        return self._mapped is not None or getattr(self, "_attached", None) is not None

    def get_array(self, ffconfig=None, data_type=None):
        if self._mapped is None:
            att = getattr(self, "_attached", None)
            if att is not None and self._live() is None:
                return att.numpy()
            self.inline_map(ffconfig)
        return self._mapped

    def get_flat_array(self, ffconfig=None, data_type=None):
        return self.get_array(ffconfig, data_type).reshape(-1)

    def attach_numpy_array(self, ffconfig, np_array):
        """Zero-copy attach of a host array (``src/runtime/model.cc:73-86``)."""
        arr = np.ascontiguousarray(np_array)
        assert tuple(arr.shape) == self.dims or arr.size == self.volume(), (arr.shape, self.dims)
        self._attached = torch.from_numpy(arr.reshape(self.dims))
        # a tensor the graph consumes (an input / label): its shards take the attached contents
        # now, or at init_layers; a host-only tensor (a full dataset) is read by the loaders
        ex = self._live()
        if ex is not None:
            ex.scatter_from_host(self, arr)
        else:
            self._pending = arr.reshape(self.dims)
        return self._attached

    def detach_numpy_array(self, ffconfig=None):
        # the loaders keep their own reference; dropping ours mirrors detach_raw_ptr
        self._attached = None
        self._mapped = None

    def get_raw_ptr(self, ffmodel=None, ffconfig=None):
        """Device address of this rank's shard buffer (``Tensor::get_raw_ptr``,
        ``src/runtime/model.cc:46-71``: the reference returned the pointer of the mapped
        region; flexmi shards are plain HIP allocations owned by the executor)."""
        buf = self._executor(ffmodel).local_buffer(self)
        return 0 if buf is None else int(buf.data_ptr())

    def attach_raw_ptr(self, ffmodel, raw_ptr, column_major=False):
        """Zero-copy attach of host memory at ``raw_ptr`` holding the whole logical tensor
        (``Tensor::attach_raw_ptr``, ``src/runtime/model.cc:73-86``).  column_major=True means
        the array is stored with the reference's internal (reversed) dim order."""
        import ctypes
        dt = np.dtype(torch.empty(0, dtype=self.torch_dtype).numpy().dtype)
        n = self.volume()
        buf = (ctypes.c_char * (n * dt.itemsize)).from_address(int(raw_ptr))
        arr = np.frombuffer(buf, dtype=dt, count=n)
        arr = arr.reshape(self.adim).transpose() if column_major else arr.reshape(self.dims)
        self._attached = torch.from_numpy(np.ascontiguousarray(arr) if column_major else arr)
        self._raw_ptr = int(raw_ptr)
        return self._attached

    def detach_raw_ptr(self, ffmodel=None, ffconfig=None):
        self._attached = None
        self._raw_ptr = None

    def get_owner_op(self):
        return self.owner_op


class Parameter(Tensor):
    """Weight tensor of an op (``include/model.h:219-231``)."""

    def __init__(self, dims, data_type=DataType.DT_FLOAT, owner_op=None, owner_idx=0,
                 model=None, name=None, initializer=None, sync_type=None):
        super().__init__(dims, data_type, owner_op, owner_idx, True, model, name)
        self.initializer = initializer
        self.pcname = name

    def set_weights(self, ffmodel, np_array):
        arr = np.asarray(np_array, dtype=np.float32)
        assert arr.size == self.volume(), (arr.shape, self.dims)
        self._executor(ffmodel).set_param_full(self, torch.from_numpy(arr.reshape(self.dims).copy()))
        return True

    def get_weights(self, ffmodel=None):
        return self._executor(ffmodel).get_param_full(self).numpy()

    # a mapped parameter is its full master copy; unmapping writes it back to every shard
    def inline_map(self, ffconfig=None):
        self._mapped = self.get_weights()
        return self._mapped

    def inline_unmap(self, ffconfig=None):
        if self._mapped is not None:
            self.set_weights(self.model, self._mapped)
        self._mapped = None

    def get_array(self, ffconfig=None, data_type=None):
        if self._mapped is None:
            self.inline_map(ffconfig)
        return self._mapped

    def __repr__(self):
        return f"Parameter({self.name}, dims={list(self.dims)})"
