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


def synthetic_pair(ffmodel, input, label, batches=4, seed=0):
    """Random full input / label arrays of ``batches`` batches (the reference loaders' random-data
    mode when no dataset is given): uniform inputs, integer labels in [0, 10) (uniform floats for
    float labels).  Returns (full_input, full_label, num_samples)."""
    rng = np.random.RandomState(seed)
    n = input.dims[0] * batches
    x = rng.rand(n, *input.dims[1:]).astype(np.float32)
    if label.data_type in (DataType.DT_INT32, DataType.DT_INT64):
        y = rng.randint(0, 10, (n,) + tuple(label.dims[1:])).astype(np.int32 if label.data_type == DataType.DT_INT32
                                                                      else np.int64)
    else:
        y = rng.rand(n, *label.dims[1:]).astype(np.float32)
    return x, y, n


def _host_array_as(arr, tdt):
    """``arr`` as a C-contiguous host array whose BYTES are elements of torch dtype ``tdt`` (the
    native ring copies raw bytes into the staging slots).  numpy has no bfloat16: a bf16 target
    is converted through torch (round to nearest even) and returned as its int16 bit pattern."""
    if tdt == torch.bfloat16:
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32)).to(torch.bfloat16)
        return t.view(torch.int16).numpy()
    npdt = torch.empty(0, dtype=tdt).numpy().dtype
    return np.ascontiguousarray(arr, dtype=npdt)


class NetConfig:
    def __init__(self):
        self.dataset_path = ""


class PrefetchLoader:
    """Multi-input prefetching loader on the native ring (``csrc/runtime/loader.{h,cc}``).

    ``pairs``: [(tensor, full host array [num_samples, ...])] or [(tensor, full 2-D array,
    (c0, c1))] -- inputs and the label; the 3-tuple form feeds columns c0:c1 of a wider array
    (zero-copy: e.g. one sparse feature of a memory-mapped ``X_cat``), and a source row narrower
    than the tensor row is zero-padded (the 13 dense features into a 16-wide GPU input).  Host
    worker threads gather each batch's rows (sequential or shuffled per epoch with ``seed``)
    into ``depth`` pinned staging slots ahead of the training loop; :meth:`next_batch` takes
    the next staged slot and issues one async H2D copy per input on the current stream, so
    the gather overlaps the previous step's compute.  Each rank stages only its shard box of
    every tensor (``python/flexflow_dataloader.cu:97-150`` gathered per shard on the GPU;
    ``dlrm.cu:19-122``)."""

    def __init__(self, ffmodel, pairs, num_samples, shuffle=False, seed=0, depth=3, threads=2):
        from flexmi import _native
        ex = ffmodel._ex()
        self.ex = ex
        self.gpu = ex.backend == "hip"
        B = pairs[0][0].dims[0]
        self.batch = B
        self.ring = _native.BatchRing(B, int(num_samples), depth, threads, bool(shuffle), int(seed))
        self.items = []
        self._keep = []
        for pair in pairs:
            t, full = pair[0], pair[1]
            cols = pair[2] if len(pair) > 2 else None
            buf = ex.local_buffer(t)
            if buf is None:
                continue
            assert t.dims[0] == B, "all inputs of a PrefetchLoader share the batch dimension"
            box = ex.home[t.guid].local_box(ex.rank)
            dims = list(t.dims)
            tdt = buf.dtype
            if cols is not None or (full.ndim == 2 and len(dims) == 2 and full.shape[1] < dims[1]):
                # column block of a 2-D source (zero-copy), zero-padded up to the tensor row
                c0, c1 = cols if cols is not None else (0, full.shape[1])
                arr = _host_array_as(np.asarray(full), tdt)
                es = arr.itemsize
                assert len(dims) == 2 and c1 - c0 <= dims[1] and box[1] == (0, dims[1]), \
                    "column-block sources feed whole rows of a 2-D input"
                self._keep.append(arr)
                si = self.ring.add_source(arr.ctypes.data, arr.shape[0], arr.shape[1] * es, c0 * es, (c1 - c0) * es,
                                          box[0][0], box[0][1], dims[1] * es)
                self._add_slots(si, buf, depth, zero=(c1 - c0) < dims[1])
                continue
            src = torch.as_tensor(np.ascontiguousarray(full)).reshape((-1,) + tuple(t.dims[1:]))
            if src.dtype != buf.dtype:
                src = src.to(buf.dtype)
            src = src.contiguous()
            self._keep.append(src)
            es = src.element_size()
            row_bytes = int(np.prod(dims[1:], dtype=np.int64)) * es
            split = [j for j in range(1, len(dims)) if box[j] != (0, dims[j])]
            if not split:
                col_off, col_bytes = 0, row_bytes
            else:
                d = split[0]
                if any(box[j][1] - box[j][0] != dims[j] for j in range(d + 1, len(dims))) or \
                        any(dims[j] != 1 for j in range(1, d)):
                    raise NotImplementedError(f"PrefetchLoader: shard box {box} of {t.name} is not a row slice")
                inner = int(np.prod(dims[d + 1:], dtype=np.int64)) * es
                col_off, col_bytes = box[d][0] * inner, (box[d][1] - box[d][0]) * inner
            si = self.ring.add_source(src.data_ptr(), src.shape[0], row_bytes, col_off, col_bytes, box[0][0], box[0][1])
            self._add_slots(si, buf, depth)
        self.pending = []
        self.depth = depth
        self.num_samples = int(num_samples)
        self.ring.start()

    def _add_slots(self, si, buf, depth, zero=False):
        stg = []
        for s in range(depth):
            st = (torch.zeros if zero else torch.empty)(tuple(buf.shape), dtype=buf.dtype, pin_memory=self.gpu)
            self.ring.set_slot(si, s, st.data_ptr())
            stg.append(st)
        self.items.append((buf, stg))

    def get_num_samples(self):
        return self.num_samples

    def _release_done(self, block=False):
        while self.pending:
            slot, ev = self.pending[0]
            if ev is not None and not ev.query():
                if not block:
                    break
                ev.synchronize()
            self.ring.release(slot)
            self.pending.pop(0)
            block = False

    def next_batch(self, ffmodel=None):
        self._release_done()
        if len(self.pending) >= self.depth - 1:
            self._release_done(block=True)
        slot = self.ring.acquire()
        for buf, stg in self.items:
            buf.copy_(stg[slot], non_blocking=self.gpu)
        ev = None
        if self.gpu:
            ev = torch.cuda.Event()
            ev.record()
        self.pending.append((slot, ev))
        if not self.gpu:
            self._release_done()

    def reset(self):
        for _, ev in self.pending:
            if ev is not None:
                ev.synchronize()
        self.pending = []
        self.ring.stop()
        self.ring.start()

    def close(self):
        self.reset()
        self.ring.stop()

    def __del__(self):
        try:
            self.ring.stop()
        except Exception:
            pass
