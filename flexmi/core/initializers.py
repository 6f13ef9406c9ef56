"""Parameter initializers (``include/initializer.h:26-101``, ``src/runtime/initializer_kernel.cu``).

MI355X design: every initializer is a *counter-based* generator -- element ``i`` of the
logical tensor gets ``f(seed, i)`` -- so any shard of a tensor is initialised directly on its
own GPU (HIP kernel ``fm_init_fill`` in ``csrc/kernels/init.hip``) and a sharded init is
bit-identical to an unsharded one.  The reference instead ran one cuRAND task over the whole
region (``initializer_kernel.cu:24-295``), which cannot work for 100 GB embedding tables.

The hash is ``lowbias32`` applied twice (64-bit element index); the CPU path below and the
HIP kernel implement the same arithmetic.
"""
from __future__ import annotations

import math

import numpy as np
import torch

KIND_ZERO, KIND_CONSTANT, KIND_UNIFORM, KIND_NORMAL = 0, 1, 2, 3


def _lowbias32(x):
    x = x & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return x


def _hash(seed, idx):
    idx = idx.astype(np.uint64)
    lo = idx & np.uint64(0xFFFFFFFF)
    hi = idx >> np.uint64(32)
    s = np.uint64(seed & 0xFFFFFFFF)
    h = _lowbias32(hi ^ _lowbias32(s ^ np.uint64(0x9E3779B9)))
    return _lowbias32(lo ^ h)


def uniform01(seed, idx):
    return (_hash(seed, idx) >> np.uint64(8)).astype(np.float64) * (1.0 / 16777216.0)


def counter_fill_cpu(kind, seed, a, b, shape, box):
    """Fill the sub-box ``box`` of a logical tensor of ``shape`` (numpy, fp32)."""
    grids = np.meshgrid(*[np.arange(lo, hi, dtype=np.int64) for lo, hi in box], indexing="ij")
    strides = np.cumprod([1] + list(reversed(shape[1:])))[::-1]
    idx = np.zeros(grids[0].shape if grids else (), dtype=np.int64)
    for g, s in zip(grids, strides):
        idx = idx + g * int(s)
    if kind == KIND_ZERO:
        return np.zeros(idx.shape, np.float32)
    if kind == KIND_CONSTANT:
        return np.full(idx.shape, a, np.float32)
    if kind == KIND_UNIFORM:
        u = uniform01(seed, idx)
        return (a + (b - a) * u).astype(np.float32)
    # normal: Box-Muller on two independent streams
    u1 = uniform01(seed, 2 * idx)
    u2 = uniform01(seed, 2 * idx + 1)
    z = np.sqrt(-2.0 * np.log(1.0 - u1)) * np.cos(2.0 * math.pi * u2)
    return (a + b * z).astype(np.float32)


_CPU = False


def _native_cpu():
    """flexmi._cpu (native CPU kernels) or None when it is not built."""
    global _CPU
    if _CPU is False:
        try:
            from flexmi import _cpu as m
            _CPU = m if hasattr(m, "counter_fill") else None
        except ImportError:
            _CPU = None
    return _CPU


class Initializer:
    kind = KIND_ZERO

    def __init__(self):
        self.seed = 0

    def params(self, dims):
        """(kind, seed, a, b) for a logical tensor of ``dims``."""
        return (self.kind, self.seed, 0.0, 0.0)

    def fill(self, dims, box, out: torch.Tensor):
        """Fill ``out`` (the shard ``box`` of a logical tensor ``dims``) in place."""
        kind, seed, a, b = self.params(dims)
        if out.is_cuda:
            from flexmi.ops import _kernels as K
            K.init_fill(out, tuple(dims), tuple(box), kind, seed, float(a), float(b))
        elif _native_cpu() is not None and out.dtype == torch.float32 and out.is_contiguous():
            # csrc/cpu/init_metrics.cc: same values as the numpy oracle, on ATen's thread pool
            _native_cpu().counter_fill(out, [int(d) for d in dims], [(int(lo), int(hi)) for lo, hi in box],
                                       int(kind), int(seed), float(a), float(b))
        else:
            out.copy_(torch.from_numpy(counter_fill_cpu(kind, seed, a, b, tuple(dims), tuple(box))).reshape(out.shape))


class GlorotUniformInitializer(Initializer):
    """``GlorotUniform::init_task`` (``initializer_kernel.cu:87-163``): U(±sqrt(6/(fan_in+fan_out)))."""
    kind = KIND_UNIFORM

    def __init__(self, seed=0):
        super().__init__()
        self.seed = seed

    def params(self, dims):
        if len(dims) == 2:          # [out, in]
            fan_out, fan_in = dims[0], dims[1]
        elif len(dims) >= 3:        # conv [out, in, kh, kw]
            rf = 1
            for d in dims[2:]:
                rf *= d
            fan_in, fan_out = dims[1] * rf, dims[0] * rf
        else:
            fan_in = fan_out = dims[0]
        s = math.sqrt(6.0 / (fan_in + fan_out))
        return (self.kind, self.seed, -s, s)


class ZeroInitializer(Initializer):
    kind = KIND_ZERO


class ConstantInitializer(Initializer):
    kind = KIND_CONSTANT

    def __init__(self, value=0.0):
        super().__init__()
        self.value = value

    def params(self, dims):
        return (self.kind, 0, self.value, 0.0)


class UniformInitializer(Initializer):
    kind = KIND_UNIFORM

    def __init__(self, seed=0, minv=0.0, maxv=1.0):
        super().__init__()
        self.seed, self.minv, self.maxv = seed, minv, maxv

    def params(self, dims):
        return (self.kind, self.seed, self.minv, self.maxv)


class NormInitializer(Initializer):
    kind = KIND_NORMAL

    def __init__(self, seed=0, meanv=0.0, stddev=1.0):
        super().__init__()
        self.seed, self.meanv, self.stddev = seed, meanv, stddev

    def params(self, dims):
        return (self.kind, self.seed, self.meanv, self.stddev)


NormalInitializer = NormInitializer


class ColumnPaddedInitializer(Initializer):
    """Initialise a [rows, cols_padded] weight exactly like a [rows, cols_logical] one (same
    fan-in/out, same counter stream) with zero padding columns.  Used when flexmi pads a narrow
    input (DLRM's 13 dense features -> 16) for 16-B aligned GEMM rows: the padded model is
    numerically the unpadded one."""

    def __init__(self, base, logical_cols):
        super().__init__()
        self.base = base
        self.logical_cols = int(logical_cols)

    def fill(self, dims, box, out):
        rows, cols = dims
        (r0, r1), (c0, c1) = box
        out.zero_()
        lc1 = min(c1, self.logical_cols)
        if lc1 <= c0:
            return
        tmp = torch.empty((r1 - r0, lc1 - c0), dtype=out.dtype, device=out.device)
        self.base.fill((rows, self.logical_cols), ((r0, r1), (c0, lc1)), tmp)
        out[:, : lc1 - c0].copy_(tmp)
