"""Per-op cost model for the simulator: measured MI355X cost DB + calibrated roofline.

Reference: ``Op::measure_compute_time`` ran each op's forward/backward kernels on GPU 0 for
a shard shape (5 warm-up + 10 timed runs, e.g. ``src/ops/linear.cu:973-1049``) and memoised
the result by (op, config) hash (``src/runtime/simulator.cc:235-273``).

flexmi separates measurement from search: ``tools/calibrate_costs.py`` measures every op of a
model on a real MI355X at the shard shapes its candidate configs produce and writes a JSON cost
DB (``flexmi/parallel/costdb/mi355x.json``).  At search time an exact (op type, shard shapes)
hit returns the measured time; a miss uses a roofline (MFMA FLOPs vs HBM bytes, plus the
kernel-boundary cost inside a hipGraph) scaled by the per-op-type ratio measured/roofline
fitted from the DB.  Searching therefore needs no GPU.
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Sequence, Tuple

from flexmi.core.types import ActiMode, OperatorType

DEFAULT_DB = os.path.join(os.path.dirname(__file__), "costdb", "mi355x.json")            # bf16 kernels
DEFAULT_DB_FP32 = os.path.join(os.path.dirname(__file__), "costdb", "mi355x_fp32.json")  # fp32 kernels


def _prod(s):
    n = 1
    for d in s:
        n *= int(d)
    return n


def op_signature(op, in_shapes, out_shapes) -> str:
    extra = ""
    if hasattr(op, "activation"):
        extra += f"|act={int(op.activation)}"
    if op.op_type == OperatorType.OP_EMBEDDING:
        extra += f"|rows={op.num_entries}"
    if op.op_type == OperatorType.OP_LINEAR and op.inputs[0].owner_op is None:
        extra += "|nodx"       # first layer: no input gradient GEMM
    return (f"{op.op_type.name}|in={';'.join('x'.join(map(str, s)) for s in in_shapes)}"
            f"|out={';'.join('x'.join(map(str, s)) for s in out_shapes)}{extra}")


class CostModel:
    def __init__(self, machine, db_path=None, dtype_bytes=2):
        self.m = machine
        self.eb = dtype_bytes
        self.db: Dict[str, Tuple[float, float]] = {}
        self.scale: Dict[str, float] = {}
        self.group_factor: Dict[str, float] = {}   # fused-launch / isolated per-op time (measured)
        path = db_path if db_path is not None else (DEFAULT_DB_FP32 if dtype_bytes == 4 else DEFAULT_DB)
        if path and os.path.exists(path):
            self.load_db(path)

    # ----------------------------------------------------------------- DB
    def load_db(self, path):
        with open(path) as f:
            d = json.load(f)
        for k, v in d.get("entries", {}).items():
            self.db[k] = (float(v[0]), float(v[1]))
        self.scale.update({k: float(v) for k, v in d.get("scale", {}).items()})
        self.group_factor.update({k: float(v) for k, v in d.get("group_factor", {}).items()})

    @staticmethod
    def fit_scales(entries: Dict[str, Tuple[float, float]], roofline: Dict[str, Tuple[float, float]]):
        """Per op type geometric mean of measured/roofline (fwd+bwd)."""
        acc: Dict[str, List[float]] = {}
        for k, (f, b) in entries.items():
            if k not in roofline:
                continue
            rf, rb = roofline[k]
            if rf + rb <= 0 or f + b <= 0:
                continue
            acc.setdefault(k.split("|")[0], []).append(math.log((f + b) / (rf + rb)))
        return {t: math.exp(sum(v) / len(v)) for t, v in acc.items()}

    # ----------------------------------------------------------------- model
    def _gemm_us(self, M, N, K):
        m = self.m
        tiles = math.ceil(M / 128) * math.ceil(N / 64)
        fill = min(1.0, tiles / 256.0)
        eff = m.mfma_eff * max(0.2, fill)
        peak = m.peak_bf16_tflops if self.eb == 2 else m.peak_fp32_tflops
        t_c = 2.0 * M * N * K / (peak * 1e12 * eff) * 1e6
        t_m = (M * K + N * K + M * N) * self.eb / (m.hbm_GBps * 1e9 * m.hbm_eff) * 1e6
        return max(t_c, t_m)

    def _bytes_us(self, nbytes):
        return nbytes / (self.m.hbm_GBps * 1e9 * self.m.hbm_eff) * 1e6

    def roofline(self, op, in_shapes: Sequence[Sequence[int]], out_shapes: Sequence[Sequence[int]]):
        """(fwd_us, bwd_us) of one shard without DB scaling."""
        t = op.op_type
        L = self.m.launch_us
        eb = self.eb
        peak = self.m.peak_bf16_tflops if eb == 2 else self.m.peak_fp32_tflops
        if getattr(op, "is_view", False) or t in (OperatorType.OP_FLAT, OperatorType.OP_RESHAPE):
            return 0.0, 0.0
        if t == OperatorType.OP_LINEAR:
            K = in_shapes[0][-1]
            N = out_shapes[0][-1]
            M = _prod(out_shapes[0][:-1])
            f = L + self._gemm_us(M, N, K)
            b = 2 * L + self._gemm_us(N, K, M) + self._gemm_us(M, K, N)
            if op.activation != ActiMode.AC_MODE_NONE:
                b += self._bytes_us(2 * M * N * eb) * 0.5
            return f, b
        if t == OperatorType.OP_EMBEDDING:
            B = in_shapes[0][0]
            bag = in_shapes[0][1] if len(in_shapes[0]) > 1 else 1
            D = out_shapes[0][-1]
            # grouped launches: one kernel per placement, so a small per-table share of a boundary
            f = 0.25 * L + self._bytes_us(B * bag * D * 4 * 1.25 + B * D * eb)
            b = 0.25 * L + B * bag * D * 4 / (self.m.atomic_TBps * 1e12) * 1e6 + self._bytes_us(B * D * eb)
            return f, b
        if t == OperatorType.OP_BATCHMATMUL:
            a, bb = in_shapes[0], in_shapes[1]
            nb = _prod(a[:-2])
            M, K, N = a[-2], a[-1], bb[-1]
            fl = 2.0 * nb * M * N * K
            tc = fl / (peak * 1e12 * self.m.mfma_eff) * 1e6
            tm = self._bytes_us((nb * (M * K + K * N + M * N)) * eb)
            return L + max(tc, tm), 2 * L + 2 * max(tc, tm)
        if t == OperatorType.OP_CONV2D:
            n, c, h, w = in_shapes[0]
            _, k, p, q = out_shapes[0]
            kh, kw = getattr(op, "kh", 3), getattr(op, "kw", 3)
            fl = 2.0 * n * k * p * q * c * kh * kw
            tc = fl / (peak * 1e12 * self.m.mfma_eff) * 1e6
            tm = self._bytes_us((n * c * h * w + n * k * p * q) * eb)
            return L + max(tc, tm), 3 * L + 2 * max(tc, tm)
        if t == OperatorType.OP_DOT_INTERACTION:
            fl = 2.0 * in_shapes[0][0] * op.F * op.F * op.d
            byt = sum(_prod(s) for s in list(in_shapes) + list(out_shapes)) * eb
            tc = fl / (peak * 1e12 * self.m.mfma_eff * 0.5) * 1e6
            return L + max(tc, self._bytes_us(byt)), L + 2 * max(tc, self._bytes_us(byt))
        # bandwidth-bound ops (elementwise, concat/split, softmax, pool, BN, transpose, ...)
        byt = sum(_prod(s) for s in list(in_shapes) + list(out_shapes)) * eb
        return L + self._bytes_us(byt), L + self._bytes_us(2 * byt)

    @staticmethod
    def kernels(op):
        """(forward, backward) kernel launches of one op shard in a captured step (grouped
        embedding tables share one launch per group: a quarter each)."""
        t = op.op_type
        if getattr(op, "is_view", False) or t in (OperatorType.OP_FLAT, OperatorType.OP_RESHAPE):
            return 0.0, 0.0
        if t == OperatorType.OP_LINEAR:
            return 1.0, 2.0 if op.inputs[0].owner_op is None else 3.0
        if t == OperatorType.OP_EMBEDDING:
            return 0.25, 0.25
        if t in (OperatorType.OP_CONV2D,):
            return 1.0, 3.0
        if t == OperatorType.OP_BATCHMATMUL:
            return 1.0, 2.0
        return 1.0, 1.0

    def op_cost(self, op, in_shapes, out_shapes):
        """Measured (DB hit) or scaled roofline time of one shard.  A roofline miss scales only
        its work terms by the fitted measured/roofline ratio, not its kernel boundaries, and no
        launch runs shorter than the machine's kernel floor: the small-batch configs are
        launch-bound (criteo_kaggle projected -57 % before)."""
        key = op_signature(op, in_shapes, out_shapes)
        hit = self.db.get(key)
        nkf, nkb = self.kernels(op)
        floor = getattr(self.m, "kernel_floor_us", 0.0)
        if hit is not None:
            gf = self.group_factor.get(op.op_type.name, 1.0)
            return max(hit[0] * gf, nkf * floor), max(hit[1] * gf, nkb * floor)
        f, b = self.roofline(op, in_shapes, out_shapes)
        s = self.scale.get(op.op_type.name, 1.0)
        L = self.m.launch_us
        ff, fb = min(f, nkf * L), min(b, nkb * L)
        f = ff + s * (f - ff)
        b = fb + s * (b - fb)
        return max(f, nkf * floor), max(b, nkb * floor)

    def update_us(self, dense_param_bytes_fp32, nstates):
        """Fused optimizer update over a device's dense parameters (read master+grad+states,
        write master+states+bf16 copy)."""
        n = dense_param_bytes_fp32 / 4
        byt = n * (4 + 4 + 2 + 8 * nstates)
        return self._bytes_us(byt)

    def memory_bytes(self, weight_numel_dense, weight_numel_sparse, act_numel, nstates):
        return (weight_numel_dense * (4 + 4 + 2 + 4 * nstates) + weight_numel_sparse * 4
                + act_numel * self.eb * 2)
