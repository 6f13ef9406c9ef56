"""Embedding bag (``OP_EMBEDDING``).

Reference: ``src/ops/embedding.cu`` -- lookup ``out[b,:] = Σ_j W[idx[b,j],:]`` (``:173-197``),
backward = atomicAdd of the output grad into a dense ``W_grad`` (``:199-224``), partitions
allow only the sample dim or whole-table placement (``:108-135``).  AVG divided inside the bag
loop (bug, ``:187-195``); here AVG divides once.

MI355X: ``csrc/kernels/embedding.hip`` -- lanes gather whole rows with 16-B loads and write bf16
activations; the executor fuses all embedding ops of one placement into ONE launch (descriptor
table).  The backward never materialises a dense gradient for SGD: rows are updated in place
(W[idx] -= lr*dy).  Mostly-unique (large) tables use owner-computes: each row is claimed by one
lookup (CAS), duplicates add with atomics, the owner applies a plain 16-B read-modify-write;
other tables use 256-B-contiguous fp32 atomics; tiny tables accumulate in LDS first.
SOAP: sample split, **column (parameter) split** of the table and whole-table placement
(``dims=[1,1]``, device k) -- a 100 M-row table fits one MI355X's 288 GB of HBM.
"""
from __future__ import annotations

import math
import os

import torch

from flexmi.core.initializers import UniformInitializer
from flexmi.core.types import AggrMode, DataType, OperatorType
from flexmi.parallel.layout import Layout

from .base import Op, OpCtx, store
from . import _kernels as K


class Embedding(Op):
    op_type = OperatorType.OP_EMBEDDING
    name_prefix = "Embed"

    def __init__(self, model, input, num_entries, out_dim, aggr=AggrMode.AGGR_MODE_SUM,
                 kernel_initializer=None, name=None):
        super().__init__(model, [input], name)
        self.num_entries = int(num_entries)
        self.out_dim = int(out_dim)
        self.aggr = AggrMode(aggr)
        if self.name is None:
            self.name = self.auto_name(f"{num_entries}x{out_dim}")
        if kernel_initializer is None:
            r = math.sqrt(1.0 / self.num_entries)
            kernel_initializer = UniformInitializer(model._next_seed() if model else 0, -r, r)
        self._add_weight((self.num_entries, self.out_dim), kernel_initializer, "weight")
        self._finish([(input.dims[0], self.out_dim)])
        # set by the executor when a fused sparse optimizer applies to this table
        self.sparse_sgd = False

    def splittable_dims(self):
        return {0, 1}

    def input_layouts(self, pc):
        out = Layout.from_pc(self.outputs[0].dims, pc)
        n, c = out.degrees
        holders = [tuple(out.holders[i * c + j][0] for j in range(c)) for i in range(n)]
        return [Layout(self.inputs[0].dims, (n, 1), holders)]

    def weight_layouts(self, pc):
        out = Layout.from_pc(self.outputs[0].dims, pc)
        n, c = out.degrees
        holders = [tuple(out.holders[i * c + j][0] for i in range(n)) for j in range(c)]
        return [Layout(self.weights[0].dims, (1, c), holders)]

    def needs_input_grad(self, i):
        return False

    # ---------------------------------------------------------- compute
    def forward(self, ctx: OpCtx):
        idx = ctx.inputs[0]
        w = ctx.weights[0]
        out = ctx.outputs[0]
        if ctx.hip:
            K.embedding_forward(idx, w, out, int(self.aggr))
        else:
            bag = idx.shape[1]
            rows = w.index_select(0, idx.reshape(-1).long()).view(idx.shape[0], bag, -1)
            r = rows.sum(1)
            if self.aggr == AggrMode.AGGR_MODE_AVG:
                r = r / bag
            out.copy_(r)

    def backward(self, ctx: OpCtx):
        idx = ctx.inputs[0]
        dy = ctx.out_grads[0]
        if self.sparse_sgd:
            # fused sparse SGD (no dense grad): W[idx] -= lr * dy  (duplicates summed first)
            if ctx.hip:
                Embedding.backward_group([self], [ctx])
            else:
                g = dy.float()
                if self.aggr == AggrMode.AGGR_MODE_AVG:
                    g = g / idx.shape[1]
                bag = idx.shape[1]
                flat = idx.reshape(-1).long()
                gg = g.repeat_interleave(bag, dim=0)
                upd = torch.zeros_like(ctx.weights[0])
                upd.index_add_(0, flat, gg)
                ctx.weights[0].sub_(ctx.lr.to(upd.dtype) * upd)
            return
        dw = ctx.weight_grads[0]
        if ctx.hip:
            K.embedding_backward_dense(idx, dy, dw, int(self.aggr))
        else:
            g = dy.float()
            if self.aggr == AggrMode.AGGR_MODE_AVG:
                g = g / idx.shape[1]
            bag = idx.shape[1]
            dw.zero_()
            dw.index_add_(0, idx.reshape(-1).long(), g.repeat_interleave(bag, dim=0))

    # ---------------------------------------------------------- fused groups
    @staticmethod
    def can_group(a, b, ca, cb):
        """Executor fusion: independent embeddings with the same placement run as ONE launch."""
        return (ca.outputs[0].dtype == cb.outputs[0].dtype and a.sparse_sgd == b.sparse_sgd
                and ca.inputs[0].shape[0] == cb.inputs[0].shape[0])

    @staticmethod
    def forward_group(ops, ctxs):
        if not ctxs[0].hip:
            for op, c in zip(ops, ctxs):
                op.forward(c)
            return
        K.C().embedding_fwd_multi([c.weights[0] for c in ctxs], [c.inputs[0] for c in ctxs],
                                  [c.outputs[0] for c in ctxs], [c.outputs[0].stride(0) for c in ctxs],
                                  [1.0 / c.inputs[0].shape[1] if op.aggr == AggrMode.AGGR_MODE_AVG else 1.0
                                   for op, c in zip(ops, ctxs)])

    @staticmethod
    def backward_group(ops, ctxs):
        if not ctxs[0].hip:
            for op, c in zip(ops, ctxs):
                op.backward(c)
            return
        scales = [1.0 / c.inputs[0].shape[1] if op.aggr == AggrMode.AGGR_MODE_AVG else 1.0 for op, c in zip(ops, ctxs)]
        if ops[0].sparse_sgd:
            tables = [c.weights[0] for c in ctxs]
            lr = ctxs[0].lr
        else:
            tables = [c.weight_grads[0] for c in ctxs]
            for t in tables:
                t.zero_()
            lr = None
        claim = None
        if ops[0].sparse_sgd:
            bufs = [op._claim_buffers(c) for op, c in zip(ops, ctxs)]
            if any(b is not None for b in bufs):
                claim = []
                for b in bufs:
                    claim.extend(b if b is not None else (None, None, None))
        K.C().embedding_bwd_multi(tables, [c.inputs[0] for c in ctxs], [c.out_grads[0] for c in ctxs],
                                  [c.out_grads[0].stride(0) for c in ctxs], scales, lr, claim)

    CLAIM = os.environ.get("FM_EMB_CLAIM", "1") != "0"

    def _claim_buffers(self, ctx):
        """Owner-computes sparse SGD buffers for a mostly-unique table (rows > lookups per step):
        a per-row claim slot (int32, -1 = free; restored after every step), the duplicate list
        and its counter.  Smaller tables keep the atomic / LDS-privatised kernels."""
        if not Embedding.CLAIM:
            return None
        s = ctx.saved
        if "claim" not in s:
            w, idx = ctx.weights[0], ctx.inputs[0]
            if w.shape[0] > idx.numel() and self.out_dim % 4 == 0:
                dev = w.device
                s["claim"] = (torch.full((w.shape[0],), -1, dtype=torch.int32, device=dev),
                              torch.empty(idx.numel(), dtype=torch.int32, device=dev),
                              torch.zeros(1, dtype=torch.int32, device=dev))
            else:
                s["claim"] = None
        return s["claim"]

    def flops(self, in_shapes, out_shapes):
        return float(in_shapes[0][0] * in_shapes[0][1] * out_shapes[0][1])

    def bytes_moved(self, in_shapes, out_shapes, elem=2):
        b, bag = in_shapes[0]
        d = out_shapes[0][1]
        return float(b * bag * d * 4 + b * d * elem + b * bag * 8)
