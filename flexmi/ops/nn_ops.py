"""Softmax, Dropout, BatchMatmul and the DLRM dot interaction.

Reference: ``src/ops/softmax.cu`` (cuDNN channel softmax; backward = copy because the CE loss
gradient already is ``p - y``, ``:223-266``), ``dropout.cu`` (cuDNN dropout, seed 0 -> random),
``batch_matmul.cu`` (cuBLAS strided-batched GEMM, ``O[b] = A[b]·B[b]`` with A ``(batch,n,k)``,
B ``(batch,k,m)``, ``:180-204``).  The reference DLRM supports only the ``cat`` interaction
(caveat C3, ``examples/cpp/DLRM/dlrm.cc:49-65``); :class:`DotInteraction` adds the DLRM ``dot``
interaction as one fused MFMA op (``csrc/kernels/interaction.hip``).
"""
from __future__ import annotations

import random

import torch

from flexmi.core.types import OperatorType
from flexmi.parallel.layout import Layout

from .base import Op, OpCtx, store
from . import _kernels as K


class Softmax(Op):
    op_type = OperatorType.OP_SOFTMAX
    name_prefix = "Softmax"

    def __init__(self, model, input, name=None):
        super().__init__(model, [input], name)
        if self.name is None:
            self.name = self.auto_name("")
        self._finish([input.dims])

    def splittable_dims(self):
        return set(range(self.out_ndims - 1))  # channel (last) dim unsplit

    def forward(self, ctx: OpCtx):
        x, y = ctx.inputs[0], ctx.outputs[0]
        if ctx.hip:
            K.softmax_forward(x, y)
        else:
            y.copy_(torch.softmax(x.float(), dim=-1))

    def backward(self, ctx: OpCtx):
        # identity: the loss already produced dL/dlogits (softmax.cu:251-253)
        if not ctx.in_grads or ctx.in_grads[0] is None:
            return
        if ctx.hip:
            K.copy_or_add(ctx.out_grads[0], ctx.in_grads[0], ctx.in_grad_accumulate[0])
        else:
            store(ctx.in_grads[0], ctx.out_grads[0], ctx.in_grad_accumulate[0])


class Dropout(Op):
    op_type = OperatorType.OP_DROPOUT
    name_prefix = "Dropout"

    def __init__(self, model, input, rate, seed=0, name=None):
        super().__init__(model, [input], name)
        self.rate = float(rate)
        self.seed = int(seed) if seed else random.randrange(1, 1 << 30)
        if self.name is None:
            self.name = self.auto_name("")
        self._finish([input.dims])
        self.step = 0

    def splittable_dims(self):
        return set(range(self.out_ndims))

    def forward(self, ctx: OpCtx):
        x, y = ctx.inputs[0], ctx.outputs[0]
        if not ctx.training or self.rate == 0.0:
            y.copy_(x)
            return
        ctx.saved["step"] = ctx.saved.get("step", 0) + 1
        if ctx.hip:
            K.dropout_forward(x, y, self.rate, self.seed, ctx)
        else:
            g = torch.Generator().manual_seed(self.seed * 7919 + ctx.saved["step"] + 131 * ctx.rank)
            mask = (torch.rand(x.shape, generator=g) >= self.rate).to(x.dtype) / (1.0 - self.rate)
            ctx.saved["mask"] = mask
            y.copy_(x * mask)

    def backward(self, ctx: OpCtx):
        if not ctx.in_grads or ctx.in_grads[0] is None:
            return
        dy, dx = ctx.out_grads[0], ctx.in_grads[0]
        if not ctx.training or self.rate == 0.0:
            store(dx, dy, ctx.in_grad_accumulate[0])
            return
        if ctx.hip:
            K.dropout_backward(dy, dx, self.rate, self.seed, ctx, ctx.in_grad_accumulate[0])
        else:
            store(dx, dy.float() * ctx.saved["mask"], ctx.in_grad_accumulate[0])


class BatchMatmul(Op):
    op_type = OperatorType.OP_BATCHMATMUL
    name_prefix = "BatchMatmul"

    def __init__(self, model, A, B, name=None):
        super().__init__(model, [A, B], name)
        assert len(A.dims) == len(B.dims) and len(A.dims) >= 3
        assert A.dims[:-2] == B.dims[:-2] and A.dims[-1] == B.dims[-2], (A.dims, B.dims)
        if self.name is None:
            self.name = self.auto_name("")
        self._finish([tuple(A.dims[:-1]) + (B.dims[-1],)])

    def splittable_dims(self):
        return set(range(self.out_ndims - 2))  # batch (outer) dims only

    def input_layouts(self, pc):
        lo = Layout.from_pc(self.outputs[0].dims, pc)
        return [Layout(t.dims, lo.degrees, lo.holders) for t in self.inputs]

    def forward(self, ctx: OpCtx):
        a, b, o = ctx.inputs[0], ctx.inputs[1], ctx.outputs[0]
        if ctx.hip:
            K.bmm(a, b, o, False, False, False)
        else:
            o.copy_(torch.matmul(a.float(), b.float()))

    def backward(self, ctx: OpCtx):
        a, b, do = ctx.inputs[0], ctx.inputs[1], ctx.out_grads[0]
        da = ctx.in_grads[0] if len(ctx.in_grads) > 0 else None
        db = ctx.in_grads[1] if len(ctx.in_grads) > 1 else None
        if ctx.hip:
            if da is not None:   # dA = dO · Bᵀ
                K.bmm(do, b, da, False, True, ctx.in_grad_accumulate[0])
            if db is not None:   # dB = Aᵀ · dO
                K.bmm(a, do, db, True, False, ctx.in_grad_accumulate[1])
            return
        if da is not None:
            store(da, torch.matmul(do.float(), b.float().transpose(-1, -2)), ctx.in_grad_accumulate[0])
        if db is not None:
            store(db, torch.matmul(a.float().transpose(-1, -2), do.float()), ctx.in_grad_accumulate[1])

    def flops(self, i, o):
        a = i[0]
        n = 1
        for d in a[:-1]:
            n *= d
        return 2.0 * n * a[-1] * i[1][-1]


class DotInteraction(Op):
    """DLRM feature interaction ``dot`` (absent in the reference, caveat C3).

    Inputs: the bottom-MLP output ``x[B,d]`` and F-1 embedding outputs ``e_i[B,d]``.
    Output ``[B, d + F(F-1)/2 (+pad)]`` = concat(x, strictly-lower-triangle of Z·Zᵀ) with
    ``Z[b] = [x; e_1; ...]``, the layout of facebookresearch/dlrm ``interact_features``.
    On MI355X one wave computes a 32x32 Gram tile per sample with
    ``v_mfma_f32_32x32x16_bf16`` (F ≤ 32), K = d.
    """
    op_type = OperatorType.OP_DOT_INTERACTION
    name_prefix = "DotInteraction"

    def __init__(self, model, bottom, embs, pad_to=16, self_interaction=False, name=None):
        super().__init__(model, [bottom] + list(embs), name)
        d = bottom.dims[-1]
        for e in embs:
            assert e.dims == bottom.dims, (e.dims, bottom.dims)
        self.d = d
        self.F = 1 + len(embs)
        self.self_interaction = self_interaction
        npairs = self.F * (self.F + 1) // 2 if self_interaction else self.F * (self.F - 1) // 2
        width = d + npairs
        self.out_width = ((width + pad_to - 1) // pad_to) * pad_to
        self.npairs = npairs
        if self.name is None:
            self.name = self.auto_name(str(self.F))
        self._finish([(bottom.dims[0], self.out_width)])

    def splittable_dims(self):
        return {0}

    def input_layouts(self, pc):
        lo = Layout.from_pc(self.outputs[0].dims, pc)
        return [Layout(t.dims, lo.degrees, lo.holders) for t in self.inputs]

    def pair_index(self):
        li, lj = [], []
        off = 0 if self.self_interaction else -1
        for i in range(self.F):
            for j in range(i + 1 + off):
                li.append(i)
                lj.append(j)
        return li, lj

    def forward(self, ctx: OpCtx):
        y = ctx.outputs[0]
        if ctx.hip:
            K.dot_interaction_forward(list(ctx.inputs), y, self.self_interaction)
            return
        Z = torch.stack([t.float() for t in ctx.inputs], dim=1)  # [B,F,d]
        G = torch.bmm(Z, Z.transpose(1, 2))
        li, lj = self.pair_index()
        flat = G[:, li, lj]
        y.zero_()
        y[:, : self.d] = ctx.inputs[0]
        y[:, self.d: self.d + self.npairs] = flat

    def backward(self, ctx: OpCtx):
        dy = ctx.out_grads[0]
        if ctx.hip:
            K.dot_interaction_backward(list(ctx.inputs), dy, list(ctx.in_grads),
                                       list(ctx.in_grad_accumulate), self.self_interaction,
                                       ctx.saved.get("act0", 10))
            return
        Z = torch.stack([t.float() for t in ctx.inputs], dim=1)
        B = Z.shape[0]
        dG = torch.zeros(B, self.F, self.F)
        li, lj = self.pair_index()
        dG[:, li, lj] = dy[:, self.d: self.d + self.npairs].float()
        dZ = torch.bmm(dG + dG.transpose(1, 2), Z)
        dZ[:, 0] += dy[:, : self.d].float()
        for i, g in enumerate(ctx.in_grads):
            if g is not None:
                store(g, dZ[:, i], ctx.in_grad_accumulate[i])

    def flops(self, i, o):
        return 2.0 * i[0][0] * self.F * self.F * self.d
