"""Linear / Dense (``OP_LINEAR``).

Reference: ``src/ops/linear.cu`` -- builder ``:19-57``, forward = cuBLAS Sgemm + bias rank-1
Sgemm + cuDNN activation (``:424-447``), backward = relu/sigmoid-bwd kernel, Sgemm dW, Sgemv db,
Sgemm dX (``:592-635``), channel-parallel input-grad replicas summed by ``backward2``
(``:766-794``).

MI355X: one MFMA GEMM kernel (``csrc/kernels/gemm.hip``) with the bias + activation fused in
its epilogue; backward = one fused act-backward + bias-grad pass, then dX and dW MFMA GEMMs
whose transposed operands are read with ``ds_read_b64_tr_b16`` (no transposed copies).
SOAP: sample (n) and out-channel (c) splits; c>1 replicates the input over the channel group
and its gradient becomes a partial-sum layout that the executor reduces (the ``replica``
tensor of the reference, done as an RCCL reduce inside the reshard).
"""
from __future__ import annotations

import torch

from flexmi.core.initializers import GlorotUniformInitializer, ZeroInitializer
from flexmi.core.types import ActiMode, OperatorType
from flexmi.parallel.layout import Layout

from .base import Op, OpCtx, store
from . import _kernels as K


def act_forward_torch(y, act):
    if act == ActiMode.AC_MODE_RELU:
        return torch.relu(y)
    if act == ActiMode.AC_MODE_SIGMOID:
        return torch.sigmoid(y)
    if act == ActiMode.AC_MODE_TANH:
        return torch.tanh(y)
    return y


def act_backward_torch(dy, y, act):
    """Activation gradient from the activation *output* (as the reference's kernels do)."""
    if act == ActiMode.AC_MODE_RELU:
        return dy * (y > 0).to(dy.dtype)
    if act == ActiMode.AC_MODE_SIGMOID:
        return dy * y * (1 - y)
    if act == ActiMode.AC_MODE_TANH:
        return dy * (1 - y * y)
    return dy


def _armed_sgd(ctx):
    """The FusedSGD of this op's weight while the executor runs its fused training step
    (Executor._plan_fused_sgd), else None."""
    upd = getattr(ctx, "fused_sgd", None)
    return upd if upd is not None and ctx.fused_sgd_state["on"] else None


class Linear(Op):
    op_type = OperatorType.OP_LINEAR
    name_prefix = "Dense"

    def __init__(self, model, input, out_dim, activation=ActiMode.AC_MODE_NONE, use_bias=True,
                 kernel_initializer=None, bias_initializer=None, name=None):
        super().__init__(model, [input], name)
        self.in_dim = input.dims[-1]
        self.out_dim = int(out_dim)
        self.activation = ActiMode(activation)
        self.use_bias = use_bias
        if self.name is None:
            self.name = self.auto_name(str(out_dim))
        kinit = kernel_initializer or GlorotUniformInitializer(model._next_seed() if model else 0)
        self._add_weight((self.out_dim, self.in_dim), kinit, "weight")
        if use_bias:
            self._add_weight((self.out_dim,), bias_initializer or ZeroInitializer(), "bias")
        self._finish([tuple(input.dims[:-1]) + (self.out_dim,)])

    # ---------------------------------------------------------- parallel
    def splittable_dims(self):
        return {0, self.out_ndims - 1}

    def _degrees(self, pc):
        return Layout.from_pc(self.outputs[0].dims, pc).degrees

    def input_layouts(self, pc):
        out = Layout.from_pc(self.outputs[0].dims, pc)
        deg = list(out.degrees)
        c = deg[-1]
        deg[-1] = 1
        holders = []
        for p in range(out.num_parts() // c):
            holders.append(tuple(out.holders[p * c + j][0] for j in range(c)))
        return [Layout(self.inputs[0].dims, tuple(deg), holders)]

    def weight_layouts(self, pc):
        out = Layout.from_pc(self.outputs[0].dims, pc)
        c = out.degrees[-1]
        n = out.num_parts() // c
        holders = [tuple(out.holders[i * c + j][0] for i in range(n)) for j in range(c)]
        lays = [Layout(self.weights[0].dims, (c, 1), holders)]
        if self.use_bias:
            lays.append(Layout(self.weights[1].dims, (c,), holders))
        return lays

    # ---------------------------------------------------------- compute
    def forward(self, ctx: OpCtx):
        x = ctx.inputs[0]
        y = ctx.outputs[0]
        x2 = x.reshape(-1, x.shape[-1])
        y2 = y.view(-1, y.shape[-1])
        b = ctx.weights[1] if self.use_bias else None
        if ctx.hip:
            K.linear_forward(x2, ctx.wcompute[0], b, int(self.activation), y2)
        else:
            out = torch.nn.functional.linear(x2.float(), ctx.wcompute[0].float(), None if b is None else b.float())
            y2.copy_(act_forward_torch(out, self.activation))

    def backward(self, ctx: OpCtx, phase="all"):
        """phase "dx": input gradient (and the shared act-bwd); "dw": weight / bias gradients --
        the executor runs dW later to overlap a pending gradient exchange; "all": both."""
        x = ctx.inputs[0]
        x2 = x.reshape(-1, x.shape[-1])
        y2 = ctx.outputs[0].view(-1, ctx.outputs[0].shape[-1])
        dy2 = ctx.out_grads[0].view(y2.shape)
        dx = ctx.in_grads[0] if ctx.in_grads else None
        dx2 = None if dx is None else dx.view(-1, dx.shape[-1])
        dw = ctx.weight_grads[0]
        db = ctx.weight_grads[1] if self.use_bias else None
        act = ActiMode.AC_MODE_NONE if getattr(self, "skip_act_grad", False) else self.activation
        if ctx.hip:
            K.linear_backward(x2, ctx.wcompute[0], y2, dy2, int(act), dx2,
                              bool(ctx.in_grad_accumulate[0]) if dx2 is not None else False, dw, db,
                              ctx.workspace, ctx.saved.get("grad_is_dpre", False), ctx.saved.get("fuse_below"), phase,
                              upd=_armed_sgd(ctx))
        else:
            dpre = act_backward_torch(dy2.float(), y2.float(), act)
            if phase != "dx":
                dw.add_(dpre.t() @ x2.float())
                if db is not None:
                    db.add_(dpre.sum(0))
            if dx2 is not None and phase != "dw":
                store(dx2, dpre @ ctx.wcompute[0].float(), ctx.in_grad_accumulate[0])

    def flops(self, in_shapes, out_shapes):
        b = 1
        for d in out_shapes[0][:-1]:
            b *= d
        return 2.0 * b * in_shapes[0][-1] * out_shapes[0][-1]
