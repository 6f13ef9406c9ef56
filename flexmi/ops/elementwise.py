"""Element-wise unary / binary ops.

Reference: ``src/ops/element_unary.cu`` (cuDNN activations + custom ``exp`` kernel, ``:283-302``,
``:384-404``) and ``src/ops/element_binary.cu`` (cuDNN OpTensor ADD/MUL, SUB via α=-1, DIV
asserts -- caveat C9).  MI355X: vectorised HIP kernels ``csrc/kernels/elementwise.hip`` for all
of relu/sigmoid/tanh/elu/exp and add/sub/mul/div (DIV works).  Any dim may be split.
"""
from __future__ import annotations

import torch

from flexmi.core.types import OperatorType
from flexmi.parallel.layout import Layout

from .base import Op, OpCtx, store
from . import _kernels as K

UNARY_CODES = {OperatorType.OP_RELU: 0, OperatorType.OP_SIGMOID: 1, OperatorType.OP_TANH: 2,
               OperatorType.OP_ELU: 3, OperatorType.OP_EXP: 4}
BINARY_CODES = {OperatorType.OP_EW_ADD: 0, OperatorType.OP_EW_SUB: 1, OperatorType.OP_EW_MUL: 2,
                OperatorType.OP_EW_DIV: 3}
_UNARY_NAMES = {OperatorType.OP_RELU: "Relu", OperatorType.OP_SIGMOID: "Sigmoid",
                OperatorType.OP_TANH: "Tanh", OperatorType.OP_ELU: "Elu", OperatorType.OP_EXP: "Exp"}
_BINARY_NAMES = {OperatorType.OP_EW_ADD: "Add", OperatorType.OP_EW_SUB: "Sub",
                 OperatorType.OP_EW_MUL: "Mul", OperatorType.OP_EW_DIV: "Div"}


def unary_fwd_torch(code, x):
    if code == 0:
        return torch.relu(x)
    if code == 1:
        return torch.sigmoid(x)
    if code == 2:
        return torch.tanh(x)
    if code == 3:
        return torch.nn.functional.elu(x)
    return torch.exp(x)


def unary_bwd_torch(code, x, y, dy):
    if code == 0:
        return dy * (x > 0).to(dy.dtype)
    if code == 1:
        return dy * y * (1 - y)
    if code == 2:
        return dy * (1 - y * y)
    if code == 3:
        return dy * torch.where(x > 0, torch.ones_like(x), y + 1)
    return dy * y


class ElementUnary(Op):
    def __init__(self, model, op_type, input, name=None):
        super().__init__(model, [input], name)
        self.op_type = OperatorType(op_type)
        self.code = UNARY_CODES[self.op_type]
        self.name_prefix = _UNARY_NAMES[self.op_type]
        if self.name is None:
            self.name = self.auto_name("")
        self._finish([input.dims])

    def splittable_dims(self):
        return set(range(self.out_ndims))

    def forward(self, ctx: OpCtx):
        if ctx.saved.get("fused_into_binary"):   # the producing ElementBinary wrote relu(a op b) here
            return
        x, y = ctx.inputs[0], ctx.outputs[0]
        if ctx.hip:
            K.unary_forward(self.code, x, y)
        else:
            y.copy_(unary_fwd_torch(self.code, x.float()))

    def backward(self, ctx: OpCtx):
        if not ctx.in_grads or ctx.in_grads[0] is None or ctx.saved.get("fused_into_binary"):
            return
        x, y, dy, dx = ctx.inputs[0], ctx.outputs[0], ctx.out_grads[0], ctx.in_grads[0]
        if getattr(self, "skip_act_grad", False):   # fused sigmoid + BCE (loss emitted dL/dz)
            if ctx.hip:
                K.copy_or_add(dy, dx, ctx.in_grad_accumulate[0])
            else:
                store(dx, dy, ctx.in_grad_accumulate[0])
            return
        if ctx.hip:
            K.unary_backward(self.code, x, y, dy, dx, ctx.in_grad_accumulate[0])
        else:
            store(dx, unary_bwd_torch(self.code, x.float(), y.float(), dy.float()), ctx.in_grad_accumulate[0])


class ElementBinary(Op):
    def __init__(self, model, op_type, x, y, name=None):
        super().__init__(model, [x, y], name)
        self.op_type = OperatorType(op_type)
        self.code = BINARY_CODES[self.op_type]
        self.name_prefix = _BINARY_NAMES[self.op_type]
        assert tuple(x.dims) == tuple(y.dims), "ElementBinary requires same-shape inputs (reference semantics)"
        if self.name is None:
            self.name = self.auto_name("")
        self._finish([x.dims])

    def splittable_dims(self):
        return set(range(self.out_ndims))

    def forward(self, ctx: OpCtx):
        a, b, y = ctx.inputs[0], ctx.inputs[1], ctx.outputs[0]
        fused = ctx.saved.get("fused_relu")      # (relu output, its gradient): executor fusion
        if ctx.hip and fused is not None:
            K.binary_forward(self.code, a, b, fused[0], relu=True)
            return
        if ctx.hip:
            K.binary_forward(self.code, a, b, y)
        else:
            a, b = a.float(), b.float()
            y.copy_([a + b, a - b, a * b, a / b][self.code])

    def backward(self, ctx: OpCtx):
        a, b, dy = ctx.inputs[0], ctx.inputs[1], ctx.out_grads[0]
        da = ctx.in_grads[0] if len(ctx.in_grads) > 0 else None
        db = ctx.in_grads[1] if len(ctx.in_grads) > 1 else None
        if ctx.hip:
            fused = ctx.saved.get("fused_relu")
            if fused is not None:
                K.binary_backward(self.code, a, b, fused[1], da, db, ctx.in_grad_accumulate[0], ctx.in_grad_accumulate[1],
                                  ymask=fused[0])
                return
            K.binary_backward(self.code, a, b, dy, da, db,
                              ctx.in_grad_accumulate[0], ctx.in_grad_accumulate[1])
            return
        a, b, g = a.float(), b.float(), dy.float()
        if self.code == 0:
            ga, gb = g, g
        elif self.code == 1:
            ga, gb = g, -g
        elif self.code == 2:
            ga, gb = g * b, g * a
        else:
            ga, gb = g / b, -g * a / (b * b)
        if da is not None:
            store(da, ga, ctx.in_grad_accumulate[0])
        if db is not None:
            store(db, gb, ctx.in_grad_accumulate[1])
