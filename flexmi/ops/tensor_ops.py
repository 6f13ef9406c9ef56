"""Data-movement ops: Concat, Split, Flat, Reshape, Transpose, Reverse.

Reference: ``src/ops/concat.cu`` (strided copy fwd ``:159-235``, ``add_with_stride`` bwd
``:263-317``), ``split.cu``, ``flat.cu`` (memcpy), ``reshape.cu`` (memcpy), ``transpose.cu``
(one-thread-per-element permute ``:135-159``), ``reverse.cu``.  Axis arguments are in user
order (the reference converts with ``numDim-1-axis``).

MI355X: Flat/Reshape are zero-copy views of their input buffer (``is_view``); Concat/Split
move all pieces in ONE launch of ``fm_strided_copy`` (pointer table); Transpose uses an
LDS-tiled 64x64 kernel; Reverse a vectorised gather kernel.
"""
from __future__ import annotations

import torch

from flexmi.core.types import OperatorType
from flexmi.parallel.layout import Layout

from .base import Op, OpCtx, store
from . import _kernels as K


def _norm_axis(axis, nd):
    return axis + nd if axis < 0 else axis


class Concat(Op):
    op_type = OperatorType.OP_CONCAT
    name_prefix = "Concat"

    def __init__(self, model, tensors, axis, name=None):
        super().__init__(model, list(tensors), name)
        nd = len(tensors[0].dims)
        self.axis = _norm_axis(axis, nd)
        dims = list(tensors[0].dims)
        for t in tensors[1:]:
            assert len(t.dims) == nd
            for j in range(nd):
                if j != self.axis:
                    assert t.dims[j] == dims[j], (t.dims, dims)
            dims[self.axis] += t.dims[self.axis]
        if self.name is None:
            self.name = self.auto_name(str(self.axis))
        self._finish([tuple(dims)])

    def splittable_dims(self):
        return set(range(self.out_ndims)) - {self.axis}

    def input_layouts(self, pc):
        lo = Layout.from_pc(self.outputs[0].dims, pc)
        return [Layout(t.dims, lo.degrees, lo.holders) for t in self.inputs]

    def forward(self, ctx: OpCtx):
        y = ctx.outputs[0]
        if ctx.hip:
            K.concat_forward(list(ctx.inputs), y, self.axis)
        else:
            torch.cat([x.to(y.dtype) for x in ctx.inputs], dim=self.axis, out=y)

    def backward(self, ctx: OpCtx):
        dy = ctx.out_grads[0]
        if ctx.hip:
            K.concat_backward(dy, list(ctx.in_grads), list(ctx.in_grad_accumulate), self.axis,
                              [tuple(x.shape) for x in ctx.inputs])
            return
        off = 0
        for i, x in enumerate(ctx.inputs):
            n = x.shape[self.axis]
            if i < len(ctx.in_grads) and ctx.in_grads[i] is not None:
                store(ctx.in_grads[i], dy.narrow(self.axis, off, n), ctx.in_grad_accumulate[i])
            off += n

    def bytes_moved(self, in_shapes, out_shapes, elem=2):
        return 2.0 * super().bytes_moved([], out_shapes, elem)


class Split(Op):
    op_type = OperatorType.OP_SPLIT
    name_prefix = "Split"

    def __init__(self, model, input, sizes, axis, name=None):
        super().__init__(model, [input], name)
        nd = len(input.dims)
        self.axis = _norm_axis(axis, nd)
        if isinstance(sizes, int):
            n = sizes
            assert input.dims[self.axis] % n == 0
            sizes = [input.dims[self.axis] // n] * n
        self.sizes = list(sizes)
        assert sum(self.sizes) == input.dims[self.axis]
        if self.name is None:
            self.name = self.auto_name(str(self.axis))
        outs = []
        for s in self.sizes:
            d = list(input.dims)
            d[self.axis] = s
            outs.append(tuple(d))
        self._finish(outs)

    def splittable_dims(self):
        return set(range(self.out_ndims)) - {self.axis}

    def forward(self, ctx: OpCtx):
        x = ctx.inputs[0]
        if ctx.hip:
            K.split_forward(x, list(ctx.outputs), self.axis)
            return
        off = 0
        for y in ctx.outputs:
            n = y.shape[self.axis]
            y.copy_(x.narrow(self.axis, off, n))
            off += n

    def backward(self, ctx: OpCtx):
        if not ctx.in_grads or ctx.in_grads[0] is None:
            return
        dx = ctx.in_grads[0]
        ogs = list(ctx.out_grads)
        acc = ctx.in_grad_accumulate[0]
        if any(g is None for g in ogs):       # unused outputs contribute zero blocks
            if all(g is None for g in ogs):
                if not acc:
                    dx.zero_()
                return
            if not acc:
                dx.zero_()
                acc = True
        if ctx.hip:
            K.split_backward(ogs, dx, acc, self.axis, [tuple(y.shape) for y in ctx.outputs])
            return
        g = torch.cat([d.float() if d is not None else torch.zeros(y.shape) for d, y in zip(ogs, ctx.outputs)],
                      dim=self.axis)
        store(dx, g, acc)


class _ViewOp(Op):
    """Ops whose output is a zero-copy view of the input buffer."""
    is_view = True

    def splittable_dims(self):
        return {0}

    def input_layouts(self, pc):
        lo = Layout.from_pc(self.outputs[0].dims, pc)
        deg = [1] * len(self.inputs[0].dims)
        deg[0] = lo.degrees[0]
        return [Layout(self.inputs[0].dims, tuple(deg), lo.holders)]

    def valid_pc(self, pc):
        if not super().valid_pc(pc):
            return False
        d = Layout.from_pc(self.outputs[0].dims, pc).degrees[0]
        return self.inputs[0].dims[0] % d == 0 and self.outputs[0].dims[0] % d == 0

    def forward(self, ctx: OpCtx):
        y = ctx.outputs[0]
        x = ctx.inputs[0]
        if y.data_ptr() != x.data_ptr():
            y.copy_(x.reshape(y.shape))

    def backward(self, ctx: OpCtx):
        if not ctx.in_grads or ctx.in_grads[0] is None:
            return
        dx = ctx.in_grads[0]
        dy = ctx.out_grads[0]
        if dx.data_ptr() == dy.data_ptr():
            return
        if ctx.hip:
            K.copy_or_add(dy.reshape(dx.shape), dx, ctx.in_grad_accumulate[0])
        else:
            store(dx, dy.reshape(dx.shape), ctx.in_grad_accumulate[0])


class Flat(_ViewOp):
    op_type = OperatorType.OP_FLAT
    name_prefix = "Flat"

    def __init__(self, model, input, name=None):
        super().__init__(model, [input], name)
        v = 1
        for d in input.dims[1:]:
            v *= d
        if self.name is None:
            self.name = self.auto_name("")
        self._finish([(input.dims[0], v)])

    def flops(self, i, o):
        return 0.0


class Reshape(_ViewOp):
    op_type = OperatorType.OP_RESHAPE
    name_prefix = "Reshape"

    def __init__(self, model, input, shape, name=None):
        super().__init__(model, [input], name)
        shape = list(shape)
        v = input.volume()
        if -1 in shape:
            k = shape.index(-1)
            rest = 1
            for j, s in enumerate(shape):
                if j != k:
                    rest *= s
            shape[k] = v // rest
        p = 1
        for s in shape:
            p *= s
        assert p == v, (shape, input.dims)
        if self.name is None:
            self.name = self.auto_name("")
        self._finish([tuple(shape)])


class Transpose(Op):
    op_type = OperatorType.OP_TRANSPOSE
    name_prefix = "Transpose"

    def __init__(self, model, input, perm, name=None):
        super().__init__(model, [input], name)
        assert sorted(perm) == list(range(len(input.dims)))
        self.perm = list(perm)
        if self.name is None:
            self.name = self.auto_name("")
        self._finish([tuple(input.dims[p] for p in self.perm)])

    def splittable_dims(self):
        return {i for i, p in enumerate(self.perm) if p == i}

    def forward(self, ctx: OpCtx):
        x, y = ctx.inputs[0], ctx.outputs[0]
        if ctx.hip:
            K.permute(x, y, self.perm, False)
        else:
            y.copy_(x.permute(*self.perm))

    def backward(self, ctx: OpCtx):
        if not ctx.in_grads or ctx.in_grads[0] is None:
            return
        inv = [0] * len(self.perm)
        for i, p in enumerate(self.perm):
            inv[p] = i
        dy, dx = ctx.out_grads[0], ctx.in_grads[0]
        if ctx.hip:
            K.permute(dy, dx, inv, ctx.in_grad_accumulate[0])
        else:
            store(dx, dy.permute(*inv), ctx.in_grad_accumulate[0])


class Reverse(Op):
    op_type = OperatorType.OP_REVERSE
    name_prefix = "Reverse"

    def __init__(self, model, input, axis, name=None):
        super().__init__(model, [input], name)
        self.axis = _norm_axis(axis, len(input.dims))
        if self.name is None:
            self.name = self.auto_name(str(self.axis))
        self._finish([input.dims])

    def splittable_dims(self):
        return set(range(self.out_ndims)) - {self.axis}

    def forward(self, ctx: OpCtx):
        x, y = ctx.inputs[0], ctx.outputs[0]
        if ctx.hip:
            K.reverse(x, y, self.axis, False)
        else:
            y.copy_(torch.flip(x, [self.axis]))

    def backward(self, ctx: OpCtx):
        if not ctx.in_grads or ctx.in_grads[0] is None:
            return
        dy, dx = ctx.out_grads[0], ctx.in_grads[0]
        if ctx.hip:
            K.reverse(dy, dx, self.axis, ctx.in_grad_accumulate[0])
        else:
            store(dx, torch.flip(dy, [self.axis]), ctx.in_grad_accumulate[0])
