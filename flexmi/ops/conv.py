"""CNN ops: Conv2D, Pool2D, BatchNorm (NCHW, like the reference).

Reference: ``src/ops/conv_2d.cu`` (cuDNN conv fwd/bwd-filter/bwd-data, autotuned algos, relu
epilogue; spatial H/W splits use disjoint partitions WITHOUT halos so shard borders are
approximate -- caveat C10), ``pool_2d.cu`` (cuDNN max/avg-exclude-pad), ``batch_norm.cu``
(training-mode spatial BN, running stats zeroed every call, optional relu).

flexmi: attribute (spatial) parallelism is EXACT -- a consumer shard's input box includes the
halo rows/columns its kernel window needs, so the reshard moves the halos and each shard runs a
convolution with per-side padding.  MI355X kernels: implicit-GEMM conv on MFMA
(``csrc/kernels/conv.hip``), pool and BN kernels (``csrc/kernels/cnn.hip``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from flexmi.core.initializers import GlorotUniformInitializer, ZeroInitializer
from flexmi.core.types import ActiMode, OperatorType, PoolType
from flexmi.parallel.layout import Layout, split_extent

from .base import Op, OpCtx, store
from .linear import act_backward_torch, act_forward_torch
from . import _kernels as K


def _halo_box(out_box, in_dims, kh, kw, sh, sw, ph, pw):
    (n0, n1), (c0, c1), (h0, h1), (w0, w1) = out_box
    ih0 = max(0, h0 * sh - ph)
    ih1 = min(in_dims[2], (h1 - 1) * sh - ph + kh)
    iw0 = max(0, w0 * sw - pw)
    iw1 = min(in_dims[3], (w1 - 1) * sw - pw + kw)
    return ((n0, n1), (0, in_dims[1]), (ih0, ih1), (iw0, iw1))


def _local_pads(out_box, in_box, kh, kw, sh, sw, ph, pw):
    (h0, h1), (w0, w1) = out_box[2], out_box[3]
    (ih0, ih1), (iw0, iw1) = in_box[2], in_box[3]
    top = ih0 - (h0 * sh - ph)
    left = iw0 - (w0 * sw - pw)
    bottom = ((h1 - 1) * sh - ph + kh) - ih1
    right = ((w1 - 1) * sw - pw + kw) - iw1
    return top, bottom, left, right


class _SpatialOp(Op):
    """Shared halo logic for Conv2D / Pool2D."""
    # the kernels take only the top / left pads and the output extent, so a local input box
    # larger than the halo box works unchanged (the executor then skips the halo copy)
    superset_input_ok = True

    def splittable_dims(self):
        return {0, 2, 3}

    def input_layouts(self, pc):
        lo = Layout.from_pc(self.outputs[0].dims, pc)
        boxes = [_halo_box(lo.part_box(p), self.inputs[0].dims, self.kh, self.kw, self.sh, self.sw,
                           self.ph, self.pw) for p in range(lo.num_parts())]
        deg = (lo.degrees[0], 1, lo.degrees[2], lo.degrees[3])
        return [Layout(self.inputs[0].dims, deg, lo.holders, False, boxes)]

    def _pads(self, ctx):
        return _local_pads(ctx.out_boxes[0], ctx.in_boxes[0], self.kh, self.kw, self.sh, self.sw,
                           self.ph, self.pw)


class Conv2D(_SpatialOp):
    op_type = OperatorType.OP_CONV2D
    name_prefix = "Conv2D"

    def __init__(self, model, input, out_channels, kernel_h, kernel_w, stride_h, stride_w,
                 padding_h, padding_w, activation=ActiMode.AC_MODE_NONE, use_bias=True,
                 kernel_initializer=None, bias_initializer=None, name=None, groups=1):
        super().__init__(model, [input], name)
        assert len(input.dims) == 4, "Conv2D expects NCHW"
        n, c, h, w = input.dims
        self.in_channels, self.out_channels = c, int(out_channels)
        self.kh, self.kw, self.sh, self.sw, self.ph, self.pw = kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w
        self.activation = ActiMode(activation)
        self.use_bias = use_bias
        self.groups = groups
        oh = 1 + (h + 2 * padding_h - kernel_h) // stride_h
        ow = 1 + (w + 2 * padding_w - kernel_w) // stride_w
        if self.name is None:
            self.name = self.auto_name(f"{c}_{out_channels}_{kernel_h}x{kernel_w}")
        kinit = kernel_initializer or GlorotUniformInitializer(model._next_seed() if model else 0)
        self._add_weight((self.out_channels, c // groups, kernel_h, kernel_w), kinit, "weight")
        if use_bias:
            self._add_weight((self.out_channels,), bias_initializer or ZeroInitializer(), "bias")
        self._finish([(n, self.out_channels, oh, ow)])

    def forward(self, ctx: OpCtx):
        x, y = ctx.inputs[0], ctx.outputs[0]
        pads = self._pads(ctx)
        b = ctx.weights[1] if self.use_bias else None
        if ctx.hip:
            K.conv2d_forward(x, ctx.wcompute[0], b, y, (self.sh, self.sw), pads, int(self.activation), self.groups,
                             ctx.saved)
            return
        xp = F.pad(x.float(), (pads[2], pads[3], pads[0], pads[1]))
        out = F.conv2d(xp, ctx.wcompute[0].float(), None if b is None else b.float(), (self.sh, self.sw), 0, 1, self.groups)
        y.copy_(act_forward_torch(out, self.activation))

    def backward(self, ctx: OpCtx):
        x, y, dy = ctx.inputs[0], ctx.outputs[0], ctx.out_grads[0]
        dx = ctx.in_grads[0] if ctx.in_grads else None
        pads = self._pads(ctx)
        dw = ctx.weight_grads[0]
        db = ctx.weight_grads[1] if self.use_bias else None
        if ctx.hip:
            K.conv2d_backward(x, ctx.wcompute[0], y, dy, dx, dw, db, (self.sh, self.sw), pads,
                              int(self.activation), self.groups,
                              bool(ctx.in_grad_accumulate[0]) if dx is not None else False, ctx.saved)
            return
        g = act_backward_torch(dy.float(), y.float(), self.activation)
        xl = x.float().detach().requires_grad_(dx is not None)
        w = ctx.wcompute[0].float().detach().requires_grad_(True)
        with torch.enable_grad():
            # pads may be negative (a local box bigger than the halo box): F.pad crops those sides
            xp = F.pad(xl, (pads[2], pads[3], pads[0], pads[1]))
            out = F.conv2d(xp, w, None, (self.sh, self.sw), 0, 1, self.groups)
            grads = torch.autograd.grad(out, [w] + ([xl] if dx is not None else []), g)
        dw.add_(grads[0])          # accumulate: the executor zeroes gradients once per step
        if db is not None:
            db.add_(g.sum((0, 2, 3)))
        if dx is not None:
            store(dx, grads[1], ctx.in_grad_accumulate[0])

    def flops(self, i, o):
        n, c, oh, ow = o[0]
        return 2.0 * n * c * oh * ow * (self.in_channels // self.groups) * self.kh * self.kw


class Pool2D(_SpatialOp):
    op_type = OperatorType.OP_POOL2D
    name_prefix = "Pool2D"

    def __init__(self, model, input, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
                 pool_type=PoolType.POOL_MAX, activation=ActiMode.AC_MODE_NONE, name=None):
        super().__init__(model, [input], name)
        n, c, h, w = input.dims
        self.kh, self.kw, self.sh, self.sw, self.ph, self.pw = kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w
        self.pool_type = PoolType(pool_type)
        self.activation = ActiMode(activation)
        oh = 1 + (h + 2 * padding_h - kernel_h) // stride_h
        ow = 1 + (w + 2 * padding_w - kernel_w) // stride_w
        if self.name is None:
            self.name = self.auto_name(f"{kernel_h}x{kernel_w}")
        self._finish([(n, c, oh, ow)])

    def splittable_dims(self):
        return {0, 1, 2, 3}

    def input_layouts(self, pc):
        lo = Layout.from_pc(self.outputs[0].dims, pc)
        boxes = []
        for p in range(lo.num_parts()):
            ob = lo.part_box(p)
            hb = _halo_box(ob, self.inputs[0].dims, self.kh, self.kw, self.sh, self.sw, self.ph, self.pw)
            boxes.append((hb[0], ob[1], hb[2], hb[3]))
        return [Layout(self.inputs[0].dims, lo.degrees, lo.holders, False, boxes)]

    def _torch_fwd(self, x, pads):
        if self.pool_type == PoolType.POOL_MAX:
            xp = F.pad(x, (pads[2], pads[3], pads[0], pads[1]), value=float("-inf"))
            return F.max_pool2d(xp, (self.kh, self.kw), (self.sh, self.sw))
        # average excluding padding (cuDNN AVERAGE_COUNT_EXCLUDE_PADDING)
        xp = F.pad(x, (pads[2], pads[3], pads[0], pads[1]))
        ones = F.pad(torch.ones_like(x[:1, :1]), (pads[2], pads[3], pads[0], pads[1]))
        s = F.avg_pool2d(xp, (self.kh, self.kw), (self.sh, self.sw), divisor_override=1)
        cnt = F.avg_pool2d(ones, (self.kh, self.kw), (self.sh, self.sw), divisor_override=1)
        return s / cnt

    def forward(self, ctx: OpCtx):
        x, y = ctx.inputs[0], ctx.outputs[0]
        pads = self._pads(ctx)
        if ctx.hip:
            K.pool2d_forward(x, y, (self.kh, self.kw), (self.sh, self.sw), pads,
                             int(self.pool_type), int(self.activation), ctx.saved)
            return
        y.copy_(act_forward_torch(self._torch_fwd(x.float(), pads), self.activation))

    def backward(self, ctx: OpCtx):
        if not ctx.in_grads or ctx.in_grads[0] is None:
            return
        x, y, dy, dx = ctx.inputs[0], ctx.outputs[0], ctx.out_grads[0], ctx.in_grads[0]
        pads = self._pads(ctx)
        if ctx.hip:
            K.pool2d_backward(x, y, dy, dx, (self.kh, self.kw), (self.sh, self.sw), pads,
                              int(self.pool_type), int(self.activation), ctx.in_grad_accumulate[0], ctx.saved)
            return
        g = act_backward_torch(dy.float(), y.float(), self.activation)
        xx = x.float().detach().requires_grad_(True)
        with torch.enable_grad():
            out = self._torch_fwd(xx, pads)
            gx, = torch.autograd.grad(out, [xx], g)
        store(dx, gx, ctx.in_grad_accumulate[0])


class BatchNorm(Op):
    """Training-mode spatial batch norm (``src/ops/batch_norm.cu:348-503``); statistics over
    the local shard (DP only, like the reference)."""
    op_type = OperatorType.OP_BATCHNORM
    name_prefix = "BatchNorm"
    eps = 1e-5

    def __init__(self, model, input, relu=True, name=None):
        super().__init__(model, [input], name)
        assert len(input.dims) == 4
        self.relu = relu
        c = input.dims[1]
        if self.name is None:
            self.name = self.auto_name("")
        from flexmi.core.initializers import ConstantInitializer
        self._add_weight((c,), ConstantInitializer(1.0), "scale")
        self._add_weight((c,), ZeroInitializer(), "bias")
        self._finish([input.dims])

    def splittable_dims(self):
        return {0}

    def forward(self, ctx: OpCtx):
        x, y = ctx.inputs[0], ctx.outputs[0]
        if ctx.hip:
            K.batchnorm_forward(x, ctx.weights[0], ctx.weights[1], y, self.relu, self.eps, ctx.saved)
            return
        xf = x.float()
        mean = xf.mean((0, 2, 3))
        var = xf.var((0, 2, 3), unbiased=False)
        inv = torch.rsqrt(var + self.eps)
        xhat = (xf - mean[None, :, None, None]) * inv[None, :, None, None]
        out = xhat * ctx.weights[0][None, :, None, None] + ctx.weights[1][None, :, None, None]
        ctx.saved["inv"] = inv
        ctx.saved["xhat"] = xhat
        y.copy_(torch.relu(out) if self.relu else out)

    def backward(self, ctx: OpCtx):
        x, y, dy = ctx.inputs[0], ctx.outputs[0], ctx.out_grads[0]
        dx = ctx.in_grads[0] if ctx.in_grads else None
        if ctx.hip:
            K.batchnorm_backward(x, ctx.weights[0], y, dy, dx, ctx.weight_grads[0], ctx.weight_grads[1],
                                 self.relu, self.eps, ctx.saved,
                                 bool(ctx.in_grad_accumulate[0]) if dx is not None else False)
            return
        g = dy.float()
        if self.relu:
            g = g * (y.float() > 0)
        xhat, inv = ctx.saved["xhat"], ctx.saved["inv"]
        m = g.shape[0] * g.shape[2] * g.shape[3]
        dgamma = (g * xhat).sum((0, 2, 3))
        dbeta = g.sum((0, 2, 3))
        ctx.weight_grads[0].copy_(dgamma)
        ctx.weight_grads[1].copy_(dbeta)
        if dx is not None:
            gam = ctx.weights[0][None, :, None, None]
            gx = gam * inv[None, :, None, None] / m * (m * g - dbeta[None, :, None, None] - xhat * dgamma[None, :, None, None])
            store(dx, gx, ctx.in_grad_accumulate[0])
