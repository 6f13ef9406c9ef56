"""LSTM (``OP_LSTM``) for the NMT workload (``nmt/lstm.cu:1-574``: cuDNN LSTM over 10-step chunks).

One op runs a whole (chunk of a) sequence: input x [B, T, I], optional initial state h0, c0
[B, H]; outputs y [B, T, H], hT, cT [B, H] (so chunks chain like the reference's per-chunk LSTM
nodes, ``nmt/rnn.cu:300-317``).  Gates i, f, g, o (PyTorch order); weights W_ih [4H, I],
W_hh [4H, H], bias [4H].  Sample (batch) parallel; chunk placement along T gives the reference's
sequence/operator parallelism.

MI355X (``csrc/kernels/lstm.hip``): the input projection of all T steps is ONE MFMA GEMM into
fp32 gates; each step adds h_{t-1}.W_hh^T with a beta=1 GEMM and runs a fused pointwise cell
kernel; the backward runs the pointwise backward + one recurrent GEMM per step and then the
three weight/input-gradient GEMMs over all B*T rows at once (db from the dW_ih GEMM's row sums).
"""
from __future__ import annotations

import torch

from flexmi.core.initializers import UniformInitializer, ZeroInitializer
from flexmi.core.types import OperatorType
from flexmi.parallel.layout import Layout

from .base import Op, OpCtx, store
from . import _kernels as K


def _lstm_torch(x, w_ih, w_hh, b, h, c):
    """fp32 reference recurrence; x [B,T,I] -> y [B,T,H], hT, cT."""
    T = x.shape[1]
    H = w_hh.shape[1]
    gi = torch.matmul(x, w_ih.t()) + b
    ys = []
    for t in range(T):
        g = gi[:, t] + h @ w_hh.t()
        i, f, gg, o = torch.sigmoid(g[:, :H]), torch.sigmoid(g[:, H:2 * H]), torch.tanh(g[:, 2 * H:3 * H]), \
            torch.sigmoid(g[:, 3 * H:])
        c = f * c + i * gg
        h = o * torch.tanh(c)
        ys.append(h)
    return torch.stack(ys, 1), h, c


class LSTM(Op):
    op_type = OperatorType.OP_LSTM
    name_prefix = "LSTM"

    def __init__(self, model, x, hidden, h0=None, c0=None, name=None, seed=None):
        ins = [x] + ([h0, c0] if h0 is not None else [])
        super().__init__(model, ins, name)
        assert len(x.dims) == 3, "LSTM input is [batch, time, features]"
        assert (h0 is None) == (c0 is None), "give both h0 and c0 or neither"
        B, T, I = x.dims
        self.H, self.T, self.I = int(hidden), T, I
        self.has_state = h0 is not None
        if self.name is None:
            self.name = self.auto_name(str(hidden))
        r = 1.0 / (self.H ** 0.5)   # PyTorch's LSTM init range
        sd = model._next_seed() if seed is None else seed
        self._add_weight((4 * self.H, I), UniformInitializer(sd, -r, r), "w_ih")
        self._add_weight((4 * self.H, self.H), UniformInitializer(sd + 1, -r, r), "w_hh")
        self._add_weight((4 * self.H,), ZeroInitializer(), "bias")
        self._finish([(B, T, self.H), (B, self.H), (B, self.H)])

    def splittable_dims(self):
        return {0}

    def input_layouts(self, pc):
        return [Layout.from_pc(t.dims, pc) for t in self.inputs]

    # ------------------------------------------------------------------ compute
    def forward(self, ctx: OpCtx):
        x = ctx.inputs[0]
        y, hT, cT = ctx.outputs
        if ctx.hip:
            self._forward_hip(ctx)
            return
        B = x.shape[0]
        h0 = ctx.inputs[1].float() if self.has_state else torch.zeros(B, self.H)
        c0 = ctx.inputs[2].float() if self.has_state else torch.zeros(B, self.H)
        w_ih, w_hh, b = (w.float() for w in ctx.wcompute)
        yy, h, c = _lstm_torch(x.float(), w_ih, w_hh, b, h0, c0)
        y.copy_(yy)
        hT.copy_(h)
        cT.copy_(c)

    def backward(self, ctx: OpCtx):
        if ctx.hip:
            self._backward_hip(ctx)
            return
        x = ctx.inputs[0].float().detach().requires_grad_(True)
        B = x.shape[0]
        ins = [x]
        if self.has_state:
            h0 = ctx.inputs[1].float().detach().requires_grad_(True)
            c0 = ctx.inputs[2].float().detach().requires_grad_(True)
            ins += [h0, c0]
        else:
            h0 = torch.zeros(B, self.H)
            c0 = torch.zeros(B, self.H)
        ws = [w.float().detach().requires_grad_(True) for w in ctx.wcompute]
        with torch.enable_grad():
            y, h, c = _lstm_torch(x, ws[0], ws[1], ws[2], h0, c0)
            outs, gouts = [], []
            for o, g in ((y, ctx.out_grads[0]), (h, ctx.out_grads[1]), (c, ctx.out_grads[2])):
                if g is not None:
                    outs.append(o)
                    gouts.append(g.float())
            grads = torch.autograd.grad(outs, ws + ins, gouts, allow_unused=True)
        for dw, g in zip(ctx.weight_grads, grads[:3]):
            dw.add_(g)
        for i, g in enumerate(grads[3:]):
            if ctx.in_grads[i] is not None and g is not None:
                store(ctx.in_grads[i], g, ctx.in_grad_accumulate[i])

    # ------------------------------------------------------------------ MI355X path
    def _bufs(self, ctx, B):
        s = ctx.saved
        if "G" not in s:
            dev = ctx.inputs[0].device
            T, H = self.T, self.H
            s["G"] = torch.empty(B * T * 4 * H, dtype=torch.float32, device=dev)
            s["C"] = torch.empty(B * T * H, dtype=torch.float32, device=dev)
            adt = ctx.inputs[0].dtype          # activation dtype (bf16, or fp32 in reference-precision mode)
            s["Hp"] = torch.empty(B * T * H, dtype=adt, device=dev)
            s["cinit"] = torch.empty(B * H, dtype=torch.float32, device=dev)
            s["dG"] = torch.empty(B * T * 4 * H, dtype=adt, device=dev)
            s["dh"] = torch.empty(B * H, dtype=torch.float32, device=dev)
            s["dc"] = torch.empty(B * H, dtype=torch.float32, device=dev)
        return s

    def _forward_hip(self, ctx):
        C = K.C()
        x = ctx.inputs[0]
        y, hT, cT = ctx.outputs
        B, T, I = x.shape
        H = self.H
        s = self._bufs(ctx, B)
        w_ih, w_hh, bias = ctx.wcompute[0], ctx.wcompute[1], ctx.weights[2]
        G, Cs, Hp = s["G"], s["C"], s["Hp"]
        K.gemm(x.reshape(B * T, I), I, True, w_ih, I, True, G, 4 * H, B * T, 4 * H, I, bias=bias)
        C.lstm_init(ctx.inputs[1] if self.has_state else None, ctx.inputs[2] if self.has_state else None,
                    Hp, T * H, s["cinit"], B, H)
        yf = y.view(-1)
        for t in range(T):
            K.gemm(Hp[t * H:], T * H, True, w_hh, H, True, G[t * 4 * H:], T * 4 * H, B, 4 * H, H, beta=True)
            last = t == T - 1
            cprev, cp_off, ldcp = (s["cinit"], 0, H) if t == 0 else (Cs, (t - 1) * H, T * H)
            C.lstm_cell_fwd(G, t * 4 * H, T * 4 * H, cprev, cp_off, ldcp, Cs, t * H, T * H, yf, t * H, T * H,
                            Hp, -1 if last else (t + 1) * H, T * H, hT if last else None, cT if last else None, B, H)

    def _backward_hip(self, ctx):
        C = K.C()
        x = ctx.inputs[0]
        B, T, I = x.shape
        H = self.H
        s = self._bufs(ctx, B)
        G, Cs, Hp, dG, dh, dc = s["G"], s["C"], s["Hp"], s["dG"], s["dh"], s["dc"]
        w_ih, w_hh = ctx.wcompute[0], ctx.wcompute[1]
        dy = ctx.out_grads[0]
        dhT, dcT = ctx.out_grads[1], ctx.out_grads[2]
        if dhT is not None:
            dh.copy_(dhT.reshape(-1))
        else:
            dh.zero_()
        if dcT is not None:
            dc.copy_(dcT.reshape(-1))
        else:
            dc.zero_()
        dyf = dy.reshape(-1) if dy is not None else None
        for t in range(T - 1, -1, -1):
            cprev, cp_off, ldcp = (s["cinit"], 0, H) if t == 0 else (Cs, (t - 1) * H, T * H)
            C.lstm_cell_bwd(G, t * 4 * H, T * 4 * H, Cs, t * H, T * H, cprev, cp_off, ldcp, dyf, t * H, T * H, dh, dc,
                            dG, t * 4 * H, T * 4 * H, B, H)
            # dh_{t-1} = dG_t . W_hh   (W_hh stored [4H][H]: MN-contiguous B operand)
            K.gemm(dG[t * 4 * H:], T * 4 * H, True, w_hh, H, False, dh, H, B, H, 4 * H)
        dW_ih, dW_hh, db = ctx.weight_grads
        dG2 = dG.view(B * T, 4 * H)
        # dW_ih = dG^T X (+ db = column sums of dG), dW_hh = dG^T Hprev
        K.gemm(dG2, 4 * H, False, x.reshape(B * T, I), I, False, dW_ih, I, 4 * H, I, B * T, rowsum_a=db)
        K.gemm(dG2, 4 * H, False, Hp.view(B * T, H), H, False, dW_hh, H, 4 * H, H, B * T)
        if ctx.in_grads[0] is not None:
            dx = ctx.in_grads[0]
            K.gemm(dG2, 4 * H, True, w_ih, I, False, dx.view(B * T, I), I, B * T, I, 4 * H,
                   beta=bool(ctx.in_grad_accumulate[0]))
        if self.has_state:
            if ctx.in_grads[1] is not None:
                store(ctx.in_grads[1], dh.view(B, H), ctx.in_grad_accumulate[1])
            if ctx.in_grads[2] is not None:
                store(ctx.in_grads[2], dc.view(B, H), ctx.in_grad_accumulate[2])

    def flops(self, in_shapes, out_shapes):
        B, T, I = in_shapes[0]
        return 2.0 * B * T * 4 * self.H * (I + self.H)
