"""Python entry points of the HIP kernels (``flexmi._C``, built from ``csrc/kernels/*.hip``).

On a GPU run the extension MUST be present: every call goes through :func:`C` which raises if
``flexmi._C`` cannot be imported -- there is no silent eager fallback for the hot ops (GEMM,
embedding, interaction, optimizer, loss, element-wise, data movement, and the CNN ops: GEMM
convolution = implicit-GEMM MFMA kernels on NCHW, HIP pooling and batch norm).
:data:`LIBRARY_FALLBACK` lists ops routed to vendor libraries instead: none by default (the big fp32
dW GEMMs went to hipBLASLt until the split-bf16 kernel beat it; ``FM_DW_LIB=1`` restores that).
"""
from __future__ import annotations

import os
import threading

import torch

_C = None
_lock = threading.Lock()
# ops routed to a vendor library instead of a flexmi kernel by default (none: opt-in FM_DW_LIB=1 only)
LIBRARY_FALLBACK = {}


def C():
    global _C
    if _C is None:
        with _lock:
            if _C is None:
                try:
                    from flexmi import _C as mod
                except ImportError as e:
                    raise RuntimeError(
                        "flexmi._C (HIP kernels for gfx950) is not built: run `python tools/build_ext.py` "
                        f"or `python -c 'import __graft_entry__ as g; g.build()'` ({e})") from e
                _C = mod
    return _C


def available():
    try:
        C()
        return True
    except RuntimeError:
        return False


# ------------------------------------------------------------------ workspace (split-K slabs)
_ws = {}


def workspace(device, nbytes):
    """Grow-only split-K slab workspace of ``device``.  The GEMMs of a step never run concurrently
    (the executor's second stream carries only the embedding-group kernels), so one workspace per
    device serves them all; keyed by device, not by stream handle -- a hipGraph capture creates
    fresh streams and must not leave a 64 MiB workspace behind per stream."""
    key = str(device)
    t = _ws.get(key)
    if t is None or t.numel() * 4 < nbytes:
        t = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=device)
        _ws[key] = t
    return t


GEMM_WS_BYTES = 64 << 20

from flexmi.ops import gemm_tune as _tune  # noqa: E402


def gemm(A, lda, a_kcontig, B, ldb, b_kcontig, Cout, ldc, M, N, K, bias=None, act=10, beta=False, alpha=1.0,
         batch=1, sA=0, sB=0, sC=0, ksplit=0, use_ws=True, act_y=None, bwd_act=10, colsum=None, rowsum_a=None):
    """C = epi(A·B).  Optional fused backward epilogue of the layer below (act_y/bwd_act/colsum):
    C = act'(act_y) * (A·B) and colsum += column sums of C (its bias gradient)."""
    ws = workspace(Cout.device, GEMM_WS_BYTES) if use_ws else None
    lday = act_y.stride(0) if act_y is not None else 0
    if ksplit == 0 and use_ws:
        # a configuration measured for this GEMM (flexmi/ops/gemm_tune.py), else the heuristic
        dt = "fp32" if A.dtype == torch.float32 else "bf16"
        k = _tune.key(dt, M, N, K, a_kcontig, b_kcontig, batch, act_y is not None, colsum is not None,
                      rowsum_a is not None, False, Cout.dtype == torch.float32)
        ksplit = _tune.lookup(k)
        if _tune.RECORD is not None:
            _tune.RECORD.append(dict(key=k, dtype=dt, M=M, N=N, K=K, a_k=bool(a_kcontig), b_k=bool(b_kcontig), lda=lda,
                                     ldb=ldb, ldc=ldc, batch=batch, sA=sA, sB=sB, sC=sC, bias=bias is not None,
                                     act=act, beta=bool(beta), act_y=act_y is not None, bwd_act=bwd_act,
                                     colsum=colsum is not None, rowsum=rowsum_a is not None,
                                     c_fp32=Cout.dtype == torch.float32, sgd=None))
    return C().gemm(A, lda, sA, a_kcontig, B, ldb, sB, b_kcontig, Cout, ldc, sC, bias, M, N, K, batch, alpha, beta, act,
                    ws, ksplit, act_y, lday, bwd_act, colsum, rowsum_a)


# ------------------------------------------------------------------ init
def init_fill(out, dims, box, kind, seed, a, b):
    dims = tuple(dims)
    if len(dims) == 1:
        rows, cols, r0, c0, ldg = 1, box[0][1] - box[0][0], 0, box[0][0], dims[0]
    else:
        inner = 1
        for d in dims[2:]:
            inner *= d
        for (lo, hi), d in zip(box[2:], dims[2:]):
            assert lo == 0 and hi == d, "sharded init supports splits on the two outer dims only"
        rows = box[0][1] - box[0][0]
        cols = (box[1][1] - box[1][0]) * inner
        r0, c0 = box[0][0], box[1][0] * inner
        ldg = dims[1] * inner
    C().init_fill(out.view(-1) if out.is_contiguous() else out, rows, cols, r0, c0, ldg, kind, seed & 0xFFFFFFFF, a, b)


# ------------------------------------------------------------------ linear
def linear_forward(x2, w, b, act, y2):
    assert x2.stride(1) == 1 and y2.stride(1) == 1 and w.is_contiguous()
    M, K = x2.shape
    N = w.shape[0]
    if N == 1:
        C().skinny_fwd(x2, w, b, y2, act)
        return
    if _smallk(x2, K) and C().smallk_fwd(x2, w, b, y2, act):
        return
    gemm(x2, x2.stride(0), True, w, K, True, y2, y2.stride(0), M, N, K, bias=b, act=act)


# FM_DW_LIB=auto/1/0: the fp32 weight-gradient GEMM dW += dpre^T x of the big layers is a plain
# library GEMM (hipBLASLt, beta = 1 accumulate; bias gradient from the act-backward pass or one
# column-sum pass).  auto = the shapes where hipBLASLt measured faster than the flexmi kernel plus
# its split-K reduce (profiles/gemm_fp32_vs_hipblaslt.jsonl: 480->1024 66 vs 85 us, 1024->1024 125
# vs 150, 1024->512 68 vs 84; the 256/128/16-wide ones stay on flexmi, where it wins)
DW_LIB = os.environ.get("FM_DW_LIB", "auto")


def _dw_lib(M, N, K, dtype):
    if DW_LIB == "0" or dtype != torch.float32:
        return False
    if DW_LIB == "auto" and C().gemm_f32_get_split() in (2, 3, 4, 5):
        return False               # the split-bf16 kernel (gemm_x3.hip) takes the big fp32 dW GEMMs
    return DW_LIB == "1" or (N >= 512 and K >= 480 and M >= 4096)


# FM_SMALLK=1/0: thin-input Linear layers (fp32 or bf16; in_features <= 32, the 13->512 bottom layer of
# DLRM) on the VALU kernels of gemm_small.hip instead of a 1-2 step K loop of MFMA tiles (forward)
# and a split-K GEMM + reduce (dW)
SMALLK = os.environ.get("FM_SMALLK", "1") == "1"


def _smallk(x2, K):
    return SMALLK and K <= 32 and K % 4 == 0 and x2.stride(0) % 4 == 0


def _dw_smallk(dpre, x2, dw, db, upd):
    """dW (+ db) of a thin-input layer on gemm_small.hip; with upd the SGD step is applied to the
    weight in the same launch pair.  False when the kernel does not apply."""
    ws = workspace(dpre.device, GEMM_WS_BYTES)
    if upd is None:
        return C().smallk_dw(dpre, x2, dw, db, ws, None, None, None, 0.0, 0.0, False)
    return C().smallk_dw(dpre, x2, upd.w, db, ws, upd.v, upd.wc, upd.lr, upd.wd, upd.mom, upd.nesterov)


class FusedSGD:
    """The SGD update of one Linear weight, fused into its weight-gradient GEMM (``upd`` of
    linear_backward): fp32 master ``w``, bf16 mirror ``wc`` (or None), momentum ``v`` (or None),
    device-side ``lr`` and the optimizer's constants.  Only for weights whose gradient has no
    other consumer (not all-reduced, not tied, single dW GEMM) -- Executor._plan_fused_sgd."""
    __slots__ = ("w", "wc", "v", "lr", "wd", "mom", "nesterov")

    def __init__(self, w, wc, v, lr, wd, mom, nesterov):
        self.w, self.wc, self.v, self.lr = w, wc, v, lr
        self.wd, self.mom, self.nesterov = float(wd), float(mom), bool(nesterov)

    def apply(self, grad):
        """Unfused fallback: the optimizer kernel over this weight's consumed gradient."""
        sgd_update(self.w, grad, self.v, self.wc, self.lr, self.wd, self.mom, self.nesterov, zero_grad=True)


def _dw_fused_sgd(dpre, x2, dw, db, upd):
    """dW GEMM + SGD in one kernel (csrc/kernels/gemm.hip fm_gemm_dw_sgd, gemm_f32.hip
    fm_gemm_f32_dw_sgd); False when it does not apply (misaligned views, ldw % 4 != 0) and the
    caller must compute dW itself."""
    dt = "fp32" if dpre.dtype == torch.float32 else "bf16"
    B, Nout = dpre.shape
    Kin = x2.shape[1]
    k = _tune.key(dt, Nout, Kin, B, False, False, 1, False, False, db is not None, True, True)
    if _tune.RECORD is not None:
        _tune.RECORD.append(dict(key=k, dtype=dt, M=Nout, N=Kin, K=B, ldd=dpre.stride(0), ldx=x2.stride(0),
                                 rowsum=db is not None, sgd=dict(mom=upd.mom, nesterov=upd.nesterov, wd=upd.wd,
                                                                 mirror=upd.wc is not None)))
    ks = C().gemm_dw_sgd(dpre, x2, upd.w, upd.wc, upd.v, upd.lr, upd.wd, upd.mom, upd.nesterov, db,
                         workspace(dpre.device, GEMM_WS_BYTES), _tune.lookup(k))
    return ks >= 0


def linear_backward(x2, w, y2, dy2, act, dx2, dx_acc, dw, db, ws, grad_is_dpre=False, fuse_below=None, phase="all",
                    upd=None):
    """Weight/bias grads ACCUMULATE into dw/db (the executor zeroes the flat gradient buffer once
    per step).  grad_is_dpre: dy2 already holds act'(y)*dy (written by the consumer's fused dX
    epilogue).  fuse_below = (y_below, act_below): apply the activation backward of the layer
    below in this layer's dX GEMM epilogue.
    upd (FusedSGD): the weight is updated in place by this call (after its dX GEMM, which reads
    it) and dw stays zero; the bias gradient is still accumulated into db."""
    M, K = x2.shape
    N = w.shape[0]
    vec = 4 if x2.dtype == torch.float32 else 8
    if N == 1 and K % vec == 0 and x2.stride(0) % vec == 0 and (dx2 is None or dx2.stride(0) % vec == 0):
        if phase != "dw":          # the skinny kernel does dX, dW and db together in the "dx" phase
            # fuse_below: the layer below's activation backward applied to dX in the same pass
            bact = int(fuse_below[1]) if (dx2 is not None and fuse_below is not None) else 10
            assert bact == 10 or not dx_acc
            C().skinny_bwd(x2, w, y2, dy2, dx2, bool(dx_acc), dw, None if grad_is_dpre else db,
                           10 if grad_is_dpre else act, bact)
        if upd is not None and phase != "dx":
            upd.apply(dw)
        return
    lib = _dw_lib(M, N, K, x2.dtype)
    fold_db = lib and not (grad_is_dpre or act == 10)    # db from the act-backward pass below
    if grad_is_dpre or act == 10:
        dpre = dy2
    elif phase == "dw":            # computed by this op's "dx" phase (per-op workspace)
        dpre = ws["dpre"]
    else:
        dpre = ws.get("dpre")
        if dpre is None or dpre.shape != (M, N) or dpre.dtype != dy2.dtype:
            dpre = torch.empty((M, N), dtype=dy2.dtype, device=x2.device)
            ws["dpre"] = dpre
        C().act_bwd_bias(y2, dy2, dpre, db if fold_db else None, M, N, act)
    if upd is not None:
        # dX first (it reads W), then dW with the update fused in (or dW + the optimizer kernel)
        if phase != "dw" and dx2 is not None:
            _linear_dx(dpre, w, dx2, dx_acc, fuse_below, M, N, K)
        if phase == "dx":
            return
        if _smallk(x2, K) and _dw_smallk(dpre, x2, dw, db, upd):
            return
        if not lib and M > 0 and _dw_fused_sgd(dpre, x2, dw, db, upd):
            return
        if lib:
            dw.addmm_(dpre.t(), x2)
            if db is not None and not fold_db:
                C().act_bwd_bias(dpre, dpre, None, db, M, N, 10)
        else:
            gemm(dpre, dpre.stride(0), False, x2, x2.stride(0), False, dw, K, N, K, M, beta=True, rowsum_a=db)
        upd.apply(dw)
        return
    if lib and phase != "dx":
        dw.addmm_(dpre.t(), x2)                          # hipBLASLt, accumulates (beta = 1)
        if db is not None and not fold_db:
            C().act_bwd_bias(dpre, dpre, None, db, M, N, 10)   # column sums of dpre
        if phase == "dw":
            return
    # dW[N,K] = dpre^T x (both operands MN-contiguous: transposing LDS reads); the bias gradient
    # db = column sums of dpre is accumulated from the staged A tiles of the same GEMM
    # dW ACCUMULATES (beta): the executor zeroes the flat gradient buffer once per step, so weights
    # used by several ops sum their gradients
    if phase != "dx" and not lib and not (_smallk(x2, K) and _dw_smallk(dpre, x2, dw, db, None)):
        gemm(dpre, dpre.stride(0), False, x2, x2.stride(0), False, dw, K, N, K, M, beta=True, rowsum_a=db)
    if phase == "dw":
        return
    if dx2 is not None:
        _linear_dx(dpre, w, dx2, dx_acc, fuse_below, M, N, K)


def _linear_dx(dpre, w, dx2, dx_acc, fuse_below, M, N, K):
    # dX[M,K] = dpre W   (+ fused activation backward of the layer below)
    if dx2 is not None:
        if fuse_below is not None:
            yb, actb = fuse_below[0], fuse_below[1]
            assert not dx_acc
            gemm(dpre, dpre.stride(0), True, w, K, False, dx2, dx2.stride(0), M, K, N,
                 act_y=yb.view(M, K), bwd_act=int(actb))
        else:
            gemm(dpre, dpre.stride(0), True, w, K, False, dx2, dx2.stride(0), M, K, N, beta=bool(dx_acc))


def bmm(a, b, out, transA, transB, acc):
    batch = 1
    for d in out.shape[:-2]:
        batch *= d
    M, N = out.shape[-2], out.shape[-1]
    K = a.shape[-2] if transA else a.shape[-1]
    lda = a.shape[-1]
    ldb = b.shape[-1]
    gemm(a, lda, not transA, b, ldb, transB, out, N, M, N, K, beta=bool(acc), batch=batch,
         sA=a.shape[-1] * a.shape[-2], sB=b.shape[-1] * b.shape[-2], sC=M * N, use_ws=False)


# ------------------------------------------------------------------ embedding
def embedding_forward(idx, w, out, aggr):
    bag = idx.shape[1]
    scale = 1.0 / bag if aggr == 22 else 1.0
    C().embedding_fwd(idx, w, out, out.stride(0), scale)


def embedding_backward_sgd(idx, dy, w, lr, aggr, ws):
    bag = idx.shape[1]
    scale = 1.0 / bag if aggr == 22 else 1.0
    C().embedding_bwd(idx, dy, dy.stride(0), w, lr, scale)


def embedding_backward_dense(idx, dy, dw, aggr):
    bag = idx.shape[1]
    scale = 1.0 / bag if aggr == 22 else 1.0
    dw.zero_()
    C().embedding_bwd(idx, dy, dy.stride(0), dw, None, scale)


# ------------------------------------------------------------------ DLRM interaction
def dot_interaction_forward(inputs, y, self_inter):
    D = inputs[0].shape[-1]
    C().dot_fwd(list(inputs), inputs[0].stride(0), y, y.stride(0), D, y.shape[1], bool(self_inter))


def dot_interaction_backward(inputs, dy, in_grads, accs, self_inter, act0=10):
    """act0 (fp32): the activation backward of input 0's producer applied to its gradient (the
    executor's bottom-MLP fusion: that Linear then takes the gradient as its pre-activation one)."""
    D = inputs[0].shape[-1]
    mask = 0
    for i, a in enumerate(accs):
        if a and in_grads[i] is not None:
            mask |= 1 << i
    ld = next((g.stride(0) for g in in_grads if g is not None), D)
    C().dot_bwd(list(inputs), inputs[0].stride(0), dy, dy.stride(0), list(in_grads), ld, mask, D, bool(self_inter),
                int(act0))


# ------------------------------------------------------------------ optimizers / loss
def sgd_update(master, grad, v, compute, lr_tensor, wd, momentum, nesterov, zero_grad=False):
    """zero_grad: the kernel writes the consumed gradient back as zeros (no separate memset)."""
    C().sgd(master, grad, v, compute, lr_tensor, wd, momentum, nesterov, zero_grad)


def adam_update(master, grad, m, v, compute, alpha_t, b1, b2, wd, eps, zero_grad=False):
    C().adam(master, grad, m, v, compute, alpha_t, b1, b2, wd, eps, zero_grad)


def loss_forward_backward(loss_type, logits, labels, grad, scale, acc, mask, clamp=0.0):
    """clamp in (0, 0.5): predictions clamped to [clamp, 1-clamp] (DLRM --loss-threshold)."""
    C().loss(loss_type, logits, labels, grad, scale, acc, mask, float(clamp))


# ------------------------------------------------------------------ element-wise & data movement
def unary_forward(code, x, y):
    C().unary_fwd(code, x, y)


def unary_backward(code, x, y, dy, dx, acc):
    C().unary_bwd(code, x, y, dy, dx, bool(acc))


def binary_forward(code, a, b, y, relu=False):
    C().binary_fwd(code, a, b, y, bool(relu))


def binary_backward(code, a, b, dy, da, db, acca, accb, ymask=None):
    C().binary_bwd(code, a, b, dy, ymask, da, db, bool(acca), bool(accb))


def _outer_inner(shape, axis):
    outer = 1
    for d in shape[:axis]:
        outer *= d
    inner = 1
    for d in shape[axis:]:
        inner *= d
    return outer, inner


def concat_forward(inputs, y, axis):
    outer, tot = _outer_inner(y.shape, axis)
    src, so, dst, do, rows, cols, lds, ldd = [], [], [], [], [], [], [], []
    off = 0
    for x in inputs:
        _, inner = _outer_inner(x.shape, axis)
        src.append(x); so.append(0); dst.append(y); do.append(off)
        rows.append(outer); cols.append(inner); lds.append(inner); ldd.append(tot)
        off += inner
    C().multi_copy(src, so, dst, do, rows, cols, lds, ldd, 0)


def concat_backward(dy, in_grads, accs, axis, in_shapes=None):
    """in_shapes: shapes of the concatenated inputs -- an input without a gradient (e.g. a model
    input) still occupies its slice of dy, so later slices start after it."""
    outer, tot = _outer_inner(dy.shape, axis)
    src, so, dst, do, rows, cols, lds, ldd = [], [], [], [], [], [], [], []
    mask = 0
    off = 0
    k = 0
    for i, (g, a) in enumerate(zip(in_grads, accs)):
        if g is None:
            assert in_shapes is not None, "concat_backward: input shapes needed to skip a gradient-less input"
            off += _outer_inner(in_shapes[i], axis)[1]
            continue
        _, inner = _outer_inner(g.shape, axis)
        src.append(dy); so.append(off); dst.append(g); do.append(0)
        rows.append(outer); cols.append(inner); lds.append(tot); ldd.append(inner)
        if a:
            mask |= 1 << k
        k += 1
        off += inner
    if src:
        C().multi_copy(src, so, dst, do, rows, cols, lds, ldd, mask)


def split_forward(x, outs, axis):
    outer, tot = _outer_inner(x.shape, axis)
    src, so, dst, do, rows, cols, lds, ldd = [], [], [], [], [], [], [], []
    off = 0
    for y in outs:
        _, inner = _outer_inner(y.shape, axis)
        src.append(x); so.append(off); dst.append(y); do.append(0)
        rows.append(outer); cols.append(inner); lds.append(tot); ldd.append(inner)
        off += inner
    C().multi_copy(src, so, dst, do, rows, cols, lds, ldd, 0)


def split_backward(out_grads, dx, acc, axis, out_shapes=None):
    """dx = concat(out_grads) along axis; a None grad (an unused split output) is a zero
    block -- the caller zeroes dx first when it does not accumulate."""
    outer, tot = _outer_inner(dx.shape, axis)
    src, so, dst, do, rows, cols, lds, ldd = [], [], [], [], [], [], [], []
    off = 0
    mask = 0
    for k, g in enumerate(out_grads):
        if g is None:
            off += _outer_inner(out_shapes[k], axis)[1]
            continue
        _, inner = _outer_inner(g.shape, axis)
        src.append(g); so.append(0); dst.append(dx); do.append(off)
        rows.append(outer); cols.append(inner); lds.append(inner); ldd.append(tot)
        if acc:
            mask |= 1 << k
        off += inner
    if src:
        C().multi_copy(src, so, dst, do, rows, cols, lds, ldd, mask)


def copy_or_add(src, dst, acc):
    n = src.numel()
    C().multi_copy([src.contiguous()], [0], [dst], [0], [1], [n], [n], [n], 1 if acc else 0)


def permute(x, y, perm, acc):
    out_dims = list(y.shape)
    strides = [x.stride(p) for p in perm]
    C().permute(x, y, out_dims, strides, bool(acc))


def reverse(x, y, axis, acc):
    outer, _ = _outer_inner(x.shape, axis)
    inner = 1
    for d in x.shape[axis + 1:]:
        inner *= d
    C().reverse(x, y, outer, x.shape[axis], inner, bool(acc))


def softmax_forward(x, y):
    C().softmax(x, y, x.numel() // x.shape[-1], x.shape[-1])


def dropout_forward(x, y, rate, seed, ctx):
    ctx.saved["step"] = ctx.saved.get("step", 0)
    C().dropout(x, y, rate, seed + 131 * ctx.rank, ctx.saved["step"], False)


def dropout_backward(dy, dx, rate, seed, ctx, acc):
    C().dropout(dy, dx, rate, seed + 131 * ctx.rank, ctx.saved.get("step", 0), bool(acc))


# ------------------------------------------------------------------ CNN
_scratch = {}


def scratch(device, name, numel, dtype=torch.bfloat16):
    """Grow-only per-device scratch buffers shared by ops that run back to back on one stream
    (im2col columns, NHWC GEMM outputs, ...).  Sizes settle during the eager warm-up steps, so
    captured hipGraphs keep valid pointers."""
    key = (str(device), name, dtype)
    t = _scratch.get(key)
    if t is None or t.numel() < numel:
        t = torch.empty(max(numel, 1), dtype=dtype, device=device)
        _scratch[key] = t
    return t[:numel]


def _s2d_plan(x, w, y, stride):
    """Space-to-depth for a strided bf16 conv whose re-laid kernel costs <= 1.5x the MACs (the
    AlexNet / ResNet stems on 3 channels): returns (s, Hs, Ws, Rs, Ss) or None."""
    s_ = stride[0]
    if s_ < 2 or stride[1] != s_ or x.dtype != torch.bfloat16:
        return None
    Kout, Cg, R, S = w.shape
    Rs, Ss = -(-R // s_), -(-S // s_)
    if Cg * s_ * s_ * Rs * Ss > 1.5 * Cg * R * S:
        return None
    return s_, y.shape[2] + (R - 1) // s_, y.shape[3] + (S - 1) // s_, Rs, Ss


def _s2d_operands(x, w, plan, pads, saved):
    s_, Hs, Ws, Rs, Ss = plan
    N, Cin = x.shape[0], x.shape[1]
    Kout = w.shape[0]
    shp = (N, Cin * s_ * s_, Hs, Ws)
    xs = saved.get("s2d_x") if saved is not None else None
    if xs is None or tuple(xs.shape) != shp or xs.dtype != x.dtype:
        xs = torch.empty(shp, dtype=x.dtype, device=x.device)
        if saved is not None:
            saved["s2d_x"] = xs
    ws = scratch(x.device, "conv_s2d_w", Kout * Cin * s_ * s_ * Rs * Ss, w.dtype).view(Kout, Cin * s_ * s_, Rs, Ss)
    return xs, ws


# ---- per-layer measured convolution algorithms ---------------------------------------------------
# The reference times cuDNN's candidate algorithms per conv layer at init and keeps the fastest for the
# forward, filter-gradient and data-gradient passes (src/ops/conv_2d.cu:216-243, :332-347, :872-930:
# cudnnFind*AlgorithmEx).  flexmi does the same over its own MFMA convolution forms: the first eager
# call of a layer's forward / backward times every applicable form on the layer's real operands
# (CUDA events, outputs into scratch, accumulating gradients untouched) and records the fastest in the
# op's context; later calls (and the hipGraph capture) run the recorded form.  Forms:
#   nhwc      NHWC-staged implicit GEMM (conv_nhwc.hip; >= 16 input channels, bf16)
#   igemm     NCHW implicit GEMM (conv_igemm.hip; any shape) -- strided 1x1 forward and strided
#             backward through the stride-phase decomposition when phase=True
#   s2d       space-to-depth of a strided few-channel stem onto the stride-1 NCHW kernels
#   s2d_nhwc  the same re-laid stem on the NHWC kernels (the space-to-depth input has s*s*Cin channels)
#   stem      the dedicated stem kernels: the input tile staged into LDS in space-to-depth NHWC order
#             by the convolution kernel itself (no re-laid image in HBM), 64 filters, few channels
# FM_CONV_TUNE=0: no timing, the fixed heuristic order (nhwc > s2d > igemm).  Layers whose NHWC images
# are shared with a neighbour (the executor's conv chain fusion) keep the nhwc form.
CONV_TUNE = os.environ.get("FM_CONV_TUNE", "1") != "0"
CONV_TUNE_LOG = []      # (direction, key, {form: us}, chosen): what the tuner measured (tests, reports)


def _chained(saved):
    return saved is not None and any(k in saved for k in ("nhwc_out2", "nhwc_x_prestaged", "nhwc_dgrad_out2",
                                                          "nhwc_g_prestaged"))


# the dedicated stem kernels (csrc/kernels/conv_stem.hip) for strided few-channel first layers
# (tests switch them off to compare with the generic forms)
STEM_CONV = True


def _stem_ok(x, w, stride, groups):
    return (STEM_CONV and x.dtype == torch.bfloat16 and groups == 1 and stride[0] == stride[1]
            and C().stem_supported(x.shape[1], w.shape[0], w.shape[2], w.shape[3], stride[0], stride[1]))


def conv_forms(x, w, y, stride, groups, direction="fwd", need_dx=False):
    """Applicable convolution forms of one layer, in the heuristic's preference order (the stem
    kernels compute no input gradient: backward candidates only for a layer on the network input)."""
    out = []
    if _stem_ok(x, w, stride, groups) and not (direction == "bwd" and need_dx):
        out.append("stem")
    if _nhwc_ok(x, w, groups):
        out.append("nhwc")
    plan = _s2d_plan(x, w, y, stride)
    if plan is not None:
        out.append("s2d")
        if NHWC_CONV and w.shape[1] * plan[0] * plan[0] >= 16:
            out.append("s2d_nhwc")
    out.append("igemm")
    return out


def _time_us(fn, reps=3):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def _conv_choose(saved, direction, forms, run, key):
    """The form recorded for this layer and direction, measuring the candidates on first use."""
    name = "conv_form_" + direction
    if saved is not None and saved.get(name) in forms:
        return saved[name]
    pick = forms[0]
    if (CONV_TUNE and len(forms) > 1 and saved is not None and not _chained(saved) and torch.cuda.is_available()
            and not torch.cuda.is_current_stream_capturing()):
        times = {}
        for f in forms:
            if run(f) is False:     # the form does not apply to this layout (a backward fell through)
                continue
            times[f] = _time_us(lambda f=f: run(f))
        pick = min(times, key=times.get) if times else forms[0]
        CONV_TUNE_LOG.append((direction, key, times, pick))
    if saved is not None:
        saved[name] = pick
    return pick


def conv2d_forward(x, w, b, y, stride, pads, act, groups, saved=None, form=None):
    """Implicit-GEMM convolution on MFMA: the form measured fastest for this layer (see
    conv_forms / _conv_choose; ``form`` forces one).  pads = (top, bottom, left, right) of this
    shard (bottom / right are implied by y's extent)."""
    assert groups == 1, "grouped convolution is not supported on the HIP path"
    w = w.contiguous()
    forms = conv_forms(x, w, y, stride, groups)
    if form is None:
        if _chained(saved) or len(forms) == 1:
            # a layer whose NHWC images are shared with a neighbour keeps the NHWC form
            form = "nhwc" if "nhwc" in forms else forms[0]
        else:
            # candidates write a scratch output and keep no staged state for the backward
            ys = scratch(y.device, "conv_tune_y", y.numel(), y.dtype).view(y.shape)
            key = (tuple(x.shape), tuple(w.shape), tuple(stride), tuple(pads), str(x.dtype))
            form = _conv_choose(saved, "fwd", forms, lambda f: _conv_fwd_run(f, x, w, b, ys, stride, pads, act, None), key)
    _conv_fwd_run(form, x, w, b, y, stride, pads, act, saved)


def _conv_fwd_run(form, x, w, b, y, stride, pads, act, saved):
    if form == "stem":
        Kout, Cin, R, S = w.shape
        wf = scratch(x.device, "stem_wf", C().stem_wf_elems(Cin, Kout, R, S, stride[0]), torch.bfloat16)
        C().stem_fwd(x, w, wf, b, y, stride[0], pads[0], pads[2], int(act))
        return
    if form == "nhwc":
        _nhwc_forward(x, w, b, y, stride, pads, act, saved)
        return
    if form in ("s2d", "s2d_nhwc"):
        plan = _s2d_plan(x, w, y, stride)
        xs, ws = _s2d_operands(x, w, plan, pads, saved)
        C().conv_s2d(x, xs, plan[0], pads[0], pads[2], False, False)
        C().conv_w_s2d(w, ws, ws, ws, plan[0], False)
        if saved is not None:
            saved["s2d_ready"] = True
        if form == "s2d_nhwc":
            # the re-laid stem's NHWC staging is not kept (its geometry is the s2d image's, not x's)
            _nhwc_forward(xs, ws, b, y, (1, 1), (0, 0, 0, 0), act, None)
            return
        x, w, stride, pads = xs, ws, (1, 1), (0, 0, 0, 0)
    Kout, Cg, R, S = w.shape
    if (PHASE_CONV and R == 1 and S == 1 and stride[0] == stride[1] and stride[0] > 1 and x.dtype == torch.bfloat16):
        # a strided 1x1 conv reads ONE input phase: gather x[:, :, a::s, b::s] and run the
        # stride-1 pixel-vector kernel on it (the ResNet downsampling shortcuts)
        s_ = stride[0]
        N, Cin, H, W = x.shape
        a, b_ = (-pads[0]) % s_, (-pads[2]) % s_
        Ha, Wb = -(-(H - a) // s_), -(-(W - b_) // s_)
        xa = scratch(x.device, "conv_phase_xf", N * Cin * Ha * Wb, x.dtype).view(N, Cin, Ha, Wb)
        _strided(x, xa, (N, Cin, Ha, Wb), (Cin * H * W, H * W, s_ * W, s_), (Cin * Ha * Wb, Ha * Wb, Wb, 1), a * W + b_,
                 0, False)
        x, stride, pads = xa, (1, 1), ((pads[0] + a) // s_, 0, (pads[2] + b_) // s_, 0)
    wpad = scratch(x.device, "conv_wpad", C().conv_scratch(Kout, Cg * R * S), w.dtype)
    C().conv_fwd(x, w, wpad, b, y, stride[0], stride[1], pads[0], pads[2], int(act))


def conv2d_backward(x, w, y, dy, dx, dw, db, stride, pads, act, groups, acc, saved=None, form=None):
    """G = act'(y) * dY with db = sum G, then dW += G (x) X and dX (+)= Wt (x) G, in the form measured
    fastest for this layer's backward (candidates run on scratch gradients: dW / db / an accumulated
    dX are touched only by the chosen form)."""
    assert groups == 1, "grouped convolution is not supported on the HIP path"
    w = w.contiguous()
    forms = conv_forms(x, w, y, stride, groups, "bwd", need_dx=dx is not None)
    if form is None:
        if _chained(saved) or len(forms) == 1:
            # a layer whose NHWC images are shared with a neighbour keeps the NHWC form
            form = "nhwc" if "nhwc" in forms else forms[0]
        else:
            dws = scratch(x.device, "conv_tune_dw", dw.numel(), dw.dtype).view(dw.shape)
            dbs = scratch(x.device, "conv_tune_db", db.numel(), db.dtype).view(db.shape) if db is not None else None
            dxs = scratch(x.device, "conv_tune_dx", dx.numel(), dx.dtype).view(dx.shape) if dx is not None else None
            key = (tuple(x.shape), tuple(w.shape), tuple(stride), tuple(pads), str(x.dtype), dx is not None)
            form = _conv_choose(saved, "bwd", forms,
                                lambda f: _conv_bwd_run(f, x, w, y, dy, dxs, dws, dbs, stride, pads, act, False, None),
                                key)
    if not _conv_bwd_run(form, x, w, y, dy, dx, dw, db, stride, pads, act, acc, saved):
        _conv_bwd_run("igemm", x, w, y, dy, dx, dw, db, stride, pads, act, acc, saved)


def _conv_bwd_run(form, x, w, y, dy, dx, dw, db, stride, pads, act, acc, saved):
    """One backward form; False when it does not apply to this layout (the caller falls back)."""
    if form == "stem":
        if dx is not None:
            return False
        Kout, Cin, R, S = w.shape
        ws = scratch(x.device, "stem_ws", C().stem_wgrad_ws(Cin, Kout, R, S, stride[0]), torch.float32)
        C().stem_wgrad(x, y, dy, dw.view(-1), db, ws, R, S, stride[0], pads[0], pads[2], int(act))
        return True
    if form == "nhwc":
        return _nhwc_backward(x, w, y, dy, int(act), db, dx, dw, stride, pads, acc, saved)
    plan = _s2d_plan(x, w, y, stride) if form in ("s2d", "s2d_nhwc") else None
    if plan is not None and form == "s2d_nhwc":
        s_, Hs, Ws, Rs, Ss = plan
        xs, ws = _s2d_operands(x, w, plan, pads, saved)
        if not (saved is not None and saved.get("s2d_ready")):
            C().conv_s2d(x, xs, s_, pads[0], pads[2], False, False)
        C().conv_w_s2d(w, ws, ws, ws, s_, False)
        dws = scratch(x.device, "conv_s2d_dw", ws.numel(), torch.float32).view(ws.shape)
        dws.zero_()
        dxs = scratch(x.device, "conv_s2d_dx", xs.numel(), xs.dtype).view(xs.shape) if dx is not None else None
        if not _nhwc_backward(xs, ws, y, dy, int(act), db, dxs, dws, (1, 1), (0, 0, 0, 0), False, None):
            return False
        C().conv_w_s2d(w, ws, dws.view(-1), dw.view(-1), s_, True)
        if dx is not None:
            if not acc:
                dx.zero_()
            C().conv_s2d(dx, dxs, s_, pads[0], pads[2], True, True)
        return True
    g = dy
    if int(act) != 10 or db is not None:
        g = scratch(x.device, "conv_g", dy.numel(), dy.dtype).view(dy.shape) if int(act) != 10 else dy
        C().conv_act_bwd(dy, y, g, db, int(act))
    if plan is not None:
        s_, Hs, Ws, Rs, Ss = plan
        xs, ws = _s2d_operands(x, w, plan, pads, saved)
        if not (saved is not None and saved.get("s2d_ready")):
            C().conv_s2d(x, xs, s_, pads[0], pads[2], False, False)
        C().conv_w_s2d(w, ws, ws, ws, s_, False)
        dws = scratch(x.device, "conv_s2d_dw", ws.numel(), torch.float32)
        dws.zero_()
        C().conv_wgrad(g, xs, dws, Rs, Ss, 1, 1, 0, 0)
        C().conv_w_s2d(w, ws, dws, dw.view(-1), s_, True)
        if dx is not None:
            dxs = scratch(x.device, "conv_s2d_dx", xs.numel(), xs.dtype).view(xs.shape)
            wt = scratch(x.device, "conv_wt", C().conv_scratch(ws.shape[1], ws.shape[0] * Rs * Ss), w.dtype)
            C().conv_dgrad(g, ws, wt, dxs, 1, 1, 0, 0, False)
            if not acc:
                dx.zero_()
            C().conv_s2d(dx, dxs, s_, pads[0], pads[2], True, True)
        return True
    Kout, Cg, R, S = w.shape
    if PHASE_CONV and stride[0] == stride[1] and stride[0] > 1 and x.dtype == torch.bfloat16:
        _conv_backward_phases(x, w, g, dx, dw, stride[0], pads, acc)
        return True
    # dW / db ACCUMULATE into the per-step zeroed gradient buffer (tied weights sum their grads)
    C().conv_wgrad(g, x, dw.view(-1), R, S, stride[0], stride[1], pads[0], pads[2])
    if dx is not None:
        wt = scratch(x.device, "conv_wt", C().conv_scratch(Cg, Kout * R * S), w.dtype)
        C().conv_dgrad(g, w, wt, dx, stride[0], stride[1], pads[0], pads[2], bool(acc))
    return True


# Stride-phase decomposition of a strided convolution's backward (PHASE_CONV; tests switch it off to
# compare with the strided element-gather kernels).  For input phase (a, b) -- rows h = a + s*h', columns
# w = b + s*w' -- only the taps r = r0 + s*i (r0 = (a + pt) mod s) and t = t0 + s*j reach it, and
#   dX[:, :, a::s, b::s] = dgrad_stride1(G, W[:, :, r0::s, t0::s], pads (oa, ob))
#   dW[:, :, r0::s, t0::s] += wgrad_stride1(G, X[:, :, a::s, b::s], pads (oa, ob))
# with oa = (a + pt - r0) / s: s*s stride-1 problems on the pixel-vector MFMA path that together do
# exactly the convolution's useful MACs (the strided element path computes every tap of every
# output position and keeps a quarter: 567 us per ResNet-50 b64 downsampling dgrad,
# profiles/prof_r3_resnet50_b64_bf16_kernels.txt).
PHASE_CONV = True


def _strided(src, dst, d, ss, ts, so, to, acc):
    C().strided_copy4(src, dst, list(d), list(ss), list(ts), int(so), int(to), bool(acc))


def _conv_backward_phases(x, w, g, dx, dw, s_, pads, acc):
    N, Cin, H, W = x.shape
    Kout, _, R, S = w.shape
    pt, pl = pads[0], pads[2]
    dev = x.device
    for a in range(s_):
        r0 = (a + pt) % s_
        nr = -(-(R - r0) // s_) if r0 < R else 0
        oa = (a + pt - r0) // s_
        Ha = -(-(H - a) // s_) if a < H else 0
        for b in range(s_):
            t0 = (b + pl) % s_
            nt = -(-(S - t0) // s_) if t0 < S else 0
            ob = (b + pl - t0) // s_
            Wb = -(-(W - b) // s_) if b < W else 0
            if Ha == 0 or Wb == 0:
                continue
            box = (N, Cin, Ha, Wb)
            xstr = (Cin * H * W, H * W, s_ * W, s_)          # x[:, :, a::s, b::s] in x's storage
            if nr == 0 or nt == 0:                           # no tap reaches this phase
                if dx is not None and not acc:
                    z = scratch(dev, "conv_phase_zero", 1, dx.dtype).zero_()
                    _strided(z, dx, box, (0, 0, 0, 0), xstr, 0, a * W + b, False)
                continue
            # sub-kernel W[:, :, r0::s, t0::s] -> contiguous [K, C, nr, nt]
            wsub = scratch(dev, "conv_phase_w", Kout * Cin * nr * nt, w.dtype).view(Kout, Cin, nr, nt)
            _strided(w, wsub, (Kout, Cin, nr, nt), (Cin * R * S, R * S, s_ * S, s_), (Cin * nr * nt, nr * nt, nt, 1),
                     r0 * S + t0, 0, False)
            # weight gradient: wgrad(G, x phase) into a fp32 [K, C, nr, nt] block, added to dW's taps
            xa = scratch(dev, "conv_phase_x", N * Cin * Ha * Wb, x.dtype).view(box)
            _strided(x, xa, box, xstr, (Cin * Ha * Wb, Ha * Wb, Wb, 1), a * W + b, 0, False)
            dws = scratch(dev, "conv_phase_dw", Kout * Cin * nr * nt, torch.float32).view(Kout, Cin, nr, nt)
            dws.zero_()
            C().conv_wgrad(g, xa, dws.view(-1), nr, nt, 1, 1, oa, ob)
            _strided(dws, dw, (Kout, Cin, nr, nt), (Cin * nr * nt, nr * nt, nt, 1), (Cin * R * S, R * S, s_ * S, s_),
                     0, r0 * S + t0, True)
            if dx is None:
                continue
            dxa = scratch(dev, "conv_phase_dx", N * Cin * Ha * Wb, dx.dtype).view(box)
            wt = scratch(dev, "conv_wt", C().conv_scratch(Cin, Kout * nr * nt), w.dtype)
            C().conv_dgrad(g, wsub, wt, dxa, 1, 1, oa, ob, False)
            _strided(dxa, dx, box, (Cin * Ha * Wb, Ha * Wb, Wb, 1), xstr, 0, a * W + b, acc)


# FM_CONV_NHWC=1/0 (default 1): bf16 convolutions on >= 16 input channels run on the NHWC-staged
# implicit GEMM (csrc/kernels/conv_nhwc.hip): the image operand is re-laid ONCE per pass into a
# zero-padded NHWC copy, so every 16-B operand chunk of the GEMM is 8 channels of one pixel (no
# per-element gather math, no halo masks).  The forward's staged input is kept in ``saved`` for
# the weight gradient.  Stems on few channels keep the NCHW kernels (space-to-depth).
NHWC_CONV = os.environ.get("FM_CONV_NHWC", "1") != "0"
# STRIDE_PHASE_DGRAD (tests compare both): strided NHWC data gradients as one GEMM per stride phase
# instead of one GEMM over the stride-dilated G (s*s the MACs)
STRIDE_PHASE_DGRAD = True


def _r8(v):
    return (v + 7) // 8 * 8


def _nhwc_ok(x, w, groups):
    return NHWC_CONV and groups == 1 and x.dtype == torch.bfloat16 and w.shape[1] >= 16


def _nhwc_stage_x(x, w, y, stride, pads, saved):
    """Stage x into its zero-padded NHWC window image [N][Hp][Wp][Cp] (output (p, q) reads rows
    p*sh .. p*sh+R-1); kept in ``saved`` (one buffer per op) for the backward."""
    N, Cin = x.shape[0], x.shape[1]
    R, S = w.shape[2], w.shape[3]
    P, Q = y.shape[2], y.shape[3]
    Cp, Hp, Wp = _r8(Cin), (P - 1) * stride[0] + R, (Q - 1) * stride[1] + S
    shp = (N, Hp, Wp, Cp)
    if saved is not None:
        xs = saved.get("nhwc_x")
        if xs is not None and saved.get("nhwc_x_prestaged") and tuple(xs.shape) == shp:
            return xs, Cp, Hp, Wp     # the producing conv's epilogue already wrote it (conv chain fusion)
        if xs is None or tuple(xs.shape) != shp or xs.device != x.device:
            xs = torch.empty(shp, dtype=x.dtype, device=x.device)
            saved["nhwc_x"] = xs
    else:
        xs = scratch(x.device, "cn_xs", N * Hp * Wp * Cp, x.dtype).view(shp)
    C().nhwc_stage(x, xs, Cp, Hp, Wp, pads[0], pads[2], 1, 1)
    return xs, Cp, Hp, Wp


def nhwc_x_geometry(x_shape, w_shape, y_shape, stride, pads):
    """(N, Hp, Wp, Cp, top, left) of a conv's staged input (see _nhwc_stage_x)."""
    R, S = w_shape[2], w_shape[3]
    P, Q = y_shape[2], y_shape[3]
    return x_shape[0], (P - 1) * stride[0] + R, (Q - 1) * stride[1] + S, _r8(x_shape[1]), pads[0], pads[2]


def nhwc_g_geometry(x_shape, w_shape, y_shape, stride, pads, need_dx):
    """(N, Hg, Wg, Kp, gt, gl, dh, dw) of a conv's staged output gradient (see _nhwc_backward), or
    None where the staging does not apply."""
    N, Cin, H, W = x_shape
    Kout, _, R, S = w_shape
    P, Q = y_shape[2], y_shape[3]
    sh, sw = stride
    pt, pl = pads[0], pads[2]
    if need_dx:
        gt, gl = R - 1 - pt, S - 1 - pl
        if gt < 0 or gl < 0:
            return None
        return (N, max(H + R - 1, gt + (P - 1) * sh + 1), max(W + S - 1, gl + (Q - 1) * sw + 1), _r8(Kout), gt, gl, sh, sw)
    return (N, P, Q, _r8(Kout), 0, 0, 1, 1)


def _nhwc_wbufs(saved, w):
    """This layer's forward matrix [K][R*S*Cp] and dgrad matrix [C][R*S*Kp] (kept in ``saved``)."""
    Kout, Cin, R, S = w.shape
    nwf, nwd = Kout * R * S * _r8(Cin), Cin * R * S * _r8(Kout)
    wf, wd = saved.get("nhwc_wf"), saved.get("nhwc_wd")
    if wf is None or wf.numel() != nwf or wf.device != w.device:
        wf = saved["nhwc_wf"] = torch.empty(nwf, dtype=w.dtype, device=w.device)
    if wd is None or wd.numel() != nwd or wd.device != w.device:
        wd = saved["nhwc_wd"] = torch.empty(nwd, dtype=w.dtype, device=w.device)
    return wf, wd


def conv_wprep_all(layers):
    """The weight re-layouts of every convolution whose last forward ran the NHWC form, in ONE launch
    at the start of the step's forward (weights change only at the update): ``layers`` = [(w,
    saved)].  Each such layer's next _nhwc_forward finds ``saved["nhwc_wf_ready"]`` and skips its own
    re-layout launch (ResNet-50: 53 launches of ~7 us per step -> 1)."""
    ws, wfs, wds, cps, kps, marks = [], [], [], [], [], []
    for w, saved in layers:
        if saved is None or not saved.get("nhwc_fwd_used") or w.dtype != torch.bfloat16 or not w.is_contiguous():
            continue
        wf, wd = _nhwc_wbufs(saved, w)
        ws.append(w)
        wfs.append(wf)
        wds.append(wd)
        cps.append(_r8(w.shape[1]))
        kps.append(_r8(w.shape[0]))
        marks.append(saved)
    if ws:
        C().cnhwc_wprep_multi(ws, wfs, wds, cps, kps)
    for sv in marks:
        sv["nhwc_wf_ready"] = True


def _nhwc_forward(x, w, b, y, stride, pads, act, saved):
    Kout, Cin, R, S = w.shape
    xs, Cp, Hp, Wp = _nhwc_stage_x(x, w, y, stride, pads, saved)
    if saved is not None:
        saved["nhwc_x_ready"] = True
        saved["nhwc_fwd_used"] = True
        # the backward's flipped / transposed matrix comes out of the same launch (weights do not
        # change between an op's forward and backward), or both came from this step's conv_wprep_all
        wf, wd = _nhwc_wbufs(saved, w)
        if not saved.pop("nhwc_wf_ready", False):
            C().cnhwc_wprep(w, wf, wd, w, w, Cp, _r8(Kout), 3, 1)
    else:
        wf = scratch(x.device, "cn_wf", Kout * R * S * Cp, w.dtype)
        C().cnhwc_wprep(w, wf, w, w, w, Cp, _r8(Kout), 0, 1)
    o2 = saved.get("nhwc_out2") if saved is not None else None   # conv chain fusion: the consumer's staged input
    C().conv_nhwc_fwd(xs, wf, b, y, R, S, Cp, Hp, Wp, stride[0], stride[1], int(act), o2[0] if o2 else None,
                      list(o2[1]) if o2 else [])


def _nhwc_backward(x, w, y, dy, act, db, dx, dw, stride, pads, acc, saved):
    """Weight gradient (and, for any stride, the data gradient) on the NHWC-staged kernels.
    G = act'(y) * dY is staged once (the bias gradient db (+)= sum G is summed by the wgrad kernel):
    placed at (R-1-pt, S-1-pl) and dilated by the stride when dX is needed (the data gradient is
    then a stride-1 convolution of the flipped kernel over it), unpadded otherwise.  Returns False
    (nothing done; the caller falls back) when the layout is outside what the staging supports."""
    N, Cin, H, W = x.shape
    Kout, _, R, S = w.shape
    P, Q = dy.shape[2], dy.shape[3]
    sh, sw = stride
    pt, pl = pads[0], pads[2]
    Kp = _r8(Kout)
    dev = x.device
    geo_g = nhwc_g_geometry(x.shape, w.shape, dy.shape, stride, pads, dx is not None)
    if geo_g is None:
        return False
    _, Hg, Wg, _, gt, gl, dh, dwl = geo_g
    gs = saved.get("nhwc_gs") if saved is not None and saved.get("nhwc_g_prestaged") else None
    if gs is None or tuple(gs.shape) != (N, Hg, Wg, Kp):
        gs = scratch(dev, "cn_gs", N * Hg * Wg * Kp, dy.dtype).view(N, Hg, Wg, Kp)
        C().nhwc_stage_grad(dy, y, gs, act, Kp, Hg, Wg, gt, gl, dh, dwl)
    # else: the consumer conv's data-gradient epilogue already wrote G here (conv chain fusion)
    if saved is not None and saved.get("nhwc_x_ready") and "nhwc_x" in saved:
        xs = saved["nhwc_x"]
        Cp, Hp, Wp = xs.shape[3], xs.shape[1], xs.shape[2]
    else:
        # no forward staging to reuse (eager backward without a saved context): stage again
        xs, Cp, Hp, Wp = _nhwc_stage_x(x, w, dy, stride, pads, None)
    # weight gradient: fp32 [K][R*S*Cp] over the output pixels; in a dilated G, pixel (p, q) sits at
    # (gt + p*sh, gl + q*sw)
    # (split-K fp32 slabs summed by the fold into dW[K,C,R,S]; db (+)= sum G from the same kernel)
    g2 = scratch(dev, "cn_g2", C().conv_nhwc_wgrad_ws(N, Kout, P, Q, R, S, Cp), torch.float32)
    # the pixel-origin table depends on the geometry only: an op builds it once
    geo = (N, P, Q, Hg, Wg, gt, gl, dh, dwl, Hp, Wp, Cp, Kp, sh, sw)
    build = True
    if saved is not None:
        ptab = saved.get("nhwc_ptab")
        if ptab is not None and saved.get("nhwc_ptab_geo") == geo and ptab.device == dev:
            build = False
        else:
            ptab = torch.empty(2 * N * P * Q, dtype=torch.int32, device=dev)
            saved["nhwc_ptab"], saved["nhwc_ptab_geo"] = ptab, geo
    else:
        ptab = scratch(dev, "cn_ptab", 2 * N * P * Q, torch.int32)
    nsplit = C().conv_nhwc_wgrad(gs, xs, g2, db, N, Kout, Kp, P, Q, Hg, Wg, gt, gl, dh, dwl, R, S, Cp, Hp, Wp, sh, sw, ptab,
                                 build)
    C().cnhwc_wprep(w, w, w, g2, dw.view(-1), Cp, Kp, 2, nsplit)
    if dx is not None:
        o2 = saved.get("nhwc_dgrad_out2") if saved is not None and not acc else None   # the producer's staged G
        if (dh > 1 or dwl > 1) and STRIDE_PHASE_DGRAD:
            # strided: one dense GEMM per stride phase over its sub-kernel (no dilation waste)
            wsub = scratch(dev, "cn_wsub", Cin * R * S * Kp, w.dtype)
            C().conv_nhwc_dgrad_strided(gs, w, wsub, dx, Kp, Hg, Wg, gt, gl, dh, dwl, bool(acc), o2[0] if o2 else None,
                                        list(o2[1]) if o2 else [])
            return True
        wd = saved.get("nhwc_wd") if saved is not None and saved.get("nhwc_x_ready") else None
        if wd is None or wd.numel() != Cin * R * S * Kp:
            wd = scratch(dev, "cn_wd", Cin * R * S * Kp, w.dtype)
            C().cnhwc_wprep(w, wd, w, w, w, _r8(Cin), Kp, 1, 1)
        C().conv_nhwc_dgrad(gs, wd, dx, R, S, Kp, Hg, Wg, bool(acc), o2[0] if o2 else None, list(o2[1]) if o2 else [])
    return True


def _pool_code(saved, y):
    c = saved.get("pool_code")
    if c is None or c.numel() < y.numel() or c.device != y.device:
        c = torch.empty(y.numel(), dtype=torch.uint8, device=y.device)
        saved["pool_code"] = c
    return c


def pool2d_forward(x, y, k, stride, pads, pool_type, act, saved=None):
    """Max pooling also records each window's argmax byte in the op's saved state (for backward)."""
    is_max = int(pool_type) == 30
    code = _pool_code(saved, y) if (is_max and saved is not None) else None
    C().pool_fwd(x, y, code, k[0], k[1], stride[0], stride[1], pads[0], pads[2], is_max, int(act))
    if saved is not None:
        saved["pool_code_ready"] = code is not None


def pool2d_backward(x, y, dy, dx, k, stride, pads, pool_type, act, acc, saved=None):
    saved = {} if saved is None else saved
    ready = bool(saved.get("pool_code_ready", False))
    code = _pool_code(saved, y)
    C().pool_bwd(x, y, dy, dx, code, ready, k[0], k[1], stride[0], stride[1], pads[0], pads[2], int(pool_type) == 30,
                 int(act), bool(acc))


def _bn_bufs(saved, C_, device):
    if "bn_stats" not in saved:
        saved["bn_stats"] = torch.zeros(2 * C_, dtype=torch.float32, device=device)
        saved["bn_meaninv"] = torch.zeros(2 * C_, dtype=torch.float32, device=device)
        saved["bn_gsum"] = torch.zeros(2 * C_, dtype=torch.float32, device=device)
    return saved["bn_stats"], saved["bn_meaninv"], saved["bn_gsum"]


def batchnorm_forward(x, scale, bias, y, relu, eps, saved):
    stats, meaninv, _ = _bn_bufs(saved, x.shape[1], x.device)
    C().bn_fwd(x, y, scale, bias, stats, meaninv, float(eps), bool(relu))


def batchnorm_backward(x, scale, y, dy, dx, dscale, dbias, relu, eps, saved, acc):
    _, meaninv, gsum = _bn_bufs(saved, x.shape[1], x.device)
    C().bn_bwd(x, y, dy, meaninv, scale, gsum, dscale, dbias, dx, bool(relu), bool(acc))
