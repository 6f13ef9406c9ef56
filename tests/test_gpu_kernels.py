"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op (MI355X only)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def bf(x):
    return x.to(torch.bfloat16)


def rel_err(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 200, 130), (1024, 512, 256), (33, 1, 64), (8192, 64, 16)])
def test_gemm_orientations(gpu, a_k, b_k, M, N, K):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(0)
    A = torch.randn(M, K, device=gpu)
    B = torch.randn(K, N, device=gpu)
    Ab = bf(A) if a_k else bf(A.t().contiguous())      # [M,K] or [K,M]
    Bb = bf(B.t().contiguous()) if b_k else bf(B)      # [N,K] or [K,N]
    lda = K if a_k else M
    ldb = K if b_k else N
    C = torch.empty(M, N, device=gpu, dtype=torch.float32)
    Kk.gemm(Ab, lda, a_k, Bb, ldb, b_k, C, N, M, N, K)
    ref = bf(A).float() @ bf(B).float()
    assert rel_err(C, ref) < 2e-3, (a_k, b_k, M, N, K)


def test_gemm_epilogue_bias_relu_bf16_beta(gpu):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(1)
    M, N, K = 512, 384, 192
    A, W = torch.randn(M, K, device=gpu), torch.randn(N, K, device=gpu)
    b = torch.randn(N, device=gpu)
    C = torch.randn(M, N, device=gpu).to(torch.bfloat16)
    C0 = C.float().clone()
    Kk.gemm(bf(A), K, True, bf(W), K, True, C, N, M, N, K, bias=b, act=11, beta=True)
    ref = torch.relu(bf(A).float() @ bf(W).float().t() + b) + C0
    assert rel_err(C, ref) < 1e-2


def test_gemm_splitk_and_batch(gpu):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(2)
    M, N, K = 64, 128, 4096
    A, B = torch.randn(K, M, device=gpu), torch.randn(K, N, device=gpu)
    C = torch.empty(M, N, device=gpu)
    ks = Kk.gemm(bf(A), M, False, bf(B), N, False, C, N, M, N, K, ksplit=8)
    assert ks == 8
    ref = bf(A).float().t() @ bf(B).float()
    assert rel_err(C, ref) < 2e-3
    # batched
    bs = 5
    X, Y = torch.randn(bs, 40, 72, device=gpu), torch.randn(bs, 72, 24, device=gpu)
    O = torch.empty(bs, 40, 24, device=gpu, dtype=torch.bfloat16)
    Kk.bmm(bf(X), bf(Y), O, False, False, False)
    assert rel_err(O, bf(X).float() @ bf(Y).float()) < 1e-2



@pytest.mark.parametrize("B,K,act,dx_acc", [(8192, 256, 12, False), (256, 64, 11, True), (1000, 128, 10, False),
                                            (37, 16, 12, True), (512, 4096, 11, False), (300, 2056, 12, True)])
def test_skinny_layer_backward(gpu, B, K, act, dx_acc):
    """out_features == 1 layer backward (DLRM click layer): d = act'(y) * dy, dX = d w, dW += x^T d,
    db += sum d -- rows processed four at a time with their loads issued first."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(7)
    x = torch.randn(B, K, device=gpu).to(torch.bfloat16)
    w = torch.randn(1, K, device=gpu).to(torch.bfloat16)
    pre = x.float() @ w.float().t()
    y = (torch.sigmoid(pre) if act == 12 else torch.relu(pre) if act == 11 else pre).to(torch.bfloat16)
    dy = torch.randn(B, 1, device=gpu).to(torch.bfloat16)
    yf, dyf = y.float(), dy.float()
    d = dyf * yf * (1 - yf) if act == 12 else dyf * (yf > 0) if act == 11 else dyf
    dx = torch.randn(B, K, device=gpu).to(torch.bfloat16)
    dx0 = dx.float().clone()
    dw = torch.zeros(K, device=gpu)
    db = torch.zeros(1, device=gpu)
    Kk.C().skinny_bwd(x, w, y, dy, dx, dx_acc, dw, db, act)
    ref_dx = d * w.float() + (dx0 if dx_acc else 0)
    assert rel_err(dx, ref_dx) < 1e-2
    assert rel_err(dw, (x.float() * d).sum(0)) < 1e-3
    assert rel_err(db, d.sum().reshape(1)) < 1e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,K", [(8192, 256), (1000, 128), (300, 2056)])
def test_skinny_backward_fused_below(gpu, dtype, B, K):
    """The layer below's ReLU backward fused into the skinny layer's dX (bact): dX = (x > 0) * d w."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(8)
    x = torch.relu(torch.randn(B, K, device=gpu)).to(dtype)
    w = torch.randn(1, K, device=gpu).to(dtype)
    y = torch.sigmoid(x.float() @ w.float().t()).to(dtype)
    dy = torch.randn(B, 1, device=gpu).to(dtype)
    d = dy.float() * y.float() * (1 - y.float())
    dx = torch.empty(B, K, device=gpu, dtype=dtype)
    dw = torch.zeros(K, device=gpu)
    db = torch.zeros(1, device=gpu)
    Kk.C().skinny_bwd(x, w, y, dy, dx, False, dw, db, 12, 11)
    tol = 1e-4 if dtype == torch.float32 else 1e-2
    assert rel_err(dx, (d * w.float()) * (x.float() > 0)) < tol
    assert rel_err(dw, (x.float() * d).sum(0)) < (1e-4 if dtype == torch.float32 else 1e-3)


def test_init_fill_matches_cpu(gpu):
    from flexmi.core.initializers import NormInitializer, UniformInitializer
    for init in [UniformInitializer(7, -0.5, 0.5), NormInitializer(9, 0.0, 2.0)]:
        dims = (300, 40)
        box = ((100, 220), (8, 40))
        cpu = torch.empty(120, 32)
        init.fill(dims, box, cpu)
        g = torch.empty(120, 32, device=gpu)
        init.fill(dims, box, g)
        assert torch.allclose(g.cpu(), cpu, atol=1e-5), type(init)


@pytest.mark.parametrize("bag,D,rows", [(1, 128, 100000), (3, 64, 50), (2, 16, 7), (1, 128, 3), (1, 128, 30), (1, 128, 100), (4, 24, 5), (1, 200, 9)])
def test_embedding_fwd_bwd(gpu, bag, D, rows):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(3)
    B = 1000
    W = torch.randn(rows, D, device=gpu)
    idx = torch.randint(0, rows, (B, bag), device=gpu)
    out = torch.empty(B, D, device=gpu, dtype=torch.bfloat16)
    Kk.embedding_forward(idx, W, out, 21)
    ref = W[idx].sum(1)
    assert rel_err(out, ref) < 1e-2
    # fused sparse SGD
    dy = torch.randn(B, D, device=gpu).to(torch.bfloat16)
    lr = torch.tensor([0.1], device=gpu)
    W2 = W.clone()
    Kk.embedding_backward_sgd(idx, dy, W2, lr, 21, {})
    upd = torch.zeros_like(W)
    upd.index_add_(0, idx.reshape(-1), dy.float().repeat_interleave(bag, 0))
    assert torch.allclose(W2, W - 0.1 * upd, atol=1e-4)
    # dense grad
    dW = torch.empty_like(W)
    Kk.embedding_backward_dense(idx, dy, dW, 21)
    assert torch.allclose(dW, upd, atol=1e-3)


@pytest.mark.parametrize("dy_dtype", [torch.float32, torch.bfloat16])
def test_embedding_small_tables_lds_atomics(gpu, dy_dtype):
    """The small-table backward (<= 160 rows: block-shared LDS copy, LDS float atomics, one global
    atomic per touched element and block) at the MLPerf batch on the 3 / 63 / 108 / 155-row sizes
    (and a bag of 2 with a row shard), fused SGD against a float64 index_add oracle."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(11)
    B = 8192
    for rows, bag, D in [(3, 1, 128), (63, 1, 128), (108, 1, 128), (155, 1, 128), (40, 2, 64)]:
        W = torch.randn(rows, D, device=gpu)
        idx = torch.randint(0, rows, (B, bag), device=gpu)
        dy = (torch.randn(B, D, device=gpu) * 1e-2).to(dy_dtype)
        lr = torch.tensor([0.05], device=gpu)
        W2 = W.clone()
        Kk.embedding_backward_sgd(idx, dy, W2, lr, 21, {})
        upd = torch.zeros(rows, D, dtype=torch.float64, device=gpu)
        upd.index_add_(0, idx.reshape(-1), dy.double().repeat_interleave(bag, 0))
        ref = W.double() - 0.05 * upd
        assert (W2.double() - ref).abs().max().item() < 2e-5 * (1 + ref.abs().max().item()), (rows, bag, D)


@pytest.mark.parametrize("F,D,self_i", [(27, 128, False), (9, 64, True), (4, 32, False)])
def test_dot_interaction(gpu, F, D, self_i):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(4)
    B = 300
    zs = [torch.randn(B, D, device=gpu).to(torch.bfloat16) for _ in range(F)]
    npairs = F * (F + 1) // 2 if self_i else F * (F - 1) // 2
    W = ((D + npairs + 15) // 16) * 16
    y = torch.empty(B, W, device=gpu, dtype=torch.bfloat16)
    Kk.dot_interaction_forward(zs, y, self_i)
    Z = torch.stack([z.float() for z in zs], 1)
    G = Z @ Z.transpose(1, 2)
    li, lj = [], []
    for i in range(F):
        for j in range(i + 1 if self_i else i):
            li.append(i)
            lj.append(j)
    ref = torch.zeros(B, W, device=gpu)
    ref[:, :D] = Z[:, 0]
    ref[:, D:D + npairs] = G[:, li, lj]
    assert rel_err(y, ref) < 1e-2
    # backward
    dy = torch.randn(B, W, device=gpu).to(torch.bfloat16)
    grads = [torch.empty(B, D, device=gpu, dtype=torch.bfloat16) for _ in range(F)]
    Kk.dot_interaction_backward(zs, dy, grads, [False] * F, self_i)
    dG = torch.zeros(B, F, F, device=gpu)
    dG[:, li, lj] = dy[:, D:D + npairs].float()
    dZ = (dG + dG.transpose(1, 2)) @ Z
    dZ[:, 0] += dy[:, :D].float()
    for i in range(F):
        assert rel_err(grads[i], dZ[:, i]) < 2e-2, i


def test_sgd_adam(gpu):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(5)
    n = 10007
    W, G, V = torch.randn(n, device=gpu), torch.randn(n, device=gpu), torch.randn(n, device=gpu)
    Wc = torch.empty(n, device=gpu, dtype=torch.bfloat16)
    W0, V0 = W.clone(), V.clone()
    lr = torch.tensor([0.05], device=gpu)
    Kk.sgd_update(W, G, V, Wc, lr, 1e-4, 0.9, True)
    g = G + 1e-4 * W0
    v = 0.9 * V0 + g
    g = g + 0.9 * v
    assert torch.allclose(W, W0 - 0.05 * g, atol=1e-5) and torch.allclose(V, v, atol=1e-5)
    assert torch.allclose(Wc.float(), W, atol=2e-2)
    M_, V_ = torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
    W1 = W.clone()
    Kk.adam_update(W, G, M_, V_, None, torch.tensor([0.01], device=gpu), 0.9, 0.999, 0.0, 1e-8)
    m = 0.1 * G
    vv = 0.001 * G * G
    assert torch.allclose(W, W1 - 0.01 * m / (vv.sqrt() + 1e-8), atol=1e-4)


@pytest.mark.parametrize("loss,C", [(54, 1), (52, 1), (51, 10), (50, 7)])
def test_loss_metrics(gpu, loss, C):
    from flexmi.core.loss_metrics import loss_and_metrics_torch
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(6)
    B = 777
    if C == 1:
        p = torch.rand(B, 1, device=gpu)
        lab = torch.randint(0, 2, (B, 1), device=gpu).float()
    else:
        p = torch.softmax(torch.randn(B, C, device=gpu), -1)
        if loss == 51:
            lab = torch.randint(0, C, (B, 1), device=gpu, dtype=torch.int32)
        else:
            lab = torch.nn.functional.one_hot(torch.randint(0, C, (B,), device=gpu), C).float()
    g = torch.empty(B, C, device=gpu)
    acc = torch.zeros(8, device=gpu)
    Kk.loss_forward_backward(loss, p, lab, g, 1.0 / B, acc, 63)
    gr = torch.empty(B, C)
    accr = torch.zeros(8)
    loss_and_metrics_torch(loss, p.cpu(), lab.cpu(), gr, 1.0 / B, accr, 63)
    assert torch.allclose(g.cpu(), gr, atol=1e-6)
    for s in [0, 1, 4, 6, 7]:
        assert abs(acc[s].item() - accr[s].item()) <= 1e-3 * max(1.0, abs(accr[s].item())), (s, acc, accr)


def test_elementwise_and_movement(gpu):
    from flexmi.ops import _kernels as Kk
    from flexmi.ops.elementwise import unary_bwd_torch, unary_fwd_torch
    torch.manual_seed(7)
    x = torch.randn(64, 33, device=gpu)
    for code in range(5):
        y = torch.empty_like(x)
        Kk.unary_forward(code, x, y)
        assert torch.allclose(y, unary_fwd_torch(code, x), atol=1e-5, rtol=1e-4)
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        Kk.unary_backward(code, x, y, dy, dx, False)
        assert torch.allclose(dx, unary_bwd_torch(code, x, y, dy), atol=1e-5, rtol=1e-4)
    a, b = torch.randn(1000, device=gpu), torch.rand(1000, device=gpu) + 0.5
    for code, f in enumerate([torch.add, torch.sub, torch.mul, torch.div]):
        y = torch.empty_like(a)
        Kk.binary_forward(code, a, b, y)
        assert torch.allclose(y, f(a, b), atol=1e-5)
    # concat / split
    xs = [torch.randn(8, k, 5, device=gpu) for k in (3, 4, 2)]
    y = torch.empty(8, 9, 5, device=gpu)
    Kk.concat_forward(xs, y, 1)
    assert torch.equal(y, torch.cat(xs, 1))
    gs = [torch.empty_like(t) for t in xs]
    Kk.concat_backward(y, gs, [False] * 3, 1)
    for gg, t in zip(gs, xs):
        assert torch.equal(gg, t)
    # permute / reverse / softmax
    t = torch.randn(4, 5, 6, device=gpu)
    o = torch.empty(6, 4, 5, device=gpu)
    Kk.permute(t, o, [2, 0, 1], False)
    assert torch.equal(o, t.permute(2, 0, 1))
    r = torch.empty_like(t)
    Kk.reverse(t, r, 1, False)
    assert torch.equal(r, torch.flip(t, [1]))
    s = torch.empty(17, 300, device=gpu)
    xx = torch.randn(17, 300, device=gpu)
    Kk.softmax_forward(xx, s)
    assert torch.allclose(s, torch.softmax(xx, -1), atol=1e-6)


@pytest.mark.parametrize("B,N,act", [(1000, 260, 11), (8192, 128, 11), (8192, 1024, 12), (256, 1024, 11), (37, 20, 13),
                                     (4096, 64, 10)])
def test_act_bwd_bias(gpu, B, N, act):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(8)
    pre = torch.randn(B, N, device=gpu)
    y = (torch.relu(pre) if act == 11 else torch.sigmoid(pre) if act == 12 else torch.tanh(pre) if act == 13
         else pre).to(torch.bfloat16)
    dy = torch.randn(B, N, device=gpu).to(torch.bfloat16)
    dpre = torch.empty(B, N, device=gpu, dtype=torch.bfloat16)
    db = torch.zeros(N, device=gpu)
    Kk.C().act_bwd_bias(y, dy, dpre, db, B, N, act)
    yf, g = y.float(), dy.float()
    ref = {11: g * (yf > 0), 12: g * yf * (1 - yf), 13: g * (1 - yf * yf), 10: g}[act]
    assert rel_err(dpre, ref) < 1e-2
    assert torch.allclose(db, ref.sum(0), atol=2e-2, rtol=1e-3)


@pytest.mark.parametrize("N,C,H,W,K,R,S,st,pads", [
    (2, 3, 19, 19, 16, 11, 11, 4, (2, 2, 2, 2)),      # AlexNet conv1-like (CRS=363: padded columns)
    (3, 16, 9, 9, 24, 3, 3, 1, (1, 1, 1, 1)),
    (2, 8, 8, 8, 16, 1, 1, 1, (0, 0, 0, 0)),
    (2, 8, 10, 7, 8, 3, 3, 2, (0, 1, 1, 0)),           # asymmetric (halo-shard) pads
])
def test_conv2d_hip(gpu, N, C, H, W, K, R, S, st, pads):
    import torch.nn.functional as F
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(5)
    x = torch.randn(N, C, H, W, device=gpu).bfloat16()
    w = (torch.randn(K, C, R, S, device=gpu) * 0.1).bfloat16()
    b = torch.randn(K, device=gpu)
    xp = F.pad(x.float(), (pads[2], pads[3], pads[0], pads[1]))
    ref = torch.relu(F.conv2d(xp, w.float(), b, st))
    y = torch.empty(ref.shape, device=gpu, dtype=torch.bfloat16)
    Kk.conv2d_forward(x, w, b, y, (st, st), pads, 11, 1)
    assert rel_err(y, ref) < 2e-2
    dy = torch.randn(ref.shape, device=gpu).bfloat16()
    dx = torch.empty_like(x)
    dw = torch.zeros(K, C, R, S, device=gpu)
    db = torch.zeros(K, device=gpu)
    Kk.conv2d_backward(x, w, y, dy, dx, dw, db, (st, st), pads, 11, 1, False)
    g = dy.float() * (y.float() > 0)
    xr = xp.clone().requires_grad_(True)
    wr = w.float().clone().requires_grad_(True)
    out = F.conv2d(xr, wr, None, st)
    gx, gw = torch.autograd.grad(out, [xr, wr], g)
    gx = gx[:, :, pads[0]: pads[0] + H, pads[2]: pads[2] + W]
    assert rel_err(dw, gw) < 2e-2
    assert rel_err(db, g.sum((0, 2, 3))) < 2e-2
    assert rel_err(dx, gx) < 2e-2


@pytest.mark.parametrize("saved", [False, True], ids=["argmax-in-bwd", "argmax-from-fwd"])
@pytest.mark.parametrize("kind", [30, 31])
def test_pool2d_hip(gpu, kind, saved):
    import torch.nn.functional as F
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(6)
    x = torch.randn(2, 5, 13, 11, device=gpu).bfloat16()
    k, st, pads = (3, 3), (2, 2), (1, 1, 1, 1)
    xf = x.float().requires_grad_(True)
    if kind == 30:
        ref = F.max_pool2d(F.pad(xf, (1, 1, 1, 1), value=float("-inf")), k, st)
    else:
        s_ = F.avg_pool2d(F.pad(xf, (1, 1, 1, 1)), k, st, divisor_override=1)
        cnt = F.avg_pool2d(F.pad(torch.ones_like(xf[:1, :1]), (1, 1, 1, 1)), k, st, divisor_override=1)
        ref = s_ / cnt
    y = torch.empty(ref.shape, device=gpu, dtype=torch.bfloat16)
    st_ = {} if saved else None
    Kk.pool2d_forward(x, y, k, st, pads, kind, 10, st_)
    assert rel_err(y, ref) < 1e-2
    dy = torch.randn(ref.shape, device=gpu).bfloat16()
    gx, = torch.autograd.grad(ref, [xf], dy.float())
    dx = torch.empty_like(x)
    Kk.pool2d_backward(x, y, dy, dx, k, st, pads, kind, 10, False, st_)
    assert rel_err(dx, gx) < 2e-2


def test_batchnorm_hip(gpu):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(7)
    x = torch.randn(4, 6, 7, 5, device=gpu).bfloat16()
    gam = torch.rand(6, device=gpu) + 0.5
    bet = torch.randn(6, device=gpu)
    xf = x.float().requires_grad_(True)
    mean = xf.mean((0, 2, 3), keepdim=True)
    var = xf.var((0, 2, 3), unbiased=False, keepdim=True)
    ref = torch.relu((xf - mean) / torch.sqrt(var + 1e-5) * gam[None, :, None, None] + bet[None, :, None, None])
    y = torch.empty_like(x)
    saved = {}
    Kk.batchnorm_forward(x, gam, bet, y, True, 1e-5, saved)
    assert rel_err(y, ref) < 1e-2
    dy = torch.randn_like(ref).bfloat16()
    gx, = torch.autograd.grad(ref, [xf], dy.float())
    dx = torch.empty_like(x)
    dg = torch.empty(6, device=gpu)
    dbt = torch.empty(6, device=gpu)
    Kk.batchnorm_backward(x, gam, y, dy, dx, dg, dbt, True, 1e-5, saved, False)
    g = dy.float() * (ref > 0)
    xhat = (xf - mean) / torch.sqrt(var + 1e-5)
    assert rel_err(dbt, g.sum((0, 2, 3))) < 2e-2
    assert rel_err(dg, (g * xhat).sum((0, 2, 3))) < 2e-2
    assert rel_err(dx, gx) < 3e-2


@pytest.mark.parametrize("idx_dtype", [torch.int64, torch.int32])
def test_embedding_owner_computes_sgd(gpu, idx_dtype):
    """Owner-computes sparse SGD for mostly-unique tables (claim CAS -> duplicate atomics ->
    owner 16-B RMW): matches the dense reference over two consecutive steps (the claim slots
    and duplicate counters must be restored after every step), mixed with atomic-path tables."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(5)
    B = 1000
    specs = [(100000, 1, 128), (1500, 1, 128), (5000, 2, 64), (40, 1, 128), (3, 1, 128)]   # rows, bag, D
    tables, idxs, claim, refs = [], [], [], []
    for rows, bag, D in specs:
        W = torch.randn(rows, D, device=gpu)
        tables.append(W)
        refs.append(W.clone())
        idxs.append(torch.randint(0, rows, (B, bag), device=gpu, dtype=idx_dtype))
        if rows > B * bag:
            claim += [torch.full((rows,), -1, dtype=torch.int32, device=gpu),
                      torch.empty(B * bag, dtype=torch.int32, device=gpu), torch.zeros(1, dtype=torch.int32, device=gpu)]
        else:
            claim += [None, None, None]
    lr = torch.tensor([0.05], device=gpu)
    for step in range(2):
        dys = [torch.randn(B, D, device=gpu).to(torch.bfloat16) for _, _, D in specs]
        Kk.C().embedding_bwd_multi(tables, idxs, dys, [d.stride(0) for d in dys], [1.0] * len(specs), lr, claim)
        for k, ((rows, bag, D), W) in enumerate(zip(specs, refs)):
            upd = torch.zeros_like(W)
            upd.index_add_(0, idxs[k].reshape(-1).long(), dys[k].float().repeat_interleave(bag, 0))
            W -= 0.05 * upd
        torch.cuda.synchronize()
        for k in range(len(specs)):
            assert torch.allclose(tables[k], refs[k], atol=1e-4), (step, specs[k])
        for k in range(0, len(claim), 3):
            if claim[k] is not None:
                assert int((claim[k] != -1).sum()) == 0 and int(claim[k + 2].item()) == 0, "claims not released"


@pytest.mark.parametrize("dy_dtype", [torch.float32, torch.bfloat16])
def test_embedding_owner_computes_duplicate_heavy(gpu, dy_dtype):
    """the DEFAULT claim rule (Embedding.CLAIM_RATIO = 0.2) puts owner-computes on
    tables with 0.2 x lookups < rows < lookups -- the 2208 / 7420-row MLPerf tables at B = 8192,
    where most lookups are duplicates and the dup-atomic path does most of the work.  Two steps
    against the dense reference, incl. the slot / duplicate-counter release."""
    from flexmi.ops import _kernels as Kk
    from flexmi.ops.embedding import Embedding
    torch.manual_seed(11)
    B = 8192
    specs = [(2208, 1, 128), (7420, 1, 128), (5000, 2, 64)]   # rows, bag, D: all in (0.2, 1) x lookups
    tables, idxs, claim, refs = [], [], [], []
    for rows, bag, D in specs:
        assert Embedding.CLAIM_RATIO * B * bag < rows < B * bag
        W = torch.randn(rows, D, device=gpu)
        tables.append(W)
        refs.append(W.clone())
        idxs.append(torch.randint(0, rows, (B, bag), device=gpu, dtype=torch.int64))
        claim += [torch.full((rows,), -1, dtype=torch.int32, device=gpu),
                  torch.empty(B * bag, dtype=torch.int32, device=gpu), torch.zeros(1, dtype=torch.int32, device=gpu)]
    lr = torch.tensor([0.05], device=gpu)
    for step in range(2):
        dys = [torch.randn(B, D, device=gpu).to(dy_dtype) for _, _, D in specs]
        Kk.C().embedding_bwd_multi(tables, idxs, dys, [d.stride(0) for d in dys], [1.0] * len(specs), lr, claim)
        for k, ((rows, bag, D), W) in enumerate(zip(specs, refs)):
            upd = torch.zeros_like(W)
            upd.index_add_(0, idxs[k].reshape(-1).long(), dys[k].float().repeat_interleave(bag, 0))
            W -= 0.05 * upd
        torch.cuda.synchronize()
        for k in range(len(specs)):
            assert torch.allclose(tables[k], refs[k], atol=2e-4), (step, specs[k])
        for k in range(0, len(claim), 3):
            assert int((claim[k] != -1).sum()) == 0 and int(claim[k + 2].item()) == 0, "claims not released"


@pytest.mark.parametrize("dy_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("idx_dtype", [torch.int64, torch.int32])
def test_embedding_count_update_sgd(gpu, idx_dtype, dy_dtype):
    """Count / update sparse SGD (FM_EMB_BWD=count: slot = lookups - 1, plain RMW for single-lookup
    rows, atomics for repeated rows) on every table above 16 rows, incl. a row shard, over three
    steps: matches the dense reference and leaves every slot free (-1) after each step."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(9)
    B = 2000
    specs = [(400000, 1, 128, 0), (1500, 1, 128, 0), (5000, 2, 64, 0), (40, 1, 128, 0), (3, 1, 128, 0),
             (30000, 1, 128, 10000)]    # rows, bag, D, first row held (row shard of a 40000-row table)
    tables, idxs, claim, refs, los = [], [], [], [], []
    for rows, bag, D, lo in specs:
        W = torch.randn(rows, D, device=gpu)
        tables.append(W)
        refs.append(W.clone())
        idxs.append(torch.randint(0, rows + lo, (B, bag), device=gpu, dtype=idx_dtype))
        los.append(lo)
        if rows > 16:
            claim += [torch.full((rows,), -1, dtype=torch.int32, device=gpu),
                      torch.empty(B * bag, dtype=torch.int32, device=gpu), torch.zeros(1, dtype=torch.int32, device=gpu)]
        else:
            claim += [None, None, None]
    lr = torch.tensor([0.05], device=gpu)
    Kk.C().embedding_set_bwd_mode(True)
    try:
        for step in range(3):
            dys = [torch.randn(B, D, device=gpu).to(dy_dtype) for _, _, D, _ in specs]
            Kk.C().embedding_bwd_multi(tables, idxs, dys, [d.stride(0) for d in dys], [1.0] * len(specs), lr, claim,
                                       los)
            for k, ((rows, bag, D, lo), W) in enumerate(zip(specs, refs)):
                flat = idxs[k].reshape(-1).long() - lo
                keep = (flat >= 0) & (flat < rows)
                upd = torch.zeros_like(W)
                upd.index_add_(0, flat[keep], dys[k].float().repeat_interleave(bag, 0)[keep])
                W -= 0.05 * upd
            torch.cuda.synchronize()
            for k in range(len(specs)):
                assert torch.allclose(tables[k], refs[k], atol=1e-4), (step, specs[k])
            for k in range(0, len(claim), 3):
                if claim[k] is not None:
                    assert int((claim[k] != -1).sum()) == 0, ("slots not freed", step, k // 3)
    finally:
        Kk.C().embedding_set_bwd_mode(False)


@pytest.mark.parametrize("dy_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("idx_dtype", [torch.int64, torch.int32])
def test_embedding_small_and_mid_tables(gpu, idx_dtype, dy_dtype):
    """The MLPerf set's non-claimed table sizes (3 .. 7420 rows at B = 8192) through the atomic /
    tiny kernels, plus D = 256 / 200 / 24 columns, a bag of 3 and a row shard, over two steps, for
    the fused sparse SGD and the dense gradient, against a float64 oracle."""
    _embedding_small_tables_case(gpu, idx_dtype, dy_dtype)


def _embedding_small_tables_case(gpu, idx_dtype, dy_dtype):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(12)
    B = 8192
    specs = [(7420, 1, 128, 0), (976, 1, 128, 0), (155, 1, 128, 0), (36, 1, 128, 0), (3, 1, 128, 0),
             (300, 3, 256, 0), (90, 1, 200, 0), (500, 2, 24, 0), (1000, 1, 128, 400)]   # rows, bag, D, lo
    tables, idxs, refs = [], [], []
    for rows, bag, D, lo in specs:
        W = torch.randn(rows, D, device=gpu)
        tables.append(W)
        refs.append(W.double())
        idxs.append(torch.randint(0, rows + lo, (B, bag), device=gpu, dtype=idx_dtype))
    lr = torch.tensor([0.05], device=gpu)
    none = [None] * (3 * len(specs))
    for step in range(2):
        dys = [torch.randn(B, D, device=gpu).to(dy_dtype) for _, _, D, _ in specs]
        Kk.C().embedding_bwd_multi(tables, idxs, dys, [d.stride(0) for d in dys], [1.0] * len(specs), lr, none,
                                   [s[3] for s in specs])
        grads = [torch.zeros_like(W) for W in tables]
        Kk.C().embedding_bwd_multi(grads, idxs, dys, [d.stride(0) for d in dys], [0.5] * len(specs), None, None,
                                   [s[3] for s in specs])
        torch.cuda.synchronize()
        for k, (rows, bag, D, lo) in enumerate(specs):
            flat = idxs[k].reshape(-1).long() - lo
            keep = (flat >= 0) & (flat < rows)
            upd = torch.zeros(rows, D, device=gpu, dtype=torch.float64)
            upd.index_add_(0, flat[keep], dys[k].double().repeat_interleave(bag, 0)[keep])
            refs[k] -= 0.05 * upd
            assert torch.allclose(tables[k].double(), refs[k], atol=2e-4), (step, specs[k], "sgd")
            assert torch.allclose(grads[k].double(), 0.5 * upd, atol=2e-3, rtol=1e-5), (step, specs[k], "dense")


@pytest.mark.parametrize("idx_dtype", [torch.int64, torch.int32])
def test_embedding_row_shards(gpu, idx_dtype):
    """Row-sharded tables (a shard holds rows [lo, lo+rows)): forward sums only the lookups the
    shard holds, and every backward path (owner-computes, atomics, tiny-table LDS, dense grad)
    touches only them -- the shards of a table together equal the unsharded table."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(6)
    B = 1000
    specs = [(100000, 1, 128), (2000, 2, 64), (12, 1, 128)]   # rows, bag, D
    lr = torch.tensor([0.05], device=gpu)
    for rows, bag, D in specs:
        W = torch.randn(rows, D, device=gpu)
        idx = torch.randint(0, rows, (B, bag), device=gpu, dtype=idx_dtype)
        dy = torch.randn(B, D, device=gpu).to(torch.bfloat16)
        cut = [0, rows // 3, rows]
        shards = [W[cut[k]:cut[k + 1]].clone() for k in range(2)]
        # forward: partial sums add up to the full lookup
        outs = [torch.empty(B, D, device=gpu) for _ in range(2)]
        Kk.C().embedding_fwd_multi(shards, [idx, idx], outs, [D, D], [1.0, 1.0], [cut[0], cut[1]])
        ref = W[idx.long()].sum(1)
        assert torch.allclose(outs[0] + outs[1], ref, atol=1e-4), (rows, "fwd")
        # fused sparse SGD (owner-computes for the big table, atomics / tiny otherwise)
        claim = []
        for k in range(2):
            r = cut[k + 1] - cut[k]
            if r > B * bag:
                claim += [torch.full((r,), -1, dtype=torch.int32, device=gpu),
                          torch.empty(B * bag, dtype=torch.int32, device=gpu), torch.zeros(1, dtype=torch.int32, device=gpu)]
            else:
                claim += [None, None, None]
        Kk.C().embedding_bwd_multi(shards, [idx, idx], [dy, dy], [D, D], [1.0, 1.0], lr, claim, [cut[0], cut[1]])
        upd = torch.zeros_like(W)
        upd.index_add_(0, idx.reshape(-1).long(), dy.float().repeat_interleave(bag, 0))
        Wn = W - 0.05 * upd
        torch.cuda.synchronize()
        assert torch.allclose(torch.cat(shards), Wn, atol=1e-4), (rows, "sgd")
        # dense gradient
        grads = [torch.zeros_like(s) for s in shards]
        Kk.C().embedding_bwd_multi(grads, [idx, idx], [dy, dy], [D, D], [1.0, 1.0], None, None, [cut[0], cut[1]])
        assert torch.allclose(torch.cat(grads), upd, atol=1e-3), (rows, "dense")


@pytest.mark.parametrize("B,bag,D", [(256, 100, 64), (37, 20, 128), (5, 16, 48), (300, 33, 256)])
@pytest.mark.parametrize("out_dt", [torch.float32, torch.bfloat16])
def test_embedding_fwd_long_bag_split(gpu, B, bag, D, out_dt):
    """Long bags on small batches (summit_large: 256 x 100) run the bag-split forward
    (embedding.hip fm_emb_fwd_split): several tables, row shards, avg scale, vs a float64 oracle."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(B + bag)
    rows = 5000
    Ws = [torch.randn(rows, D, device=gpu) for _ in range(3)]
    idxs = [torch.randint(0, rows, (B, bag), device=gpu) for _ in range(3)]
    lo = [0, 0, 1000]            # third table: a row shard holding [1000, 6000)
    scales = [1.0, 1.0 / bag, 1.0]
    outs = [torch.empty(B, D, device=gpu, dtype=out_dt) for _ in range(3)]
    Kk.C().embedding_fwd_multi(Ws, idxs, outs, [D] * 3, scales, lo)
    torch.cuda.synchronize()
    for W, idx, l, sc, o in zip(Ws, idxs, lo, scales, outs):
        r = idx.long() - l
        ok = (r >= 0) & (r < rows)
        ref = (W.double()[r.clamp(0, rows - 1)] * ok[..., None]).sum(1) * sc
        tol = 1e-5 if out_dt == torch.float32 else 1e-2
        assert rel_err(o, ref) < tol, (B, bag, D)


