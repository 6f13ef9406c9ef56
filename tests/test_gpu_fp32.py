"""Reference-precision (fp32) HIP path: every fp32 kernel vs a float64 PyTorch oracle at <= 1e-4
relative error, and whole models on the GPU in fp32 vs the fp32 CPU executor (reference
``src/ops/tests/test_harness.py:78-94``: golden forward + one SGD step at ``assert_allclose``
tolerances).  The reference computes in fp32 everywhere (cublasSgemm, cuDNN FLOAT)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 1e-4          # max-normalised relative error bound of every fp32 kernel test


def rel_err(a, b):
    a = a.double()
    b = b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


# ---------------------------------------------------------------- GEMM
@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 200, 130), (1024, 512, 256), (8192, 64, 16),
                                   (4096, 1024, 1024), (77, 33, 13), (2048, 479, 512), (8192, 1024, 480),
                                   (1000, 1020, 8192), (8192, 96, 256)])
def test_gemm_f32_orientations(gpu, a_k, b_k, M, N, K):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(0)
    A = torch.randn(M, K, device=gpu)
    B = torch.randn(K, N, device=gpu)
    Ag = A if a_k else A.t().contiguous()
    Bg = B.t().contiguous() if b_k else B
    C = torch.empty(M, N, device=gpu)
    Kk.gemm(Ag, K if a_k else M, a_k, Bg, K if b_k else N, b_k, C, N, M, N, K)
    ref = A.double() @ B.double()
    assert rel_err(C, ref) < TOL, (a_k, b_k, M, N, K, rel_err(C, ref))


def test_gemm_f32_epilogue_bias_act_beta(gpu):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(1)
    M, N, K = 1000, 384, 192
    A, W, b = torch.randn(M, K, device=gpu), torch.randn(N, K, device=gpu), torch.randn(N, device=gpu)
    for act, fn in ((11, torch.relu), (12, torch.sigmoid), (13, torch.tanh)):
        C = torch.randn(M, N, device=gpu)
        C0 = C.double().clone()
        Kk.gemm(A, K, True, W, K, True, C, N, M, N, K, bias=b, act=act, beta=True)
        ref = fn(A.double() @ W.double().t() + b.double()) + C0
        assert rel_err(C, ref) < TOL, act


@pytest.mark.parametrize("ks", [2, 4, 8, 16, 64])      # >= 16: the slab-parallel reduce
def test_gemm_f32_splitk_and_batch(gpu, ks):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(2)
    M, N, K = 256, 128, 8192
    A, B = torch.randn(K, M, device=gpu), torch.randn(K, N, device=gpu)
    bias = torch.randn(N, device=gpu)
    C = torch.empty(M, N, device=gpu)
    assert Kk.gemm(A, M, False, B, N, False, C, N, M, N, K, bias=bias, ksplit=ks) == ks
    assert rel_err(C, A.double().t() @ B.double() + bias.double()) < TOL
    bs = 5
    X, Y = torch.randn(bs, 40, 72, device=gpu), torch.randn(bs, 72, 24, device=gpu)
    O = torch.empty(bs, 40, 24, device=gpu)
    Kk.bmm(X, Y, O, False, False, False)
    assert rel_err(O, X.double() @ Y.double()) < TOL
    Kk.bmm(X, O, Y.new_empty(bs, 72, 24), True, False, False)    # transposed A operand


@pytest.mark.parametrize("M,K,N", [(2048, 512, 256), (8192, 1024, 1024), (8192, 480, 1024)])
def test_gemm_f32_fused_backward_epilogue(gpu, M, K, N):
    """dX GEMM with the activation backward of the layer below (y fp32) and its bias-gradient
    column sums fused; dW GEMM with the bias gradient as row sums of the staged MN-contiguous A."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(3)
    _fused_backward_epilogue(Kk, gpu, M, K, N)


def _fused_backward_epilogue(Kk, gpu, M, K, N):     # dpre [M,N], W [N,K] -> dX [M,K]
    dpre = torch.randn(M, N, device=gpu)
    W = torch.randn(N, K, device=gpu)
    yb = torch.randn(M, K, device=gpu).relu()
    dx = torch.empty(M, K, device=gpu)
    colsum = torch.zeros(K, device=gpu)
    Kk.gemm(dpre, N, True, W, K, False, dx, K, M, K, N, act_y=yb, bwd_act=11, colsum=colsum)
    ref = (dpre.double() @ W.double()) * (yb.double() > 0)
    assert rel_err(dx, ref) < TOL
    assert rel_err(colsum, ref.sum(0)) < TOL
    x = torch.randn(M, K, device=gpu)
    dw = torch.randn(N, K, device=gpu)
    dw0 = dw.double().clone()
    db = torch.zeros(N, device=gpu)
    Kk.gemm(dpre, N, False, x, K, False, dw, K, N, K, M, beta=True, rowsum_a=db)
    assert rel_err(dw, dw0 + dpre.double().t() @ x.double()) < TOL
    assert rel_err(db, dpre.double().sum(0)) < TOL


# ---------------------------------------------------------------- skinny / act-bwd / interaction
@pytest.mark.parametrize("B,K,act,dx_acc", [(8192, 256, 12, False), (256, 64, 11, True), (37, 16, 10, True),
                                            (512, 4096, 11, False), (300, 1036, 12, True)])
def test_skinny_f32(gpu, B, K, act, dx_acc):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(7)
    x, w, b = torch.randn(B, K, device=gpu), torch.randn(1, K, device=gpu), torch.randn(1, device=gpu)
    y = torch.empty(B, 1, device=gpu)
    Kk.linear_forward(x, w, b, act, y)
    pre = x.double() @ w.double().t() + b.double()
    yr = torch.sigmoid(pre) if act == 12 else torch.relu(pre) if act == 11 else pre
    assert rel_err(y, yr) < TOL
    dy = torch.randn(B, 1, device=gpu)
    yd = y.double()
    d = dy.double() * yd * (1 - yd) if act == 12 else dy.double() * (yd > 0) if act == 11 else dy.double()
    dx = torch.randn(B, K, device=gpu)
    dx0 = dx.double().clone()
    dw, db = torch.zeros(1, K, device=gpu), torch.zeros(1, device=gpu)
    Kk.linear_backward(x, w, y, dy, act, dx, dx_acc, dw, db, {})
    assert rel_err(dx, d @ w.double() + (dx0 if dx_acc else 0)) < TOL
    assert rel_err(dw, d.t() @ x.double()) < TOL
    assert rel_err(db, d.sum(0)) < TOL


def test_act_bwd_bias_f32(gpu):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(8)
    for (B, N) in ((8192, 1024), (300, 77)):
        y = torch.rand(B, N, device=gpu)
        dy = torch.randn(B, N, device=gpu)
        dpre = torch.empty(B, N, device=gpu)
        db = torch.zeros(N, device=gpu)
        Kk.C().act_bwd_bias(y, dy, dpre, db, B, N, 12)
        ref = dy.double() * y.double() * (1 - y.double())
        assert rel_err(dpre, ref) < TOL
        assert rel_err(db, ref.sum(0)) < TOL


@pytest.mark.parametrize("F,D,selfi", [(27, 128, False), (27, 16, False), (9, 64, True), (5, 24, False), (32, 32, False),
                                       (28, 128, True), (2, 64, False), (27, 32, True)])
def test_dot_interaction_f32(gpu, F, D, selfi):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(9)
    B = 1000
    zs = [torch.randn(B, D, device=gpu) for _ in range(F)]
    npairs = F * (F + 1) // 2 if selfi else F * (F - 1) // 2
    W = (D + npairs + 15) // 16 * 16
    y = torch.full((B, W), 7.0, device=gpu)
    Kk.dot_interaction_forward(zs, y, selfi)
    Z = torch.stack([z.double() for z in zs], 1)
    G = Z @ Z.transpose(1, 2)
    li, lj = zip(*[(i, j) for i in range(F) for j in range(i + (1 if selfi else 0))])
    ref = torch.zeros(B, W, dtype=torch.float64, device=gpu)
    ref[:, :D] = Z[:, 0]
    ref[:, D:D + npairs] = G[:, li, lj]
    assert rel_err(y, ref) < TOL
    dy = torch.randn(B, W, device=gpu)
    dz = [torch.randn(B, D, device=gpu) for _ in range(F)]
    old = [g.double().clone() for g in dz]
    accs = [i % 2 == 1 for i in range(F)]
    Kk.dot_interaction_backward(zs, dy, dz, accs, selfi)
    dG = torch.zeros(B, F, F, dtype=torch.float64, device=gpu)
    dG[:, li, lj] = dy[:, D:D + npairs].double()
    dZ = (dG + dG.transpose(1, 2)) @ Z
    dZ[:, 0] += dy[:, :D].double()
    for i in range(F):
        exp = dZ[:, i] + (old[i] if accs[i] else 0)
        assert rel_err(dz[i], exp) < TOL, i


@pytest.mark.parametrize("F,D,selfi", [(27, 128, False), (9, 64, True), (32, 32, False), (28, 128, True)])
def test_dot_interaction_f32_split_forward(gpu, monkeypatch, F, D, selfi):
    """fp32 interaction forward with the Gram on the bf16 matrix cores through the exact
    three-way split (the only fp32 forward form), incl. operands spanning many binades, vs float64."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(19)
    B = 777
    zs = [torch.randn(B, D, device=gpu) * torch.exp2(torch.randint(-12, 12, (B, D), device=gpu).float())
          for _ in range(F)]
    npairs = F * (F + 1) // 2 if selfi else F * (F - 1) // 2
    W = (D + npairs + 15) // 16 * 16
    y = torch.full((B, W), 7.0, device=gpu)
    Kk.dot_interaction_forward(zs, y, selfi)
    Z = torch.stack([z.double() for z in zs], 1)
    G = Z @ Z.transpose(1, 2)
    li, lj = zip(*[(i, j) for i in range(F) for j in range(i + (1 if selfi else 0))])
    ref = torch.zeros(B, W, dtype=torch.float64, device=gpu)
    ref[:, :D] = Z[:, 0]
    ref[:, D:D + npairs] = G[:, li, lj]
    # per-element error against the magnitude the fp32 product sums carry (|Z||Z|^T)
    A = Z.abs() @ Z.abs().transpose(1, 2)
    scale = torch.zeros_like(ref)
    scale[:, :D] = Z[:, 0].abs()
    scale[:, D:D + npairs] = A[:, li, lj]
    err = ((y.double() - ref).abs() / scale.clamp_min(1e-30))[:, :D + npairs].max().item()
    assert err < 1e-5, err


@pytest.mark.parametrize("F,D,selfi", [(27, 128, False), (27, 64, False), (9, 24, True), (5, 128, True)])
def test_dot_interaction_f32_act0(gpu, F, D, selfi):
    """act0: the bottom MLP's ReLU backward applied to feature 0's gradient inside the interaction
    backward (fast and fallback kernels), vs a float64 oracle."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(10)
    B = 1000
    zs = [torch.randn(B, D, device=gpu) for _ in range(F)]
    zs[0] = torch.relu(zs[0])                          # a ReLU output: about half the entries 0
    npairs = F * (F + 1) // 2 if selfi else F * (F - 1) // 2
    W = (D + npairs + 15) // 16 * 16
    Z = torch.stack([z.double() for z in zs], 1)
    li, lj = zip(*[(i, j) for i in range(F) for j in range(i + (1 if selfi else 0))])
    dy = torch.randn(B, W, device=gpu)
    dz = [torch.empty(B, D, device=gpu) for _ in range(F)]
    Kk.dot_interaction_backward(zs, dy, dz, [False] * F, selfi, act0=11)
    dG = torch.zeros(B, F, F, dtype=torch.float64, device=gpu)
    dG[:, li, lj] = dy[:, D:D + npairs].double()
    dZ = (dG + dG.transpose(1, 2)) @ Z
    dZ[:, 0] += dy[:, :D].double()
    dZ[:, 0] *= (Z[:, 0] > 0).double()
    for i in range(F):
        assert rel_err(dz[i], dZ[:, i]) < TOL, i


def _dlrm_run(dev, dcfg, B, steps, seed=0, graph=False, lr=0.1):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer, LossType, MetricsType
    from flexmi.models.dlrm import build_dlrm
    rng = np.random.RandomState(seed)
    cfg = FFConfig()
    cfg.batchSize = B
    cfg.device = dev
    cfg.compute_dtype = "fp32"
    cfg.seed = 5
    m = FFModel(cfg)
    d, s, p = build_dlrm(m, dcfg)
    m.compile(SGDOptimizer(m, lr), LossType.LOSS_BINARY_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    batches = []
    for _ in range(steps):
        dd = np.zeros((B, d.dims[1]), np.float32)
        dd[:, :13] = rng.rand(B, 13)
        # skewed indices: hot rows repeat (atomic / duplicate paths), tails stay mostly unique
        sp = [np.minimum((rng.zipf(1.2, (B, dcfg.embedding_bag_size)) - 1), r - 1).astype(np.int64)
              if r > 64 else rng.randint(0, r, (B, dcfg.embedding_bag_size)).astype(np.int64)
              for r in dcfg.embedding_size]
        lab = rng.randint(0, 2, (B, 1)).astype(np.float32)
        batches.append((dd, sp, lab))

    def feed(k):
        dd, sp, lab = batches[k]
        ex.scatter_from_host(d, dd)
        for t, a in zip(s, sp):
            ex.scatter_from_host(t, a)
        ex.scatter_from_host(m.get_label_tensor(), lab)

    if graph and dev == "gpu":
        feed(0)
        ex.train_step()
        run = ex.capture_step()
        for k in range(1, steps):
            feed(k)          # host scatter into the captured input buffers, then replay
            run()
        torch.cuda.synchronize()
    else:
        for k in range(steps):
            feed(k)
            ex.train_step()
    ws = [w.get_weights(m) for w in m.parameters]
    ws[0] = ws[0][:, :13]   # the GPU pads the 13 dense features (zero input columns) for aligned loads
    return ws, m.get_perf_metrics().get_loss(), ex


def _assert_params_close(a_list, b_list, rtol):
    for a, b in zip(a_list, b_list):
        err = np.abs(a - b).max() / max(np.abs(a).max(), 1e-6)
        assert err < rtol, (a.shape, err)


def test_dlrm_tiny_fp32_gpu_matches_cpu(gpu):
    from flexmi.models.dlrm import DLRMConfig
    dcfg = DLRMConfig.preset("tiny")
    cpu = _dlrm_run("cpu", dcfg, 256, 5)
    g = _dlrm_run("gpu", dcfg, 256, 5)
    _assert_params_close(cpu[0], g[0], 1e-4)
    assert abs(cpu[1] - g[1]) < 1e-4 * max(1.0, abs(cpu[1]))


@pytest.mark.parametrize("graph", [False, True])
def test_dlrm_mlperf_widths_fp32_gpu_matches_cpu(gpu, graph):
    """The headline's code paths at MLPerf widths (D=128, 26 tables, bottom 13-512-256-128, top
    479-1024-1024-512-256-1) and batch 4096, so the production GEMM dispatch (128x128 tiles,
    split-K dW, fused act-bwd epilogues, skinny click layer), the second-stream embedding/MLP
    overlap (auto for D >= 128), the tiny-table LDS, atomic and owner-computes sparse-SGD kernels
    all run -- eager and as a captured hipGraph step -- and agree with the fp32 CPU executor after
    5 SGD steps at rtol 1e-4."""
    from flexmi.models.dlrm import DLRMConfig
    from flexmi.runtime import executor as E
    dcfg = DLRMConfig.preset("mlperf")
    # rows scaled so all three sparse-SGD kernels run: <= 16 rows (tiny LDS), <= 4096 (atomic),
    # > 4096 = lookups per step (owner-computes claim)
    dcfg.embedding_size = [max(3, min(r, int(r * 2e-3))) if r > 100000 else r for r in dcfg.embedding_size]
    rows = dcfg.embedding_size
    assert min(rows) <= 16 and any(16 < r <= 4096 for r in rows) and max(rows) > 4096
    B = 4096
    cpu = _dlrm_run("cpu", dcfg, B, 5, lr=0.05)
    g = _dlrm_run("gpu", dcfg, B, 5, graph=graph, lr=0.05)
    assert E.overlap_embeddings_enabled(g[2]), "second-stream embedding overlap not active at D=128"
    _assert_params_close(cpu[0], g[0], 1e-4)
    assert abs(cpu[1] - g[1]) < 1e-4 * max(1.0, abs(cpu[1]))


def _zoo_params(name, dev, steps, perturb=0.0, **kw):
    from tests.test_cpu_models import _zoo_feed, _zoo_model
    m, built = _zoo_model(name, device=dev, B=8, dtype="fp32", **kw)
    m.init_layers()
    if perturb:
        p = m.parameters[0]
        w = p.get_weights(m)
        p.set_weights(m, (w * (1 + perturb * np.random.RandomState(0).randn(*w.shape))).astype(np.float32))
    for it in range(steps):
        _zoo_feed(m, built, it)
        m._ex().train_step()
    return [p.get_weights(m) for p in m.parameters]


def _max_rel(a_list, b_list):
    return max(np.abs(a - b).max() / max(np.abs(a).max(), 1e-6) for a, b in zip(a_list, b_list))


@pytest.mark.parametrize("name,steps,kw", [("mnist_cnn", 3, {}), ("alexnet", 2, {}), ("resnet50", 2, {}),
                                           ("inception_v3", 1, {}), ("resnet50", 2, {"batch_norm": True}),
                                           ("candle_uno", 3, {}), ("nmt", 3, {})])
def test_zoo_fp32_gpu_matches_cpu(gpu, name, steps, kw):
    """fp32 GPU vs fp32 CPU after a few SGD steps.  Deep batch-norm nets at batch 8 are chaotic
    (ResNet-50+BN: a 1e-6 relative change of ONE weight tensor moves parameters by ~10 % after two
    steps), so the bound is max(2e-4, 20 x the CPU run's own sensitivity to a 1e-6 perturbation):
    parity to within what fp32 rounding differences can produce on that graph."""
    cpu = _zoo_params(name, "cpu", steps, **kw)
    gpu_p = _zoo_params(name, "gpu", steps, **kw)
    tol = 2e-4
    if name in ("inception_v3",) or kw.get("batch_norm"):
        tol = max(tol, 20 * _max_rel(cpu, _zoo_params(name, "cpu", steps, perturb=1e-6, **kw)))
    err = _max_rel(cpu, gpu_p)
    assert err < tol, (name, err, tol)


@pytest.mark.parametrize("state", [False, True])
def test_lstm_fp32_gpu_matches_cpu(gpu, state):
    from tests.test_cpu_models import _lstm_model
    B, T, I, H = 8, 7, 24, 32
    rng = np.random.RandomState(1)
    xin = rng.randn(B, T, I).astype(np.float32)
    hin = 0.5 * rng.randn(B, H).astype(np.float32)
    cin = 0.5 * rng.randn(B, H).astype(np.float32)
    lab = 0.3 * rng.randn(B, T * H).astype(np.float32)
    res = {}
    for dev in ("cpu", "gpu"):
        m, x, h0, c0, out = _lstm_model(dev, B, T, I, H, state=state, dtype="fp32")
        ex = m.init_layers()
        ex.scatter_from_host(x, xin)
        if state:
            ex.scatter_from_host(h0, hin)
            ex.scatter_from_host(c0, cin)
        ex.scatter_from_host(m.get_label_tensor(), lab)
        m.forward()
        y = ex.gather_to_host(out)
        for _ in range(2):
            ex.train_step()
        res[dev] = (y, [p.get_weights(m) for p in m.parameters])
    np.testing.assert_allclose(res["gpu"][0], res["cpu"][0], atol=1e-5)
    _assert_params_close(res["cpu"][1], res["gpu"][1], 1e-4)


def test_embedding_overlap_on_off_equivalent(gpu, monkeypatch):
    """Captured steps with the fused embedding groups on a second HIP stream (OVERLAP_EMB=1) train
    exactly like the single-stream schedule: multi-table group, >= 128-wide tables, bottom MLP."""
    from flexmi.models.dlrm import DLRMConfig
    from flexmi.runtime import executor as E
    dcfg = DLRMConfig(128, [5000, 300, 12, 70000, 40], [13, 256, 128], [256, 256, 1], 1, -1, -1, 0.0, "dot", "", -1,
                      "bce", "overlap")
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(E, "OVERLAP_EMB", mode)
        ws, loss, ex = _dlrm_run("gpu", dcfg, 2048, 4, graph=True)
        assert E.overlap_embeddings_enabled(ex) == (mode == "1")
        res[mode] = (ws, loss)
    _assert_params_close(res["0"][0], res["1"][0], 1e-5)
    assert abs(res["0"][1] - res["1"][1]) < 1e-5


# ---------------------------------------------------------------- CNN kernels (fp32)
@pytest.mark.parametrize("shape,relu", [((8, 64, 16, 16), True), ((8, 256, 4, 4), False), ((8, 2048, 1, 1), True),
                                        ((3, 5, 7, 9), False)])
def test_batchnorm_f32(gpu, shape, relu):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(10)
    x = (torch.randn(*shape, device=gpu) * 2 + 0.5)
    C_ = shape[1]
    gamma, beta = torch.rand(C_, device=gpu) + 0.5, torch.randn(C_, device=gpu)
    y = torch.empty_like(x)
    saved = {}
    Kk.batchnorm_forward(x, gamma, beta, y, relu, 1e-5, saved)
    xd = x.double().requires_grad_(True)
    gd, bd = gamma.double().requires_grad_(True), beta.double().requires_grad_(True)
    yr = torch.nn.functional.batch_norm(xd, None, None, gd, bd, training=True, eps=1e-5)
    if relu:
        yr = torch.relu(yr)
    assert rel_err(y, yr.detach()) < TOL
    dy = torch.randn_like(x)
    dx, dgam, dbet = torch.empty_like(x), torch.empty(C_, device=gpu), torch.empty(C_, device=gpu)
    Kk.batchnorm_backward(x, gamma, y, dy, dx, dgam, dbet, relu, 1e-5, saved, False)
    yr.backward(dy.double())
    assert rel_err(dx, xd.grad) < TOL
    assert rel_err(dgam, gd.grad) < TOL
    assert rel_err(dbet, bd.grad) < TOL


@pytest.mark.parametrize("k,s,p,is_max", [(3, 2, 1, True), (2, 2, 0, True), (3, 1, 1, False), (7, 1, 0, False)])
def test_pool_f32(gpu, k, s, p, is_max):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(11)
    x = torch.randn(4, 8, 14, 14, device=gpu)
    xd = x.double().requires_grad_(True)
    if is_max:
        yr = torch.nn.functional.max_pool2d(xd, k, s, p)
    else:
        yr = torch.nn.functional.avg_pool2d(xd, k, s, p, count_include_pad=False)
    y = torch.empty(yr.shape, device=gpu)
    Kk.pool2d_forward(x, y, (k, k), (s, s), (p, p, p, p), 30 if is_max else 31, 10)
    assert rel_err(y, yr.detach()) < TOL
    dy = torch.randn_like(y)
    yr.backward(dy.double())
    dx = torch.empty_like(x)
    Kk.pool2d_backward(x, y, dy, dx, (k, k), (s, s), (p, p, p, p), 30 if is_max else 31, 10, False)
    assert rel_err(dx, xd.grad) < TOL


@pytest.mark.parametrize("cin,cout,hw,k,s,p", [(3, 64, 32, 7, 2, 3), (64, 64, 16, 3, 1, 1), (32, 48, 9, 1, 1, 0),
                                               (5, 7, 11, 3, 2, 1)])
def test_conv2d_f32(gpu, cin, cout, hw, k, s, p):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(12)
    x = torch.randn(4, cin, hw, hw, device=gpu)
    w = torch.randn(cout, cin, k, k, device=gpu) * 0.1
    b = torch.randn(cout, device=gpu)
    xd, wd, bd = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = torch.relu(torch.nn.functional.conv2d(xd, wd, bd, s, p))
    y = torch.empty(yr.shape, device=gpu)
    Kk.conv2d_forward(x, w, b, y, (s, s), (p, p, p, p), 11, 1)
    assert rel_err(y, yr.detach()) < TOL
    dy = torch.randn_like(y)
    yr.backward(dy.double())
    dx, dw, db = torch.empty_like(x), torch.zeros_like(w), torch.zeros_like(b)
    Kk.conv2d_backward(x, w, y, dy, dx, dw, db, (s, s), (p, p, p, p), 11, 1, False)
    assert rel_err(dx, xd.grad) < TOL
    assert rel_err(dw, wd.grad) < TOL
    assert rel_err(db, bd.grad) < TOL


def test_loss_threshold_kernel_f32(gpu):
    """HIP loss with the DLRM --loss-threshold clamp vs the fp32 torch oracle (C == 1 and C > 1)."""
    from flexmi.core.loss_metrics import NUM_SLOTS, loss_and_metrics_torch
    from flexmi.core.types import LossType
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(13)
    for C_, lt in ((1, LossType.LOSS_BINARY_CROSSENTROPY), (1, LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE),
                   (5, LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE)):
        p = torch.rand(4096, C_, device=gpu)
        y = torch.randint(0, 2, (4096, C_), device=gpu).float()
        g, acc = torch.empty_like(p), torch.zeros(NUM_SLOTS, device=gpu)
        Kk.loss_forward_backward(int(lt), p, y, g, 0.5, acc, 0xFF, 0.05)
        g2, acc2 = torch.empty(4096, C_), torch.zeros(NUM_SLOTS)
        loss_and_metrics_torch(lt, p.cpu(), y.cpu(), g2, 0.5, acc2, 0xFF, clamp=0.05)
        assert rel_err(g.cpu(), g2) < TOL
        assert (g.cpu()[(p.cpu() < 0.05) | (p.cpu() > 0.95)] == 0).all()
        assert abs(acc[4].item() - acc2[4].item()) < 1e-3 * acc2[4].item()


def test_dlrm_hdf5_dataset_fp32_gpu_matches_cpu(gpu, tmp_path):
    """--dataset path on the GPU: the 13 dense features are zero-padded into the 16-wide input by
    the prefetch ring, sparse inputs are column blocks of the memory-mapped X_cat."""
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.models.dlrm import DLRMConfig, HDF5DLRMData, build_dlrm
    from flexmi.utils.hdf5 import write_h5
    rng = np.random.RandomState(0)
    tables, B, n = [500, 40, 9000, 7], 256, 256 * 4
    write_h5(str(tmp_path / "d.h5"), {
        "X_int": np.log(rng.randint(0, 1000, (n, 13)).astype(np.float32) + 1),
        "X_cat": np.concatenate([rng.randint(0, r, (n, 1)) for r in tables], 1).astype(np.int64),
        "y": rng.randint(0, 2, n).astype(np.float32)})
    res = {}
    for dev in ("cpu", "gpu"):
        cfg = FFConfig()
        cfg.batchSize, cfg.device, cfg.compute_dtype, cfg.seed = B, dev, "fp32", 5
        m = FFModel(cfg)
        dcfg = DLRMConfig(16, tables, [13, 64, 16], [64, 32, 1], 1, -1, -1, 0.0, "dot", "", -1, "bce", "h5")
        d, s, p = build_dlrm(m, dcfg)
        m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_BINARY_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
        ex = m.init_layers()
        data = HDF5DLRMData(m, d, s, dcfg, str(tmp_path / "d.h5"))
        for _ in range(6):
            data.next_batch()
            ex.train_step()
        data.close()
        ws = [w.get_weights(m) for w in m.parameters]
        ws[0] = ws[0][:, :13]
        res[dev] = ws
    _assert_params_close(res["cpu"], res["gpu"], 1e-4)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fused_backward_epilogue_split_k_small_batch(gpu, dtype):
    """Small-batch dX GEMM with the fused backward epilogue (summit_large: 256 x 4096 x 4096): the
    grid is small, so K is split and the act-bwd + bias-gradient column sums run in the split-K
    reduce (fm_gemm_f32_reduce_bwd / fm_gemm_splitk_reduce_bwd) -- same results as the oracle."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(9)
    dt = torch.float32 if dtype == "fp32" else torch.bfloat16
    tol = TOL if dtype == "fp32" else 2e-2
    M, K, N = 256, 2048, 4096          # dpre [M, N] . W [N, K] -> dX [M, K]
    dpre = torch.randn(M, N, device=gpu).to(dt)
    W = (torch.randn(N, K, device=gpu) * 0.05).to(dt)
    yb = torch.randn(M, K, device=gpu).relu().to(dt)
    dx = torch.empty(M, K, device=gpu, dtype=dt)
    colsum = torch.zeros(K, device=gpu)
    ks = Kk.gemm(dpre, N, True, W, K, False, dx, K, M, K, N, act_y=yb, bwd_act=11, colsum=colsum)
    assert ks > 1
    ref = (dpre.double() @ W.double()) * (yb.double() > 0)
    assert rel_err(dx, ref) < tol
    assert rel_err(colsum, ref.sum(0)) < tol


# ---------------------------------------------------------------- thin-input Linear (gemm_small.hip)
@pytest.mark.parametrize("act", [10, 11, 12])
@pytest.mark.parametrize("M,K,N", [(8192, 16, 512), (1000, 4, 12), (333, 32, 1024), (4096, 20, 260)])
def test_smallk_forward(gpu, act, M, K, N):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(11)
    x, w, b = torch.randn(M, K, device=gpu), torch.randn(N, K, device=gpu), torch.randn(N, device=gpu)
    y = torch.full((M, N), float("nan"), device=gpu)
    assert Kk.C().smallk_fwd(x, w, b, y, act)
    ref = x.double() @ w.double().t() + b.double()
    ref = {10: ref, 11: ref.clamp_min(0), 12: torch.sigmoid(ref)}[act]
    assert rel_err(y, ref) < TOL
    # outside the limits nothing is launched and the caller falls back
    assert not Kk.C().smallk_fwd(torch.randn(M, 13, device=gpu), torch.randn(N, 13, device=gpu), b, y, act)


@pytest.mark.parametrize("M,K,N", [(8192, 16, 512), (1000, 4, 12), (333, 32, 1032), (77, 8, 4), (8192, 28, 2052)])
def test_smallk_dw(gpu, M, K, N):
    """dW += dpre^T x and db += colsum(dpre) (accumulating, two-pass deterministic)."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(12)
    dpre, x = torch.randn(M, N, device=gpu), torch.randn(M, K, device=gpu)
    dw0, db0 = torch.randn(N, K, device=gpu), torch.randn(N, device=gpu)
    dw, db = dw0.clone(), db0.clone()
    ws = Kk.workspace(dpre.device, Kk.GEMM_WS_BYTES)
    assert Kk.C().smallk_dw(dpre, x, dw, db, ws, None, None, None, 0.0, 0.0, False)
    assert rel_err(dw - dw0, dpre.double().t() @ x.double()) < TOL
    assert rel_err(db - db0, dpre.double().sum(0)) < TOL
    dw2, db2 = dw0.clone(), db0.clone()
    assert Kk.C().smallk_dw(dpre, x, dw2, db2, ws, None, None, None, 0.0, 0.0, False)
    assert torch.equal(dw2, dw) and torch.equal(db2, db)          # fixed summation order


@pytest.mark.parametrize("M,K,N", [(8192, 16, 512), (1000, 4, 12), (77, 8, 4)])
def test_smallk_bf16(gpu, M, K, N):
    """The bf16 forms (bf16 x / w / y and dpre, fp32 accumulate and dW): against float64 of the same
    bf16 values."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(14)
    x = torch.randn(M, K, device=gpu).bfloat16()
    w = torch.randn(N, K, device=gpu).bfloat16()
    b = torch.randn(N, device=gpu)
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    assert Kk.C().smallk_fwd(x, w, b, y, 11)
    ref = (x.double() @ w.double().t() + b.double()).clamp_min(0)
    assert rel_err(y, ref) < 1e-2
    dpre = torch.randn(M, N, device=gpu).bfloat16()
    dw, db = torch.zeros(N, K, device=gpu), torch.zeros(N, device=gpu)
    ws = Kk.workspace(gpu, Kk.GEMM_WS_BYTES)
    assert Kk.C().smallk_dw(dpre, x, dw, db, ws, None, None, None, 0.0, 0.0, False)
    assert rel_err(dw, dpre.double().t() @ x.double()) < 1e-5
    assert rel_err(db, dpre.double().sum(0)) < 1e-5


@pytest.mark.parametrize("mom,nesterov,mirror", [(0.0, False, False), (0.9, False, True), (0.9, True, False)])
def test_smallk_dw_fused_sgd(gpu, mom, nesterov, mirror):
    """The SGD step applied in the dW reduce == gradient + optim.hip SGD kernel."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(13)
    M, K, N, lr, wd = 8192, 16, 512, 0.05, 1e-3
    dpre, x = torch.randn(M, N, device=gpu), torch.randn(M, K, device=gpu)
    w = torch.randn(N, K, device=gpu)
    v = torch.randn(N, K, device=gpu) if mom > 0 else None
    wc = torch.empty(N, K, device=gpu, dtype=torch.bfloat16) if mirror else None
    db = torch.zeros(N, device=gpu)
    lr_t = torch.tensor([lr], device=gpu)
    g = dpre.double().t() @ x.double() + wd * w.double()
    if mom > 0:
        v_ref = v.double() * mom + g
        g = g + mom * v_ref if nesterov else v_ref
    w_ref = w.double() - lr * g
    ws = Kk.workspace(dpre.device, Kk.GEMM_WS_BYTES)
    assert Kk.C().smallk_dw(dpre, x, w, db, ws, v, wc, lr_t, wd, mom, nesterov)
    assert rel_err(w, w_ref) < TOL
    assert rel_err(db, dpre.double().sum(0)) < TOL
    if mom > 0:
        assert rel_err(v, v_ref) < TOL
    if mirror:
        assert torch.equal(wc, w.to(torch.bfloat16))
