"""SGD fused into the weight-gradient GEMM (csrc/kernels/gemm.hip fm_gemm_dw_sgd, Executor.
_plan_fused_sgd): the kernel against the unfused pair (dW GEMM + fm_sgd kernel) and against a
float64 oracle, over the in-tile epilogue, the split-K reduce, tails and momentum / Nesterov / weight
decay; and whole training steps (eager and hipGraph-captured) with the fusion on vs off."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


# B (= GEMM K), out (= M), in (= N): split-K through the reduce (small grids, long K), unsplit tiles
# through the LDS-staged update (128x128 / 64x64 tiles, M / N tails), in % 8 != 0 (scalar loads)
SHAPES = [(256, 512, 384), (8192, 256, 128), (96, 100, 36), (64, 40, 20), (64, 2000, 1028), (256, 2048, 2048),
          (128, 4096, 512)]


@pytest.mark.parametrize("shape", SHAPES, ids=[f"s{i}" for i in range(len(SHAPES))])
@pytest.mark.parametrize("mom,nest,wd,mirror", [(0.0, False, 0.0, True), (0.9, True, 1e-3, True), (0.5, False, 0.0, False)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_gemm_dw_sgd_matches_unfused(gpu, shape, mom, nest, wd, mirror, dt):
    from flexmi.ops import _kernels as K
    B, out, inp = shape
    torch.manual_seed(B + out + inp)
    dpre = (torch.randn(B, out, device=gpu) * 0.1).to(dt)
    x = torch.randn(B, inp, device=gpu).to(dt)
    w0 = torch.randn(out, inp, device=gpu) * 0.05
    v0 = torch.randn(out, inp, device=gpu) * 0.01 if mom > 0 else None
    lr = torch.tensor([0.05], device=gpu)
    # unfused: gradient into a zeroed buffer, then the optimizer kernel
    wu, gu = w0.clone(), torch.zeros_like(w0)
    vu = v0.clone() if v0 is not None else None
    cu = torch.empty(out, inp, device=gpu, dtype=torch.bfloat16) if mirror else None
    dbu = torch.zeros(out, device=gpu)
    K.gemm(dpre, out, False, x, inp, False, gu, inp, out, inp, B, beta=True, rowsum_a=dbu)
    K.sgd_update(wu, gu, vu, cu, lr, wd, mom, nest, zero_grad=True)
    # fused
    wf = w0.clone()
    vf = v0.clone() if v0 is not None else None
    cf = torch.empty(out, inp, device=gpu, dtype=torch.bfloat16) if mirror else None
    dbf = torch.zeros(out, device=gpu)
    upd = K.FusedSGD(wf, cf, vf, lr, wd, mom, nest)
    assert K._dw_fused_sgd(dpre, x, None, dbf, upd)
    torch.cuda.synchronize()
    assert torch.equal(gu, torch.zeros_like(gu))
    torch.testing.assert_close(wf, wu, rtol=1e-6, atol=1e-7)
    if mom > 0:
        torch.testing.assert_close(vf, vu, rtol=1e-6, atol=1e-7)
    if mirror:
        assert (cf.float() - cu.float()).abs().max().item() <= 2 ** -7 * wu.abs().max().item()
        torch.testing.assert_close(cf.float(), wf.bfloat16().float(), rtol=0, atol=0)
    torch.testing.assert_close(dbf, dbu, rtol=1e-5, atol=1e-5)
    # float64 oracle of one SGD step
    g = dpre.double().t() @ x.double() + wd * w0.double()
    if mom > 0:
        vv = v0.double() * mom + g
        g = g + mom * vv if nest else vv
    ref = w0.double() - 0.05 * g
    assert ((wf.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5


def _train(monkeypatch, fused, graph, momentum, dtype="bf16"):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer, LossType, MetricsType
    from flexmi.models.dlrm import DLRMConfig, build_dlrm, SyntheticDLRMData
    monkeypatch.setenv("FM_FUSED_SGD", "1" if fused else "0")
    from flexmi.runtime import executor as _E
    monkeypatch.setattr(_E, "FUSED_SGD_MIN", 0)      # the tiny model's layers are below the default size
    cfg = FFConfig()
    cfg.batchSize = 512
    cfg.seed = 5
    cfg.compute_dtype = dtype
    m = FFModel(cfg)
    dcfg = DLRMConfig.preset("tiny")
    d, s, p = build_dlrm(m, dcfg)
    m.compile(SGDOptimizer(m, 0.05, momentum=momentum, nesterov=momentum > 0, weight_decay=1e-4 if momentum else 0.0),
              LossType.LOSS_BINARY_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    data = SyntheticDLRMData(m, d, s, dcfg, num_batches=1)
    data.next_batch()
    if graph:
        ex.train_step()
        run = ex.capture_step()
        for _ in range(3):
            run()
    else:
        for _ in range(4):
            ex.train_step()
    torch.cuda.synchronize()
    n_fused = len(ex.fused_sgd_entries)
    return [w.get_weights(m) for w in m.parameters], n_fused, ex


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_fused_sgd_training_matches_unfused(gpu, monkeypatch, graph, momentum):
    ref, n0, _ = _train(monkeypatch, False, graph, momentum)
    got, n1, ex = _train(monkeypatch, True, graph, momentum)
    assert n0 == 0 and n1 >= 3, (n0, n1)
    # fused weights never materialise a gradient
    for e in ex.fused_sgd_entries:
        assert float(e.grad.abs().max()) == 0.0
    for a, b in zip(ref, got):
        assert np.allclose(a, b, rtol=1e-5, atol=1e-6), (a.shape, np.abs(a - b).max())


def test_fused_sgd_fp32_training_matches_unfused(gpu, monkeypatch):
    """fp32 compute (the reference precision): fused fp32 dW GEMM (gemm_f32.hip) vs the unfused step."""
    ref, _, _ = _train(monkeypatch, False, False, 0.0, dtype="fp32")
    got, n1, _ = _train(monkeypatch, True, False, 0.0, dtype="fp32")
    assert n1 >= 3
    for a, b in zip(ref, got):
        assert np.allclose(a, b, rtol=1e-6, atol=1e-7), a.shape


def test_separate_backward_update_keeps_gradients(gpu, monkeypatch):
    """backward() / update() called separately stay unfused: gradients are materialised."""
    from flexmi.core import FFConfig, FFModel, SGDOptimizer, LossType, MetricsType
    from flexmi.models.dlrm import DLRMConfig, build_dlrm, SyntheticDLRMData
    monkeypatch.setenv("FM_FUSED_SGD", "1")
    from flexmi.runtime import executor as _E
    monkeypatch.setattr(_E, "FUSED_SGD_MIN", 0)
    cfg = FFConfig()
    cfg.batchSize = 256
    m = FFModel(cfg)
    dcfg = DLRMConfig.preset("tiny")
    d, s, p = build_dlrm(m, dcfg)
    m.compile(SGDOptimizer(m, 0.05), LossType.LOSS_BINARY_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    data = SyntheticDLRMData(m, d, s, dcfg, num_batches=1)
    data.next_batch()
    ex.forward()
    ex.backward()
    torch.cuda.synchronize()
    assert ex.fused_sgd_entries
    assert any(float(e.grad.abs().max()) > 0 for e in ex.fused_sgd_entries)
    ex.update()


@pytest.mark.parametrize("mom", [0.0, 0.9])
def test_sgd_segs_matches_full_update(gpu, mom):
    """The segmented optimizer launch (ranges off the 4-element grain, tiny and long ranges) updates
    exactly the listed ranges like fm_sgd, and leaves everything else untouched."""
    from flexmi.ops import _kernels as K
    torch.manual_seed(2)
    n = 100003
    w0 = torch.randn(n, device=gpu)
    g0 = torch.randn(n, device=gpu)
    v0 = torch.randn(n, device=gpu) if mom > 0 else None
    lr = torch.tensor([0.1], device=gpu)
    segs = [(0, 5), (7, 1), (13, 40000), (40021, 3), (50001, 49999), (100000, 3)]
    w, g = w0.clone(), g0.clone()
    v = v0.clone() if v0 is not None else None
    c = torch.zeros(n, device=gpu, dtype=torch.bfloat16)
    K.C().sgd_segs(w, g, v, c, lr, [a for a, _ in segs], [b for _, b in segs], 1e-3, mom, True, True)
    wr, gr = w0.clone(), g0.clone()
    vr = v0.clone() if v0 is not None else None
    cr = torch.zeros(n, device=gpu, dtype=torch.bfloat16)
    for a, b in segs:
        K.sgd_update(wr[a:a + b], gr[a:a + b], vr[a:a + b] if vr is not None else None, cr[a:a + b], lr, 1e-3, mom, True,
                     zero_grad=True)
    torch.cuda.synchronize()
    torch.testing.assert_close(w, wr, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(g, gr, rtol=0, atol=0)
    torch.testing.assert_close(c.float(), cr.float(), rtol=0, atol=0)
    if v is not None:
        torch.testing.assert_close(v, vr, rtol=1e-6, atol=1e-7)
    untouched = torch.ones(n, dtype=torch.bool, device=gpu)
    for a, b in segs:
        untouched[a:a + b] = False
    assert torch.equal(w[untouched], w0[untouched])
