"""Native CPU kernels (flexmi/_cpu, csrc/cpu/cpu_ops.cc) against the torch reference path:
embedding-bag forward (sum / avg, row shards, out-of-shard lookups, strided output rows), the
dense gradient and the fused sparse SGD update, and a whole DLRM CPU training run with the native
kernels on vs off (reference: src/ops/embedding.cc:87-163, embedding_avx2.cc)."""
import numpy as np
import pytest
import torch

cpu = pytest.importorskip("flexmi._cpu")


@pytest.mark.parametrize("D,bag,idt", [(64, 1, torch.int32), (13, 3, torch.int64), (128, 100, torch.int64),
                                       (40, 7, torch.int32)])
def test_embedding_kernels_vs_torch(D, bag, idt):
    torch.manual_seed(0)
    R, lo, B = 500, 100, 257
    W = torch.randn(R, D)
    idx = torch.randint(0, 700, (B, bag), dtype=idt)          # shard holds rows [100, 600)
    li = (idx.long() - lo)
    ok = ((li >= 0) & (li < R)).float()
    li = li.clamp(0, R - 1)
    out = torch.zeros(B, D + 5)[:, :D]                         # strided output rows
    cpu.embedding_fwd(W, idx, out, lo, 0.5)
    ref = (W[li] * ok[..., None]).sum(1) * 0.5
    assert torch.allclose(out, ref, atol=1e-5)
    dy = torch.randn(B, D)
    G = torch.zeros(R, D)
    cpu.embedding_bwd(G, idx, dy, lo, 0.25)
    upd = torch.zeros(R, D)
    upd.index_add_(0, li.reshape(-1), dy.repeat_interleave(bag, 0) * ok.reshape(-1, 1))
    assert torch.allclose(G, 0.25 * upd, atol=1e-4)


def _train(native, steps=3):
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.models.dlrm import DLRMConfig, build_dlrm
    from flexmi.ops import embedding as E
    old = E.NATIVE_CPU
    E.NATIVE_CPU = native
    try:
        cfg = FFConfig()
        cfg.batchSize, cfg.device, cfg.seed = 32, "cpu", 5
        m = FFModel(cfg)
        dcfg = DLRMConfig(16, [300, 50, 1000], [13, 32, 16], [64, 16, 1], 2, -1, -1, 0.0, "cat", "", -1, "mse", "n")
        d, s, _ = build_dlrm(m, dcfg)
        m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, [MetricsType.METRICS_ACCURACY])
        ex = m.init_layers()
        rng = np.random.RandomState(1)
        for _ in range(steps):
            ex.scatter_from_host(d, rng.rand(32, 13).astype(np.float32))
            for t, r in zip(s, dcfg.embedding_size):
                ex.scatter_from_host(t, rng.randint(0, r, t.dims).astype(np.int64))
            ex.scatter_from_host(m.get_label_tensor(), rng.randint(0, 2, (32, 1)).astype(np.float32))
            ex.train_step()
        return [p.get_weights(m) for p in m.parameters]
    finally:
        E.NATIVE_CPU = old


def test_dlrm_cpu_native_matches_torch_path():
    a, b = _train(True), _train(False)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-6)


def test_native_cpu_kernels_are_used(monkeypatch):
    """The CPU backend's embedding really dispatches to flexmi._cpu (not a silent torch path)."""
    from flexmi.ops import embedding as E
    calls = []
    real = E._cpu_ext()

    class Spy:
        def embedding_fwd(self, *a):
            calls.append("fwd")
            return real.embedding_fwd(*a)

        def embedding_bwd(self, *a):
            calls.append("bwd")
            return real.embedding_bwd(*a)

    monkeypatch.setattr(E, "_CPU_MOD", [Spy()])
    _train(True, steps=1)
    assert "fwd" in calls and "bwd" in calls
