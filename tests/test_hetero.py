"""Heterogeneous CPU placement (reference src/runtime/dlrm_strategy_hetero.cc and the
CPU embedding task variants, src/ops/embedding.cc:87-163): embedding tables placed on the host
(device_type CPU in the strategy) train exactly like tables placed on the device."""
import numpy as np
import pytest


def _run(hetero, device, steps=3):
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.models.dlrm import DLRMConfig, build_dlrm
    from flexmi.parallel.layout import ParallelConfig
    cfg = FFConfig()
    cfg.device, cfg.batchSize = device, 16
    if device == "cpu":
        cfg.compute_dtype = "fp32"
    m = FFModel(cfg)
    dcfg = DLRMConfig.preset("tiny")
    d, s, _ = build_dlrm(m, dcfg)
    strat = {}
    if hetero:
        for op in m.layers:
            if op.op_type.name == "OP_EMBEDDING":
                strat[op.name] = ParallelConfig([1, 1], [0], ParallelConfig.CPU)
    m.strategies = strat
    m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_BINARY_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    m.strategies = strat
    ex = m.init_layers()
    if hetero:
        embs = [op for op in m.layers if getattr(op, "host_exec", False)]
        assert len(embs) == len(s), "every table must be host-placed"
        assert all(not ex.wentries[op.weights[0].guid].master.is_cuda for op in embs)
    rng = np.random.RandomState(0)
    for _ in range(steps):
        dd = np.zeros((16, d.dims[1]), np.float32)
        dd[:, :13] = rng.rand(16, 13)
        ex.scatter_from_host(d, dd)
        for t, r in zip(s, dcfg.embedding_size):
            ex.scatter_from_host(t, rng.randint(0, r, t.dims).astype(np.int64))
        ex.scatter_from_host(m.get_label_tensor(), rng.randint(0, 2, (16, 1)).astype(np.float32))
        ex.train_step()
    return [p.get_weights(m) for p in m.parameters], m.get_perf_metrics().get_loss()


def test_cpu_placed_embeddings_match_device_tables():
    ref, lref = _run(False, "cpu")
    got, lgot = _run(True, "cpu")
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    assert abs(lref - lgot) < 1e-5


def test_cpu_placement_rejects_dense_optimizer():
    from flexmi.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexmi.models.dlrm import DLRMConfig, build_dlrm
    from flexmi.parallel.layout import ParallelConfig
    cfg = FFConfig()
    cfg.device, cfg.compute_dtype, cfg.batchSize = "cpu", "fp32", 16
    m = FFModel(cfg)
    build_dlrm(m, DLRMConfig.preset("tiny"))
    emb = next(op for op in m.layers if op.op_type.name == "OP_EMBEDDING")
    m.strategies = {emb.name: ParallelConfig([1, 1], [0], ParallelConfig.CPU)}
    m.compile(AdamOptimizer(m, 0.01), LossType.LOSS_BINARY_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    with pytest.raises(NotImplementedError):
        m.init_layers()


@pytest.mark.gpu
def test_cpu_placed_embeddings_on_gpu():
    """Host tables next to a GPU model: lookups on the host, H2D of the bag sums, host sparse SGD
    (the items stay outside hipGraph segments)."""
    ref, lref = _run(False, "gpu")
    got, lgot = _run(True, "gpu")
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=2e-4)
    assert abs(lref - lgot) < 1e-3
