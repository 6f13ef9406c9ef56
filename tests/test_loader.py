"""Native prefetching data loader (csrc/runtime/loader.cc): batch order, shuffling, per-rank
shard gather, and training equivalence with the plain SingleDataLoader."""
import numpy as np
import pytest


def test_ring_order_and_shuffle():
    from flexmi import _native
    n, B = 40, 8
    data = np.arange(n * 3, dtype=np.float32).reshape(n, 3)
    for shuffle in (False, True):
        r = _native.BatchRing(B, n, 3, 3, shuffle, 11)
        bufs = [np.zeros((B, 3), np.float32) for _ in range(3)]
        si = r.add_source(data.ctypes.data, n, 12, 0, 12, 0, B)
        for s, b in enumerate(bufs):
            r.set_slot(si, s, b.ctypes.data)
        r.start()
        seen = []
        for k in range(10):          # two epochs
            slot = r.acquire()
            ids = r.batch_ids(k)
            np.testing.assert_array_equal(bufs[slot], data[ids])
            seen.append(ids)
            r.release(slot)
        r.stop()
        ep0 = np.concatenate(seen[:5])
        assert sorted(ep0) == list(range(n))                 # an epoch visits every sample once
        if shuffle:
            assert list(ep0) != list(range(n))
            assert list(np.concatenate(seen[5:])) != list(ep0)  # new permutation per epoch
        else:
            assert list(ep0) == list(range(n))


def test_ring_column_and_row_shard():
    from flexmi import _native
    n, B = 16, 8
    data = np.arange(n * 6, dtype=np.int64).reshape(n, 6)
    r = _native.BatchRing(B, n, 2, 1, True, 3)
    bufs = [np.zeros((4, 2), np.int64) for _ in range(2)]
    si = r.add_source(data.ctypes.data, n, 48, 2 * 8, 2 * 8, 4, 8)   # rows 4..8, cols 2..4
    for s, b in enumerate(bufs):
        r.set_slot(si, s, b.ctypes.data)
    r.start()
    for k in range(4):
        slot = r.acquire()
        ids = r.batch_ids(k)[4:8]
        np.testing.assert_array_equal(bufs[slot], data[ids][:, 2:4])
        r.release(slot)
    r.stop()


def test_prefetch_loader_trains_like_single_loader():
    from flexmi.core import (ActiMode, FFConfig, FFModel, LossType, MetricsType, PrefetchLoader, SGDOptimizer,
                             SingleDataLoader)
    rng = np.random.RandomState(0)
    n, B = 48, 8
    xs = rng.rand(n, 10).astype(np.float32)
    ys = rng.randint(0, 3, (n, 1)).astype(np.int32)
    res = []
    for kind in ("single", "prefetch"):
        cfg = FFConfig()
        cfg.device, cfg.compute_dtype, cfg.batchSize = "cpu", "fp32", B
        m = FFModel(cfg)
        x = m.create_tensor([B, 10], name="x")
        o = m.softmax(m.dense(m.dense(x, 8, ActiMode.AC_MODE_RELU, name="a"), 3, name="b"))
        m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
        m.init_layers()
        if kind == "single":
            dls = [SingleDataLoader(m, x, xs, n), SingleDataLoader(m, m.get_label_tensor(), ys, n)]
        else:
            dls = [PrefetchLoader(m, [(x, xs), (m.get_label_tensor(), ys)], n, depth=3, threads=2)]
        m.train(dls, epochs=2)
        res.append([p.get_weights(m) for p in m.parameters])
        if kind == "prefetch":
            dls[0].close()
    for a, b in zip(*res):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
