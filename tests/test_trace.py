"""begin_trace / end_trace (reference Legion tracing, examples/cpp/DLRM/dlrm.cc:178-185): the first
traced iteration records its call sequence; on MI355X later iterations of a training-step trace
replay it as hipGraph segments, on CPU every iteration runs eagerly.  Either way the training
result equals an untraced loop."""
import numpy as np
import pytest


def _train(device, traced, steps=5):
    from flexmi.core import ActiMode, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    cfg = FFConfig()
    cfg.device, cfg.batchSize = device, 32
    if device == "cpu":
        cfg.compute_dtype = "fp32"
    m = FFModel(cfg)
    x = m.create_tensor([32, 64])
    t = m.dense(x, 128, ActiMode.AC_MODE_RELU)
    t = m.softmax(m.dense(t, 10))
    m.compile(SGDOptimizer(m, 0.05), LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    rng = np.random.RandomState(0)
    for it in range(steps):
        ex.scatter_from_host(x, rng.rand(32, 64).astype(np.float32))
        ex.scatter_from_host(m.get_label_tensor(), rng.randint(0, 10, (32, 1)).astype(np.int32))
        if traced:
            cfg.begin_trace(111)
        m.forward()
        m.zero_gradients()
        m.backward()
        m.update()
        if traced:
            cfg.end_trace(111)
    st = m._traces.get(111)
    return [p.get_weights(m) for p in m.parameters], st, ex


def test_trace_cpu_runs_eagerly():
    ref, _, _ = _train("cpu", False)
    got, st, _ = _train("cpu", True)
    assert st is not None and st["seq"] == ["forward", "zero_gradients", "backward", "update"]
    assert not st["replayable"] and st["replay"] is None
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_trace_gpu_replays_hipgraph():
    ref, _, _ = _train("gpu", False)
    got, st, ex = _train("gpu", True)
    assert st["replayable"] and st["replay"] is not None, "the trace must be replayed as hipGraph segments"
    assert ex.step_count == 5
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
