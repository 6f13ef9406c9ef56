"""The NHWC convolutions' weight re-layouts as one launch per step (flexmi/ops/_kernels.py
conv_wprep_all -> fm_cnhwc_wprep_multi, issued by the executor's conv.wprep_all item): the batched
launch writes exactly the per-layer fm_cnhwc_wprep layouts, and a CNN trained with it ends with the
parameters of one trained with the per-layer launches (a re-layout is a copy; the tolerance only absorbs the
order of the float atomics some gradient epilogues use)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_multi_wprep_equals_per_layer(gpu):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(3)
    shapes = [(64, 64, 3, 3), (256, 64, 1, 1), (48, 20, 5, 5), (8, 16, 1, 1), (192, 64, 5, 5)]
    layers = []
    for sh in shapes:
        w = torch.randn(*sh, device=gpu).bfloat16()
        layers.append((w, {"nhwc_fwd_used": True}))
    Kk.conv_wprep_all(layers)
    for w, sv in layers:
        assert sv.pop("nhwc_wf_ready")
        K, C, R, S = w.shape
        wf = torch.empty(K * R * S * Kk._r8(C), device=gpu, dtype=torch.bfloat16)
        wd = torch.empty(C * R * S * Kk._r8(K), device=gpu, dtype=torch.bfloat16)
        Kk.C().cnhwc_wprep(w, wf, wd, w, w, Kk._r8(C), Kk._r8(K), 3, 1)
        assert torch.equal(sv["nhwc_wf"], wf) and torch.equal(sv["nhwc_wd"], wd), w.shape


def test_layers_without_an_nhwc_forward_are_left_alone(gpu):
    from flexmi.ops import _kernels as Kk
    w = torch.randn(16, 16, 3, 3, device=gpu).bfloat16()
    sv = {}
    Kk.conv_wprep_all([(w, sv), (w, None)])
    assert "nhwc_wf_ready" not in sv and "nhwc_wf" not in sv


def _train(gpu, batched, steps=3):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer
    from flexmi.models import zoo
    from flexmi.runtime import executor as E
    old = E.CONV_WPREP_ALL
    E.CONV_WPREP_ALL = batched
    try:
        cfg = FFConfig()
        cfg.batchSize = 8
        cfg.compute_dtype = "bf16"
        m = FFModel(cfg)
        built = zoo.build("resnet50", m, small=True)
        m.compile(SGDOptimizer(m, 0.01), built.loss, built.metrics)
        ex = m.init_layers()
        rng = np.random.RandomState(0)
        for t in built.inputs.values():
            ex.scatter_from_host(t, rng.rand(*t.dims).astype(np.float32))
        lab = m.get_label_tensor()
        ex.scatter_from_host(lab, rng.randint(0, built.output.dims[-1], lab.dims).astype(np.int32))
        for _ in range(steps):
            ex.train_step()
        torch.cuda.synchronize()
        return [p.get_weights(m).copy() for p in m.parameters]
    finally:
        E.CONV_WPREP_ALL = old


def test_resnet_trains_identically_with_the_batched_relayout(gpu):
    a = _train(gpu, True)
    b = _train(gpu, False)
    assert len(a) == len(b)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-3, atol=1e-4)
