"""Native CPU counter-based init and loss/metrics (csrc/cpu/init_metrics.cc, flexmi._cpu) against
the numpy / torch oracles of flexmi/core/initializers.py and flexmi/core/loss_metrics.py
(reference: src/runtime/initializer.cc CPU init tasks, src/metrics_functions/metrics_functions.cc
CPU metrics)."""
import numpy as np
import pytest
import torch

from flexmi.core import initializers as I
from flexmi.core.loss_metrics import NUM_SLOTS, loss_and_metrics_torch
from flexmi.core.types import LossType

cpu = pytest.importorskip("flexmi._cpu")
if not hasattr(cpu, "counter_fill"):
    pytest.skip("flexmi._cpu predates counter_fill", allow_module_level=True)


@pytest.mark.parametrize("kind,a,b", [(I.KIND_ZERO, 0, 0), (I.KIND_CONSTANT, 0.7, 0), (I.KIND_UNIFORM, -0.3, 0.5),
                                      (I.KIND_NORMAL, 0.1, 2.0)])
@pytest.mark.parametrize("shape,box", [((37, 19), ((0, 37), (0, 19))), ((40, 24), ((5, 33), (8, 20))),
                                       ((3, 4, 5, 6), ((1, 3), (0, 4), (2, 5), (1, 6))), ((1000,), ((123, 877),))])
def test_counter_fill_matches_numpy(kind, a, b, shape, box):
    ref = I.counter_fill_cpu(kind, 1234, a, b, shape, box)
    out = torch.empty(ref.shape, dtype=torch.float32)
    cpu.counter_fill(out, list(shape), list(box), kind, 1234, a, b)
    if kind == I.KIND_NORMAL:
        np.testing.assert_allclose(out.numpy(), ref, rtol=1e-6, atol=1e-6)
    else:
        assert np.array_equal(out.numpy(), ref)


def test_sharded_fill_equals_unsharded():
    full = torch.empty(64, 48)
    cpu.counter_fill(full, [64, 48], [(0, 64), (0, 48)], I.KIND_UNIFORM, 9, -1.0, 1.0)
    for r0, r1, c0, c1 in [(0, 32, 0, 48), (32, 64, 0, 24), (7, 50, 13, 40)]:
        part = torch.empty(r1 - r0, c1 - c0)
        cpu.counter_fill(part, [64, 48], [(r0, r1), (c0, c1)], I.KIND_UNIFORM, 9, -1.0, 1.0)
        assert torch.equal(part, full[r0:r1, c0:c1])


def test_initializer_fill_uses_native():
    init = I.GlorotUniformInitializer(seed=5)
    out = torch.empty(20, 30)
    init.fill((20, 30), ((0, 20), (0, 30)), out)
    kind, seed, a, b = init.params((20, 30))
    assert np.array_equal(out.numpy(), I.counter_fill_cpu(kind, seed, a, b, (20, 30), ((0, 20), (0, 30))))


@pytest.mark.parametrize("loss,C", [(LossType.LOSS_BINARY_CROSSENTROPY, 1), (LossType.LOSS_CATEGORICAL_CROSSENTROPY, 7),
                                    (LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, 10),
                                    (LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, 3),
                                    (LossType.LOSS_MEAN_SQUARED_ERROR_SUM_REDUCE, 1)])
@pytest.mark.parametrize("clamp", [0.0, 0.05])
def test_loss_metrics_matches_torch(loss, C, clamp):
    torch.manual_seed(C)
    B = 1000
    if loss in (LossType.LOSS_CATEGORICAL_CROSSENTROPY, LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY):
        p = torch.softmax(torch.randn(B, C), 1)
    else:
        p = torch.rand(B, C)
    if loss == LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY:
        y = torch.randint(0, C, (B, 1), dtype=torch.int32)
    elif loss == LossType.LOSS_CATEGORICAL_CROSSENTROPY:
        y = torch.nn.functional.one_hot(torch.randint(0, C, (B,)), C).float()
    else:
        y = (torch.rand(B, C) > 0.5).float()
    mask = 63
    g_ref, acc_ref = torch.empty(B, C), torch.zeros(NUM_SLOTS)
    loss_and_metrics_torch(loss, p, y, g_ref, 1.0 / B, acc_ref, mask, clamp=clamp)
    g, acc = torch.empty(B, C), torch.zeros(NUM_SLOTS)
    cpu.loss_metrics(int(loss), p, y, g, 1.0 / B, acc, mask, clamp)
    torch.testing.assert_close(g, g_ref, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(acc, acc_ref, rtol=2e-5, atol=1e-3)
    acc2 = torch.zeros(NUM_SLOTS)
    cpu.loss_metrics(int(loss), p, y, None, 1.0 / B, acc2, mask, clamp)
    torch.testing.assert_close(acc2, acc)
