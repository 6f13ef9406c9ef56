"""Functional "no-inout" builders + init_inout (include/model.h:402-436) and the raw-pointer
tensor API (Tensor::get_raw_ptr / attach_raw_ptr, src/runtime/model.cc:46-93) on the CPU."""
import ctypes

import numpy as np
import pytest

from flexmi.core import ActiMode, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexmi.core.model import DeferredOp


def _cfg(b=8):
    c = FFConfig()
    c.device = "cpu"
    c.compute_dtype = "fp32"
    c.batchSize = b
    return c


def test_deferred_builders_match_direct():
    outs = []
    for functional in (False, True):
        m = FFModel(_cfg())
        x = m.create_tensor([8, 3, 8, 8], name="x")
        if functional:
            conv = m.conv2d(3, 4, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
            assert isinstance(conv, DeferredOp)
            h = conv.init_inout(m, x)
            h = m.pool2d(2, 2, 2, 2, 0, 0).init_inout(m, h)
            h = m.flat().init_inout(m, h)
            d1 = m.dense(64, 16)
            a = d1.init_inout(m, h)
            a = m.relu().init_inout(m, a)
            b = m.dense(64, 16).init_inout(m, h)
            o = m.add().init_inout(m, [a, b])
            assert d1.get_weight_tensor().dims == (16, 64)
        else:
            h = m.conv2d(x, 4, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
            h = m.pool2d(h, 2, 2, 2, 2, 0, 0)
            h = m.flat(h)
            a = m.relu(m.dense(h, 16))
            b = m.dense(h, 16)
            o = m.add(a, b)
        o = m.softmax(m.dense(o, 4))
        m.compile(SGDOptimizer(m, 0.05), LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
        ex = m.init_layers()
        rng = np.random.RandomState(0)
        for _ in range(2):
            ex.scatter_from_host(x, rng.rand(8, 3, 8, 8).astype(np.float32))
            ex.scatter_from_host(m.get_label_tensor(), rng.randint(0, 4, (8, 1)).astype(np.int32))
            ex.train_step()
        outs.append([p.get_weights(m) for p in m.parameters])
    assert len(outs[0]) == len(outs[1])
    for a, b in zip(*outs):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)


def test_deferred_checks_and_errors():
    m = FFModel(_cfg())
    x = m.create_tensor([8, 10])
    d = m.dense(12, 4)
    with pytest.raises(AttributeError):
        d.get_weight_tensor()
    with pytest.raises(AssertionError):
        d.init_inout(m, x)          # built for 12 input features
    e = m.embedding(100, 8)
    idx = m.create_tensor([8, 1], data_type=43)
    y = e.init_inout(m, idx)
    assert y.dims == (8, 8) and e.num_entries == 100


def test_raw_ptr_attach_and_get():
    m = FFModel(_cfg(4))
    x = m.create_tensor([4, 6], name="x")
    o = m.dense(x, 2)
    m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, [])
    ex = m.init_layers()
    assert x.get_raw_ptr(m) == ex.local_buffer(x).data_ptr() != 0
    host = np.arange(24, dtype=np.float32).reshape(4, 6)
    t = x.attach_raw_ptr(m, host.ctypes.data)
    np.testing.assert_array_equal(t.numpy(), host)
    host[0, 0] = 42.0                      # zero-copy: the attached view sees host writes
    assert float(t[0, 0]) == 42.0
    cm = np.ascontiguousarray(host.T)      # reference-internal (column-major) storage
    t2 = x.attach_raw_ptr(m, cm.ctypes.data, column_major=True)
    np.testing.assert_array_equal(t2.numpy(), host)
    x.detach_raw_ptr(m)


def test_shared_op_ties_weights_like_torch():
    """dense(..., shared_op=op): one set of weights used by two layers; gradients of both uses are
    summed and applied once (checked against torch autograd with a literally shared module)."""
    import torch
    B, D = 8, 6
    m = FFModel(_cfg(B))
    x = m.create_tensor([B, D], name="x")
    h = m.dense(x, D, ActiMode.AC_MODE_RELU, name="fc")
    owner = h.owner_op
    h2 = m.dense(h, D, ActiMode.AC_MODE_NONE, shared_op=owner, name="fc_tied")
    assert h2.owner_op.weights[0] is owner.weights[0] and len(m.parameters) == 2
    o = m.softmax(m.dense(h2, 3, name="head"))
    m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    W0 = owner.weights[0].get_weights(m).copy()
    b0 = owner.weights[1].get_weights(m).copy()
    Wh = m.layers[-2].weights[0].get_weights(m).copy()
    bh = m.layers[-2].weights[1].get_weights(m).copy()
    fc = torch.nn.Linear(D, D)
    head = torch.nn.Linear(D, 3)
    with torch.no_grad():
        fc.weight.copy_(torch.from_numpy(W0)); fc.bias.copy_(torch.from_numpy(b0))
        head.weight.copy_(torch.from_numpy(Wh)); head.bias.copy_(torch.from_numpy(bh))
    opt = torch.optim.SGD(list(fc.parameters()) + list(head.parameters()), lr=0.1)
    rng = np.random.RandomState(2)
    for _ in range(3):
        xa = rng.rand(B, D).astype(np.float32)
        ya = rng.randint(0, 3, (B, 1)).astype(np.int32)
        ex.scatter_from_host(x, xa)
        ex.scatter_from_host(m.get_label_tensor(), ya)
        ex.train_step()
        opt.zero_grad()
        logits = head(fc(torch.relu(fc(torch.from_numpy(xa)))))
        torch.nn.functional.cross_entropy(logits, torch.from_numpy(ya[:, 0]).long(), reduction="sum").div(B).backward()
        opt.step()
    np.testing.assert_allclose(owner.weights[0].get_weights(m), fc.weight.detach().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(owner.weights[1].get_weights(m), fc.bias.detach().numpy(), rtol=1e-4, atol=1e-5)
