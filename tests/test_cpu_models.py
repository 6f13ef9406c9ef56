"""CPU (world_size=1) end-to-end training vs PyTorch autograd oracles (reference test style:
src/ops/tests/test_harness.py -- PyTorch/numpy golden values, one SGD step included)."""
import numpy as np
import pytest
import torch

from flexmi.core import (ActiMode, AdamOptimizer, DataType, FFConfig, FFModel, LossType, MetricsType,
                         SGDOptimizer, SingleDataLoader)


def _cfg(B):
    c = FFConfig()
    c.batchSize = B
    c.device = "cpu"
    c.compute_dtype = "fp32"
    return c


def _params(m):
    return [torch.tensor(p.get_weights(m)) for p in m.parameters]


@pytest.mark.parametrize("opt", ["sgd", "sgd_mom", "adam"])
def test_mlp_matches_torch(opt):
    B = 32
    m = FFModel(_cfg(B))
    x = m.create_tensor([B, 20])
    t = m.dense(x, 64, ActiMode.AC_MODE_RELU)
    t = m.dense(t, 32, ActiMode.AC_MODE_TANH)
    t = m.dense(t, 10)
    t = m.softmax(t)
    if opt == "sgd":
        o = SGDOptimizer(m, 0.1)
    elif opt == "sgd_mom":
        o = SGDOptimizer(m, 0.05, momentum=0.9, nesterov=True, weight_decay=1e-3)
    else:
        o = AdamOptimizer(m, 0.01)
    m.compile(o, LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    m.init_layers()
    rng = np.random.RandomState(0)
    X = rng.randn(128, 20).astype(np.float32)
    Y = rng.randint(0, 10, (128, 1)).astype(np.int32)
    ps = [p.clone().requires_grad_(True) for p in _params(m)]
    if opt == "sgd":
        topt = torch.optim.SGD(ps, lr=0.1)
    elif opt == "sgd_mom":
        topt = torch.optim.SGD(ps, lr=0.05, momentum=0.9, nesterov=True, weight_decay=1e-3)
    else:
        class RefAdam:
            """Reference Adam (src/runtime/optimizer.cc:167-173, optimizer_kernel.cu:134-154):
            eps added to sqrt(v) without bias correction -- differs from torch.optim.Adam."""
            def __init__(self, ps):
                self.ps, self.t = ps, 0
                self.m = [torch.zeros_like(p) for p in ps]
                self.v = [torch.zeros_like(p) for p in ps]

            def zero_grad(self):
                for p in self.ps:
                    p.grad = None

            def step(self):
                self.t += 1
                at = 0.01 * (1 - 0.999 ** self.t) ** 0.5 / (1 - 0.9 ** self.t)
                with torch.no_grad():
                    for p, m_, v_ in zip(self.ps, self.m, self.v):
                        m_.mul_(0.9).add_(0.1 * p.grad)
                        v_.mul_(0.999).add_(0.001 * p.grad * p.grad)
                        p -= at * m_ / (v_.sqrt() + 1e-8)
        topt = RefAdam(ps)
    dx = SingleDataLoader(m, x, X, 128)
    dy = SingleDataLoader(m, m.get_label_tensor(), Y, 128)
    for it in range(6):
        dx.next_batch(m)
        dy.next_batch(m)
        m.forward()
        m.zero_gradients()
        m.backward()
        m.update()
        s = (it % 4) * B
        xb, yb = torch.tensor(X[s:s + B]), torch.tensor(Y[s:s + B]).long().view(-1)
        h = torch.relu(xb @ ps[0].t() + ps[1])
        h = torch.tanh(h @ ps[2].t() + ps[3])
        out = torch.softmax(h @ ps[4].t() + ps[5], -1)
        loss = torch.nn.functional.nll_loss(torch.log(out), yb)
        topt.zero_grad()
        loss.backward()
        topt.step()
    for a, b in zip(_params(m), ps):
        assert torch.allclose(a, b.detach(), atol=2e-5), (a - b).abs().max()


def _torch_dlrm(params, dense, sparse, D, F, inter, bot_n, top_n):
    """Pure-PyTorch DLRM (facebookresearch/dlrm semantics) on the same parameters."""
    i = 0
    x = dense
    for k in range(bot_n):
        x = torch.relu(x @ params[i].t() + params[i + 1])
        i += 2
    embs = []
    for t in range(F - 1):
        embs.append(params[i][sparse[t].view(-1)])
        i += 1
    if inter == "dot":
        Z = torch.stack([x] + embs, 1)
        G = Z @ Z.transpose(1, 2)
        li, lj = np.tril_indices(F, -1)
        z = torch.cat([x, G[:, li, lj]], 1)
        pad = params[i].shape[1] - z.shape[1]
        if pad:
            z = torch.cat([z, torch.zeros(z.shape[0], pad)], 1)
    else:
        z = torch.cat([x] + embs, 1)
    for k in range(top_n):
        z = z @ params[i].t() + params[i + 1]
        z = torch.sigmoid(z) if k == top_n - 1 else torch.relu(z)
        i += 2
    return z


@pytest.mark.parametrize("inter,loss", [("dot", "bce"), ("cat", "mse")])
def test_dlrm_matches_torch(inter, loss):
    from flexmi.models.dlrm import DLRMConfig, build_dlrm
    B = 64
    dcfg = DLRMConfig.preset("tiny")
    dcfg.arch_interaction_op = inter
    dcfg.loss = loss
    m = FFModel(_cfg(B))
    d, s, p = build_dlrm(m, dcfg)
    lt = LossType.LOSS_BINARY_CROSSENTROPY if loss == "bce" else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE
    m.compile(SGDOptimizer(m, 0.5), lt, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    # parameters in builder order: bottom linears, embeddings, top linears
    ps = [p_.clone().requires_grad_(True) for p_ in _params(m)]
    rng = np.random.RandomState(3)
    for it in range(3):
        dense = rng.rand(B, 13).astype(np.float32)
        sp = [rng.randint(0, r, (B, 1)) for r in dcfg.embedding_size]
        lab = rng.randint(0, 2, (B, 1)).astype(np.float32)
        ex.scatter_from_host(d, dense)
        for t, a in zip(s, sp):
            ex.scatter_from_host(t, a)
        ex.scatter_from_host(m.get_label_tensor(), lab)
        ex.train_step()
        out = _torch_dlrm(ps, torch.tensor(dense), [torch.tensor(a) for a in sp], dcfg.sparse_feature_size,
                          len(sp) + 1, inter, len(dcfg.mlp_bot) - 1, len(dcfg.mlp_top) - 1)
        y = torch.tensor(lab)
        if loss == "bce":
            L = torch.nn.functional.binary_cross_entropy(out, y)
        else:
            L = ((out - y) ** 2).sum() / (2 * B)   # reference MSE_AVG grad = (p - y)/B
        g = torch.autograd.grad(L, ps)
        with torch.no_grad():
            for a, gg in zip(ps, g):
                a -= 0.5 * gg
    for a, b in zip(_params(m), ps):
        assert torch.allclose(a, b.detach(), atol=1e-5), (a.shape, (a - b.detach()).abs().max())


def test_metrics_and_eval():
    B = 16
    m = FFModel(_cfg(B))
    x = m.create_tensor([B, 4])
    t = m.dense(x, 3)
    t = m.softmax(t)
    m.compile(SGDOptimizer(m, 0.0), LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              [MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    m.init_layers()
    X = np.random.RandomState(1).randn(64, 4).astype(np.float32)
    Y = np.random.RandomState(2).randint(0, 3, (64, 1)).astype(np.int32)
    dx = SingleDataLoader(m, x, X, 64)
    dy = SingleDataLoader(m, m.get_label_tensor(), Y, 64)
    m.eval((dx, dy))
    pm = m.get_perf_metrics()
    assert pm.train_all == 64
    W, b = m.parameters[0].get_weights(m), m.parameters[1].get_weights(m)
    pred = (X @ W.T + b).argmax(1)
    assert pm.train_correct == int((pred == Y[:, 0]).sum())
    assert "accuracy" in str(pm)


def test_set_get_weights_and_inline_map():
    B = 8
    m = FFModel(_cfg(B))
    x = m.create_tensor([B, 4])
    t = m.dense(x, 2)
    m.compile(SGDOptimizer(m, 0.1), LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, [])
    m.init_layers()
    W = np.arange(8, dtype=np.float32).reshape(2, 4)
    m.parameters[0].set_weights(m, W)
    assert np.array_equal(m.parameters[0].get_weights(m), W)
    arr = x.get_array(m.config, DataType.DT_FLOAT)
    arr[:] = 1.0
    x.inline_unmap(m.config)
    m.forward()
    out = m.layers[-1].outputs[0].get_array(m.config)
    assert np.allclose(out, W.sum(1)[None, :] + m.parameters[1].get_weights(m)[None, :])


# ---------------------------------------------------------------------------- model zoo
def _zoo_model(name, device="cpu", B=4, dtype=None, **kw):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer
    from flexmi.models import zoo
    cfg = FFConfig()
    cfg.batchSize = B
    cfg.device = device
    cfg.compute_dtype = dtype or ("bf16" if device == "gpu" else "fp32")
    cfg.seed = 11
    m = FFModel(cfg)
    built = zoo.build(name, m, small=True, **kw)
    m.compile(SGDOptimizer(m, built.lr * 10), built.loss, built.metrics)
    return m, built


def _zoo_feed(m, built, seed=0):
    from flexmi.core import DataType
    rng = np.random.RandomState(seed)
    ex = m._ex()
    if "dlrm" in built.extra:
        dcfg = built.extra["dlrm"]
        for i, (name, t) in enumerate(built.inputs.items()):
            if name == "dense":
                a = np.zeros(t.dims, np.float32)
                a[:, :13] = rng.rand(t.dims[0], 13)
                ex.scatter_from_host(t, a)
            else:
                ex.scatter_from_host(t, rng.randint(0, dcfg.embedding_size[i - 1], t.dims).astype(np.int64))
    elif "int_range" in built.extra:     # word ids (NMT): the label is the dst sequence itself
        for t in built.inputs.values():
            ex.scatter_from_host(t, rng.randint(0, built.extra["int_range"], t.dims).astype(np.int32))
        lab = m.get_label_tensor()
        ex.scatter_from_host(lab, rng.randint(0, built.output.dims[-1], lab.dims).astype(np.int32))
        return
    else:
        for t in built.inputs.values():
            ex.scatter_from_host(t, rng.rand(*t.dims).astype(np.float32))
    lab = m.get_label_tensor()
    if lab.data_type == DataType.DT_INT32:
        ex.scatter_from_host(lab, rng.randint(0, built.output.dims[-1], lab.dims).astype(np.int32))
    else:
        ex.scatter_from_host(lab, rng.randint(0, 2, lab.dims).astype(np.float32))


@pytest.mark.parametrize("name", ["mlp", "mnist_cnn", "cifar10_cnn", "alexnet", "inception_v3", "resnet50",
                                  "candle_uno", "dlrm", "nmt", "densenet121"])
def test_zoo_models_train_cpu(name):
    m, built = _zoo_model(name)
    m.init_layers()
    losses = []
    for it in range(2):
        _zoo_feed(m, built, it)
        m.reset_metrics()
        m._ex().train_step()
        losses.append(m.get_perf_metrics().get_loss())
    assert all(np.isfinite(losses)), losses


def test_cifar10_cnn_matches_torch():
    """flexmi CPU executor vs a plain PyTorch re-implementation (same weights): forward loss and
    one SGD step of every parameter (the reference op tests' golden style)."""
    import torch.nn.functional as F
    m, built = _zoo_model("cifar10_cnn", B=6)
    ex = m.init_layers()
    _zoo_feed(m, built, 3)
    x = torch.from_numpy(ex.gather_to_host(built.inputs["input"]))
    y = torch.from_numpy(ex.gather_to_host(m.get_label_tensor())).long().view(-1)
    params = [torch.from_numpy(p.get_weights(m)).requires_grad_(True) for p in m.parameters]
    ex.train_step()
    t = x
    pi = iter(params)
    for op in m.layers:
        kind = type(op).__name__
        if kind == "Conv2D":
            w, b = next(pi), next(pi)
            t = torch.relu(F.conv2d(t, w, b, op.sh, op.ph))
        elif kind == "Pool2D":
            t = F.max_pool2d(t, op.kh, op.sh)
        elif kind == "Flat":
            t = t.reshape(t.shape[0], -1)
        elif kind == "Linear":
            w, b = next(pi), next(pi)
            t = F.linear(t, w, b)
            if int(op.activation) == 11:
                t = torch.relu(t)
        elif kind == "Softmax":
            pass
    loss = F.cross_entropy(t, y)
    grads = torch.autograd.grad(loss, params)
    lr = m.optimizer.lr
    for p, g, prm in zip(params, grads, m.parameters):
        np.testing.assert_allclose(prm.get_weights(m), (p - lr * g).detach().numpy(), rtol=1e-4, atol=1e-5)


# ---------------------------------------------------------------------------- LSTM / NMT
def _lstm_model(device, B=4, T=5, I=8, H=16, state=False, dtype=None):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer, LossType, MetricsType
    cfg = FFConfig()
    cfg.batchSize, cfg.device = B, device
    cfg.compute_dtype = dtype or ("bf16" if device == "gpu" else "fp32")
    m = FFModel(cfg)
    x = m.create_tensor([B, T, I], name="x")
    h0 = c0 = None
    if state:
        h0 = m.create_tensor([B, H], name="h0")
        c0 = m.create_tensor([B, H], name="c0")
    y, hT, cT = m.lstm(x, H, h0, c0, name="lstm")
    out = m.reshape(y, [B, T * H], name="flat")
    m.compile(SGDOptimizer(m, 0.5), LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, [MetricsType.METRICS_MEAN_SQUARED_ERROR])
    return m, x, h0, c0, out


def test_lstm_matches_torch_lstm():
    """flexmi LSTM (CPU executor) vs torch.nn.LSTM: forward output and one SGD step."""
    B, T, I, H = 4, 5, 8, 16
    m, x, h0, c0, out = _lstm_model("cpu", B, T, I, H)
    ex = m.init_layers()
    ref = torch.nn.LSTM(I, H, batch_first=True)
    op = m.get_layer_by_name("lstm")
    with torch.no_grad():
        op.weights[0].set_weights(m, ref.weight_ih_l0.numpy())
        op.weights[1].set_weights(m, ref.weight_hh_l0.numpy())
        op.weights[2].set_weights(m, (ref.bias_ih_l0 + ref.bias_hh_l0).numpy())
    rng = np.random.RandomState(0)
    xin = rng.randn(B, T, I).astype(np.float32)
    lab = rng.randn(B, T * H).astype(np.float32)
    ex.scatter_from_host(x, xin)
    ex.scatter_from_host(m.get_label_tensor(), lab)
    m.forward()
    yr, _ = ref(torch.from_numpy(xin))
    np.testing.assert_allclose(ex.gather_to_host(out), yr.reshape(B, -1).detach().numpy(), rtol=1e-5, atol=1e-6)
    m.backward()
    m.update()
    loss = ((yr.reshape(B, -1) - torch.from_numpy(lab)) ** 2).sum(1).mean() / 2 / 1
    loss = torch.nn.functional.mse_loss(yr.reshape(B, -1), torch.from_numpy(lab), reduction="sum") / (2 * B)
    gih, ghh, gb = torch.autograd.grad(loss, [ref.weight_ih_l0, ref.weight_hh_l0, ref.bias_ih_l0])
    np.testing.assert_allclose(op.weights[0].get_weights(m), (ref.weight_ih_l0 - 0.5 * gih).detach().numpy(),
                               rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(op.weights[1].get_weights(m), (ref.weight_hh_l0 - 0.5 * ghh).detach().numpy(),
                               rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(op.weights[2].get_weights(m),
                               (ref.bias_ih_l0 + ref.bias_hh_l0 - 0.5 * gb).detach().numpy(), rtol=1e-4, atol=1e-6)
