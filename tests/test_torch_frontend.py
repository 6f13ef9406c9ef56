"""PyTorch frontend: torch.fx -> .ff -> FFModel reproduces the module's output."""
import numpy as np
import torch


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = torch.nn.Conv2d(3, 8, 3, 1, 1)
        self.conv2 = torch.nn.Conv2d(3, 8, 3, 1, 1)
        self.pool = torch.nn.MaxPool2d(2, 2)
        self.relu = torch.nn.ReLU()
        self.flat = torch.nn.Flatten()
        self.fc1 = torch.nn.Linear(16 * 4 * 4, 32)
        self.fc2 = torch.nn.Linear(32, 5)
        self.sm = torch.nn.Softmax(dim=1)

    def forward(self, x):
        a = self.relu(self.conv1(x))
        b = self.conv2(x)
        t = torch.cat([a, b], dim=1)
        t = self.pool(t)
        t = self.flat(t)
        h = self.relu(self.fc1(t))
        return self.sm(self.fc2(h) + self.fc2(h))


def test_fx_roundtrip_matches_torch(tmp_path):
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.torch import copy_weights, from_torch
    torch.manual_seed(0)
    net = Net()
    cfg = FFConfig()
    cfg.batchSize, cfg.device, cfg.compute_dtype = 4, "cpu", "fp32"
    m = FFModel(cfg)
    x = m.create_tensor([4, 3, 8, 8])
    outs, pm = from_torch(net, m, [x], filename=str(tmp_path / "net.ff"))
    text = (tmp_path / "net.ff").read_text()
    assert "2011" in text and "2016, 1" in text and "2051" in text   # conv2d, concat(axis 1), output
    m.compile(SGDOptimizer(m, 0.01), LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    copy_weights(net, m, pm)
    xin = np.random.RandomState(1).rand(4, 3, 8, 8).astype(np.float32)
    ex.scatter_from_host(x, xin)
    m.forward()
    got = ex.gather_to_host(outs[0])
    ref = net(torch.from_numpy(xin)).detach().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
