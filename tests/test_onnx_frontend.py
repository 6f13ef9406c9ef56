"""ONNX frontend: a hand-encoded ONNX graph (Conv/Relu/MaxPool/Flatten/Gemm/
Softmax + initializers) lowered onto FFModel reproduces the same network run in PyTorch."""
import numpy as np
import torch
import torch.nn.functional as F


def test_onnx_graph_matches_torch(tmp_path):
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.onnx import ONNXModel, encode_model, encode_node
    rng = np.random.RandomState(0)
    W1 = rng.randn(4, 3, 3, 3).astype(np.float32) * 0.3
    b1 = rng.randn(4).astype(np.float32)
    W2 = rng.randn(5, 64).astype(np.float32) * 0.1
    b2 = rng.randn(5).astype(np.float32)
    nodes = [
        encode_node("Conv", ["x", "W1", "b1"], ["c"], kernel_shape=[3, 3], pads=[1, 1, 1, 1], strides=[1, 1]),
        encode_node("Relu", ["c"], ["r"]),
        encode_node("MaxPool", ["r"], ["p"], kernel_shape=[2, 2], strides=[2, 2], pads=[0, 0, 0, 0]),
        encode_node("Flatten", ["p"], ["f"], axis=1),
        encode_node("Gemm", ["f", "W2", "b2"], ["g"], transB=1),
        encode_node("Softmax", ["g"], ["y"], axis=1),
    ]
    blob = encode_model(nodes, [("x", [2, 3, 8, 8])], [("y", [2, 5])], {"W1": W1, "b1": b1, "W2": W2, "b2": b2})
    path = tmp_path / "net.onnx"
    path.write_bytes(blob)
    cfg = FFConfig()
    cfg.batchSize, cfg.device, cfg.compute_dtype = 2, "cpu", "fp32"
    m = FFModel(cfg)
    x = m.create_tensor([2, 3, 8, 8])
    om = ONNXModel(str(path))
    y = om.apply(m, {"x": x})
    m.compile(SGDOptimizer(m, 0.01), LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY])
    ex = m.init_layers()
    om.copy_weights(m)
    xin = rng.rand(2, 3, 8, 8).astype(np.float32)
    ex.scatter_from_host(x, xin)
    m.forward()
    got = ex.gather_to_host(y)
    t = F.max_pool2d(torch.relu(F.conv2d(torch.from_numpy(xin), torch.from_numpy(W1), torch.from_numpy(b1), 1, 1)), 2)
    ref = torch.softmax(F.linear(t.reshape(2, -1), torch.from_numpy(W2), torch.from_numpy(b2)), 1).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
