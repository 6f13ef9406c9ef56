"""CNN model builders with the reference example architectures.

* AlexNet      -- ``examples/cpp/AlexNet/alexnet.cc:60-77`` (5 conv + 3 pool + 3 dense + softmax,
  input 3x229x229, 10 classes, SGD lr 0.001, sparse CCE)
* InceptionV3  -- ``examples/cpp/InceptionV3/inception.cc:26-174`` (stem, A x3, B, C x4, D, E x2,
  8x8 avg pool, dense 10; input 3x299x299)
* ResNet-50    -- ``examples/cpp/ResNet/resnet.cc:34-110`` (bottlenecks 3-4-6-3 with additive
  residuals; batch norm commented out in the reference, optional here)

All take an FFModel and return (input tensor, output tensor).  ``scale`` shrinks the image side
(tests use tiny images; the architecture is unchanged).
"""
from __future__ import annotations

from flexmi.core.types import ActiMode, PoolType

RELU = ActiMode.AC_MODE_RELU
NONE = ActiMode.AC_MODE_NONE


def alexnet(model, batch=None, image=229, num_classes=10):
    b = batch or model.config.batchSize
    x = model.create_tensor([b, 3, image, image], name="input")
    t = model.conv2d(x, 64, 11, 11, 4, 4, 2, 2, RELU, name="conv1")
    t = model.pool2d(t, 3, 3, 2, 2, 0, 0, name="pool1")
    t = model.conv2d(t, 192, 5, 5, 1, 1, 2, 2, RELU, name="conv2")
    t = model.pool2d(t, 3, 3, 2, 2, 0, 0, name="pool2")
    t = model.conv2d(t, 384, 3, 3, 1, 1, 1, 1, RELU, name="conv3")
    t = model.conv2d(t, 256, 3, 3, 1, 1, 1, 1, RELU, name="conv4")
    t = model.conv2d(t, 256, 3, 3, 1, 1, 1, 1, RELU, name="conv5")
    t = model.pool2d(t, 3, 3, 2, 2, 0, 0, name="pool3")
    t = model.flat(t, name="flat")
    t = model.dense(t, 4096, RELU, name="fc6")
    t = model.dense(t, 4096, RELU, name="fc7")
    t = model.dense(t, num_classes, name="fc8")
    t = model.softmax(t, name="softmax")
    return x, t


def _inception_a(m, x, pool_features):
    t1 = m.conv2d(x, 64, 1, 1, 1, 1, 0, 0, RELU)
    t2 = m.conv2d(x, 48, 1, 1, 1, 1, 0, 0, RELU)
    t2 = m.conv2d(t2, 64, 5, 5, 1, 1, 2, 2, RELU)
    t3 = m.conv2d(x, 64, 1, 1, 1, 1, 0, 0, RELU)
    t3 = m.conv2d(t3, 96, 3, 3, 1, 1, 1, 1, RELU)
    t3 = m.conv2d(t3, 96, 3, 3, 1, 1, 1, 1, RELU)
    t4 = m.pool2d(x, 3, 3, 1, 1, 1, 1, PoolType.POOL_AVG)
    t4 = m.conv2d(t4, pool_features, 1, 1, 1, 1, 0, 0, RELU)
    return m.concat([t1, t2, t3, t4], 1)


def _inception_b(m, x):
    t1 = m.conv2d(x, 384, 3, 3, 2, 2, 0, 0)
    t2 = m.conv2d(x, 64, 1, 1, 1, 1, 0, 0)
    t2 = m.conv2d(t2, 96, 3, 3, 1, 1, 1, 1)
    t2 = m.conv2d(t2, 96, 3, 3, 2, 2, 0, 0)
    t3 = m.pool2d(x, 3, 3, 2, 2, 0, 0)
    return m.concat([t1, t2, t3], 1)


def _inception_c(m, x, ch):
    t1 = m.conv2d(x, 192, 1, 1, 1, 1, 0, 0)
    t2 = m.conv2d(x, ch, 1, 1, 1, 1, 0, 0)
    t2 = m.conv2d(t2, ch, 1, 7, 1, 1, 0, 3)
    t2 = m.conv2d(t2, 192, 7, 1, 1, 1, 3, 0)
    t3 = m.conv2d(x, ch, 1, 1, 1, 1, 0, 0)
    t3 = m.conv2d(t3, ch, 7, 1, 1, 1, 3, 0)
    t3 = m.conv2d(t3, ch, 1, 7, 1, 1, 0, 3)
    t3 = m.conv2d(t3, ch, 7, 1, 1, 1, 3, 0)
    t3 = m.conv2d(t3, 192, 1, 7, 1, 1, 0, 3)
    t4 = m.pool2d(x, 3, 3, 1, 1, 1, 1, PoolType.POOL_AVG)
    t4 = m.conv2d(t4, 192, 1, 1, 1, 1, 0, 0)
    return m.concat([t1, t2, t3, t4], 1)


def _inception_d(m, x):
    t1 = m.conv2d(x, 192, 1, 1, 1, 1, 0, 0)
    t1 = m.conv2d(t1, 320, 3, 3, 2, 2, 0, 0)
    t2 = m.conv2d(x, 192, 1, 1, 1, 1, 0, 0)
    t2 = m.conv2d(t2, 192, 1, 7, 1, 1, 0, 3)
    t2 = m.conv2d(t2, 192, 7, 1, 1, 1, 3, 0)
    t2 = m.conv2d(t2, 192, 3, 3, 2, 2, 0, 0)
    t3 = m.pool2d(x, 3, 3, 2, 2, 0, 0)
    return m.concat([t1, t2, t3], 1)


def _inception_e(m, x):
    t1 = m.conv2d(x, 320, 1, 1, 1, 1, 0, 0)
    t2i = m.conv2d(x, 384, 1, 1, 1, 1, 0, 0)
    t2 = m.conv2d(t2i, 384, 1, 3, 1, 1, 0, 1)
    t3 = m.conv2d(t2i, 384, 3, 1, 1, 1, 1, 0)
    t3i = m.conv2d(x, 448, 1, 1, 1, 1, 0, 0)
    t3i = m.conv2d(t3i, 384, 3, 3, 1, 1, 1, 1)
    t4 = m.conv2d(t3i, 384, 1, 3, 1, 1, 0, 1)
    t5 = m.conv2d(t3i, 384, 3, 1, 1, 1, 1, 0)
    t6 = m.pool2d(x, 3, 3, 1, 1, 1, 1, PoolType.POOL_AVG)
    t6 = m.conv2d(t6, 192, 1, 1, 1, 1, 0, 0)
    return m.concat([t1, t2, t3, t4, t5, t6], 1)


def inception_v3(model, batch=None, image=299, num_classes=10):
    b = batch or model.config.batchSize
    x = model.create_tensor([b, 3, image, image], name="input")
    m = model
    t = m.conv2d(x, 32, 3, 3, 2, 2, 0, 0, RELU)
    t = m.conv2d(t, 32, 3, 3, 1, 1, 0, 0, RELU)
    t = m.conv2d(t, 64, 3, 3, 1, 1, 1, 1, RELU)
    t = m.pool2d(t, 3, 3, 2, 2, 0, 0)
    t = m.conv2d(t, 80, 1, 1, 1, 1, 0, 0, RELU)
    t = m.conv2d(t, 192, 3, 3, 1, 1, 1, 1, RELU)
    t = m.pool2d(t, 3, 3, 2, 2, 0, 0)
    t = _inception_a(m, t, 32)
    t = _inception_a(m, t, 64)
    t = _inception_a(m, t, 64)
    t = _inception_b(m, t)
    t = _inception_c(m, t, 128)
    t = _inception_c(m, t, 160)
    t = _inception_c(m, t, 160)
    t = _inception_c(m, t, 192)
    t = _inception_d(m, t)
    t = _inception_e(m, t)
    t = _inception_e(m, t)
    k = t.dims[2]      # 8 at 299x299
    t = m.pool2d(t, k, k, 1, 1, 0, 0, PoolType.POOL_AVG)
    t = m.flat(t)
    t = m.dense(t, num_classes)
    t = m.softmax(t)
    return x, t


def _bottleneck(m, x, out_channels, stride, batch_norm):
    t = m.conv2d(x, out_channels, 1, 1, 1, 1, 0, 0, NONE)
    if batch_norm:
        t = m.batch_norm(t)
    t = m.conv2d(t, out_channels, 3, 3, stride, stride, 1, 1, NONE)
    if batch_norm:
        t = m.batch_norm(t)
    t = m.conv2d(t, 4 * out_channels, 1, 1, 1, 1, 0, 0)
    if batch_norm:
        t = m.batch_norm(t, relu=False)
    if stride > 1 or x.dims[1] != 4 * out_channels:
        x = m.conv2d(x, 4 * out_channels, 1, 1, stride, stride, 0, 0, NONE)
        if batch_norm:
            x = m.batch_norm(x, relu=False)
    t = m.add(x, t)
    return m.relu(t)


def resnet50(model, batch=None, image=229, num_classes=10, batch_norm=False, blocks=(3, 4, 6, 3)):
    b = batch or model.config.batchSize
    x = model.create_tensor([b, 3, image, image], name="input")
    m = model
    t = m.conv2d(x, 64, 7, 7, 2, 2, 3, 3)
    if batch_norm:
        t = m.batch_norm(t)
    t = m.pool2d(t, 3, 3, 2, 2, 1, 1)
    for stage, (n, ch) in enumerate(zip(blocks, (64, 128, 256, 512))):
        for i in range(n):
            t = _bottleneck(m, t, ch, 2 if (i == 0 and stage > 0) else 1, batch_norm)
    k = t.dims[2]      # 7 at 229x229
    t = m.pool2d(t, k, k, 1, 1, 0, 0, PoolType.POOL_AVG)
    t = m.flat(t)
    t = m.dense(t, num_classes)
    t = m.softmax(t)
    return x, t


# ------------------------------------------------------------------ DenseNet-121
# The reference's standalone SOAP simulator builds DenseNet-121 (scripts/simulator.cc model
# builders): dense blocks of (BN-ReLU-Conv1x1(4k)-BN-ReLU-Conv3x3(k)) whose outputs are
# concatenated onto the block input, transitions BN-Conv1x1(theta=0.5)-AvgPool2, growth k = 32.
def _dense_layer(m, x, growth):
    t = m.batch_norm(x)
    t = m.conv2d(t, 4 * growth, 1, 1, 1, 1, 0, 0, NONE, use_bias=False)
    t = m.batch_norm(t)
    t = m.conv2d(t, growth, 3, 3, 1, 1, 1, 1, NONE, use_bias=False)
    return m.concat([x, t], 1)


def densenet121(model, batch=None, image=224, num_classes=10, growth=32, blocks=(6, 12, 24, 16)):
    b = batch or model.config.batchSize
    x = model.create_tensor([b, 3, image, image], name="input")
    m = model
    t = m.conv2d(x, 2 * growth, 7, 7, 2, 2, 3, 3, NONE, use_bias=False)
    t = m.batch_norm(t)
    t = m.pool2d(t, 3, 3, 2, 2, 1, 1)
    for bi, n in enumerate(blocks):
        for _ in range(n):
            t = _dense_layer(m, t, growth)
        if bi != len(blocks) - 1:
            c = t.dims[1] // 2
            t = m.batch_norm(t)
            t = m.conv2d(t, c, 1, 1, 1, 1, 0, 0, NONE, use_bias=False)
            t = m.pool2d(t, 2, 2, 2, 2, 0, 0, PoolType.POOL_AVG)
    t = m.batch_norm(t)
    k = t.dims[2]
    t = m.pool2d(t, k, k, 1, 1, 0, 0, PoolType.POOL_AVG)
    t = m.flat(t)
    t = m.dense(t, num_classes)
    t = m.softmax(t)
    return x, t


def resnet101(model, batch=None, image=224, num_classes=10, batch_norm=True):
    """ResNet-101 (bottlenecks 3-4-23-3), the standalone simulator's ResNet builder."""
    return resnet50(model, batch, image, num_classes, batch_norm, blocks=(3, 4, 23, 3))
