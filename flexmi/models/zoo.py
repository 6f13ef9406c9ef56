"""Model zoo: every workload of the reference behind one builder.

``build(name, model, **kw)`` adds the layers to ``model`` and returns a :class:`Built` with the
input tensors, the output, and the loss / metrics / learning rate the reference example uses.
Names: ``mlp`` / ``mnist_mlp`` (examples/python/native/mnist_mlp.py), ``mnist_cnn``,
``cifar10_cnn`` (examples/python/native/{mnist,cifar10}_cnn.py), ``alexnet``, ``inception_v3``,
``resnet50`` (examples/cpp/*), ``resnet101`` / ``densenet121`` (the standalone simulator's
builders, scripts/simulator.cc), ``nmt`` (nmt/), ``candle_uno`` (examples/cpp/candle_uno), ``dlrm-<preset>``
(examples/cpp/DLRM; presets in flexmi.models.dlrm).  ``small=True`` gives a reduced-size
instance of the same architecture for tests.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List

from flexmi.core.types import ActiMode, LossType, MetricsType

SCCE = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
ACC = [MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY]


@dataclass
class Built:
    inputs: Dict[str, object]
    output: object
    loss: LossType
    metrics: List[MetricsType] = field(default_factory=list)
    lr: float = 0.01
    extra: dict = field(default_factory=dict)


def _mlp(m, small):
    b = m.config.batchSize
    x = m.create_tensor([b, 64 if small else 784], name="input")
    t = m.dense(x, 32 if small else 512, ActiMode.AC_MODE_RELU)
    t = m.dense(t, 32 if small else 512, ActiMode.AC_MODE_RELU)
    t = m.dense(t, 10)
    t = m.softmax(t)
    return Built({"input": x}, t, SCCE, ACC, 0.01)


def _mnist_cnn(m, small):
    b = m.config.batchSize
    x = m.create_tensor([b, 1, 28, 28], name="input")
    t = m.conv2d(x, 8 if small else 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = m.conv2d(t, 16 if small else 64, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0)
    t = m.flat(t)
    t = m.dense(t, 32 if small else 128, ActiMode.AC_MODE_RELU)
    t = m.dense(t, 10)
    t = m.softmax(t)
    return Built({"input": x}, t, SCCE, ACC, 0.01)


def _cifar10_cnn(m, small):
    b = m.config.batchSize
    x = m.create_tensor([b, 3, 32, 32], name="input")
    c1, c2, d = (8, 16, 64) if small else (32, 64, 512)
    t = m.conv2d(x, c1, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = m.conv2d(t, c1, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0)
    t = m.conv2d(t, c2, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = m.conv2d(t, c2, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0)
    t = m.flat(t)
    t = m.dense(t, d, ActiMode.AC_MODE_RELU)
    t = m.dense(t, 10)
    t = m.softmax(t)
    return Built({"input": x}, t, SCCE, ACC, 0.01)


def build(name, model, small=False, **kw):
    from . import candle_uno as cu
    from . import cnn
    if name in ("mlp", "mnist_mlp"):
        return _mlp(model, small)
    if name == "mnist_cnn":
        return _mnist_cnn(model, small)
    if name == "cifar10_cnn":
        return _cifar10_cnn(model, small)
    if name == "alexnet":
        x, t = cnn.alexnet(model, image=kw.get("image", 67 if small else 229))
        return Built({"input": x}, t, SCCE, ACC, 0.001)
    if name in ("inception_v3", "inception"):
        x, t = cnn.inception_v3(model, image=kw.get("image", 139 if small else 299))
        return Built({"input": x}, t, SCCE, ACC, 0.001)
    if name in ("resnet50", "resnet"):
        x, t = cnn.resnet50(model, image=kw.get("image", 64 if small else 229), batch_norm=kw.get("batch_norm", False),
                            blocks=(1, 1, 1, 1) if small else (3, 4, 6, 3))
        return Built({"input": x}, t, SCCE, ACC, 0.001)
    if name == "densenet121":
        x, t = cnn.densenet121(model, image=kw.get("image", 32 if small else 224),
                               blocks=(1, 2, 2, 1) if small else (6, 12, 24, 16), growth=8 if small else 32)
        return Built({"input": x}, t, SCCE, ACC, 0.001)
    if name == "resnet101":
        x, t = cnn.resnet101(model, image=kw.get("image", 64 if small else 224),
                             batch_norm=kw.get("batch_norm", True))
        return Built({"input": x}, t, SCCE, ACC, 0.001)
    if name == "candle_uno":
        ins, out = cu.candle_uno(model, cu.CandleConfig.small() if small else cu.CandleConfig())
        return Built(ins, out, LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE,
                     [MetricsType.METRICS_MEAN_SQUARED_ERROR], 0.001)
    if name == "nmt":
        from . import nmt as N
        ncfg = N.NMTConfig.small() if small else N.NMTConfig()
        ins, out = N.nmt(model, ncfg)
        return Built(ins, out, SCCE, ACC, 0.01, {"int_range": ncfg.vocab})
    if name.startswith("dlrm"):
        from .dlrm import DLRMConfig, build_dlrm
        preset = name.split("-", 1)[1] if "-" in name else ("tiny" if small else "run_random")
        dcfg = DLRMConfig.preset(preset)
        d, s, out = build_dlrm(model, dcfg)
        ins = {"dense": d}
        ins.update({f"sparse{i}": t for i, t in enumerate(s)})
        loss = LossType.LOSS_BINARY_CROSSENTROPY if dcfg.loss == "bce" else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE
        return Built(ins, out, loss, [MetricsType.METRICS_ACCURACY, MetricsType.METRICS_MEAN_SQUARED_ERROR], 0.01,
                     {"dlrm": dcfg})
    raise KeyError(f"unknown model {name!r}")


NAMES = ["mlp", "mnist_cnn", "cifar10_cnn", "alexnet", "inception_v3", "resnet50", "resnet101", "densenet121",
         "candle_uno", "dlrm", "nmt"]
