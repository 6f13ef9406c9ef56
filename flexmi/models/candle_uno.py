"""CANDLE-Uno (``examples/cpp/candle_uno/candle_uno.cc:48-166``, ``candle_uno.h:22-37``).

Per-input feature towers (3 x dense 1000 relu) for cell / drug features, concat with the raw
dose inputs, 3 x dense 1000 relu, dense 1, MSE-average loss, SGD lr 0.001.  Inputs are visited
in the reference's ``std::map`` (sorted key) order.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List

from flexmi.core.types import ActiMode


@dataclass
class CandleConfig:
    dense_layers: List[int] = field(default_factory=lambda: [1000, 1000, 1000])
    dense_feature_layers: List[int] = field(default_factory=lambda: [1000, 1000, 1000])
    feature_shapes: Dict[str, int] = field(default_factory=lambda: {
        "dose": 1, "cell.rnaseq": 942, "drug.descriptors": 5270, "drug.fingerprints": 2048})
    input_features: Dict[str, str] = field(default_factory=lambda: {
        "dose1": "dose", "dose2": "dose", "cell.rnaseq": "cell.rnaseq",
        "drug1.descriptors": "drug.descriptors", "drug1.fingerprints": "drug.fingerprints",
        "drug2.descriptors": "drug.descriptors", "drug2.fingerprints": "drug.fingerprints"})

    @staticmethod
    def small():
        c = CandleConfig([32, 32], [16, 16])
        c.feature_shapes = {"dose": 1, "cell.rnaseq": 24, "drug.descriptors": 40, "drug.fingerprints": 16}
        return c


def candle_uno(model, cfg: CandleConfig = None, batch=None):
    """Returns (inputs dict name -> tensor, output tensor)."""
    cfg = cfg or CandleConfig()
    b = batch or model.config.batchSize
    towers = {k for k in cfg.feature_shapes if k.split(".")[0] in ("cell", "drug") and "." in k}
    inputs, encoded = {}, []
    for name in sorted(cfg.input_features):
        ftype = cfg.input_features[name]
        t = model.create_tensor([b, cfg.feature_shapes[ftype]], name=name)
        inputs[name] = t
        if ftype in towers:
            for i, d in enumerate(cfg.dense_feature_layers):
                t = model.dense(t, d, ActiMode.AC_MODE_RELU, name=f"{name}.dense{i}")
        encoded.append(t)
    out = model.concat(encoded, 1, name="concat")
    for i, d in enumerate(cfg.dense_layers):
        out = model.dense(out, d, ActiMode.AC_MODE_RELU, name=f"dense{i}")
    out = model.dense(out, 1, name="out")
    return inputs, out
