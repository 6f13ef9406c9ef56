"""CANDLE-Uno drug-response regression in the Keras API (reference
examples/python/keras/candle_uno/{candle_uno,uno}.py): one shared-shape dense tower per feature type
applied to every input of that type, concat with the raw dose inputs, a dense trunk, 1 output,
mean-squared-error.  Random features (the reference downloads the Uno data, which needs network).

    python examples/python/keras/candle_uno/candle_uno.py -b 64 [--small]
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import common  # noqa: E402

import numpy as np  # noqa: E402
from flexmi.keras import Model, optimizers  # noqa: E402
from flexmi.keras.layers import Concatenate, Dense, Input  # noqa: E402
from flexmi.models.candle_uno import CandleConfig  # noqa: E402


def build(cfg):
    inputs, encoded = [], []
    for name in sorted(cfg.input_features):
        ftype = cfg.input_features[name]
        i = Input(shape=(cfg.feature_shapes[ftype],), dtype="float32", name=name)
        inputs.append(i)
        t = i
        if ftype != "dose":
            for w in cfg.dense_feature_layers:
                t = Dense(w, activation="relu")(t)
        encoded.append(t)
    t = Concatenate(axis=1)(encoded)
    for w in cfg.dense_layers:
        t = Dense(w, activation="relu")(t)
    return Model(inputs, Dense(1)(t))


def main():
    cfg = CandleConfig.small() if "--small" in sys.argv else CandleConfig()
    n = common.num_samples(4096)
    model = build(cfg)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    rng = np.random.RandomState(0)
    xs = [rng.rand(n, cfg.feature_shapes[cfg.input_features[k]]).astype("float32") for k in sorted(cfg.input_features)]
    y = rng.rand(n, 1).astype("float32")
    hist = model.fit(xs, y, epochs=common.epochs(1))
    assert all(np.isfinite(h["loss"]) for h in hist)


if __name__ == "__main__":
    print("candle uno (keras)")
    main()
