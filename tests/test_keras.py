"""Keras frontend: Sequential + functional models train through flexmi."""
import numpy as np
import pytest


def _cfg(b=64):
    from flexmi.core import FFConfig
    c = FFConfig()
    c.batchSize = b
    c.device = "cpu"
    c.compute_dtype = "fp32"
    return c


def test_sequential_mlp_learns_synthetic_mnist():
    from flexmi.keras import Sequential, datasets, optimizers
    from flexmi.keras.callbacks import VerifyMetrics
    from flexmi.keras.layers import Activation, Dense
    (x, y), _ = datasets.mnist.load_data(1024)
    x = x.reshape(len(x), 784).astype("float32") / 255
    y = y.astype("int32").reshape(-1, 1)
    model = Sequential([Dense(64, input_shape=(784,), activation="relu"), Dense(10), Activation("softmax")],
                       ffconfig=_cfg())
    model.compile(optimizer=optimizers.SGD(learning_rate=0.1), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    assert "dense" in model.summary()
    hist = model.fit(x, y, epochs=4, callbacks=[VerifyMetrics(80.0)], verbose=0)
    assert hist[-1]["accuracy"] > hist[0]["accuracy"]
    ev = model.evaluate(x, y, verbose=0)
    assert ev[0]["accuracy"] > 80.0


def test_functional_two_input_cnn_concat_and_callbacks():
    from flexmi.keras import Model, optimizers
    from flexmi.keras.callbacks import EpochVerifyMetrics, LearningRateScheduler
    from flexmi.keras.layers import Activation, Concatenate, Conv2D, Dense, Flatten, Input, MaxPooling2D, add
    rng = np.random.RandomState(0)
    n = 128
    x1 = rng.rand(n, 3, 8, 8).astype("float32")
    x2 = rng.rand(n, 3, 8, 8).astype("float32")
    y = (x1.mean((1, 2, 3)) > x2.mean((1, 2, 3))).astype("int32").reshape(-1, 1)
    i1 = Input(shape=(3, 8, 8), name="in1")
    i2 = Input(shape=(3, 8, 8), name="in2")
    a = Conv2D(filters=4, kernel_size=(3, 3), padding=(1, 1), activation="relu")(i1)
    b = Conv2D(filters=4, kernel_size=(3, 3), padding="same", activation="relu")(i2)
    t = Concatenate(axis=1)([a, b])
    t = MaxPooling2D(pool_size=(2, 2))(t)
    t = Flatten()(t)
    u = Dense(16, activation="relu")(t)
    v = Dense(16, activation="relu")(t)
    t = add([u, v])
    t = Dense(2)(t)
    out = Activation("softmax")(t)
    model = Model([i1, i2], out, ffconfig=_cfg(32))
    opt = optimizers.Adam(learning_rate=0.01)
    model.compile(optimizer=opt, loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    lrs = []
    sched = LearningRateScheduler(lambda e: 0.01 * (0.5 ** e))

    class Rec(LearningRateScheduler):
        def on_epoch_begin(self, epoch, logs=None):
            super().on_epoch_begin(epoch, logs)
            lrs.append(self.model.optimizer.lr)
    hist = model.fit([x1, x2], y, epochs=3, callbacks=[Rec(sched.schedule), EpochVerifyMetrics(101.0)], verbose=0)
    assert lrs == pytest.approx([0.01, 0.005, 0.0025])
    assert len(hist) == 3 and all(np.isfinite(h["loss"]) for h in hist)
    assert [lay.name for lay in model.layers][:2] != []
