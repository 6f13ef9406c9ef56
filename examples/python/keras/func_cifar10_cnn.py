"""Functional CIFAR-10 CNN (reference examples/python/keras/func_cifar10_cnn.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402,F401
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, concatenate)



def conv(filters, **kw):
    return Conv2D(filters=filters, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu", **kw)


def pool():
    return MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")


def head(t, hidden=512):
    return Activation("softmax")(Dense(10)(Dense(hidden, activation="relu")(Flatten()(t))))


def main():
    x, y = common.cifar10()
    inp = Input(shape=(3, 32, 32), dtype='float32')
    t = pool()(conv(32)(conv(32)(inp)))
    t = pool()(conv(64)(conv(64)(t)))
    model = Model(inp, head(t))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    model.fit(x, y, epochs=epochs(40), callbacks=keras_callbacks(ModelAccuracy.CIFAR10_CNN))


if __name__ == '__main__':
    main()
