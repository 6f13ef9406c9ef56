"""Functional CIFAR-10 CNN composed of two sub-models
(reference examples/python/keras/func_cifar10_cnn_nested.py)."""
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
    i1 = Input(shape=(3, 32, 32), dtype='float32')
    features = Model(i1, pool()(conv(32)(conv(32)(i1))))
    i2 = Input(shape=(32, 16, 16), dtype='float32')
    classifier = Model(i2, head(pool()(conv(64)(conv(64)(i2)))))
    inp = Input(shape=(3, 32, 32), dtype='float32')
    model = Model(inp, classifier(features(inp)))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    print(model.summary())
    model.fit(x, y, epochs=epochs(40), callbacks=keras_callbacks(ModelAccuracy.CIFAR10_CNN))


if __name__ == '__main__':
    main()
