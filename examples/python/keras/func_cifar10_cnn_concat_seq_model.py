"""Two Sequential towers whose outputs feed a functional graph
(model.input / model.output; reference examples/python/keras/func_cifar10_cnn_concat_seq_model.py)."""
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


def tower():
    s = Sequential()
    s.add(conv(32, input_shape=(3, 32, 32)))
    s.add(conv(32))
    return s


def main():
    x, y = common.cifar10()
    m1, m2 = tower(), tower()
    t = pool()(Concatenate(axis=1)([m1.output, m2.output]))
    t = pool()(conv(64)(conv(64)(t)))
    model = Model([m1.input[0], m2.input[0]], head(t))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    model.fit([x, x], y, epochs=epochs(40), callbacks=keras_callbacks(ModelAccuracy.CIFAR10_CNN))


if __name__ == '__main__':
    main()
