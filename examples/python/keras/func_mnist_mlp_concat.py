"""Functional MNIST MLP with concatenated towers over two inputs
(reference examples/python/keras/func_mnist_mlp_concat.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402,F401
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, concatenate)



def main():
    x, y = common.mnist_flat()
    a = Input(shape=(784,), dtype='float32')
    b = Input(shape=(784,), dtype='float32')
    ta = Dense(512, activation='relu')(Dense(512, activation='relu')(a))
    tb = Dense(512, activation='relu')(Dense(512, activation='relu')(b))
    t = Concatenate(axis=1)([ta, tb])
    model = Model([a, b], Activation('softmax')(Dense(10)(t)))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    model.fit([x, x], y, epochs=epochs(20), callbacks=keras_callbacks(ModelAccuracy.MNIST_MLP))


if __name__ == '__main__':
    main()
