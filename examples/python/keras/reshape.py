"""Reshape layers round-tripping 784 -> 28x28 -> 784 ahead of an MLP
(reference examples/python/keras/reshape.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, Reshape, add, concatenate, subtract)



from flexmi.keras import metrics  # noqa: E402


def main():
    x, y = common.mnist_flat()
    inp = Input(shape=(784,))
    t = Reshape(target_shape=(784,))(Reshape(target_shape=(28, 28))(inp))
    t = Dense(512, activation='relu')(t)
    t = Dense(512, activation='relu')(t)
    t = Activation('softmax')(Dense(10)(t))
    model = Model(inp, t)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy',
                  metrics=['accuracy', metrics.SparseCategoricalCrossentropy()])
    model.fit(x, y, epochs=epochs(5), callbacks=keras_callbacks(ModelAccuracy.MNIST_MLP))


if __name__ == '__main__':
    main()
