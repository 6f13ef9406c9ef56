"""Functional MLP built from sub-models (one of them itself nested), joined
with raw inputs by a 6-way concat (reference examples/python/keras/func_mnist_mlp_concat2.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402,F401
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, concatenate)



def tower(width, depth, in_dim=784):
    i = Input(shape=(in_dim,))
    t = i
    for _ in range(depth):
        t = Dense(width, activation='relu')(t)
    return Model(i, t)


def main():
    x, y = common.mnist_flat()
    inner = tower(512, 1)
    i1 = Input(shape=(784,))
    m1 = Model(i1, Dense(512, activation='relu')(inner(i1)))       # nested: tower inside a model
    towers = [m1] + [tower(512, 2) for _ in range(3)]
    inp = Input(shape=(784,))
    raw0, raw1 = Input(shape=(784,), name='input_00'), Input(shape=(784,), name='input_01')
    t = Concatenate(axis=1)([raw0, raw1] + [m(inp) for m in towers])
    model = Model([raw0, raw1, inp], Activation('softmax')(Dense(10)(t)))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    print(model.summary())
    model.fit([x, x, x], y, epochs=epochs(20), callbacks=keras_callbacks(ModelAccuracy.MNIST_MLP))


if __name__ == '__main__':
    main()
