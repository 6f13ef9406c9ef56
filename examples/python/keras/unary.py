"""Element-wise merge layers (Add / subtract) in functional graphs that are compiled and
initialised (reference examples/python/keras/unary.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, Reshape, add, concatenate, subtract)



from flexmi.keras.layers import Add  # noqa: E402


def two_branch(merge):
    a = Input(shape=(16,), dtype='float32')
    b = Input(shape=(32,), dtype='float32')
    t = merge([Dense(8, activation='relu')(a), Dense(8, activation='relu')(b)])
    model = Model([a, b], Dense(4)(t))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    print(model.summary())
    model.ffmodel.init_layers()
    return model


def main():
    two_branch(Add())
    two_branch(subtract)


if __name__ == '__main__':
    main()
