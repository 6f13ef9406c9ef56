"""Teacher -> student weight transfer between two Sequential MLPs
(reference examples/python/keras/seq_mnist_mlp_net2net.py): get_weights / set_weights per layer."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, Reshape, add, concatenate, subtract)



import numpy as np  # noqa: E402


def mlp():
    return Sequential([Dense(512, input_shape=(784,), activation='relu'), Dense(512, activation='relu'),
                       Dense(10), Activation('softmax')])


def main():
    x, y = common.mnist_flat()
    teacher = mlp()
    teacher.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    teacher.fit(x, y, epochs=epochs(1))
    weights = [teacher.get_layer(index=i).get_weights(teacher.ffmodel) for i in range(3)]
    student = mlp()
    student.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    for i, (k, b) in enumerate(weights):
        student.get_layer(index=i).set_weights(student.ffmodel, k, b)
    k, b = student.get_layer(index=2).get_weights(student.ffmodel)
    assert np.array_equal(k, weights[2][0]) and np.array_equal(b, weights[2][1])
    student.fit(x, y, epochs=epochs(5), callbacks=keras_callbacks(ModelAccuracy.MNIST_MLP))


if __name__ == '__main__':
    main()
