"""Teacher -> student weight transfer between functional MLPs
(reference examples/python/keras/func_mnist_mlp_net2net.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402,F401
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, concatenate)



def mlp():
    inp = Input(shape=(784,), dtype='float32')
    t = Dense(512, activation='relu')(inp)
    t = Dense(512, activation='relu')(t)
    return Model(inp, Activation('softmax')(Dense(10)(t)))


def main():
    x, y = common.mnist_flat()
    teacher = mlp()
    teacher.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    teacher.fit(x, y, epochs=epochs(1))
    student = mlp()
    student.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    for i in range(3):
        student.get_layer(index=i).set_weights(student.ffmodel, *teacher.get_layer(index=i).get_weights(teacher.ffmodel))
    student.fit(x, y, epochs=epochs(5), callbacks=keras_callbacks(ModelAccuracy.MNIST_MLP))


if __name__ == '__main__':
    main()
