"""Functional AlexNet on CIFAR-10 images upsampled (nearest) to 229x229
(reference examples/python/keras/func_cifar10_alexnet.py; no PIL needed: index-based resize)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402,F401
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, concatenate)



import numpy as np  # noqa: E402


def upsample(x, size=229):
    idx = (np.arange(size) * x.shape[-1]) // size
    return np.ascontiguousarray(x[:, :, idx][:, :, :, idx])


def main():
    x, y = common.cifar10()
    x = upsample(x)
    inp = Input(shape=(3, 229, 229), dtype='float32')
    t = Conv2D(filters=64, kernel_size=(11, 11), strides=(4, 4), padding=(2, 2), activation='relu')(inp)
    t = MaxPooling2D(pool_size=(3, 3), strides=(2, 2), padding='valid')(t)
    t = Conv2D(filters=192, kernel_size=(5, 5), strides=(1, 1), padding=(2, 2), activation='relu')(t)
    t = MaxPooling2D(pool_size=(3, 3), strides=(2, 2), padding='valid')(t)
    t = Conv2D(filters=384, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation='relu')(t)
    t = Conv2D(filters=256, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation='relu')(t)
    t = Conv2D(filters=256, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation='relu')(t)
    t = MaxPooling2D(pool_size=(3, 3), strides=(2, 2), padding='valid')(t)
    t = Dense(4096, activation='relu')(Flatten()(t))
    t = Dense(4096, activation='relu')(t)
    model = Model(inp, Activation('softmax')(Dense(10)(t)))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    model.fit(x, y, epochs=epochs(40), callbacks=keras_callbacks(ModelAccuracy.CIFAR10_ALEXNET))


if __name__ == '__main__':
    main()
