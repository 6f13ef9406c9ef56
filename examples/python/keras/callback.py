"""LearningRateScheduler + accuracy callbacks on a functional CIFAR-10 CNN
(reference examples/python/keras/callback.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, Reshape, add, concatenate, subtract)



from flexmi.keras.callbacks import LearningRateScheduler  # noqa: E402


def schedule(epoch):
    return 0.01 if epoch == 0 else 0.02


def main():
    x, y = common.cifar10()
    inp = Input(shape=(3, 32, 32), dtype='float32')
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation='relu')(inp)
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation='relu')(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding='valid')(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation='relu')(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation='relu')(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding='valid')(t)
    t = Activation('softmax')(Dense(10)(Dense(512, activation='relu')(Flatten()(t))))
    model = Model(inp, t)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.02), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    model.fit(x, y, epochs=epochs(40),
              callbacks=[LearningRateScheduler(schedule)] + keras_callbacks(ModelAccuracy.CIFAR10_CNN))


if __name__ == '__main__':
    main()
