"""A Sequential model whose layers are two smaller Sequential models
(reference examples/python/keras/seq_mnist_cnn_nested.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, Reshape, add, concatenate, subtract)



def main():
    x, y = common.mnist_images()
    features = Sequential()
    features.add(Conv2D(filters=32, input_shape=(1, 28, 28), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
                        activation='relu'))
    features.add(Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation='relu'))
    features.add(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding='valid'))
    head = Sequential()
    head.add(Flatten(input_shape=(64, 14, 14)))
    head.add(Dense(128, activation='relu'))
    head.add(Dense(10))
    head.add(Activation('softmax'))
    model = Sequential()
    model.add(features)
    model.add(head)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    print(model.summary())
    model.fit(x, y, epochs=epochs(5), callbacks=keras_callbacks(ModelAccuracy.MNIST_CNN))


if __name__ == '__main__':
    main()
