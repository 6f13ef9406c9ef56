"""Sequential Reuters newswire MLP, 46 topics (reference examples/python/keras/seq_reuters_mlp.py)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import common  # noqa: E402,F401
from common import ModelAccuracy, epochs, keras_callbacks  # noqa: E402

from flexmi.keras import Model, Sequential, optimizers  # noqa: E402
from flexmi.keras.layers import (Activation, Concatenate, Conv2D, Dense, Flatten, Input,  # noqa: E402,F401
                                 MaxPooling2D, Reshape, add, concatenate, subtract)



def main():
    x, y = common.reuters()
    model = Sequential([Dense(512, input_shape=(1000,), activation='relu'), Dense(46), Activation('softmax')])
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss='sparse_categorical_crossentropy', metrics=['accuracy', 'sparse_categorical_crossentropy'])
    model.fit(x, y, epochs=epochs(20), callbacks=keras_callbacks(ModelAccuracy.REUTERS_MLP))


if __name__ == '__main__':
    main()
