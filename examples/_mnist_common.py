"""Shared MNIST setup of the MNIST examples (reference examples/mnist_mlp_spark*.py:1-48).

``keras.datasets.mnist`` has no network here: ``load_data`` reads
``~/.keras/datasets/mnist.npz`` when present, else synthetic MNIST-shaped data.
``EXAMPLE_ROWS`` (env) trims the training set for quick runs.
"""
import os

from elephas_amd.keras.datasets import mnist
from elephas_amd.keras.layers import Activation, Dense, Dropout
from elephas_amd.keras.models import Sequential
from elephas_amd.keras.utils import to_categorical

batch_size = 64
nb_classes = 10


def load():
    (x_train, y_train), (x_test, y_test) = mnist.load_data()
    rows = int(os.environ.get("EXAMPLE_ROWS", "60000"))
    x_train = x_train.reshape(-1, 784)[:rows].astype("float32") / 255
    x_test = x_test.reshape(-1, 784).astype("float32") / 255
    y_train = to_categorical(y_train[:rows], nb_classes)
    y_test = to_categorical(y_test, nb_classes)
    print(x_train.shape[0], 'train samples')
    print(x_test.shape[0], 'test samples')
    return x_train, y_train, x_test, y_test


def mlp():
    model = Sequential()
    model.add(Dense(128, input_dim=784))
    model.add(Activation('relu'))
    model.add(Dropout(0.2))
    model.add(Dense(128))
    model.add(Activation('relu'))
    model.add(Dropout(0.2))
    model.add(Dense(10))
    model.add(Activation('softmax'))
    return model
