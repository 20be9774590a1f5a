"""Test configuration.

Markers: ``gpu`` = needs an MI355X (run with ``-m gpu`` on the GPU box); every
other test runs on CPU (torch reference engine, gloo for multi-process).
Fixtures mirror the reference's (reference tests/conftest.py:8-63) with
synthetic data of the same shapes (no network: MNIST/Boston are not available).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU (native HIP engine)")
    config.addinivalue_line("markers", "slow: longer-running test")


@pytest.fixture(autouse=True)
def _fresh_names():
    from elephas_amd.models.layers import clear_session
    clear_session()
    yield


@pytest.fixture(autouse=True)
def _gpu_isolation(request):
    """After every GPU test: a device synchronisation (an asynchronous device error is charged
    to the test that caused it, as a teardown error, not to whichever later test first
    touches the device) and a garbage collection (the test's trainers -- executors, loaders,
    streams -- are destroyed at the boundary, not inside a later test)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        gc.collect()
        torch.cuda.synchronize()


@pytest.fixture
def classification_model():
    from elephas_amd.models import Sequential, Dense, Activation, Dropout
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


@pytest.fixture
def regression_model():
    from elephas_amd.models import Sequential, Dense
    model = Sequential()
    model.add(Dense(64, activation='relu', input_shape=(13,)))
    model.add(Dense(64, activation='relu'))
    model.add(Dense(1, activation='linear'))
    return model


@pytest.fixture
def classification_model_functional():
    from elephas_amd.models import Input, Dense, Dropout, Model
    input_layer = Input(shape=(784,))
    hidden = Dense(128, activation='relu')(input_layer)
    dropout = Dropout(0.2)(hidden)
    hidden2 = Dense(128, activation='relu')(dropout)
    dropout2 = Dropout(0.2)(hidden2)
    output = Dense(10, activation='softmax')(dropout2)
    return Model(inputs=input_layer, outputs=output)


@pytest.fixture(scope='session')
def mnist_data():
    """Synthetic MNIST-shaped data (60000x784 would be slow on CPU: 6000/1000 rows)."""
    from elephas_amd.models.datasets import synthetic_classification
    from elephas_amd.models.utils import to_categorical
    x, y = synthetic_classification(7000, 784, 10, seed=42)
    x = (x - x.min()) / (x.max() - x.min())
    y = to_categorical(y, 10)
    return x[:6000].astype(np.float32), y[:6000], x[6000:].astype(np.float32), y[6000:]


@pytest.fixture(scope='session')
def boston_housing_dataset():
    from elephas_amd.models.datasets import boston_housing
    (x_train, y_train), (x_test, y_test) = boston_housing.load_data()
    return x_train, y_train, x_test, y_test


@pytest.fixture
def spark_context():
    from elephas_amd.data import SparkContext
    sc = SparkContext.getOrCreate()
    yield sc


@pytest.fixture
def tmp_cwd(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    return tmp_path
