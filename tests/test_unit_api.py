"""Pure unit tests mirroring the reference's (reference tests/ml/test_params.py,
tests/mllib/test_adapter.py, tests/utils/test_functional_utils.py,
tests/utils/test_model_utils.py, tests/utils/test_serialization.py,
tests/parameter/test_client.py) plus the ones the reference left as TODO
(rwlock, socket framing)."""
import threading
import time
from unittest.mock import patch

import numpy as np
import pytest

from elephas_amd.ml.params import *  # noqa: F401,F403
from elephas_amd.mllib.adapter import from_matrix, from_vector, to_matrix, to_vector
from elephas_amd.data.linalg import Matrices, Vectors
from elephas_amd.utils import functional_utils
from elephas_amd.utils.model_utils import LossModelTypeMapper, ModelType, ModelTypeEncoder, as_enum


# ---------------------------------------------------------------- params
@pytest.mark.parametrize("cls,getter,setter,default,new", [
    (HasMode, "get_mode", "set_mode", "asynchronous", "foobar"),
    (HasFrequency, "get_frequency", "set_frequency", "epoch", "foobar"),
    (HasNumberOfClasses, "get_nb_classes", "set_nb_classes", 10, 42),
    (HasCategoricalLabels, "get_categorical_labels", "set_categorical_labels", True, False),
    (HasEpochs, "get_epochs", "set_epochs", 10, 42),
    (HasBatchSize, "get_batch_size", "set_batch_size", 32, 42),
    (HasVerbosity, "get_verbosity", "set_verbosity", 0, 2),
    (HasValidationSplit, "get_validation_split", "set_validation_split", 0.1, 0.5),
    (HasNumberOfWorkers, "get_num_workers", "set_num_workers", 8, 12),
    (HasKerasOptimizerConfig, "get_optimizer_config", "set_optimizer_config", None, {"foo": "bar"}),
    (HasMetrics, "get_metrics", "set_metrics", ["acc"], ["mae"]),
    (HasCustomObjects, "get_custom_objects", "set_custom_objects", {}, {"f": 1}),
    (HasInferenceBatchSize, "get_inference_batch_size", "set_inference_batch_size", None, 100),
])
def test_param_defaults_and_setters(cls, getter, setter, default, new):
    p = cls()
    assert getattr(p, getter)() == default
    getattr(p, setter)(new)
    assert getattr(p, getter)() == new


def test_params_without_default():
    p = HasKerasModelConfig()
    p.set_keras_model_config({"foo": "bar"})
    assert p.get_keras_model_config() == {"foo": "bar"}
    q = HasLoss()
    with pytest.raises(KeyError):
        q.get_loss()
    q.set_loss("mse")
    assert q.get_loss() == "mse"


# --------------------------------------------------------- mllib adapter
def test_to_matrix():
    mat = to_matrix(np.ones((4, 2)))
    assert mat.numRows == 4 and mat.numCols == 2


def test_from_matrix():
    assert from_matrix(Matrices.dense(1, 2, [13, 37])).shape == (1, 2)


def test_matrix_column_major_roundtrip():
    a = np.arange(6.0).reshape(2, 3)
    assert np.array_equal(from_matrix(to_matrix(a, column_major=True)), a)
    # reference behaviour: row-major values into a column-major matrix
    assert not np.array_equal(from_matrix(to_matrix(a)), a)


def test_vectors():
    assert len(to_vector(np.ones((3,)))) == 3
    assert from_vector(Vectors.dense([4, 2])).shape == (2,)
    with pytest.raises(Exception):
        to_vector(np.ones((2, 2)))


# ------------------------------------------------------ functional utils
def test_functional_utils():
    p1 = [np.ones((5, 5)) for _ in range(10)]
    p2 = [np.ones((5, 5)) for _ in range(10)]
    assert functional_utils.add_params(p1, p2)[0][0, 0] == 2
    assert functional_utils.subtract_params(p1, p2)[0][4, 4] == 0
    assert functional_utils.get_neutral([np.ones((3, 4))])[0].sum() == 0
    assert functional_utils.divide_by([np.ones((3, 4))], num_workers=10)[0][0, 0] == 0.1


# ----------------------------------------------------------- model utils
@pytest.mark.parametrize("loss, model_type", [("binary_crossentropy", ModelType.CLASSIFICATION),
                                              ("mean_squared_error", ModelType.REGRESSION),
                                              ("categorical_crossentropy", ModelType.CLASSIFICATION),
                                              ("mean_absolute_error", ModelType.REGRESSION)])
def test_model_type_mapper(loss, model_type):
    assert LossModelTypeMapper().get_model_type(loss) == model_type


@pytest.mark.parametrize("loss", ["poisson", "cosine_similarity", "log_cosh", "MeanSquaredError", "hinge"])
def test_model_type_mapper_unlisted_is_none(loss):
    # the reference table has 11 names and answers None for every other loss
    assert LossModelTypeMapper().get_model_type(loss) is None


def test_model_type_mapper_custom():
    LossModelTypeMapper().register_loss("test", ModelType.REGRESSION)
    assert LossModelTypeMapper().get_model_type("test") == ModelType.REGRESSION

    def custom_loss(y_true, y_pred):
        return y_true - y_pred
    LossModelTypeMapper().register_loss(custom_loss, ModelType.REGRESSION)
    assert LossModelTypeMapper().get_model_type("custom_loss") == ModelType.REGRESSION
    assert LossModelTypeMapper() is LossModelTypeMapper()


def test_model_type_json_roundtrip():
    s = json.dumps({"t": ModelType.CLASSIFICATION}, cls=ModelTypeEncoder)
    assert json.loads(s, object_hook=as_enum)["t"] == ModelType.CLASSIFICATION


# --------------------------------------------------------- serialization
def test_model_to_dict_roundtrip():
    from elephas_amd.models import Sequential, Dense
    from elephas_amd.utils import serialization
    model = Sequential()
    model.build((1,))
    d = serialization.model_to_dict(model)
    assert list(d.keys()) == ["model", "weights"]
    assert serialization.dict_to_model(d).to_json() == model.to_json()
    m2 = Sequential([Dense(3, input_dim=2)])
    d2 = serialization.model_to_dict(m2)
    r2 = serialization.dict_to_model(d2)
    assert all(np.array_equal(a, b) for a, b in zip(r2.get_weights(), m2.get_weights()))


# ---------------------------------------------------------- client factory
@pytest.mark.parametrize("client_type, name", [("http", "HttpClient"), ("socket", "SocketClient")])
def test_client_factory_method(client_type, name):
    from elephas_amd.parameter import BaseParameterClient
    import elephas_amd.parameter.client as client_mod
    with patch("elephas_amd.parameter.client.socket"):
        assert type(BaseParameterClient.get_client(client_type, 4000)) == getattr(client_mod, name)
    with pytest.raises(ValueError):
        BaseParameterClient.get_client("pigeon", 4000)


def test_factory_unknown():
    from elephas_amd.parameter.factory import ClientServerFactory
    with pytest.raises(ValueError):
        ClientServerFactory.get_factory("carrier-pigeon")
    assert type(ClientServerFactory.get_factory("http")).__name__ == "HttpFactory"


# ------------------------------------------------------------------ rwlock
def test_rwlock_readers_share_writer_excludes():
    from elephas_amd.utils.rwlock import RWLock
    lock = RWLock()
    lock.acquire_read()
    lock.acquire_read()       # many readers
    got = []

    def writer():
        lock.acquire_write()
        got.append("w")
        lock.release()
    t = threading.Thread(target=writer)
    t.start()
    time.sleep(0.05)
    assert got == []          # writer waits for readers
    lock.release()
    lock.release()
    t.join(2)
    assert got == ["w"]


def test_rwlock_writer_priority_and_counter():
    from elephas_amd.utils.rwlock import RWLock
    lock = RWLock()
    counter = [0]

    def inc():
        for _ in range(200):
            lock.acquire_write()
            v = counter[0]
            counter[0] = v + 1
            lock.release()
    ts = [threading.Thread(target=inc) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert counter[0] == 1600
    with pytest.raises(RuntimeError):
        lock.release()


# --------------------------------------------------------- socket framing
def test_socket_framing_roundtrip():
    import socket
    from elephas_amd.utils.sockets import receive, send, encode, decode
    arrays = [np.arange(10, dtype=np.float32).reshape(2, 5), np.ones(3)]
    a, b = socket.socketpair()
    t = threading.Thread(target=send, args=(a, arrays))
    t.start()
    got = receive(b)
    t.join()
    assert all(np.array_equal(x, y) for x, y in zip(arrays, got))
    d = decode(encode({"delta": arrays}))
    assert list(d.keys()) == ["delta"] and np.array_equal(d["delta"][0], arrays[0])
    a.close()
    b.close()


def test_no_pickle_on_the_wire():
    import io
    import pickle
    from elephas_amd.utils.sockets import decode
    with pytest.raises(Exception):
        decode(pickle.dumps([np.ones(2)]))


def test_determine_master(monkeypatch):
    from elephas_amd.utils.sockets import determine_master
    monkeypatch.setenv("SPARK_LOCAL_IP", "10.1.2.3")
    assert determine_master(4000) == "10.1.2.3:4000"


import json  # noqa: E402
