"""SparkModel integration matrix (reference tests/integration/test_end_to_end.py,
test_custom_models.py, test_model_serialization.py, test_mllib_model.py) on the
CPU torch engine with synthetic MNIST/Boston-shaped data.

Asserted like the reference: consistency, not accuracy -- predict(numpy) ==
predict(RDD) == master_network.predict (argmax), distributed evaluate ==
local evaluate within abs 0.01."""
import os
from itertools import count
from math import isclose

import numpy as np
import pytest

from elephas_amd.models import Sequential, Dense
from elephas_amd.models.optimizers import SGD, RMSprop
from elephas_amd.spark_model import SparkMLlibModel, SparkModel, load_spark_model
from elephas_amd.utils.rdd_utils import to_labeled_point, to_simple_rdd

_port = count(5200 + 97 * int(os.environ.get("PYTEST_XDIST_WORKER", "gw0")[2:] or 0))

MATRIX = [("synchronous", None, None), ("synchronous", None, 2),
          ("asynchronous", "http", None), ("asynchronous", "http", 2),
          ("asynchronous", "socket", None), ("asynchronous", "socket", 2),
          ("hogwild", "http", None), ("hogwild", "http", 2),
          ("hogwild", "socket", None), ("hogwild", "socket", 2)]


@pytest.mark.parametrize("mode,parameter_server_mode,num_workers", MATRIX)
def test_training_classification(spark_context, mode, parameter_server_mode, num_workers, mnist_data,
                                 classification_model):
    x_train, y_train, x_test, y_test = mnist_data
    x_train, y_train = x_train[:1000], y_train[:1000]
    x_test, y_test = x_test[:300], y_test[:300]
    classification_model.compile(SGD(lr=0.1), "categorical_crossentropy", ["acc"])
    rdd = to_simple_rdd(spark_context, x_train, y_train)
    spark_model = SparkModel(classification_model, frequency="epoch", num_workers=num_workers, mode=mode,
                             parameter_server_mode=parameter_server_mode or "http", port=next(_port))
    spark_model.fit(rdd, epochs=2, batch_size=64, verbose=0, validation_split=0.1)
    predictions = spark_model.predict(x_test)
    evals = spark_model.evaluate(x_test, y_test)
    test_rdd = spark_context.parallelize(x_test)
    assert [np.argmax(x) for x in predictions] == [np.argmax(x) for x in spark_model.predict(test_rdd)]
    assert [np.argmax(x) for x in predictions] == \
        [np.argmax(x) for x in spark_model.master_network.predict(x_test)]
    local = spark_model.master_network.evaluate(x_test, y_test)
    assert isclose(evals[0], local[0], abs_tol=0.01)
    assert isclose(evals[1], local[1], abs_tol=0.01)
    if mode == "synchronous":
        n = num_workers or spark_context.defaultParallelism
        assert len(spark_model.training_histories) == n


@pytest.mark.parametrize("mode,parameter_server_mode,num_workers", MATRIX[:2] + MATRIX[4:6])
def test_training_regression(spark_context, mode, parameter_server_mode, num_workers, boston_housing_dataset,
                             regression_model):
    x_train, y_train, x_test, y_test = boston_housing_dataset
    rdd = to_simple_rdd(spark_context, x_train, y_train)
    regression_model.compile(SGD(lr=0.0000001), "mse", ["mae", "mean_absolute_percentage_error"])
    spark_model = SparkModel(regression_model, frequency="epoch", mode=mode, num_workers=num_workers,
                             parameter_server_mode=parameter_server_mode or "http", port=next(_port))
    spark_model.fit(rdd, epochs=3, batch_size=64, verbose=0, validation_split=0.1)
    predictions = spark_model.predict(x_test)
    evals = spark_model.evaluate(x_test, y_test)
    test_rdd = spark_context.parallelize(x_test)
    assert all(np.isclose(x, y, 0.01) for x, y in zip(predictions, spark_model.predict(test_rdd)))
    assert all(np.isclose(x, y, 0.01) for x, y in zip(predictions, spark_model.master_network.predict(x_test)))
    local = spark_model.master_network.evaluate(x_test, y_test)
    for i in range(3):
        assert isclose(evals[i], local[i], abs_tol=0.01)


def test_training_regression_no_metrics(spark_context, boston_housing_dataset, regression_model):
    x_train, y_train, x_test, y_test = boston_housing_dataset
    rdd = to_simple_rdd(spark_context, x_train, y_train)
    regression_model.compile(SGD(lr=0.0000001), "mse")
    spark_model = SparkModel(regression_model, frequency="epoch", mode="synchronous", port=next(_port))
    spark_model.fit(rdd, epochs=1, batch_size=64, verbose=0, validation_split=0.1)
    assert isclose(spark_model.evaluate(x_test, y_test), spark_model.master_network.evaluate(x_test, y_test),
                   abs_tol=0.01)


@pytest.mark.parametrize("mode", ["synchronous", "asynchronous", "hogwild"])
@pytest.mark.parametrize("frequency", ["epoch", "batch"])
def test_training_custom_activation(mode, frequency, spark_context):
    from elephas_amd.models.backend import sigmoid

    def custom_activation(x):
        return sigmoid(x) + 1
    model = Sequential()
    model.add(Dense(1, input_dim=1, activation=custom_activation))
    model.add(Dense(1, activation="sigmoid"))
    model.compile(SGD(learning_rate=0.1), "binary_crossentropy", ["acc"])
    x_train = np.random.rand(100)
    y_train = np.zeros(100)
    x_test = np.random.rand(10)
    y_test = np.zeros(10)
    y_train[:50] = 1
    rdd = to_simple_rdd(spark_context, x_train, y_train)
    spark_model = SparkModel(model, frequency=frequency, mode=mode,
                             custom_objects={"custom_activation": custom_activation}, port=next(_port))
    spark_model.fit(rdd, epochs=1, batch_size=16, verbose=0, validation_split=0.1)
    assert spark_model.predict(x_test)
    assert spark_model.evaluate(x_test, y_test)


def test_sync_average_equals_mean_of_workers(spark_context):
    """theta = theta0 - sum(delta_i)/N (reference spark_model.py:221-227), empty partitions count."""
    from elephas_amd.worker import SparkWorker
    rng = np.random.default_rng(0)
    model = Sequential([Dense(4, input_dim=3, activation="relu"), Dense(2, activation="softmax")])
    model.compile(SGD(0.1), "categorical_crossentropy")
    w0 = model.get_weights()
    x = rng.normal(size=(90, 3)).astype(np.float32)
    y = np.eye(2, dtype=np.float32)[rng.integers(0, 2, 90)]
    rdd = spark_context.parallelize(list(zip(x, y)), 3)
    parts = rdd.partitions() + [[]]                  # plus one empty worker
    sm = SparkModel(model, mode="synchronous")
    sm.fit(spark_context.parallelize(list(zip(x, y)), 3).union(spark_context.emptyRDD()), epochs=1,
           batch_size=8, verbose=0, shuffle=False)
    # recompute independently: each partition trained alone from w0
    deltas = []
    for p in parts:
        m = Sequential([Dense(4, input_dim=3, activation="relu"), Dense(2, activation="softmax")])
        m.compile(SGD(0.1), "categorical_crossentropy")
        m.set_weights(w0)
        w = SparkWorker(m.to_json(), w0, {"epochs": 1, "batch_size": 8, "shuffle": False}, SGD(0.1),
                        "categorical_crossentropy", [], {})
        deltas.append(next(w.train(iter(p)))[0])
    assert len(sm.training_histories) == 4 and sm.training_histories[-1] is None
    expected = [w - sum(d[i] for d in deltas) / 4 for i, w in enumerate(w0)]
    for a, b in zip(sm.master_network.get_weights(), expected):
        assert np.allclose(a, b, atol=1e-6)


def test_model_serialization(tmp_cwd, spark_context, classification_model):
    classification_model.compile(optimizer="sgd", loss="categorical_crossentropy", metrics=["acc"])
    spark_model = SparkModel(classification_model, frequency="epoch", mode="synchronous", foo="bar")
    spark_model.save("elephas_sequential.h5")
    loaded = load_spark_model("elephas_sequential.h5")
    assert isinstance(loaded, SparkModel) and not isinstance(loaded, SparkMLlibModel)
    assert loaded.get_config()["foo"] == "bar"
    assert loaded.master_network.to_json() == classification_model.to_json()
    with pytest.raises(AssertionError):
        spark_model.save("model.txt")


def test_mllib_model_serialization_and_fit(tmp_cwd, spark_context, classification_model, mnist_data):
    rms = RMSprop()
    classification_model.compile(rms, "categorical_crossentropy", ["acc"])
    spark_model = SparkMLlibModel(classification_model, frequency="epoch", mode="synchronous", num_workers=2)
    spark_model.save("test.h5")
    loaded = load_spark_model("test.h5")
    assert isinstance(loaded, SparkMLlibModel) and loaded.master_network.to_json()
    x_train, y_train, x_test, y_test = mnist_data
    lp_rdd = to_labeled_point(spark_context, x_train[:600], y_train[:600], categorical=True)
    spark_model.fit(lp_rdd, epochs=2, batch_size=64, verbose=0, validation_split=0.1, categorical=True,
                    nb_classes=10)
    from elephas_amd.mllib.adapter import to_matrix, to_vector
    from elephas_amd.data.linalg import DenseMatrix, DenseVector
    pm = spark_model.predict(to_matrix(x_test[:4], column_major=True))
    assert isinstance(pm, DenseMatrix) and pm.numRows == 4 and pm.numCols == 10
    pv = spark_model.predict(to_vector(x_test[0]))
    assert isinstance(pv, DenseVector) and len(pv) == 10


def test_invalid_mode(spark_context, classification_model):
    classification_model.compile("sgd", "categorical_crossentropy")
    sm = SparkModel(classification_model, mode="synchronous")
    sm.mode = "pigeon"
    with pytest.raises(ValueError):
        sm.fit(spark_context.parallelize([(np.zeros(784), np.zeros(10))]))
    with pytest.raises(Exception):
        SparkModel(Sequential([Dense(2, input_dim=2)]))  # not compiled
