"""Spark-ML API: ElephasEstimator / ElephasTransformer inside a Pipeline.

Mirrors reference tests/test_ml_model.py:29-376 (serialization round trips,
classification / functional / regression pipelines, deprecated column setters,
constructor columns, custom objects, class-probability output, batched ==
unbatched inference, pipeline save) on synthetic MNIST/Boston-shaped data.
Runs on the CPU torch engine (GPU-only paths are in test_native_gpu.py).
"""
import numpy as np
import pytest

from elephas_amd.data import Pipeline, DoubleType
from elephas_amd.data import functions as F
from elephas_amd.data.ml import MulticlassMetrics, RegressionMetrics
from elephas_amd.ml.adapter import to_data_frame
from elephas_amd.ml_model import ElephasEstimator, ElephasTransformer, load_ml_estimator, load_ml_transformer
from elephas_amd.models import optimizers
from elephas_amd.models.activations import relu
from elephas_amd.models import Dense, Sequential
from elephas_amd.utils.model_utils import ModelType


def argmax(c):
    return F.expr(f'array_position({c}, array_max({c})) - 1')


def _clf_estimator(model, epochs=1, batch_size=64, opt=None):
    opt = opt or optimizers.SGD(learning_rate=0.01, decay=1e-6, momentum=0.9, nesterov=True)
    est = ElephasEstimator()
    est.set_keras_model_config(model.to_json())
    est.set_optimizer_config(optimizers.serialize(opt))
    est.set_mode("synchronous")
    est.set_loss("categorical_crossentropy")
    est.set_metrics(['acc'])
    est.set_epochs(epochs)
    est.set_batch_size(batch_size)
    est.set_validation_split(0.1)
    est.set_categorical_labels(True)
    est.set_nb_classes(10)
    est.set_num_workers(2)
    return est


def _reg_estimator(model, **cols):
    est = ElephasEstimator(**cols)
    est.set_keras_model_config(model.to_json())
    est.set_optimizer_config(optimizers.serialize(optimizers.SGD(learning_rate=0.00001)))
    est.set_mode("synchronous")
    est.set_loss("mae")
    est.set_metrics(['mae'])
    est.set_epochs(3)
    est.set_batch_size(64)
    est.set_validation_split(0.01)
    est.set_categorical_labels(False)
    est.set_num_workers(2)
    return est


def test_serialization_transformer(tmp_cwd, classification_model):
    transformer = ElephasTransformer()
    transformer.set_keras_model_config(classification_model.to_json())
    transformer.save("test.h5")
    loaded = load_ml_transformer("test.h5")
    assert loaded.get_model().to_json() == classification_model.to_json()


def test_serialization_estimator(tmp_cwd, classification_model):
    estimator = ElephasEstimator()
    estimator.set_keras_model_config(classification_model.to_json())
    estimator.set_loss("categorical_crossentropy")
    estimator.save("test.h5")
    loaded = load_ml_estimator("test.h5")
    assert loaded.get_model().to_json() == classification_model.to_json()
    assert loaded.get_loss() == "categorical_crossentropy"


def test_serialization_transformer_and_predict(tmp_cwd, spark_context, classification_model, mnist_data):
    _, _, x_test, y_test = mnist_data
    df = to_data_frame(spark_context, x_test[:200], y_test[:200], categorical=True)
    transformer = ElephasTransformer(weights=classification_model.get_weights(),
                                     model_type=ModelType.CLASSIFICATION)
    transformer.set_keras_model_config(classification_model.to_json())
    transformer.save("test.h5")
    loaded = load_ml_transformer("test.h5")
    out = loaded.transform(df)
    assert out.count() == 200
    # the loaded weights reproduce the original network's probabilities
    # a directly constructed transformer keeps pyspark's default '<uid>__output' column
    assert out.columns[-1] == loaded.getOutputCol()
    p0 = np.asarray(out.take(1)[0][loaded.getOutputCol()])
    classification_model.compile("sgd", "categorical_crossentropy")
    ref = classification_model.predict(x_test[:1])[0]
    assert np.allclose(p0, ref, atol=1e-5)


def test_spark_ml_model_classification(spark_context, classification_model, mnist_data, capsys):
    x_train, y_train, x_test, y_test = mnist_data
    df = to_data_frame(spark_context, x_train[:1000], y_train[:1000], categorical=True)
    test_df = to_data_frame(spark_context, x_test, y_test, categorical=True)
    pipeline = Pipeline(stages=[_clf_estimator(classification_model)])
    fitted = pipeline.fit(df)
    prediction = fitted.transform(test_df)
    pnl = prediction.select("label", "prediction")
    pnl.show(5)
    assert "prediction" in capsys.readouterr().out
    pnl = pnl.select('label', argmax('prediction').astype(DoubleType()).alias('prediction'))
    metrics = MulticlassMetrics(pnl.rdd.map(lambda row: (row.label, row.prediction)))
    assert 0.0 <= metrics.accuracy <= 1.0
    # the transform is the fitted network's prediction, row for row
    stage = fitted.stages[-1] if hasattr(fitted, "stages") else fitted.getStages()[-1]
    net = stage.get_model()
    net.set_weights(stage.weights)
    ref = np.argmax(net.predict(x_test), axis=1)
    assert np.array_equal(np.array([r.prediction for r in pnl.collect()]), ref)


def test_functional_model(spark_context, classification_model_functional, mnist_data):
    x_train, y_train, x_test, y_test = mnist_data
    df = to_data_frame(spark_context, x_train[:1000], y_train[:1000], categorical=True)
    test_df = to_data_frame(spark_context, x_test[:300], y_test[:300], categorical=True)
    est = _clf_estimator(classification_model_functional, opt=optimizers.SGD())
    fitted = Pipeline(stages=[est]).fit(df)
    pnl = fitted.transform(test_df).select('label', argmax('prediction').astype(DoubleType()).alias('prediction'))
    metrics = MulticlassMetrics(pnl.rdd.map(lambda row: (row.label, row.prediction)))
    assert 0.0 <= metrics.accuracy <= 1.0


def test_regression_model(spark_context, regression_model, boston_housing_dataset):
    x_train, y_train, x_test, y_test = boston_housing_dataset
    df = to_data_frame(spark_context, x_train, y_train)
    test_df = to_data_frame(spark_context, x_test, y_test)
    fitted = Pipeline(stages=[_reg_estimator(regression_model)]).fit(df)
    pnl = fitted.transform(test_df).select("label", "prediction")
    row = pnl.take(1)[0]
    assert isinstance(row.prediction, float)   # regression -> DoubleType scalar column
    metrics = RegressionMetrics(pnl.rdd.map(lambda r: (r.label, r.prediction)))
    assert np.isfinite(metrics.r2)


def _renamed(spark_context, x, y):
    df = to_data_frame(spark_context, x, y)
    return df.withColumnRenamed('features', 'scaled_features').withColumnRenamed('label', 'ground_truth')


def test_set_cols_deprecated(spark_context, regression_model, boston_housing_dataset):
    x_train, y_train, x_test, y_test = boston_housing_dataset
    with pytest.deprecated_call():
        est = _reg_estimator(regression_model)
        est.setFeaturesCol('scaled_features')
        est.setOutputCol('output')
        est.setLabelCol('ground_truth')
    fitted = Pipeline(stages=[est]).fit(_renamed(spark_context, x_train, y_train))
    pnl = fitted.transform(_renamed(spark_context, x_test, y_test)).select("ground_truth", "output")
    metrics = RegressionMetrics(pnl.rdd.map(lambda row: (row['ground_truth'], row['output'])))
    assert np.isfinite(metrics.r2)


def test_set_cols(spark_context, regression_model, boston_housing_dataset):
    x_train, y_train, x_test, y_test = boston_housing_dataset
    est = _reg_estimator(regression_model, labelCol='ground_truth', outputCol='output',
                         featuresCol='scaled_features')
    fitted = Pipeline(stages=[est]).fit(_renamed(spark_context, x_train, y_train))
    out = fitted.transform(_renamed(spark_context, x_test, y_test))
    assert "output" in out.columns
    pnl = out.select("ground_truth", "output")
    assert pnl.count() == len(x_test)


def test_custom_objects(spark_context, boston_housing_dataset):
    def custom_activation(x):
        return 2 * relu(x)

    model = Sequential()
    model.add(Dense(64, input_shape=(13,)))
    model.add(Dense(64, activation=custom_activation))
    model.add(Dense(1, activation='linear'))
    x_train, y_train, x_test, y_test = boston_housing_dataset
    est = _reg_estimator(model)
    est.set_batch_size(32)
    est.set_custom_objects({'custom_activation': custom_activation})
    fitted = Pipeline(stages=[est]).fit(to_data_frame(spark_context, x_train, y_train))
    out = fitted.transform(to_data_frame(spark_context, x_test, y_test))
    assert out.count() == len(x_test)


def test_predict_classes_probability(spark_context, classification_model, mnist_data):
    x_train, y_train, x_test, y_test = mnist_data
    df = to_data_frame(spark_context, x_train[:1000], y_train[:1000], categorical=True)
    test_df = to_data_frame(spark_context, x_test[:100], y_test[:100], categorical=True)
    fitted = Pipeline(stages=[_clf_estimator(classification_model)]).fit(df)
    results = fitted.transform(test_df)
    probs = np.asarray(results.take(1)[0].prediction)
    assert len(probs) == 10
    assert abs(probs.sum() - 1.0) < 1e-4


def test_batch_predict_classes_probability(spark_context, classification_model, mnist_data):
    x_train, y_train, x_test, y_test = mnist_data
    df = to_data_frame(spark_context, x_train[:1000], y_train[:1000], categorical=True)
    test_df = to_data_frame(spark_context, x_test, y_test, categorical=True)
    fitted = _clf_estimator(classification_model).fit(df)
    results = fitted.transform(test_df)
    fitted.set_params(inference_batch_size=int(len(y_test) / 10))
    fitted.set_params(outputCol="prediction_via_batch_inference")
    both = fitted.transform(results)
    for r in both.take(len(y_test)):
        assert len(r.prediction) == 10 and len(r.prediction_via_batch_inference) == 10
        assert np.array_equal(r.prediction, r.prediction_via_batch_inference)


def test_save_pipeline(tmp_cwd, classification_model):
    est = _clf_estimator(classification_model, epochs=10, batch_size=10)
    pipeline = Pipeline(stages=[est])
    pipeline.save('tmp')
    loaded = Pipeline.load('tmp')
    st = loaded.getStages()[0]
    assert isinstance(st, ElephasEstimator)
    assert st.get_epochs() == 10 and st.get_batch_size() == 10
    assert st.get_model().to_json() == classification_model.to_json()
