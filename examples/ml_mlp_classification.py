"""Spark-ML Pipeline with ElephasEstimator, MNIST classification
(reference examples/ml_mlp_classification.py)."""
import os

import numpy as np
from _mnist_common import load, mlp, nb_classes

from elephas_amd.keras import optimizers
from elephas_amd.ml.adapter import to_data_frame
from elephas_amd.ml_model import ElephasEstimator
from elephas_amd.spark import SparkConf, SparkContext
from elephas_amd.spark.ml import Pipeline
from elephas_amd.spark.mllib.evaluation import MulticlassMetrics

os.environ.setdefault("EXAMPLE_ROWS", "5000")
batch_size, epochs = 64, int(os.environ.get("EXAMPLE_EPOCHS", "20"))
x_train, y_train, x_test, y_test = load()
x_test, y_test = x_test[:1000], y_test[:1000]
model = mlp()
sc = SparkContext(conf=SparkConf().setAppName('Mnist_Spark_MLP').setMaster('local[8]'))
df = to_data_frame(sc, x_train, y_train, categorical=True)
test_df = to_data_frame(sc, x_test, y_test, categorical=True)

sgd_conf = optimizers.serialize(optimizers.SGD(learning_rate=0.01, decay=1e-6, momentum=0.9, nesterov=True))
estimator = ElephasEstimator()
estimator.set_keras_model_config(model.to_json())
estimator.set_optimizer_config(sgd_conf)
estimator.set_mode("synchronous")
estimator.set_loss("categorical_crossentropy")
estimator.set_metrics(['acc'])
estimator.set_epochs(epochs)
estimator.set_batch_size(batch_size)
estimator.set_validation_split(0.1)
estimator.set_categorical_labels(True)
estimator.set_nb_classes(nb_classes)

fitted_pipeline = Pipeline(stages=[estimator]).fit(df)
prediction = fitted_pipeline.transform(test_df)
pnl = prediction.select("label", "prediction")
pnl.show(10, truncate=False)
metrics = MulticlassMetrics(pnl.rdd.map(lambda row: (row.label, float(np.argmax(row.prediction)))))
print(metrics.accuracy)
print(metrics.weightedPrecision)
print(metrics.weightedRecall)
