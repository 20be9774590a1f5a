"""Spark-ML Pipeline with ElephasEstimator, Boston-housing regression
(reference examples/ml_mlp_regression.py)."""
import os

from elephas_amd.keras import optimizers
from elephas_amd.keras.datasets import boston_housing
from elephas_amd.keras.layers import Activation, Dense
from elephas_amd.keras.models import Sequential
from elephas_amd.ml.adapter import to_data_frame
from elephas_amd.ml_model import ElephasEstimator
from elephas_amd.spark import SparkConf, SparkContext
from elephas_amd.spark.ml import Pipeline
from elephas_amd.spark.mllib.evaluation import RegressionMetrics

batch_size, epochs = 16, int(os.environ.get("EXAMPLE_EPOCHS", "100"))
(x_train, y_train), (x_test, y_test) = boston_housing.load_data()
x_train, x_test = x_train.astype("float32"), x_test.astype("float32")
model = Sequential()
model.add(Dense(64, input_shape=(x_train.shape[1],)))
model.add(Activation('relu'))
model.add(Dense(64))
model.add(Activation('relu'))
model.add(Dense(1))

sc = SparkContext(conf=SparkConf().setAppName('BostonHousing_Spark_MLP').setMaster('local[*]'))
df = to_data_frame(sc, x_train, y_train)
test_df = to_data_frame(sc, x_test, y_test)
estimator = ElephasEstimator()
estimator.set_keras_model_config(model.to_json())
estimator.set_optimizer_config(optimizers.serialize(optimizers.SGD(learning_rate=0.000001)))
estimator.set_mode("synchronous")
estimator.set_loss("mae")
estimator.set_metrics(['mse'])
estimator.set_epochs(epochs)
estimator.set_batch_size(batch_size)
estimator.set_validation_split(0.1)
estimator.set_categorical_labels(False)

fitted_pipeline = Pipeline(stages=[estimator]).fit(df)
pnl = fitted_pipeline.transform(test_df).select("label", "prediction")
pnl.show(10)
metrics = RegressionMetrics(pnl.rdd.map(lambda row: (row.label, row.prediction)))
print(metrics.r2)
print(metrics.meanAbsoluteError)
print(metrics.rootMeanSquaredError)
