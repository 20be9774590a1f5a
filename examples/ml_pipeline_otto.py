"""Otto product classification: StringIndexer + StandardScaler + ElephasEstimator
(reference examples/ml_pipeline_otto.py, Spark_ML_Pipeline.ipynb).

The Kaggle CSVs are not available offline: with no ``train.csv`` next to this
script, a synthetic Otto-shaped CSV (93 count features, 9 classes 'Class_1'..
'Class_9', 61,878 rows by default; ``OTTO_ROWS`` to change) is written first and
read back through the same textFile -> DataFrame path.
"""
import os
import random

import numpy as np

from elephas_amd.keras import optimizers
from elephas_amd.keras.layers import Activation, Dense, Dropout
from elephas_amd.keras.models import Sequential
from elephas_amd.ml_model import ElephasEstimator
from elephas_amd.spark.ml import Pipeline
from elephas_amd.spark.ml.feature import StandardScaler, StringIndexer
from elephas_amd.spark.ml.linalg import Vectors
from elephas_amd.spark.mllib.evaluation import MulticlassMetrics
from elephas_amd.spark.sql import SparkSession

data_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "")
spark_session = SparkSession.builder.appName('Otto_Spark_ML_Pipeline').getOrCreate()
sc = spark_session.sparkContext


def synth_csv(path, n, seed=0):
    rng = np.random.default_rng(seed)
    centers = rng.gamma(0.6, 2.0, size=(1, 93)) * np.exp(rng.normal(0, 0.25, size=(9, 93)))  # Otto-like overlap
    y = rng.integers(0, 9, n)
    x = rng.poisson(centers[y])
    with open(path, "w") as f:
        f.write("id," + ",".join(f"feat_{i + 1}" for i in range(93)) + ",target\n")
        for i in range(n):
            f.write(f"{i + 1}," + ",".join(map(str, x[i])) + f",Class_{y[i] + 1}\n")


def shuffle_csv(csv_file):
    lines = open(csv_file).readlines()
    header, body = lines[:1], lines[1:]
    random.shuffle(body)
    open(csv_file, 'w').writelines(header + body)


def load_data_rdd(csv_file, shuffle=True, train=True):
    if shuffle:
        shuffle_csv(data_path + csv_file)
    data = sc.textFile(data_path + csv_file)
    data = data.filter(lambda x: x.split(',')[0] != 'id').map(lambda line: line.split(','))
    if train:
        data = data.map(lambda line: (Vectors.dense(np.asarray(line[1:-1]).astype(np.float32)),
                                      str(line[-1]).replace('Class_', '')))
    else:
        data = data.map(lambda line: (Vectors.dense(np.asarray(line[1:]).astype(np.float32)), "1"))
    return data


if not os.path.exists(data_path + "train.csv"):
    synth_csv(data_path + "train.csv", int(os.environ.get("OTTO_ROWS", "61878")))
train_df = spark_session.createDataFrame(load_data_rdd("train.csv"), ['features', 'category'])

string_indexer = StringIndexer(inputCol="category", outputCol="index_category")
scaler = StandardScaler(inputCol="features", outputCol="scaled_features", withStd=True, withMean=True)
nb_classes = train_df.select("category").distinct().count()
input_dim = len(train_df.select("features").first()[0])

model = Sequential()
model.add(Dense(512, input_shape=(input_dim,)))
model.add(Activation('relu'))
model.add(Dropout(0.5))
model.add(Dense(512))
model.add(Activation('relu'))
model.add(Dropout(0.5))
model.add(Dense(512))
model.add(Activation('relu'))
model.add(Dropout(0.5))
model.add(Dense(nb_classes))
model.add(Activation('softmax'))
model.compile(loss='categorical_crossentropy', optimizer='adam')

estimator = ElephasEstimator()
estimator.set_keras_model_config(model.to_json())
estimator.set_optimizer_config(optimizers.serialize(optimizers.Adam(learning_rate=0.01)))
estimator.set_mode("synchronous")
estimator.set_loss("categorical_crossentropy")
estimator.set_metrics(['acc'])
estimator.setFeaturesCol("scaled_features")
estimator.setLabelCol("index_category")
estimator.set_epochs(int(os.environ.get("EXAMPLE_EPOCHS", "20")))
estimator.set_batch_size(128)
estimator.set_num_workers(1)
estimator.set_verbosity(0)
estimator.set_validation_split(0.15)
estimator.set_categorical_labels(True)
estimator.set_nb_classes(nb_classes)

fitted_pipeline = Pipeline(stages=[string_indexer, scaler, estimator]).fit(train_df)
prediction = fitted_pipeline.transform(train_df)
pnl = prediction.select("index_category", "prediction")
pnl.show(10)
prediction_and_label = pnl.rdd.map(lambda row: (row.index_category, float(np.argmax(row.prediction))))
metrics = MulticlassMetrics(prediction_and_label)
print("precision:", metrics.precision())
