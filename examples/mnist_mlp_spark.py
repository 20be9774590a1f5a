"""MNIST MLP with SparkModel defaults (asynchronous, epoch frequency)
(reference examples/mnist_mlp_spark.py)."""
from _mnist_common import batch_size, load, mlp

from elephas_amd.keras.optimizers import SGD
from elephas_amd.spark import SparkConf, SparkContext
from elephas_amd.spark_model import SparkModel
from elephas_amd.utils.rdd_utils import to_simple_rdd

sc = SparkContext(conf=SparkConf().setAppName('Mnist_Spark_MLP').setMaster('local[8]'))
x_train, y_train, x_test, y_test = load()
model = mlp()
model.compile(SGD(learning_rate=0.1), 'categorical_crossentropy', ['acc'])
spark_model = SparkModel(model, frequency='epoch', mode='asynchronous')
spark_model.fit(to_simple_rdd(sc, x_train, y_train), epochs=1, batch_size=batch_size, verbose=0,
                validation_split=0.1)
score = spark_model.master_network.evaluate(x_test, y_test, verbose=2)
print('Test accuracy:', score[1])
