"""MNIST MLP with SparkModel, mode='synchronous' (reference examples/mnist_mlp_spark_synchronous.py).

Spark partitions -> logical workers on the GPU(s); run on N GPUs with
`torchrun --nproc-per-node N examples/mnist_mlp_spark_synchronous.py`.
"""
from _mnist_common import batch_size, load, mlp

from elephas_amd.keras.optimizers import SGD
from elephas_amd.spark import SparkConf, SparkContext
from elephas_amd.spark_model import SparkModel
from elephas_amd.utils.rdd_utils import to_simple_rdd

epochs = 1
conf = SparkConf().setAppName('Mnist_Spark_MLP').setMaster('local[8]')
sc = SparkContext(conf=conf)
x_train, y_train, x_test, y_test = load()

model = mlp()
model.compile(SGD(learning_rate=0.1), 'categorical_crossentropy', ['acc'])
rdd = to_simple_rdd(sc, x_train, y_train)
spark_model = SparkModel(model, mode='synchronous')
spark_model.fit(rdd, epochs=epochs, batch_size=batch_size, verbose=2, validation_split=0.1)
score = spark_model.evaluate(x_test, y_test, verbose=2)
print('Test accuracy:', score[1])
