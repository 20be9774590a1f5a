"""SparkMLlibModel on an RDD of LabeledPoints (reference examples/mllib_mlp.py)."""
from _mnist_common import load, mlp, nb_classes

from elephas_amd.keras.optimizers import RMSprop
from elephas_amd.spark import SparkConf, SparkContext
from elephas_amd.spark_model import SparkMLlibModel
from elephas_amd.utils.rdd_utils import to_labeled_point

x_train, y_train, x_test, y_test = load()
model = mlp()
model.compile(RMSprop(), "categorical_crossentropy", ['acc'])
sc = SparkContext(conf=SparkConf().setAppName('Mnist_Spark_MLP').setMaster('local[8]'))
lp_rdd = to_labeled_point(sc, x_train, y_train, categorical=True)
spark_model = SparkMLlibModel(model=model, frequency='epoch', mode='synchronous')
spark_model.fit(lp_rdd, epochs=5, batch_size=32, verbose=0, validation_split=0.1, categorical=True,
                nb_classes=nb_classes)
score = spark_model.master_network.evaluate(x_test, y_test, verbose=2)
print('Test accuracy:', score[1])
