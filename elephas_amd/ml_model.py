"""Spark-ML Estimator / Transformer (reference elephas/ml_model.py:25-269).

``ElephasEstimator._fit`` turns a DataFrame into a (features, label) RDD,
compiles the Keras-compatible model from its JSON config and trains it with a
``SparkModel`` (MI355X native engine); the result is an ``ElephasTransformer``
holding the trained weights.  ``_transform`` appends a prediction column:
``DoubleType`` for regression losses, ``ArrayType(DoubleType)`` of class
probabilities for classification (reference :243-249).  ``inference_batch_size``
chunks the prediction exactly like the reference's ``batched_prediction``
(chunked and unchunked results are identical: tests/test_ml_model.py:345-354).
"""
from __future__ import annotations

import copy
import json
import warnings
from typing import Optional

import numpy as np

from .data.ml import (DefaultParamsReadable, DefaultParamsWritable, Estimator, HasFeaturesCol, HasLabelCol,
                      HasOutputCol, Model, keyword_only)
from .data.sql import ArrayType, DataFrame, DoubleType, Row, SparkSession, StructField, StructType
from .io import h5lite
from .ml.adapter import df_to_simple_rdd
from .ml.params import *  # noqa: F401,F403
from .ml.params import (HasBatchSize, HasCategoricalLabels, HasCustomObjects, HasEpochs, HasFrequency,
                        HasInferenceBatchSize, HasKerasModelConfig, HasKerasOptimizerConfig, HasLoss, HasMetrics,
                        HasMode, HasNumberOfClasses, HasNumberOfWorkers, HasValidationSplit, HasVerbosity)
from .mllib.adapter import from_vector
from .models import model_from_json
from .models import optimizers as O
from .spark_model import SparkModel
from .utils.model_utils import LossModelTypeMapper, ModelType, ModelTypeEncoder, as_enum


def _attr_json(raw):
    if isinstance(raw, (bytes, np.bytes_)):
        return bytes(raw).decode("utf8")
    return str(raw)


# get_config() keys and the getters that produce them (reference ml_model.py:40-59);
# the same dict round-trips through save() / load_ml_estimator() as constructor kwargs
_ESTIMATOR_CONFIG = (
    ("keras_model_config", "get_keras_model_config"), ("mode", "get_mode"), ("frequency", "get_frequency"),
    ("num_workers", "get_num_workers"), ("categorical", "get_categorical_labels"), ("loss", "get_loss"),
    ("metrics", "get_metrics"), ("validation_split", "get_validation_split"), ("featuresCol", "getFeaturesCol"),
    ("labelCol", "getLabelCol"), ("epochs", "get_epochs"), ("batch_size", "get_batch_size"),
    ("verbose", "get_verbosity"), ("nb_classes", "get_nb_classes"), ("outputCol", "getOutputCol"),
)


def _deprecated_col_setter(col: str):
    """Spark 3 deprecated the column setters in favour of constructor kwargs; the
    reference keeps them with a DeprecationWarning (ml_model.py:111-124)."""
    def setter(self, value):
        warnings.warn(f"set{col[0].upper()}{col[1:]} is deprecated in Spark 3.0.x+ - please supply {col} in the "
                      f"constructor i.e; ElephasEstimator({col}='foo')", DeprecationWarning)
        return self._set(**{col: value})
    setter.__name__ = f"set{col[0].upper()}{col[1:]}"
    return setter


def _read_distributed_config(file_name: str, object_hook=None) -> dict:
    """The ``distributed_config`` root attribute of an estimator / transformer file."""
    f = h5lite.File(file_name, mode="r")
    try:
        return json.loads(_attr_json(f.attrs.get("distributed_config")), object_hook=object_hook)
    finally:
        f.close()


class ElephasEstimator(Estimator, HasCategoricalLabels, HasValidationSplit, HasKerasModelConfig, HasFeaturesCol,
                       HasLabelCol, HasMode, HasEpochs, HasBatchSize, HasFrequency, HasVerbosity, HasNumberOfClasses,
                       HasNumberOfWorkers, HasOutputCol, HasLoss, HasMetrics, HasKerasOptimizerConfig,
                       HasCustomObjects, DefaultParamsReadable, DefaultParamsWritable):
    """Spark-ML Estimator wrapping a Keras-compatible model config: ``fit(df)`` trains
    a SparkModel on the native engine and returns an ``ElephasTransformer``."""

    @keyword_only
    def __init__(self, **kwargs):
        super(ElephasEstimator, self).__init__()
        self._defaultParamMap[self.outputCol] = "prediction"
        self.set_params(**kwargs)

    def get_config(self):
        return {key: getattr(self, getter)() for key, getter in _ESTIMATOR_CONFIG}

    def save(self, file_name: str):
        """HDF5 holding only the ``distributed_config`` attribute (reference :61-70)."""
        conf = {"class_name": type(self).__name__, "config": self.get_config()}
        f = h5lite.File(file_name, mode="w")
        f.attrs["distributed_config"] = json.dumps(conf).encode("utf8")
        f.flush()
        f.close()

    @keyword_only
    def set_params(self, **kwargs):
        return self._set(**kwargs)

    def get_model(self):
        return model_from_json(self.get_keras_model_config(), self.get_custom_objects())

    # -- fit: DataFrame -> (features, label) RDD -> SparkModel -> transformer
    def _training_rdd(self, df: DataFrame):
        rdd = df_to_simple_rdd(df, categorical=self.get_categorical_labels(), nb_classes=self.get_nb_classes(),
                               features_col=self.getFeaturesCol(), label_col=self.getLabelCol())
        return rdd.repartition(self.get_num_workers())

    def _compiled_model(self):
        model = self.get_model()
        model.compile(loss=self.get_loss(), optimizer=O.get(self.get_optimizer_config()),
                      metrics=self.get_metrics(), custom_objects=self.get_custom_objects())
        return model

    def _fit(self, df: DataFrame):
        rdd = self._training_rdd(df)
        spark_model = SparkModel(model=self._compiled_model(), mode=self.get_mode(), frequency=self.get_frequency(),
                                 num_workers=self.get_num_workers(), custom_objects=self.get_custom_objects())
        spark_model.fit(rdd, epochs=self.get_epochs(), batch_size=self.get_batch_size(),
                        verbose=self.get_verbosity(), validation_split=self.get_validation_split())
        trained = spark_model.master_network
        return ElephasTransformer(labelCol=self.getLabelCol(), outputCol=self.getOutputCol(),
                                  featuresCol=self.getFeaturesCol(), keras_model_config=trained.to_json(),
                                  weights=trained.get_weights(), custom_objects=self.get_custom_objects(),
                                  model_type=LossModelTypeMapper().get_model_type(self.get_loss()),
                                  history=spark_model.training_histories)

    setFeaturesCol = _deprecated_col_setter("featuresCol")
    setLabelCol = _deprecated_col_setter("labelCol")
    setOutputCol = _deprecated_col_setter("outputCol")


def load_ml_estimator(file_name: str) -> ElephasEstimator:
    """Rebuild an estimator from ElephasEstimator.save() (reference :129-133)."""
    return ElephasEstimator(**_read_distributed_config(file_name).get("config"))


class ElephasTransformer(Model, HasKerasModelConfig, HasLabelCol, HasOutputCol, HasFeaturesCol, HasCustomObjects,
                         HasInferenceBatchSize):
    """Spark-ML Model holding a trained network; ``transform`` appends predictions."""

    @keyword_only
    def __init__(self, **kwargs):
        super(ElephasTransformer, self).__init__()
        # weights / model_type / history are plain attributes, not Spark Params
        for attr in ("weights", "model_type"):
            if attr in kwargs:
                setattr(self, attr, kwargs.pop(attr))
        self._history = kwargs.pop("history", [])
        self.set_params(**kwargs)

    @property
    def history(self):
        return self._history

    @keyword_only
    def set_params(self, **kwargs):
        return self._set(**kwargs)

    def get_config(self):
        return {"keras_model_config": self.get_keras_model_config(), "labelCol": self.getLabelCol(),
                "featuresCol": self.getFeaturesCol(), "outputCol": self.getOutputCol(),
                "weights": [np.asarray(w).tolist() for w in getattr(self, "weights", [])],
                "model_type": getattr(self, "model_type", None)}

    def save(self, file_name: str):
        """HDF5 with the ``distributed_config`` attribute: config, weights as lists and
        the model type enum (reference :205-213)."""
        conf = {"class_name": type(self).__name__, "config": self.get_config()}
        f = h5lite.File(file_name, mode="w")
        f.attrs["distributed_config"] = json.dumps(conf, cls=ModelTypeEncoder).encode("utf8")
        f.flush()
        f.close()

    def get_model(self):
        return model_from_json(self.get_keras_model_config(), self.get_custom_objects())

    def _transform(self, df: DataFrame) -> DataFrame:
        """Append the network's predictions as ``outputCol`` (reference ml_model.py:223-242
        maps the prediction over the DataFrame's partitions).  The rows are split in
        contiguous blocks over the ranks of the job, each rank predicts its block on its
        GPU in ``inference_batch_size`` chunks, and one tensor all-gather (RCCL) puts the
        predictions back in row order on every rank -- the SparkModel.predict path."""
        from .parallel import dist
        output_col = self.getOutputCol()
        new_schema = copy.deepcopy(df.schema)
        rows = df.collect()
        model = self.get_model()
        model.set_weights(self.weights)
        features_col = self.getFeaturesCol()
        n = len(rows)
        lo, hi = dist.block_range(n)
        out_shape = tuple(model.output_shape[1:])
        if hi > lo:
            feats = np.array([from_vector(r[features_col]) for r in rows[lo:hi]])
            bs = self.get_inference_batch_size()
            if bs is not None and bs > 0:
                local = np.vstack([model.predict(feats[i:i + bs]) for i in range(0, len(feats), bs)])
            else:
                local = model.predict(feats)
        else:
            local = np.zeros((0,) + out_shape, np.float32)
        preds = dist.all_gather_rows(np.asarray(local, np.float32).reshape((-1,) + out_shape), n)
        if getattr(self, "model_type", None) == ModelType.REGRESSION:
            values = [float(np.asarray(p).reshape(-1)[0]) for p in preds]
            output_col_field = StructField(output_col, DoubleType(), True)
        else:
            values = [np.asarray(p, dtype=np.float64).tolist() for p in preds]
            output_col_field = StructField(output_col, ArrayType(DoubleType()), True)
        new_schema.add(output_col_field)
        names = new_schema.names
        out_rows = [Row.from_pairs(names, tuple(r) + (v,)) for r, v in zip(rows, values)]
        return DataFrame(out_rows, new_schema, df._nparts)


def load_ml_transformer(file_name: str) -> ElephasTransformer:
    """Rebuild a transformer from ElephasTransformer.save() (reference :265-269): the
    model type comes back as its enum, the weights as arrays."""
    config = _read_distributed_config(file_name, object_hook=as_enum).get("config")
    config["weights"] = [np.array(w) for w in config["weights"]]
    return ElephasTransformer(**config)
