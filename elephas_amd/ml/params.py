"""Spark-ML parameter mixins with the reference's names and defaults
(reference elephas/ml/params.py:4-259; defaults asserted by tests/ml/test_params.py).

The fifteen mixins are generated from one table -- (class, param, accessor suffix,
description, default) -- instead of fifteen hand-written copies of the same get/set
pair: each class gets ``__init__`` (declares the Param, sets the default), a setter
``set_<suffix>`` that returns ``self`` and a getter ``get_<suffix>``.
"""
import copy

from ..data.ml import Param, Params

_NO_DEFAULT = object()

#  class name,               param,                 accessor suffix,         description,                                     default
_TABLE = [
    ("HasKerasModelConfig",     "keras_model_config",   "keras_model_config",   "Serialized Keras model as json string",          _NO_DEFAULT),
    ("HasMode",                 "mode",                 "mode",                 "Elephas mode",                                   "asynchronous"),
    ("HasFrequency",            "frequency",            "frequency",            "Elephas frequency",                              "epoch"),
    ("HasNumberOfClasses",      "nb_classes",           "nb_classes",           "number of classes",                              10),
    ("HasCategoricalLabels",    "categorical",          "categorical_labels",   "Boolean to indicate if labels are categorical",  True),
    ("HasEpochs",               "epochs",               "epochs",               "Number of epochs to train",                      10),
    ("HasBatchSize",            "batch_size",           "batch_size",           "Batch size",                                     32),
    ("HasVerbosity",            "verbose",              "verbosity",            "Stdout verbosity",                               0),
    ("HasValidationSplit",      "validation_split",     "validation_split",     "validation split percentage",                    0.1),
    ("HasNumberOfWorkers",      "num_workers",          "num_workers",          "number of workers",                              8),
    ("HasKerasOptimizerConfig", "optimizer_config",     "optimizer_config",     "Serialized Keras optimizer properties",          None),
    ("HasMetrics",              "metrics",              "metrics",              "Keras metrics",                                  ["acc"]),
    ("HasLoss",                 "loss",                 "loss",                 "Keras loss",                                     _NO_DEFAULT),
    ("HasCustomObjects",        "custom_objects",       "custom_objects",       "Custom objects",                                 {}),
    ("HasInferenceBatchSize",   "inference_batch_size", "inference_batch_size", "Batch size for inference",                       None),
]


def _mixin(cls_name, param, suffix, doc, default):
    def __init__(self):
        super(cls, self).__init__()
        setattr(self, param, Param(self, param, doc))
        if default is not _NO_DEFAULT:
            # a fresh copy per instance: mutable defaults (metrics, custom_objects) are not shared
            self._setDefault(**{param: copy.deepcopy(default)})

    def setter(self, value):
        self._paramMap[getattr(self, param)] = value
        return self

    def getter(self):
        return self.getOrDefault(getattr(self, param))

    setter.__name__, getter.__name__ = f"set_{suffix}", f"get_{suffix}"
    setter.__doc__ = f"Set ``{param}`` ({doc}); returns self."
    getter.__doc__ = f"``{param}`` ({doc})" + ("" if default is _NO_DEFAULT else f", default {default!r}.")
    cls = type(cls_name, (Params,), {
        "__init__": __init__, f"set_{suffix}": setter, f"get_{suffix}": getter,
        "__doc__": f"Parameter mixin: {doc} (param ``{param}``).", "__module__": __name__})
    return cls


for _row in _TABLE:
    globals()[_row[0]] = _mixin(*_row)

__all__ = [row[0] for row in _TABLE]
