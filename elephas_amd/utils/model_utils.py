"""Loss -> model-type mapping and its JSON enum codec
(reference elephas/utils/model_utils.py:9-70)."""
import json
from enum import Enum


class ModelType(Enum):
    CLASSIFICATION = 1
    REGRESSION = 2


class _Singleton(type):
    _instances = {}

    def __call__(cls, *args):
        if cls not in cls._instances:
            cls._instances[cls] = super(_Singleton, cls).__call__(*args)
        return cls._instances[cls]


class Singleton(_Singleton("SingletonMeta", (object,), {})):
    pass


class LossModelTypeMapper(Singleton):
    """Mapper for losses -> model type."""

    def __init__(self):
        self.__mapping = {
            "mean_squared_error": ModelType.REGRESSION,
            "mean_absolute_error": ModelType.REGRESSION,
            "mse": ModelType.REGRESSION,
            "mae": ModelType.REGRESSION,
            "cosine_proximity": ModelType.REGRESSION,
            "mean_absolute_percentage_error": ModelType.REGRESSION,
            "mean_squared_logarithmic_error": ModelType.REGRESSION,
            "logcosh": ModelType.REGRESSION,
            "binary_crossentropy": ModelType.CLASSIFICATION,
            "categorical_crossentropy": ModelType.CLASSIFICATION,
            "sparse_categorical_crossentropy": ModelType.CLASSIFICATION,
        }

    def get_model_type(self, loss):
        if callable(loss):
            loss = loss.__name__
        return self.__mapping.get(loss)

    def register_loss(self, loss, model_type):
        if callable(loss):
            loss = loss.__name__
        self.__mapping.update({loss: model_type})


class ModelTypeEncoder(json.JSONEncoder):
    def default(self, obj):
        if isinstance(obj, ModelType):
            return {"__enum__": str(obj)}
        return json.JSONEncoder.default(self, obj)


def as_enum(d):
    if "__enum__" in d:
        name, member = d["__enum__"].split(".")
        return getattr(ModelType, member)
    return d
