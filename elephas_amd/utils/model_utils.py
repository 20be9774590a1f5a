"""Which kind of model a loss implies, and the JSON form of that kind.

Public contract of reference elephas/utils/model_utils.py:9-70 (``ModelType``,
``LossModelTypeMapper().get_model_type / register_loss``, ``ModelTypeEncoder``,
``as_enum``); the ``{"__enum__": "ModelType.X"}`` JSON form is what saved
ElephasTransformer files hold, so it is kept byte-compatible.

The default table holds exactly the reference's eleven loss names (regression: the
squared / absolute / percentage / logarithmic errors, log-cosh and cosine proximity;
classification: the three cross-entropies) and answers None for every other loss,
as the reference does: callers treat None like a classification loss (the full
output vector is kept), so a multi-output model trained with e.g. 'poisson' keeps
all its prediction columns.  ``register_loss`` adds or overrides entries.
"""
from __future__ import annotations

import json
from enum import Enum
from typing import Callable, Dict, Optional, Union


class ModelType(Enum):
    CLASSIFICATION = 1
    REGRESSION = 2


_REGRESSION_LOSSES = ("mean_squared_error", "mean_absolute_error", "mse", "mae", "cosine_proximity",
                      "mean_absolute_percentage_error", "mean_squared_logarithmic_error", "logcosh")
_CLASSIFICATION_LOSSES = ("binary_crossentropy", "categorical_crossentropy", "sparse_categorical_crossentropy")


def _default_table() -> Dict[str, ModelType]:
    table = dict.fromkeys(_REGRESSION_LOSSES, ModelType.REGRESSION)
    table.update(dict.fromkeys(_CLASSIFICATION_LOSSES, ModelType.CLASSIFICATION))
    return table


def _key(loss: Union[str, Callable]) -> str:
    return loss if isinstance(loss, str) else getattr(loss, "__name__", str(loss))


class LossModelTypeMapper:
    """Process-wide loss -> ModelType table (every construction returns the same object)."""

    _shared: Optional["LossModelTypeMapper"] = None

    def __new__(cls):
        if cls._shared is None:
            inst = super().__new__(cls)
            inst._table = _default_table()
            cls._shared = inst
        return cls._shared

    def get_model_type(self, loss) -> Optional[ModelType]:
        return self._table.get(_key(loss))

    def register_loss(self, loss, model_type: ModelType) -> None:
        self._table[_key(loss)] = model_type


class ModelTypeEncoder(json.JSONEncoder):
    """json.dumps(..., cls=ModelTypeEncoder) writes ModelType members as {"__enum__": "ModelType.X"}."""

    def default(self, obj):
        if isinstance(obj, ModelType):
            return {"__enum__": f"{type(obj).__name__}.{obj.name}"}
        return super().default(obj)


def as_enum(d: dict):
    """json.loads object_hook: the inverse of ModelTypeEncoder."""
    tag = d.get("__enum__")
    if tag is None:
        return d
    return ModelType[tag.rpartition(".")[2]]
