"""Which kind of model a loss implies, and the JSON form of that kind.

Public contract of reference elephas/utils/model_utils.py:9-70 (``ModelType``,
``LossModelTypeMapper().get_model_type / register_loss``, ``ModelTypeEncoder``,
``as_enum``); the ``{"__enum__": "ModelType.X"}`` JSON form is what saved
ElephasTransformer files hold, so it is kept byte-compatible.

The table is not hand-maintained: it is derived from the loss registry
(models/losses.py, names and aliases): cross-entropy, hinge and KL-divergence
losses are classification losses, every other registered loss a regression loss
(the reference lists 11 names and answers None for the rest; for those it agrees
with the reference's use of the answer, where None falls into the classification
branch).  ``register_loss`` adds or overrides entries (custom losses).
"""
from __future__ import annotations

import json
from enum import Enum
from typing import Callable, Dict, Optional, Union


class ModelType(Enum):
    CLASSIFICATION = 1
    REGRESSION = 2


# aliases the reference table lists that are not names in our loss registry
_EXTRA_REGRESSION = ("cosine_proximity",)


def _default_table() -> Dict[str, ModelType]:
    from ..models import losses
    table = {}
    for name in losses.registered_names():
        canon = losses.canonical(name).lower()
        classify = any(k in canon for k in ("crossentropy", "hinge", "kullback"))
        table[name] = ModelType.CLASSIFICATION if classify else ModelType.REGRESSION
    for name in _EXTRA_REGRESSION:
        table.setdefault(name, ModelType.REGRESSION)
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
