"""Loss registry with tf.keras 2.10 semantics.

Names/aliases follow ``keras.losses``; the model-type mapping used by the
Spark-ML layer lives in elephas_amd/utils/model_utils.py (reference
elephas/utils/model_utils.py:28-55).  Every loss returns the *per-sample* value
(Keras ``reduction=AUTO`` then averages over the batch).  ``softmax`` +
categorical cross-entropy and ``sigmoid`` + binary cross-entropy use the logits
path exactly as Keras does when ``y_pred`` carries ``_keras_logits``.
"""
from __future__ import annotations

from typing import Callable, Optional, Union

import torch
import torch.nn.functional as F

EPS = 1e-7

# id -> csrc/kernels/args.h Loss enum
LOSS_IDS = {
    "categorical_crossentropy": 0, "sparse_categorical_crossentropy": 1, "binary_crossentropy": 2,
    "mean_squared_error": 3, "mean_absolute_error": 4, "mean_absolute_percentage_error": 5,
    "mean_squared_logarithmic_error": 6, "logcosh": 7, "hinge": 8, "squared_hinge": 9,
    "kullback_leibler_divergence": 10, "poisson": 11, "cosine_similarity": 12, "categorical_hinge": 13,
}

ALIASES = {
    "mse": "mean_squared_error", "MSE": "mean_squared_error", "mae": "mean_absolute_error",
    "MAE": "mean_absolute_error", "mape": "mean_absolute_percentage_error",
    "MAPE": "mean_absolute_percentage_error", "msle": "mean_squared_logarithmic_error",
    "MSLE": "mean_squared_logarithmic_error", "kld": "kullback_leibler_divergence",
    "KLD": "kullback_leibler_divergence", "kl_divergence": "kullback_leibler_divergence",
    "log_cosh": "logcosh", "cosine_proximity": "cosine_similarity",
    "CategoricalCrossentropy": "categorical_crossentropy",
    "SparseCategoricalCrossentropy": "sparse_categorical_crossentropy",
    "BinaryCrossentropy": "binary_crossentropy", "MeanSquaredError": "mean_squared_error",
    "MeanAbsoluteError": "mean_absolute_error",
}


def canonical(name: str) -> str:
    return ALIASES.get(name, name)


def _mean_last(x):
    return x.mean(dim=-1)


def categorical_crossentropy(y_true, y_pred, logits=None):
    if logits is not None:
        return -(y_true * torch.log_softmax(logits, dim=-1)).sum(-1)
    p = y_pred / y_pred.sum(-1, keepdim=True)
    p = torch.clamp(p, EPS, 1.0 - EPS)
    return -(y_true * torch.log(p)).sum(-1)


def sparse_categorical_crossentropy(y_true, y_pred, logits=None):
    n = y_pred.shape[-1]
    yt = F.one_hot(y_true.reshape(-1).long(), n).to(y_pred.dtype)
    return categorical_crossentropy(yt, y_pred, logits)


def binary_crossentropy(y_true, y_pred, logits=None):
    if logits is not None:
        z = logits
        return _mean_last(torch.clamp(z, min=0) - z * y_true + torch.log1p(torch.exp(-torch.abs(z))))
    p = torch.clamp(y_pred, EPS, 1.0 - EPS)
    return _mean_last(-(y_true * torch.log(p + EPS) + (1 - y_true) * torch.log(1 - p + EPS)))


def mean_squared_error(y_true, y_pred, logits=None):
    return _mean_last((y_pred - y_true) ** 2)


def mean_absolute_error(y_true, y_pred, logits=None):
    return _mean_last(torch.abs(y_pred - y_true))


def mean_absolute_percentage_error(y_true, y_pred, logits=None):
    return 100.0 * _mean_last(torch.abs((y_true - y_pred) / torch.clamp(torch.abs(y_true), min=EPS)))


def mean_squared_logarithmic_error(y_true, y_pred, logits=None):
    a = torch.log1p(torch.clamp(y_pred, min=EPS)) - torch.log1p(torch.clamp(y_true, min=EPS))
    return _mean_last(a * a)


def logcosh(y_true, y_pred, logits=None):
    x = y_pred - y_true
    return _mean_last(x + F.softplus(-2.0 * x) - 0.6931471805599453)


def hinge(y_true, y_pred, logits=None):
    return _mean_last(torch.clamp(1.0 - y_true * y_pred, min=0.0))


def squared_hinge(y_true, y_pred, logits=None):
    return _mean_last(torch.clamp(1.0 - y_true * y_pred, min=0.0) ** 2)


def kullback_leibler_divergence(y_true, y_pred, logits=None):
    yt = torch.clamp(y_true, EPS, 1.0)
    yp = torch.clamp(y_pred, EPS, 1.0)
    return (yt * torch.log(yt / yp)).sum(-1)


def poisson(y_true, y_pred, logits=None):
    return _mean_last(y_pred - y_true * torch.log(y_pred + EPS))


def cosine_similarity(y_true, y_pred, logits=None):
    a = y_true / torch.sqrt(torch.clamp((y_true * y_true).sum(-1, keepdim=True), min=1e-12))
    b = y_pred / torch.sqrt(torch.clamp((y_pred * y_pred).sum(-1, keepdim=True), min=1e-12))
    return -(a * b).sum(-1)


def categorical_hinge(y_true, y_pred, logits=None):
    pos = (y_true * y_pred).sum(-1)
    neg = ((1.0 - y_true) * y_pred).max(-1).values
    return torch.clamp(neg - pos + 1.0, min=0.0)


FUNCTIONS = {
    "categorical_crossentropy": categorical_crossentropy,
    "sparse_categorical_crossentropy": sparse_categorical_crossentropy,
    "binary_crossentropy": binary_crossentropy,
    "mean_squared_error": mean_squared_error,
    "mean_absolute_error": mean_absolute_error,
    "mean_absolute_percentage_error": mean_absolute_percentage_error,
    "mean_squared_logarithmic_error": mean_squared_logarithmic_error,
    "logcosh": logcosh, "hinge": hinge, "squared_hinge": squared_hinge,
    "kullback_leibler_divergence": kullback_leibler_divergence, "poisson": poisson,
    "cosine_similarity": cosine_similarity, "categorical_hinge": categorical_hinge,
}

def registered_names():
    """Every built-in loss name and alias (alias -> canonical via ``canonical``)."""
    return list(FUNCTIONS) + list(ALIASES)


# keras convenience aliases as module attributes
mse = MSE = mean_squared_error
mae = MAE = mean_absolute_error
mape = MAPE = mean_absolute_percentage_error
msle = MSLE = mean_squared_logarithmic_error
kld = KLD = kullback_leibler_divergence


class LossSpec:
    """Resolved loss: name (for serialization), torch fn, native id (or None)."""

    def __init__(self, identifier: Union[str, Callable], custom_objects: Optional[dict] = None):
        self.identifier = identifier
        if callable(identifier) and not isinstance(identifier, str):
            name = getattr(identifier, "__name__", "custom_loss")
            builtin = FUNCTIONS.get(canonical(name))
            if builtin is identifier or (builtin is not None and getattr(identifier, "__module__", "") == __name__):
                self.name, self.fn, self.native = canonical(name), builtin, LOSS_IDS.get(canonical(name))
            else:
                self.name, self.fn, self.native = name, identifier, None
        else:
            key = canonical(str(identifier))
            if custom_objects and identifier in custom_objects:
                self.name, self.fn, self.native = identifier, custom_objects[identifier], None
            elif key in FUNCTIONS:
                self.name, self.fn, self.native = key, FUNCTIONS[key], LOSS_IDS[key]
            else:
                raise ValueError(f"Unknown loss function: {identifier}")
        self.custom = self.native is None

    @property
    def converts_binary_labels(self) -> bool:
        return self.name in ("hinge", "squared_hinge")

    def __call__(self, y_true, y_pred, logits=None):
        if self.custom:
            return self.fn(y_true, y_pred)
        return self.fn(y_true, y_pred, logits)


def get(identifier, custom_objects=None) -> LossSpec:
    return identifier if isinstance(identifier, LossSpec) else LossSpec(identifier, custom_objects)
