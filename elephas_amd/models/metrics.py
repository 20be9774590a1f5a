"""Metric registry (tf.keras 2.10 ``compile(metrics=...)`` strings).

``'acc'``/``'accuracy'`` resolves by output shape exactly as Keras'
``MetricsContainer._get_metric_object``: one output unit -> binary accuracy,
sparse integer targets -> sparse categorical accuracy, otherwise categorical
accuracy.  Loss names used as metrics evaluate the loss per sample.
The history key is the string the user passed (``'acc'`` -> ``history['acc']``).
"""
from __future__ import annotations

from typing import Callable, Optional, Union

import torch

from . import losses as L

MET_ACC_CAT, MET_ACC_SPARSE, MET_ACC_BIN = 100, 101, 102


def categorical_accuracy(y_true, y_pred, logits=None):
    return (torch.argmax(y_true, -1) == torch.argmax(y_pred, -1)).to(y_pred.dtype)


def sparse_categorical_accuracy(y_true, y_pred, logits=None):
    return (y_true.reshape(-1).long() == torch.argmax(y_pred, -1)).to(y_pred.dtype)


def binary_accuracy(y_true, y_pred, logits=None, threshold=0.5):
    return ((y_pred > threshold).to(y_pred.dtype) == y_true).to(y_pred.dtype).mean(-1)


def top_k_categorical_accuracy(y_true, y_pred, logits=None, k=5):
    topk = torch.topk(y_pred, min(k, y_pred.shape[-1]), dim=-1).indices
    return (topk == torch.argmax(y_true, -1, keepdim=True)).any(-1).to(y_pred.dtype)


def cosine_similarity_metric(y_true, y_pred, logits=None):
    return -L.cosine_similarity(y_true, y_pred)


ACC_FUNCS = {MET_ACC_CAT: categorical_accuracy, MET_ACC_SPARSE: sparse_categorical_accuracy,
             MET_ACC_BIN: binary_accuracy}


class MetricSpec:
    def __init__(self, identifier: Union[str, Callable], n_out: int, loss: "L.LossSpec",
                 custom_objects: Optional[dict] = None):
        self.identifier = identifier
        if callable(identifier) and not isinstance(identifier, str):
            self.name = getattr(identifier, "__name__", "metric")
            self.fn, self.native = identifier, None
            self.custom = True
            return
        name = str(identifier)
        self.name = name
        self.custom = False
        if name in ("acc", "accuracy"):
            if n_out == 1:
                kind = MET_ACC_BIN
            elif loss is not None and loss.name == "sparse_categorical_crossentropy":
                kind = MET_ACC_SPARSE
            else:
                kind = MET_ACC_CAT
            self.fn, self.native = ACC_FUNCS[kind], kind
        elif name == "categorical_accuracy":
            self.fn, self.native = categorical_accuracy, MET_ACC_CAT
        elif name == "sparse_categorical_accuracy":
            self.fn, self.native = sparse_categorical_accuracy, MET_ACC_SPARSE
        elif name == "binary_accuracy":
            self.fn, self.native = binary_accuracy, MET_ACC_BIN
        elif name in ("top_k_categorical_accuracy",):
            self.fn, self.native = top_k_categorical_accuracy, None
        elif name == "cosine_similarity":
            self.fn, self.native = cosine_similarity_metric, L.LOSS_IDS["cosine_similarity"]
        elif name in ("crossentropy", "ce"):
            lname = loss.name if loss is not None else "categorical_crossentropy"
            self.fn, self.native = L.FUNCTIONS.get(lname, L.categorical_crossentropy), L.LOSS_IDS.get(lname)
        else:
            key = L.canonical(name)
            if custom_objects and name in custom_objects:
                self.fn, self.native, self.custom = custom_objects[name], None, True
            elif key in L.FUNCTIONS:
                self.fn, self.native = L.FUNCTIONS[key], L.LOSS_IDS[key]
            else:
                raise ValueError(f"Unknown metric function: {name}")

    def __call__(self, y_true, y_pred, logits=None):
        if self.custom:
            return self.fn(y_true, y_pred)
        return self.fn(y_true, y_pred, logits)


def get(identifier, n_out, loss, custom_objects=None) -> MetricSpec:
    return identifier if isinstance(identifier, MetricSpec) else MetricSpec(identifier, n_out, loss, custom_objects)
