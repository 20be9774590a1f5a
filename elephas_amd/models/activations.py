"""Activation registry (tf.keras 2.10 ``keras.activations`` names).

Each built-in activation has a torch implementation (CPU engine / autograd
fallback) and an integer id understood by the fused HIP epilogues
(csrc/kernels/args.h ``Act``).  Callables that are not built-ins are "custom"
activations: they run through the torch path and serialise by ``__name__``.
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Union

import torch
import torch.nn.functional as F

ACT_IDS = {
    "linear": 0, "relu": 1, "sigmoid": 2, "tanh": 3, "softmax": 4, "elu": 5, "selu": 6,
    "softplus": 7, "softsign": 8, "exponential": 9, "hard_sigmoid": 10, "swish": 11,
    "gelu": 12, "relu6": 13,
}

_SELU_A = 1.6732632423543772
_SELU_S = 1.0507009873554805


def linear(x):
    return x


def relu(x):
    return torch.relu(x)


def sigmoid(x):
    return torch.sigmoid(x)


def tanh(x):
    return torch.tanh(x)


def softmax(x, axis=-1):
    return torch.softmax(x, dim=axis)


def elu(x, alpha=1.0):
    return F.elu(x, alpha)


def selu(x):
    return _SELU_S * torch.where(x > 0, x, _SELU_A * torch.expm1(x))


def softplus(x):
    return F.softplus(x)


def softsign(x):
    return x / (torch.abs(x) + 1.0)


def exponential(x):
    return torch.exp(x)


def hard_sigmoid(x):
    return torch.clamp(0.2 * x + 0.5, 0.0, 1.0)


def swish(x):
    return x * torch.sigmoid(x)


def gelu(x, approximate=False):
    if approximate:
        return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def relu6(x):
    return torch.clamp(x, 0.0, 6.0)


_FNS = {
    "linear": linear, "relu": relu, "sigmoid": sigmoid, "tanh": tanh, "softmax": softmax, "elu": elu,
    "selu": selu, "softplus": softplus, "softsign": softsign, "exponential": exponential,
    "hard_sigmoid": hard_sigmoid, "swish": swish, "silu": swish, "gelu": gelu, "relu6": relu6,
}

_FN_TO_NAME = {v: k for k, v in _FNS.items() if k != "silu"}


def get(identifier: Union[None, str, Callable], custom_objects: Optional[dict] = None) -> Callable:
    if identifier is None:
        return linear
    if callable(identifier):
        return identifier
    if isinstance(identifier, dict):  # {'class_name': ..., 'config': ...} legacy form
        identifier = identifier.get("config", {}).get("name", identifier.get("class_name"))
    if isinstance(identifier, str):
        if custom_objects and identifier in custom_objects:
            return custom_objects[identifier]
        if identifier in _FNS:
            return _FNS[identifier]
        raise ValueError(f"Unknown activation function: {identifier}. Please ensure it is passed in custom_objects.")
    raise TypeError(f"Could not interpret activation identifier: {identifier!r}")


def serialize(fn: Callable) -> str:
    if fn in _FN_TO_NAME:
        return _FN_TO_NAME[fn]
    return getattr(fn, "__name__", str(fn))


def native_id(fn: Callable) -> Optional[int]:
    """Id of the fused HIP activation, or None for custom callables."""
    name = _FN_TO_NAME.get(fn)
    return ACT_IDS.get(name) if name is not None else None
