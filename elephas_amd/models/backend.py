"""Backend functions for user-defined (``custom_objects``) activations and losses.

The reference tests write custom activations against ``tensorflow.keras.backend``
(reference tests/integration/test_custom_models.py:16-17 ``sigmoid(x) + 1``,
tests/test_ml_model.py:245-246 ``2 * relu(x)``).  Here they operate on torch
tensors, so a custom callable runs unchanged on the CPU engine and, through the
torch-ROCm autograd fallback, on an MI355X.
"""
from __future__ import annotations

import torch

epsilon_value = 1e-7


def epsilon() -> float:
    return epsilon_value


def sigmoid(x):
    return torch.sigmoid(x)


def relu(x, alpha=0.0, max_value=None, threshold=0.0):
    if alpha == 0.0 and max_value is None and threshold == 0.0:
        return torch.relu(x)
    y = torch.where(x >= threshold, x, alpha * (x - threshold))
    if max_value is not None:
        y = torch.clamp(y, max=max_value)
    return y


def tanh(x):
    return torch.tanh(x)


def softmax(x, axis=-1):
    return torch.softmax(x, dim=axis)


def exp(x):
    return torch.exp(x)


def log(x):
    return torch.log(x)


def square(x):
    return x * x


def sqrt(x):
    return torch.sqrt(x)


def abs(x):  # noqa: A001 - keras name
    return torch.abs(x)


def mean(x, axis=None, keepdims=False):
    return torch.mean(x) if axis is None else torch.mean(x, dim=axis, keepdim=keepdims)


def sum(x, axis=None, keepdims=False):  # noqa: A001 - keras name
    return torch.sum(x) if axis is None else torch.sum(x, dim=axis, keepdim=keepdims)


def clip(x, lo, hi):
    return torch.clamp(x, lo, hi)


def maximum(x, y):
    return torch.maximum(x, torch.as_tensor(y, dtype=x.dtype, device=x.device))


def minimum(x, y):
    return torch.minimum(x, torch.as_tensor(y, dtype=x.dtype, device=x.device))


def softplus(x):
    return torch.nn.functional.softplus(x)


def elu(x, alpha=1.0):
    return torch.nn.functional.elu(x, alpha)
