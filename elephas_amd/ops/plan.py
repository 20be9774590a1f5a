"""Lowering of a Keras-compatible model into a flat training plan.

A model is a chain ``Input -> (Dense [Activation] [Dropout])* -> loss``.  The
plan folds every Activation/Dropout into the Dense that precedes it (the HIP
epilogues apply them in the producing GEMM) and lays all weights out in one
flat fp32 vector in Keras ``get_weights()`` order (kernel ``[in,out]`` row-major,
then bias), which is also the all-reduce / parameter-server payload
(reference spark_model.py:205-227, server.py:117-132).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from ..models import activations as A
from ..models.layers import Activation, Dense, Dropout, Flatten, InputLayer


@dataclass
class DenseSpec:
    layer: Dense
    in_dim: int
    units: int
    use_bias: bool
    act_fn: object
    act_id: Optional[int]
    dropout: float = 0.0
    p_off: int = 0

    @property
    def n_params(self) -> int:
        return self.in_dim * self.units + (self.units if self.use_bias else 0)


@dataclass
class Plan:
    layers: List[DenseSpec]
    n_params: int
    native_ok: bool
    reason: str = ""
    ops: list = field(default_factory=list)  # original op chain (torch engine)

    @property
    def in_dim(self) -> int:
        return self.layers[0].in_dim

    @property
    def out_dim(self) -> int:
        return self.layers[-1].units


def chain_layers(model) -> list:
    """Ordered layers of a Sequential or chain-shaped functional model."""
    return [l for l in model.layers if not isinstance(l, InputLayer)]


def build_plan(model) -> Plan:
    ops = chain_layers(model)
    specs: List[DenseSpec] = []
    reason = ""
    off = 0
    for op in ops:
        if isinstance(op, Dense):
            s = DenseSpec(op, int(op.kernel.shape[0]), op.units, op.use_bias, op.activation,
                          A.native_id(op.activation), p_off=off)
            off += s.n_params
            specs.append(s)
        elif isinstance(op, Activation):
            if not specs:
                reason = reason or "activation before the first Dense"
                continue
            s = specs[-1]
            if s.act_id != A.ACT_IDS["linear"] or s.dropout > 0 or s.act_fn is not A.linear:
                reason = reason or "stacked activations"
            s.act_fn = op.activation
            s.act_id = A.native_id(op.activation)
        elif isinstance(op, Dropout):
            if not specs:
                reason = reason or "input dropout"
                continue
            if specs[-1].dropout > 0:
                reason = reason or "stacked dropout"
            specs[-1].dropout = op.rate
        elif isinstance(op, Flatten):
            continue
        else:
            reason = reason or f"unsupported layer {type(op).__name__}"
    if not specs:
        raise ValueError("model has no Dense layer")
    for i, s in enumerate(specs):
        if s.act_id is None:
            reason = reason or f"custom activation in {s.layer.name}"
        if s.act_id == A.ACT_IDS["softmax"] and i != len(specs) - 1:
            reason = reason or "softmax on a hidden layer"
    if len(specs) > 16:
        reason = reason or "more than 16 Dense layers"
    return Plan(specs, off, native_ok=not reason, reason=reason, ops=ops)


def flatten_weights(weights: List[np.ndarray]) -> np.ndarray:
    if not weights:
        return np.zeros(0, np.float32)
    return np.concatenate([np.asarray(w, np.float32).reshape(-1) for w in weights])


def unflatten_weights(flat: np.ndarray, like: List[np.ndarray]) -> List[np.ndarray]:
    out, o = [], 0
    for w in like:
        n = int(np.prod(w.shape))
        out.append(np.asarray(flat[o:o + n], np.float32).reshape(w.shape).copy())
        o += n
    if o != flat.size:
        raise ValueError(f"flat parameter vector has {flat.size} entries, model needs {o}")
    return out
