"""Shared trainer logic for the torch reference engine and the native HIP engine.

A trainer holds R independent replicas of one model ("logical workers"; one
per Spark partition in the reference, elephas/worker.py:26-49) with their own
weights, optimizer state and data shard, and reproduces tf.keras 2.10
``Model.fit`` semantics per replica:
  * ``validation_split`` takes the LAST fraction of the shard before shuffling
    (keras data_adapter.train_validation_split: ``split_at = floor(n*(1-vs))``);
  * training rows are reshuffled every epoch;
  * batches of ``batch_size`` rows, the last one partial;
  * the reported epoch loss/metrics are sample-weighted means over the epoch
    computed with the pre-update weights of each batch; ``val_*`` are computed
    after the epoch with dropout off.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..models import losses as L


def prepare_targets(y: np.ndarray, n_out: int, loss: "L.LossSpec") -> np.ndarray:
    y = np.asarray(y)
    if loss.name == "sparse_categorical_crossentropy":
        return y.reshape(-1, 1).astype(np.float32)
    y = y.astype(np.float32)
    if y.ndim == 1:
        y = y.reshape(-1, 1)
    if y.shape[1] != n_out:
        if y.shape[1] == 1 and n_out > 1:
            raise ValueError(f"targets have 1 column but the model has {n_out} outputs "
                             f"(one-hot encode them or use sparse_categorical_crossentropy)")
        raise ValueError(f"targets have {y.shape[1]} columns, model outputs {n_out}")
    if loss.converts_binary_labels and np.isin(y, (0.0, 1.0)).all():
        y = 2.0 * y - 1.0  # keras losses._maybe_convert_labels
    return y


def prepare_features(x: np.ndarray, in_dim: int) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32)
    if x.ndim == 1:
        x = x.reshape(-1, 1) if in_dim == 1 else x.reshape(1, -1)
    if x.ndim > 2:
        x = x.reshape(x.shape[0], -1)
    if x.shape[1] != in_dim:
        raise ValueError(f"input has {x.shape[1]} features, model expects {in_dim}")
    return x


def split_point(n: int, validation_split: float) -> int:
    if validation_split and validation_split > 0:
        return int(math.floor(n * (1.0 - validation_split)))
    return n


class TrainerBase:
    """Interface shared by TorchTrainer and NativeTrainer."""

    def __init__(self, model, plan, R: int, batch_size: int):
        self.model = model
        self.plan = plan
        self.R = int(R)
        self.B = int(batch_size)
        self.loss = model._loss_spec
        self.metrics = list(model._metric_specs)
        self.metric_names = [m.name for m in self.metrics]
        self.n_out = plan.out_dim
        self.in_dim = plan.in_dim

    # ---------------------------------------------------------------- weights
    def set_weights_flat(self, flat: np.ndarray) -> None:
        raise NotImplementedError

    def get_weights_flat(self) -> np.ndarray:
        """[R, n_params] fp32"""
        raise NotImplementedError

    def get_state_flat(self):
        """Optimizer state for checkpoints: ([R, planes, n_params] fp32, iterations [R])."""
        raise NotImplementedError

    def set_state_flat(self, state: np.ndarray, iterations) -> None:
        raise NotImplementedError

    # ------------------------------------------------------------------- data
    def set_data(self, xs: Sequence[np.ndarray], ys: Sequence[np.ndarray], validation_split: float = 0.0,
                 active: Optional[Sequence[bool]] = None, shuffle: bool = True) -> None:
        raise NotImplementedError

    def fit(self, epochs: int, verbose: int = 0) -> List[Dict[str, list]]:
        raise NotImplementedError

    def evaluate(self, x: np.ndarray, y: np.ndarray, batch_size: Optional[int] = None) -> List[float]:
        raise NotImplementedError

    def predict(self, x: np.ndarray, batch_size: Optional[int] = None) -> np.ndarray:
        raise NotImplementedError

    # shared helpers
    def _history_from_sums(self, sums: np.ndarray, prefix: str = "") -> Dict[str, float]:
        """sums = [loss_sum, count, metric sums...]"""
        cnt = max(float(sums[1]), 1.0)
        h = {prefix + "loss": float(sums[0] / cnt)}
        for i, name in enumerate(self.metric_names):
            h[prefix + name] = float(sums[2 + i] / cnt)
        return h

    @staticmethod
    def print_epoch(epoch: int, epochs: int, h: Dict[str, float], r: int = 0) -> None:
        items = " - ".join(f"{k}: {v:.4f}" for k, v in h.items())
        print(f"Epoch {epoch + 1}/{epochs} [worker {r}] - {items}", flush=True)
