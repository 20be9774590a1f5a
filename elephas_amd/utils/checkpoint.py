"""Resumable training checkpoints (an extension: the reference only saves the
final model, spark_model.py:92-134, and re-creates the optimizer every fit).

Layout of ``directory``:
  model.h5             the averaged master network as a Keras HDF5 file with the
                       ``distributed_config`` root attribute (loadable with
                       ``load_spark_model``)
  weights.npy          the same weights as one flat fp32 vector (Keras order)
  state_rank<r>.npz    rank r's optimizer state planes [R_local, planes, n] and
                       per-worker iteration counters, tagged with the epoch
  checkpoint.json      {"epoch": done, "epochs": total, "world_size": W} -- written
                       last, so a reader never sees an epoch whose weights are missing

Every file is written to a temporary name and moved into place (atomic on
POSIX). Loading uses only non-executing loaders (``numpy.load`` with
``allow_pickle=False``, JSON).
"""
from __future__ import annotations

import json
import os
from typing import Optional, Tuple

import numpy as np

META = "checkpoint.json"


def _atomic(path: str, write) -> None:
    tmp = path + ".tmp"
    write(tmp)
    os.replace(tmp, path)


def _save_npz(p, **arrays):
    with open(p, "wb") as f:
        np.savez(f, **arrays)


def _save_npy(p, a):
    with open(p, "wb") as f:
        np.save(f, a)


def _save_text(p, text):
    with open(p, "w") as f:
        f.write(text)


def exists(directory: str) -> bool:
    return os.path.exists(os.path.join(directory, META))


def save(directory: str, epoch: int, epochs: int, model, weights: np.ndarray, state, rank: int,
         distributed_config: Optional[dict] = None) -> None:
    os.makedirs(directory, exist_ok=True)
    if state is not None:
        S, iters = state
        _atomic(os.path.join(directory, f"state_rank{rank}.npz"),
                lambda p: _save_npz(p, S=np.asarray(S, np.float32), iters=np.asarray(iters, np.int64),
                                    epoch=np.int64(epoch)))
    if rank != 0:
        return
    _atomic(os.path.join(directory, "weights.npy"), lambda p: _save_npy(p, np.asarray(weights, np.float32)))

    def write_h5(p):
        model.save(p + ".h5")
        if distributed_config is not None:
            from ..io import h5lite
            f = h5lite.File(p + ".h5", mode="a")
            f.attrs["distributed_config"] = json.dumps(distributed_config).encode("utf8")
            f.flush()
            f.close()
        os.replace(p + ".h5", p)
    _atomic(os.path.join(directory, "model.h5"), write_h5)
    meta = {"epoch": int(epoch), "epochs": int(epochs)}
    _atomic(os.path.join(directory, META), lambda p: _save_text(p, json.dumps(meta)))


def load(directory: str, rank: int, n_local: int) -> Tuple[int, np.ndarray, Optional[tuple]]:
    """Returns (epochs done, flat weights, (state, iterations) or None)."""
    with open(os.path.join(directory, META)) as f:
        meta = json.load(f)
    weights = np.load(os.path.join(directory, "weights.npy"), allow_pickle=False)
    state = None
    sp = os.path.join(directory, f"state_rank{rank}.npz")
    if os.path.exists(sp):
        with np.load(sp, allow_pickle=False) as z:
            if int(z["epoch"]) == int(meta["epoch"]) and z["S"].shape[0] == max(n_local, 1):
                state = (z["S"].copy(), z["iters"].copy())
    return int(meta["epoch"]), weights, state
