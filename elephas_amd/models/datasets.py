"""Offline dataset loaders with the keras.datasets signatures.

There is no network access: ``load_data`` reads a local ``.npz`` when one
exists (``path`` argument, or ``~/.keras/datasets/<name>.npz``; loaded with
``allow_pickle=False``) and otherwise returns SYNTHETIC data of the real shape
and dtype, generated from a fixed seed, with a class-dependent signal so that
models can actually learn from it.  Benchmarks and tests state which they used.
"""
from __future__ import annotations

import os
import warnings

import numpy as np


def _local(name, path):
    cands = [path] if path else []
    cands.append(os.path.expanduser(f"~/.keras/datasets/{name}.npz"))
    for p in cands:
        if p and os.path.exists(p):
            with np.load(p, allow_pickle=False) as f:
                return {k: f[k] for k in f.files}
    return None


def synthetic_classification(n, in_dim, n_classes, seed=0, dtype=np.float32, scale=1.0):
    """Gaussian class clusters: learnable, deterministic."""
    rng = np.random.default_rng(seed)
    centers = rng.normal(0.0, 1.0, size=(n_classes, in_dim)).astype(np.float32)
    y = rng.integers(0, n_classes, size=n)
    x = centers[y] + rng.normal(0.0, 1.5, size=(n, in_dim)).astype(np.float32)
    return (x * scale).astype(dtype), y


class _MNIST:
    @staticmethod
    def load_data(path="mnist.npz"):
        d = _local("mnist", path if path and os.path.isabs(path) else None)
        if d is not None:
            return (d["x_train"], d["y_train"]), (d["x_test"], d["y_test"])
        warnings.warn("MNIST not available offline: returning synthetic MNIST-shaped data (uint8 28x28, 10 classes)")
        x, y = synthetic_classification(70000, 784, 10, seed=1234)
        x = np.clip((x - x.min()) / (x.max() - x.min()) * 255.0, 0, 255).astype(np.uint8).reshape(-1, 28, 28)
        return (x[:60000], y[:60000].astype(np.uint8)), (x[60000:], y[60000:].astype(np.uint8))


class _Boston:
    @staticmethod
    def load_data(path="boston_housing.npz", test_split=0.2, seed=113):
        d = _local("boston_housing", path if path and os.path.isabs(path) else None)
        if d is not None:
            x, y = d["x"], d["y"]
        else:
            warnings.warn("Boston housing not available offline: returning synthetic data of the same shape (506x13)")
            rng = np.random.default_rng(seed)
            x = rng.uniform(0, 100, size=(506, 13)).astype(np.float64)
            w = rng.normal(0, 0.1, size=13)
            y = np.clip(x @ w + 22.0 + rng.normal(0, 2.0, 506), 5.0, 50.0)
        n_train = int(len(x) * (1 - test_split))
        return (x[:n_train], y[:n_train]), (x[n_train:], y[n_train:])


mnist = _MNIST()
boston_housing = _Boston()
