"""Weight initializers with tf.keras 2.10 config names (Dense defaults:
GlorotUniform kernel, Zeros bias; reference tests/conftest.py:11-38)."""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

_global_rng = np.random.default_rng()


def set_seed(seed: int) -> None:
    global _global_rng
    _global_rng = np.random.default_rng(seed)


def _rng(seed):
    return np.random.default_rng(seed) if seed is not None else _global_rng


def _fans(shape):
    if len(shape) == 1:
        return shape[0], shape[0]
    return shape[0], shape[1]


class Initializer:
    def __call__(self, shape, dtype=np.float32):
        raise NotImplementedError

    def get_config(self) -> dict:
        return {}

    @classmethod
    def from_config(cls, config):
        return cls(**config)


class Zeros(Initializer):
    def __call__(self, shape, dtype=np.float32):
        return np.zeros(shape, dtype=dtype)


class Ones(Initializer):
    def __call__(self, shape, dtype=np.float32):
        return np.ones(shape, dtype=dtype)


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def __call__(self, shape, dtype=np.float32):
        return np.full(shape, self.value, dtype=dtype)

    def get_config(self):
        return {"value": self.value}


class RandomUniform(Initializer):
    def __init__(self, minval=-0.05, maxval=0.05, seed=None):
        self.minval, self.maxval, self.seed = minval, maxval, seed

    def __call__(self, shape, dtype=np.float32):
        return _rng(self.seed).uniform(self.minval, self.maxval, size=shape).astype(dtype)

    def get_config(self):
        return {"minval": self.minval, "maxval": self.maxval, "seed": self.seed}


class RandomNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05, seed=None):
        self.mean, self.stddev, self.seed = mean, stddev, seed

    def __call__(self, shape, dtype=np.float32):
        return _rng(self.seed).normal(self.mean, self.stddev, size=shape).astype(dtype)

    def get_config(self):
        return {"mean": self.mean, "stddev": self.stddev, "seed": self.seed}


class VarianceScaling(Initializer):
    def __init__(self, scale=1.0, mode="fan_in", distribution="truncated_normal", seed=None):
        self.scale, self.mode, self.distribution, self.seed = scale, mode, distribution, seed

    def __call__(self, shape, dtype=np.float32):
        fan_in, fan_out = _fans(shape)
        n = {"fan_in": fan_in, "fan_out": fan_out}.get(self.mode, (fan_in + fan_out) / 2.0)
        scale = self.scale / max(1.0, n)
        rng = _rng(self.seed)
        if self.distribution == "uniform":
            lim = math.sqrt(3.0 * scale)
            return rng.uniform(-lim, lim, size=shape).astype(dtype)
        if self.distribution == "untruncated_normal":
            return rng.normal(0.0, math.sqrt(scale), size=shape).astype(dtype)
        std = math.sqrt(scale) / 0.87962566103423978
        out = rng.normal(0.0, std, size=shape)
        bad = np.abs(out) > 2 * std
        while bad.any():
            out[bad] = rng.normal(0.0, std, size=int(bad.sum()))
            bad = np.abs(out) > 2 * std
        return out.astype(dtype)

    def get_config(self):
        return {"scale": self.scale, "mode": self.mode, "distribution": self.distribution, "seed": self.seed}


class GlorotUniform(VarianceScaling):
    def __init__(self, seed=None):
        super().__init__(1.0, "fan_avg", "uniform", seed)

    def get_config(self):
        return {"seed": self.seed}


class GlorotNormal(VarianceScaling):
    def __init__(self, seed=None):
        super().__init__(1.0, "fan_avg", "truncated_normal", seed)

    def get_config(self):
        return {"seed": self.seed}


class HeNormal(VarianceScaling):
    def __init__(self, seed=None):
        super().__init__(2.0, "fan_in", "truncated_normal", seed)

    def get_config(self):
        return {"seed": self.seed}


class HeUniform(VarianceScaling):
    def __init__(self, seed=None):
        super().__init__(2.0, "fan_in", "uniform", seed)

    def get_config(self):
        return {"seed": self.seed}


class LecunNormal(VarianceScaling):
    def __init__(self, seed=None):
        super().__init__(1.0, "fan_in", "truncated_normal", seed)

    def get_config(self):
        return {"seed": self.seed}


_CLASSES = {c.__name__: c for c in (Zeros, Ones, Constant, RandomUniform, RandomNormal, VarianceScaling,
                                    GlorotUniform, GlorotNormal, HeNormal, HeUniform, LecunNormal)}
_ALIASES = {"zeros": "Zeros", "ones": "Ones", "constant": "Constant", "random_uniform": "RandomUniform",
            "random_normal": "RandomNormal", "glorot_uniform": "GlorotUniform", "glorot_normal": "GlorotNormal",
            "he_normal": "HeNormal", "he_uniform": "HeUniform", "lecun_normal": "LecunNormal",
            "variance_scaling": "VarianceScaling"}


def get(identifier) -> Initializer:
    if isinstance(identifier, Initializer):
        return identifier
    if isinstance(identifier, str):
        return _CLASSES[_ALIASES.get(identifier, identifier)]()
    if isinstance(identifier, dict):
        cls = _CLASSES[_ALIASES.get(identifier["class_name"], identifier["class_name"])]
        return cls.from_config(identifier.get("config", {}))
    if callable(identifier):
        return identifier
    raise ValueError(f"Unknown initializer {identifier!r}")


def serialize(init: Initializer) -> dict:
    return {"class_name": type(init).__name__, "config": init.get_config()}
