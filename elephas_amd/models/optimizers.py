"""Optimizers with tf.keras 2.10 ``optimizer_v2`` configs and update rules.

``serialize``/``deserialize``/``get`` produce and accept the same
``{'class_name', 'config'}`` dicts the reference ships to workers
(reference elephas/spark_model.py:17-18,54,193,200; ml_model.py:90;
tests/test_ml_model.py:68-69 ``SGD(learning_rate=0.01, decay=1e-6,
momentum=0.9, nesterov=True)``; legacy ``lr=`` at tests/integration/
test_end_to_end.py:39).

Each optimizer also exposes:
  * ``native()``   -> (opt id, hyper-parameter dict, state planes) for the fused
                      HIP update epilogue (csrc/kernels/common.h ``opt_update``),
                      or None if only the torch engine implements it;
  * ``apply_torch``-> the same rule on torch tensors (CPU engine / fallback).
"""
from __future__ import annotations

import copy
import math
from typing import Dict, List, Optional

import torch

OPT_SGD, OPT_RMSPROP, OPT_ADAM, OPT_ADAGRAD, OPT_ADAMAX = 0, 1, 2, 3, 4


class Optimizer:
    _defaults: Dict[str, object] = {}

    def __init__(self, name=None, **kwargs):
        lr = kwargs.pop("lr", None)
        if lr is not None and "learning_rate" not in kwargs:
            kwargs["learning_rate"] = lr
        self._hyper = dict(self._defaults)
        decay = kwargs.pop("decay", 0.0)
        for k in list(kwargs):
            if k in ("clipnorm", "clipvalue", "global_clipnorm"):
                self._hyper[k] = kwargs.pop(k)
        unknown = set(kwargs) - set(self._defaults)
        if unknown:
            raise TypeError(f"Unexpected keyword argument(s) for {type(self).__name__}: {sorted(unknown)}")
        self._hyper.update(kwargs)
        self._hyper["decay"] = float(decay)
        self._name = name or type(self).__name__
        self.iterations = 0

    # ---- keras-style accessors
    @property
    def learning_rate(self):
        return self._hyper["learning_rate"]

    @learning_rate.setter
    def learning_rate(self, v):
        self._hyper["learning_rate"] = float(v)

    lr = learning_rate

    @property
    def decay(self):
        return self._hyper["decay"]

    def get_config(self) -> dict:
        cfg = {"name": self._name}
        cfg["learning_rate"] = float(self._hyper["learning_rate"])
        cfg["decay"] = float(self._hyper["decay"])
        for k, v in self._hyper.items():
            if k not in ("learning_rate", "decay"):
                cfg[k] = v
        return cfg

    @classmethod
    def from_config(cls, config):
        config = dict(config)
        if "lr" in config and "learning_rate" not in config:
            config["learning_rate"] = config.pop("lr")
        config.pop("lr", None)
        config.pop("is_legacy_optimizer", None)
        for k in ("jit_compile", "use_ema", "ema_momentum", "ema_overwrite_frequency"):
            config.pop(k, None)
        return cls(**config)

    def __getattr__(self, item):
        hyper = self.__dict__.get("_hyper", {})
        if item in hyper:
            return hyper[item]
        raise AttributeError(item)

    def decayed_lr(self, iteration: int) -> float:
        return self._hyper["learning_rate"] / (1.0 + self._hyper["decay"] * iteration)

    # ---- engines
    def native(self):
        return None

    def n_state(self) -> int:
        return 0

    def slot_names(self) -> List[str]:
        """Keras 2.10 slot-variable names of the state planes, in engine plane order
        (HDF5 ``optimizer_weights``: '<optimizer>/<layer>/<kernel|bias>/<slot>:0')."""
        return []

    def init_state(self, params: List[torch.Tensor]) -> List[List[torch.Tensor]]:
        return [[torch.zeros_like(p) for _ in range(self.n_state())] for p in params]

    def apply_torch(self, params, grads, state, iteration: int):
        raise NotImplementedError


class SGD(Optimizer):
    _defaults = {"learning_rate": 0.01, "momentum": 0.0, "nesterov": False}

    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, name="SGD", **kwargs):
        if "lr" in kwargs:  # legacy keras argument
            learning_rate = kwargs.pop("lr")
        super().__init__(name=name, learning_rate=learning_rate, momentum=momentum, nesterov=nesterov, **kwargs)

    def native(self):
        h = self._hyper
        return OPT_SGD, {"lr": h["learning_rate"], "momentum": h["momentum"], "nesterov": int(bool(h["nesterov"])),
                         "decay": h["decay"]}, self.n_state()

    def n_state(self):
        return 1 if self._hyper["momentum"] > 0 else 0

    def slot_names(self):
        return ["momentum"] if self._hyper["momentum"] > 0 else []

    @torch.no_grad()
    def apply_torch(self, params, grads, state, iteration):
        lr = self.decayed_lr(iteration)
        m = self._hyper["momentum"]
        for p, g, s in zip(params, grads, state):
            if m == 0:
                p.sub_(lr * g)
            else:
                v = s[0]
                v.mul_(m).sub_(lr * g)
                if self._hyper["nesterov"]:
                    p.add_(m * v - lr * g)
                else:
                    p.add_(v)


class RMSprop(Optimizer):
    _defaults = {"learning_rate": 0.001, "rho": 0.9, "momentum": 0.0, "epsilon": 1e-7, "centered": False}

    def __init__(self, learning_rate=0.001, rho=0.9, momentum=0.0, epsilon=1e-07, centered=False, name="RMSprop", **kwargs):
        if "lr" in kwargs:  # legacy keras argument
            learning_rate = kwargs.pop("lr")
        super().__init__(name=name, learning_rate=learning_rate, rho=rho, momentum=momentum, epsilon=epsilon, centered=centered, **kwargs)

    def native(self):
        h = self._hyper
        if h["centered"]:
            return None
        return OPT_RMSPROP, {"lr": h["learning_rate"], "rho": h["rho"], "momentum": h["momentum"],
                             "epsilon": h["epsilon"], "decay": h["decay"]}, self.n_state()

    def n_state(self):
        return 1 + (1 if self._hyper["momentum"] > 0 else 0) + (1 if self._hyper["centered"] else 0)

    def slot_names(self):
        h = self._hyper
        return ["rms"] + (["momentum"] if h["momentum"] > 0 else []) + (["mg"] if h["centered"] else [])

    @torch.no_grad()
    def apply_torch(self, params, grads, state, iteration):
        h = self._hyper
        lr = self.decayed_lr(iteration)
        for p, g, s in zip(params, grads, state):
            ms = s[0]
            ms.mul_(h["rho"]).add_((1 - h["rho"]) * g * g)
            denom = ms
            idx = 1
            if h["momentum"] > 0:
                idx = 2
            if h["centered"]:
                mg = s[idx]
                mg.mul_(h["rho"]).add_((1 - h["rho"]) * g)
                denom = ms - mg * mg
            if h["momentum"] > 0:
                # tf.raw_ops.ResourceApply(Centered)RMSProp: epsilon inside the square root
                mom = s[1]
                mom.mul_(h["momentum"]).add_(lr * g / torch.sqrt(denom + h["epsilon"]))
                p.sub_(mom)
            else:
                p.sub_(lr * g / (torch.sqrt(denom) + h["epsilon"]))


class Adam(Optimizer):
    _defaults = {"learning_rate": 0.001, "beta_1": 0.9, "beta_2": 0.999, "epsilon": 1e-7, "amsgrad": False}

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-07, amsgrad=False, name="Adam", **kwargs):
        if "lr" in kwargs:  # legacy keras argument
            learning_rate = kwargs.pop("lr")
        super().__init__(name=name, learning_rate=learning_rate, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon, amsgrad=amsgrad, **kwargs)

    def native(self):
        h = self._hyper
        if h["amsgrad"]:
            return None
        return OPT_ADAM, {"lr": h["learning_rate"], "beta_1": h["beta_1"], "beta_2": h["beta_2"],
                          "epsilon": h["epsilon"], "decay": h["decay"]}, 2

    def n_state(self):
        return 3 if self._hyper["amsgrad"] else 2

    def slot_names(self):
        return ["m", "v"] + (["vhat"] if self._hyper["amsgrad"] else [])

    @torch.no_grad()
    def apply_torch(self, params, grads, state, iteration):
        h = self._hyper
        t = iteration + 1
        lr = self.decayed_lr(iteration)
        lr_t = lr * math.sqrt(1 - h["beta_2"] ** t) / (1 - h["beta_1"] ** t)
        for p, g, s in zip(params, grads, state):
            m, v = s[0], s[1]
            m.mul_(h["beta_1"]).add_((1 - h["beta_1"]) * g)
            v.mul_(h["beta_2"]).add_((1 - h["beta_2"]) * g * g)
            if h["amsgrad"]:
                vh = s[2]
                torch.maximum(vh, v, out=vh)
                p.sub_(lr_t * m / (torch.sqrt(vh) + h["epsilon"]))
            else:
                p.sub_(lr_t * m / (torch.sqrt(v) + h["epsilon"]))


class Adagrad(Optimizer):
    _defaults = {"learning_rate": 0.001, "initial_accumulator_value": 0.1, "epsilon": 1e-7}

    def __init__(self, learning_rate=0.001, initial_accumulator_value=0.1, epsilon=1e-07, name="Adagrad", **kwargs):
        if "lr" in kwargs:  # legacy keras argument
            learning_rate = kwargs.pop("lr")
        super().__init__(name=name, learning_rate=learning_rate, initial_accumulator_value=initial_accumulator_value, epsilon=epsilon, **kwargs)

    def native(self):
        h = self._hyper
        return OPT_ADAGRAD, {"lr": h["learning_rate"], "epsilon": h["epsilon"], "decay": h["decay"],
                             "state_init": h["initial_accumulator_value"]}, 1

    def n_state(self):
        return 1

    def slot_names(self):
        return ["accumulator"]

    def init_state(self, params):
        return [[torch.full_like(p, self._hyper["initial_accumulator_value"])] for p in params]

    @torch.no_grad()
    def apply_torch(self, params, grads, state, iteration):
        lr = self.decayed_lr(iteration)
        for p, g, s in zip(params, grads, state):
            s[0].add_(g * g)
            p.sub_(lr * g / (torch.sqrt(s[0]) + self._hyper["epsilon"]))


class Adamax(Optimizer):
    def slot_names(self):
        return ["m", "v"]

    _defaults = {"learning_rate": 0.001, "beta_1": 0.9, "beta_2": 0.999, "epsilon": 1e-7}

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-07, name="Adamax", **kwargs):
        if "lr" in kwargs:  # legacy keras argument
            learning_rate = kwargs.pop("lr")
        super().__init__(name=name, learning_rate=learning_rate, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon, **kwargs)

    def native(self):
        h = self._hyper
        return OPT_ADAMAX, {"lr": h["learning_rate"], "beta_1": h["beta_1"], "beta_2": h["beta_2"],
                            "epsilon": h["epsilon"], "decay": h["decay"]}, 2

    def n_state(self):
        return 2

    @torch.no_grad()
    def apply_torch(self, params, grads, state, iteration):
        h = self._hyper
        t = iteration + 1
        lr_t = self.decayed_lr(iteration) / (1 - h["beta_1"] ** t)
        for p, g, s in zip(params, grads, state):
            m, u = s[0], s[1]
            m.mul_(h["beta_1"]).add_((1 - h["beta_1"]) * g)
            torch.maximum(h["beta_2"] * u, torch.abs(g), out=u)
            p.sub_(lr_t * m / (u + h["epsilon"]))


class Adadelta(Optimizer):
    def slot_names(self):
        return ["accum_grad", "accum_var"]

    _defaults = {"learning_rate": 0.001, "rho": 0.95, "epsilon": 1e-7}

    def __init__(self, learning_rate=0.001, rho=0.95, epsilon=1e-07, name="Adadelta", **kwargs):
        if "lr" in kwargs:  # legacy keras argument
            learning_rate = kwargs.pop("lr")
        super().__init__(name=name, learning_rate=learning_rate, rho=rho, epsilon=epsilon, **kwargs)

    def n_state(self):
        return 2

    @torch.no_grad()
    def apply_torch(self, params, grads, state, iteration):
        h = self._hyper
        lr = self.decayed_lr(iteration)
        for p, g, s in zip(params, grads, state):
            ag, ad = s[0], s[1]
            ag.mul_(h["rho"]).add_((1 - h["rho"]) * g * g)
            upd = torch.sqrt(ad + h["epsilon"]) / torch.sqrt(ag + h["epsilon"]) * g
            ad.mul_(h["rho"]).add_((1 - h["rho"]) * upd * upd)
            p.sub_(lr * upd)


class Nadam(Optimizer):
    def slot_names(self):
        return ["m", "v"]

    _defaults = {"learning_rate": 0.001, "beta_1": 0.9, "beta_2": 0.999, "epsilon": 1e-7}

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-07, name="Nadam", **kwargs):
        if "lr" in kwargs:  # legacy keras argument
            learning_rate = kwargs.pop("lr")
        super().__init__(name=name, learning_rate=learning_rate, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon, **kwargs)

    def n_state(self):
        return 2

    def init_state(self, params):
        self._m_cache = 1.0
        return super().init_state(params)

    @torch.no_grad()
    def apply_torch(self, params, grads, state, iteration):
        h = self._hyper
        lr = self.decayed_lr(iteration)
        t = iteration + 1
        b1, b2 = h["beta_1"], h["beta_2"]
        mu_t = b1 * (1.0 - 0.5 * 0.96 ** (0.004 * t))
        mu_t1 = b1 * (1.0 - 0.5 * 0.96 ** (0.004 * (t + 1)))
        m_cache = getattr(self, "_m_cache", 1.0) * mu_t
        m_cache1 = m_cache * mu_t1
        self._m_cache = m_cache
        for p, g, s in zip(params, grads, state):
            m, v = s[0], s[1]
            g_prime = g / (1.0 - m_cache)
            m.mul_(b1).add_((1 - b1) * g)
            m_prime = m / (1.0 - m_cache1)
            v.mul_(b2).add_((1 - b2) * g * g)
            v_prime = v / (1.0 - b2 ** t)
            m_bar = (1.0 - mu_t) * g_prime + mu_t1 * m_prime
            p.sub_(lr * m_bar / (torch.sqrt(v_prime) + h["epsilon"]))


_CLASSES = {c.__name__: c for c in (SGD, RMSprop, Adam, Adagrad, Adamax, Adadelta, Nadam)}
_ALIASES = {"sgd": "SGD", "rmsprop": "RMSprop", "adam": "Adam", "adagrad": "Adagrad", "adamax": "Adamax",
            "adadelta": "Adadelta", "nadam": "Nadam"}


def serialize(optimizer: Optimizer) -> dict:
    return {"class_name": type(optimizer).__name__, "config": optimizer.get_config()}


def deserialize(config: dict, custom_objects: Optional[dict] = None) -> Optimizer:
    name = config["class_name"]
    if custom_objects and name in custom_objects:
        cls = custom_objects[name]
    else:
        cls = _CLASSES.get(_ALIASES.get(name.lower(), name), None) or _CLASSES.get(name)
    if cls is None:
        raise ValueError(f"Unknown optimizer: {name}")
    return cls.from_config(config.get("config", {}))


def get(identifier) -> Optimizer:
    if isinstance(identifier, Optimizer):
        return identifier
    if isinstance(identifier, dict):
        return deserialize(identifier)
    if isinstance(identifier, str):
        key = _ALIASES.get(identifier.lower(), identifier)
        if key not in _CLASSES:
            raise ValueError(f"Could not interpret optimizer identifier: {identifier}")
        return _CLASSES[key]()
    if identifier is None:
        return RMSprop()
    raise ValueError(f"Could not interpret optimizer identifier: {identifier!r}")


def clone(optimizer: Optimizer) -> Optimizer:
    return deserialize(serialize(optimizer))
