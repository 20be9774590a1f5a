"""Engine selection: native HIP executor on an MI355X, torch reference otherwise.

``auto`` picks the native executor whenever a GPU is present and the model's
plan is fully fusable (built-in activations, loss, metrics and optimizer);
models with custom callables run on the torch engine on the same device.  With
a GPU present the native runtime must load (``native.require`` raises), so a
supported model never silently falls back.
"""
from __future__ import annotations

import logging
from typing import Optional

from .. import config
from . import native
from .plan import build_plan

log = logging.getLogger("elephas_amd")


def native_supported(model, plan=None) -> (bool, str):
    plan = plan or build_plan(model)
    if not plan.native_ok:
        return False, plan.reason
    if model._loss_spec.native is None:
        return False, f"custom loss {model._loss_spec.name}"
    if any(m.native is None for m in model._metric_specs):
        return False, "custom metric"
    if len(model._metric_specs) > 4:
        return False, "more than 4 metrics"
    if model.optimizer.native() is None:
        return False, f"optimizer {type(model.optimizer).__name__}"
    return True, ""


def make_trainer(model, replicas: int = 1, batch_size: int = 32, device=None, engine: Optional[str] = None,
                 seed: Optional[int] = None, **native_kw):
    """Native executor on a GPU when the model is supported (``native_kw`` go to
    NativeTrainer, e.g. persist=0), else the torch reference engine."""
    device = device if device is not None else config.get_device()
    engine = engine or config.get_engine()
    plan = build_plan(model)
    import torch
    dev = torch.device(device)
    if engine == "native" or (engine == "auto" and dev.type == "cuda"):
        ok, why = native_supported(model, plan)
        if ok:
            native.require()
            from .native_engine import NativeTrainer
            return NativeTrainer(model, plan, replicas, batch_size, dev, seed=seed, **native_kw)
        if engine == "native":
            raise ValueError(f"native engine cannot run this model: {why}")
        log.info("elephas_amd: torch engine on %s (%s)", dev, why)
    from .torch_engine import TorchTrainer
    return TorchTrainer(model, plan, replicas, batch_size, dev, seed=seed)
