"""Global runtime configuration: device, compute precision, engine selection.

Defaults: the first visible MI355X when there is one (native HIP engine), the
CPU otherwise (torch reference engine).  Compute precision follows Keras'
mixed-precision policy names: ``'float32'`` (exact-f32 MFMA) or
``'mixed_bfloat16'`` (bf16 MFMA operands, fp32 accumulation and fp32 master
weights / optimizer state).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

_device: Optional[torch.device] = None
_policy = os.environ.get("ELEPHAS_AMD_POLICY", "float32")
_engine = os.environ.get("ELEPHAS_AMD_ENGINE", "auto")  # auto | native | torch


def get_device() -> torch.device:
    global _device
    if _device is None:
        if torch.cuda.is_available():
            local = int(os.environ.get("LOCAL_RANK", "0"))
            _device = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        else:
            _device = torch.device("cpu")
    return _device


def set_device(device) -> None:
    global _device
    _device = torch.device(device)


def set_policy(policy: str) -> None:
    global _policy
    if policy not in ("float32", "mixed_bfloat16", "bfloat16"):
        raise ValueError(f"unsupported policy {policy}")
    _policy = "mixed_bfloat16" if policy == "bfloat16" else policy


def get_policy() -> str:
    return _policy


def set_engine(engine: str) -> None:
    global _engine
    if engine not in ("auto", "native", "torch"):
        raise ValueError(engine)
    _engine = engine


def get_engine() -> str:
    return _engine
