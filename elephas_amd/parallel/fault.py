"""Failure detection and fault injection.

The reference has none of its own (Spark task retry re-runs a failed
partition, which is not idempotent for async pushes). Here a failure is fatal and
visible instead of silent:

* collectives run with a timeout (``$ELEPHAS_AMD_COLLECTIVE_TIMEOUT`` seconds,
  default 600) and RCCL's asynchronous error handling, so a rank that dies or
  hangs makes its peers raise instead of blocking forever;
* worker threads (async / hogwild) re-raise their first exception in the driver;
* ``$ELEPHAS_AMD_FAULT_INJECT`` (``rank=R,phase=P[,after=N]``) raises
  ``InjectedFault`` on rank R the (N+1)-th time phase P is reached -- the hook the
  failure tests use. Phases: ``train``, ``allreduce``, ``push``, ``pull``, ``ps_selftest`` (the
  rank pushes a wrong delta in the device PS self-test, which must then fail),
  ``xrank_selftest`` (the rank sends a wrong tile in the in-launch rank-exchange self-test:
  every rank must then detach and keep the peer all-reduce path), ``bench_sub:<name>``
  (bench.py, at the start of a sub-measurement).  With ``stall=1`` the rank blocks
  forever instead of raising -- a hung rank, which bench.py's job-wide deadline
  (``$ELEPHAS_AMD_BENCH_DEADLINE_S``) must survive.
"""
from __future__ import annotations

import os
from typing import Dict

_counts: Dict[str, int] = {}


class InjectedFault(RuntimeError):
    pass


def collective_timeout_s(default: int = 600) -> int:
    return int(os.environ.get("ELEPHAS_AMD_COLLECTIVE_TIMEOUT", str(default)))


def enable_async_error_handling() -> None:
    """Make a hung / failed RCCL collective abort the process (torch watchdog)."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")


def _spec():
    raw = os.environ.get("ELEPHAS_AMD_FAULT_INJECT", "")
    if not raw:
        return None
    kv = dict(item.split("=", 1) for item in raw.split(",") if "=" in item)
    return (int(kv.get("rank", 0)), kv.get("phase", "train"), int(kv.get("after", 0)),
            kv.get("stall", "0") not in ("0", ""))


def maybe_inject(phase: str, rank: int) -> None:
    spec = _spec()
    if spec is None:
        return
    r, p, after, stall = spec
    if r != rank or p != phase:
        return
    n = _counts.get(phase, 0)
    _counts[phase] = n + 1
    if n >= after:
        if stall:
            import time
            while True:   # a hung rank: never returns (the caller's deadline must cope)
                time.sleep(3600)
        raise InjectedFault(f"injected fault: rank {rank}, phase {phase}, occurrence {n}")


def injection_active() -> bool:
    """True when a fault is configured (hooks must then run eagerly, not from a graph)."""
    return _spec() is not None


def reset() -> None:
    _counts.clear()
