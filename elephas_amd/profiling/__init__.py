"""Tracing, timers and metrics for training / inference runs.

The reference has no tracing at all (only Keras ``verbose``
output and ``print('>>> ...')`` markers, reference spark_model.py:181-228).
This module adds, without changing any numerics:

* ``trace_range(name)`` -- a ROCTx range (``torch.cuda.nvtx`` maps to roctx on
  ROCm builds) so ``rocprofv3 --marker-trace`` / ``--sys-trace`` shows the fit,
  epoch, all-reduce and checkpoint phases around the HIP kernels; a no-op
  without a GPU.
* ``PhaseTimer`` -- wall-clock phase accounting; on a GPU each phase is
  bracketed by device synchronisation of the given stream so the time covers the
  queued kernels, not just their launches.
* ``MetricsLogger`` -- JSON-lines sink (``$ELEPHAS_AMD_METRICS`` or an explicit
  path); rank 0 writes, one record per event (samples/s, step time, comm time).

``SparkModel.fit`` records its phases here; the result is available as
``spark_model.metrics`` and, when a sink is configured, as JSONL records.
"""
from __future__ import annotations

import contextlib
import json
import os
import time
from typing import Any, Dict, Iterator, Optional

_ENABLED = os.environ.get("ELEPHAS_AMD_TRACE", "1") != "0"


def _nvtx():
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:  # pragma: no cover - torch without ROCm
        pass
    return None


@contextlib.contextmanager
def trace_range(name: str) -> Iterator[None]:
    """ROCTx range around a host-side phase (visible in rocprofv3 marker traces)."""
    nv = _nvtx() if _ENABLED else None
    if nv is not None:
        nv.range_push(name)
    try:
        yield
    finally:
        if nv is not None:
            nv.range_pop()


def mark(name: str) -> None:
    nv = _nvtx() if _ENABLED else None
    if nv is not None:
        nv.mark(name)


class PhaseTimer:
    """Accumulates seconds per named phase: ``with timer.phase('allreduce'): ...``.

    ``sync`` is called before reading the clock at both ends of a phase (e.g.
    ``torch.cuda.synchronize``) so asynchronous device work is attributed to the
    phase that queued it.
    """

    def __init__(self, sync=None):
        self.sync = sync
        self.totals: Dict[str, float] = {}
        self.counts: Dict[str, int] = {}

    @contextlib.contextmanager
    def phase(self, name: str) -> Iterator[None]:
        with trace_range(name):
            if self.sync is not None:
                self.sync()
            t0 = time.perf_counter()
            try:
                yield
            finally:
                if self.sync is not None:
                    self.sync()
                dt = time.perf_counter() - t0
                self.totals[name] = self.totals.get(name, 0.0) + dt
                self.counts[name] = self.counts.get(name, 0) + 1

    def as_dict(self) -> Dict[str, float]:
        return {k: round(v, 6) for k, v in self.totals.items()}


def device_sync():
    """A sync function for PhaseTimer: device-wide synchronize when a GPU is in use."""
    try:
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            return torch.cuda.synchronize
    except Exception:  # pragma: no cover
        pass
    return None


class MetricsLogger:
    """JSON-lines metrics sink. ``path=None`` reads ``$ELEPHAS_AMD_METRICS``;
    with neither, records are only kept in memory (``records``)."""

    def __init__(self, path: Optional[str] = None, rank: int = 0):
        self.path = path if path is not None else os.environ.get("ELEPHAS_AMD_METRICS")
        self.rank = rank
        self.records = []

    def log(self, event: str, **fields: Any) -> Dict[str, Any]:
        rec = {"ts": round(time.time(), 6), "event": event, "rank": self.rank}
        rec.update(fields)
        self.records.append(rec)
        if self.path and self.rank == 0:
            d = os.path.dirname(os.path.abspath(self.path))
            os.makedirs(d, exist_ok=True)
            with open(self.path, "a") as f:
                f.write(json.dumps(rec, default=float) + "\n")
        return rec


__all__ = ["trace_range", "mark", "PhaseTimer", "device_sync", "MetricsLogger"]
