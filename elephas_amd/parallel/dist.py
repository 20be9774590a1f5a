"""Process-group helpers: one process per GPU, torch.distributed over RCCL.

``init_from_env`` joins the job started by ``torchrun`` (RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT); backend 'nccl' (= RCCL over xGMI on ROCm) when the
process owns a GPU, 'gloo' on CPU.  Without a launcher everything degrades to
rank 0 of a world of 1, so the same SparkModel code runs single-process.

Collectives used by the engine (SURVEY.md §2.6 call sites C1-C13):
  * ``all_reduce_sum_``  -- sync averaging of the flat parameter/delta vector
                            (C2/C3) and of evaluation sums (C10)
  * ``broadcast_``       -- initial weights / final PS weights (C1/C8)
  * ``all_gather_object``-- histories, predictions (C9/C11)
"""
from __future__ import annotations

import os
from datetime import timedelta
from typing import Any, List

import torch
import torch.distributed as dist


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def init_from_env(backend: str = None, timeout_s: int = None) -> bool:
    """Join a torchrun-style job if the environment describes one. Collectives
    time out after ``timeout_s`` (``$ELEPHAS_AMD_COLLECTIVE_TIMEOUT``, default 600 s)
    and RCCL errors abort asynchronously (see parallel/fault.py)."""
    from . import fault
    if is_initialized():
        return True
    timeout_s = fault.collective_timeout_s() if timeout_s is None else timeout_s
    fault.enable_async_error_handling()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return False
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        # ELEPHAS_AMD_DIST_BACKEND=gloo: rehearsal of a multi-rank GPU job on ONE GPU
        # (RCCL refuses two ranks on one device; the peer kernels do not)
        backend = os.environ.get("ELEPHAS_AMD_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    dist.init_process_group(backend=backend, timeout=timedelta(seconds=timeout_s))
    _detect_device_sharing()
    return True


_SHARERS = 1


def _device_key():
    import socket
    if not torch.cuda.is_available():
        return (socket.gethostname(), "cpu", os.getpid())
    p = torch.cuda.get_device_properties(torch.cuda.current_device())
    uuid = str(getattr(p, "uuid", "")) or "%x:%x" % (getattr(p, "pci_bus_id", -1), getattr(p, "pci_device_id", -1))
    return (socket.gethostname(), uuid)


def _detect_device_sharing():
    """How many ranks of the job run on this rank's GPU (same host and device UUID / PCI
    id): > 1 only in single-GPU multi-rank rehearsals.  A rank that sees ONE device of
    an 8-GPU node (HIP_VISIBLE_DEVICES per rank) is not sharing, whatever
    LOCAL_WORLD_SIZE says.  Collective: called by every rank in init_from_env."""
    global _SHARERS
    keys = all_gather_object(_device_key())
    me = keys[rank()]
    _SHARERS = max(1, sum(1 for k in keys if k == me))


def device_sharers() -> int:
    """Ranks of this job that share this process's GPU (1 when it owns it)."""
    return _SHARERS


def rank() -> int:
    return dist.get_rank() if is_initialized() else 0


def world_size() -> int:
    return dist.get_world_size() if is_initialized() else 1


def backend() -> str:
    return dist.get_backend() if is_initialized() else "none"


def _comm_device() -> torch.device:
    if is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_sum_(t: torch.Tensor) -> torch.Tensor:
    """In-place sum across ranks; moves through the backend's device if needed.
    fp32 CUDA tensors of an RCCL job go through the peer-memory all-reduce
    (parallel/p2p.py) up to its size limit."""
    if not is_initialized() or world_size() == 1:
        return t
    dev = _comm_device()
    if t.is_cuda:
        from . import p2p
        peer = p2p.get()
        if peer is not None and peer.eligible(t):
            return peer.all_reduce_(t)
    if t.device == dev or (t.device.type == dev.type == "cuda"):
        dist.all_reduce(t)
        return t
    tmp = t.to(dev)
    dist.all_reduce(tmp)
    t.copy_(tmp.to(t.device))
    return t


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if not is_initialized() or world_size() == 1:
        return t
    dev = _comm_device()
    if t.device.type == dev.type:
        dist.broadcast(t, src)
        return t
    tmp = t.to(dev)
    dist.broadcast(tmp, src)
    t.copy_(tmp.to(t.device))
    return t


def all_gather_object(obj: Any) -> List[Any]:
    if not is_initialized() or world_size() == 1:
        return [obj]
    out = [None] * world_size()
    dist.all_gather_object(out, obj)
    return out


def all_gather_rows(local, n: int):
    """Concatenate, in rank order, every rank's ``block_range(n)`` rows (numpy arrays of
    one trailing shape) with ONE tensor all-gather on the backend's device (RCCL over
    xGMI on GPUs) instead of pickling arrays through ``all_gather_object``."""
    import numpy as np
    local = np.asarray(local, np.float32)
    if not is_initialized() or world_size() == 1:
        return local
    w = world_size()
    sizes = [hi - lo for lo, hi in (block_range(n, r, w) for r in range(w))]
    mx = max(max(sizes), 1)
    dev = _comm_device()
    buf = torch.zeros((mx,) + local.shape[1:], dtype=torch.float32, device=dev)
    if len(local):
        buf[:len(local)].copy_(torch.from_numpy(np.ascontiguousarray(local)))
    out = torch.empty((w * mx,) + local.shape[1:], dtype=torch.float32, device=dev)
    dist.all_gather_into_tensor(out, buf)
    host = out.cpu().numpy()
    return np.concatenate([host[r * mx:r * mx + sizes[r]] for r in range(w)])


def broadcast_object(obj: Any, src: int = 0) -> Any:
    if not is_initialized() or world_size() == 1:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src)
    return box[0]


def barrier() -> None:
    """Host barrier.  On an RCCL job whose peer-memory all-reduce is up, a 1-element
    peer all-reduce + device sync: every rank's kernel waits for every peer's flag,
    which a peer only raises after reaching this call (~10 us instead of an RCCL
    barrier's all-reduce round trip through the proxy threads)."""
    if is_initialized() and world_size() > 1:
        if dist.get_backend() == "nccl":
            from . import p2p
            peer = p2p.current()
            if peer is not None:
                peer.barrier()
                return
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def any_failed(failed: bool) -> bool:
    """Collective failure vote (replaces a barrier at the end of a phase): every rank
    contributes whether it failed; all ranks learn whether ANY did, so the healthy
    ones raise too instead of waiting in the next collective until it times out."""
    if not is_initialized() or world_size() == 1:
        return bool(failed)
    t = torch.tensor([1.0 if failed else 0.0], dtype=torch.float32, device=_comm_device())
    dist.all_reduce(t)
    return bool(t.item() > 0)


def block_range(n: int, r: int = None, w: int = None):
    """Contiguous block [lo, hi) of n items owned by rank r of w."""
    r = rank() if r is None else r
    w = world_size() if w is None else w
    return r * n // w, (r + 1) * n // w
