"""Native MI355X training engine: device buffers + the C++ ``Executor``.

Memory layout (per replica r; everything stays resident in HBM):
  P    fp32 [R, n]            master weights, Keras flat order (all-reduce / PS payload)
  S    fp32 [R, k, n]         optimizer state planes
  G    fp32 [R, n]            gradients (per-step all-reduce path only)
  Wsh  T    [R, 2, sum K*Np]  row-major weight image, 2 parities (read by DX GEMMs)
  WTsh T    [R, 2, sum N*Kp]  transposed weight image, 2 parities (read by FWD GEMMs)
  X    T    [R, nmax, Kp0]    the replica's data shard (padded rows), Y fp32 [R, nmax, ldy]
  per layer workspaces Z/D/D^T/dZ/dZ^T for one batch
T is bf16 under the 'mixed_bfloat16' policy and fp32 otherwise.  The fused
update epilogue writes the next step's shadow parity while this step's DX
GEMMs still read the current one, so DW and DX of a layer share one launch.

A training step is 3 launches on the row-chain plan (small MLPs: every layer but
the last <= 256 wide, a last layer <= 32 wide -- csrc/kernels/rowchain.hip) and 2L
grouped launches otherwise; the step is captured once as a hipGraph (natively, in
csrc/runtime/executor.cpp) and replayed for every step of every epoch because
batch index, dropout counter and optimizer iteration are read from device counters.
"""
from __future__ import annotations

import logging
import math
import os
import threading
import weakref
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import config
from ..models import optimizers as O
from . import native
from .plan import flatten_weights
from .trainer import TrainerBase, prepare_features, prepare_targets, split_point

_log = logging.getLogger("elephas_amd.native")


class _OutputPool:
    """Pinned host buffers for large prediction arrays, recycled when the array the
    caller got is garbage-collected (weakref.finalize) -- a caching allocator for the
    outputs.  A fresh 65 MB array costs ~5.5 ms of first-touch page faults plus ~2.5 ms
    to pin it, more than the whole transfer-bound inference of Wide's 16,384 rows
    (4.5-5.7 ms into a resident array, profiles/README.md).  Every call still returns an
    array nobody else holds: a buffer is reused only after its previous array (and every
    view of it) is gone; otherwise a new one is allocated."""

    MIN_BYTES = 8 << 20
    KEEP = 2   # idle buffers kept per size

    class _Holder:
        """The base object of a handed-out array and of every view of it (numpy collapses
        view bases down to the first non-ndarray), so its finalizer runs only once no
        array referencing the buffer is left."""

        def __init__(self, buf, shape):
            self.buf = buf
            self.__array_interface__ = dict(shape=shape, typestr="<f4", data=(buf.data_ptr(), False), version=3)

    def __init__(self):
        self._free = {}
        self._lock = threading.Lock()

    def _give(self, nbytes, buf):
        with self._lock:
            lst = self._free.setdefault(nbytes, [])
            if len(lst) < self.KEEP:
                lst.append(buf)

    def take(self, shape) -> np.ndarray:
        shape = tuple(int(s) for s in shape)
        n = int(np.prod(shape))
        if n * 4 < self.MIN_BYTES or not torch.cuda.is_available():
            return np.empty(shape, np.float32)
        with self._lock:
            lst = self._free.get(n * 4)
            buf = lst.pop() if lst else None
        if buf is None:
            buf = torch.empty(n, dtype=torch.float32, pin_memory=True)
        holder = self._Holder(buf, shape)
        arr = np.asarray(holder)
        weakref.finalize(holder, self._give, n * 4, buf)
        return arr


_OUT_POOL = _OutputPool()


def _shared_cu_share(dev: torch.device) -> int:
    """CUs a persistent grid of this rank may assume when ranks of the job share its
    GPU (single-GPU multi-rank rehearsals; detected from device UUIDs at init,
    parallel/dist.py): an equal share, so the sharers' grids are co-resident.
    0 = the GPU is this process's alone."""
    from ..parallel import dist
    n = dist.device_sharers()
    if n <= 1:
        return 0
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    return max(1, ncu // n)


# The persistent chunk kernel needs every workgroup of its grid resident at once (they
# wait for each other inside the launch), so two of them in flight on different streams
# of one device can each hold part of the GPU and wait forever. Persistent launches of
# all trainers of a device are therefore serialised: each waits for the device's most
# recent one (an event) unless that one was issued on its own stream.
_PERSIST_LAST: Dict[int, tuple] = {}
# fence -> launch(es) -> mark is one critical section per device: threaded workers (one
# native trainer per thread) must not interleave it, or two grids could be in flight at once
_PERSIST_LOCKS: Dict[int, threading.Lock] = {}
_PERSIST_LOCKS_GUARD = threading.Lock()


def _persist_lock(dev_index: int) -> threading.Lock:
    with _PERSIST_LOCKS_GUARD:
        lk = _PERSIST_LOCKS.get(dev_index)
        if lk is None:
            lk = _PERSIST_LOCKS[dev_index] = threading.Lock()
        return lk


class PersistentPlanError(RuntimeError):
    """A persistent launch gave up waiting inside the kernel (its sticky error word).
    The trainer has already cleared the word and re-planned onto the row-chain plan,
    so later calls run; ``clean`` is True when the launch modified nothing (the grid was
    not resident: PERR_GRID), False when a wait timed out mid-chunk (weights may be
    partially updated -- ``fit`` restores its entry snapshot and re-runs either way)."""

    def __init__(self, code: int, rank_exchange: bool = False):
        self.code = int(code)
        self.clean = self.code in (9, 12)   # grid not resident / replica not on one XCD: nothing modified
        self.rank_exchange = bool(rank_exchange)
        super().__init__(
            f"persistent step kernel: an in-launch wait timed out (code {self.code}; "
            + ("the grid was not resident, nothing was modified" if self.clean else
               "mid-chunk: weights may be partially updated")
            + ("); the in-launch rank exchange is attached, so this rank cannot re-plan alone: the job's "
               "per-step sync must be restarted without it (ELEPHAS_AMD_XRANK=0)" if rank_exchange else
               "); the trainer now runs the row-chain plan"))


def _replica_sum(G: torch.Tensor):
    """Gradient exchange of a sync trainer's replicas (one GPU): every replica gets the
    sum (the optimizer applies grad_scale = 1/R)."""
    G.copy_(G.sum(0, keepdim=True).expand_as(G))


def pad8(n: int) -> int:
    return (int(n) + 7) // 8 * 8


class NativeTrainer(TrainerBase):
    # steps per captured graph: a power of two (run_steps splits a remainder into the
    # binary fractions of it), ELEPHAS_AMD_GRAPH_CHUNK rounded down to one
    GRAPH_CHUNK = 1 << (max(1, int(os.environ.get("ELEPHAS_AMD_GRAPH_CHUNK", "16"))).bit_length() - 1)
    # the persistent plan runs a whole chunk in one launch (its fill / drain and the
    # launch's P / S / weight-image round trip are paid once per chunk): longer chunks
    PERSIST_CHUNK = max(1, int(os.environ.get("ELEPHAS_AMD_PERSIST_CHUNK", "128")))

    def __del__(self):
        # the trainer's tensors live in torch's caching allocator, its kernels on its own
        # stream: a dropped trainer must not hand its memory to the next allocation while
        # work it enqueued still runs (torch only orders reuse on the allocating stream)
        try:
            st = self.__dict__.get("stream")
            if st is not None:
                st.synchronize()
        except Exception:  # noqa: BLE001 - interpreter shutdown, CUDA already torn down
            pass

    def __init__(self, model, plan, R: int = 1, batch_size: int = 32, device=None, seed: Optional[int] = None,
                 policy: Optional[str] = None, eval_batch: int = 2048, rowchain: Optional[int] = None,
                 persist: Optional[int] = None, stream: Optional[torch.cuda.Stream] = None,
                 persist_cus: Optional[int] = None, sync: bool = False, ps_hook: bool = False):
        super().__init__(model, plan, R, batch_size)
        self.C = native.require()
        # sync: the R replicas are ONE model trained with per-step synchronous data
        # parallelism (reference SURVEY §2.3 DP-sync 'batch'): every step each replica's
        # gradient over its own batch, summed over the replicas, scaled 1/R, applied by all.
        # On the persistent plan the exchange happens inside the launch (persist.hip
        # xchg_sum); otherwise forward/backward -> replica sum -> apply per step.
        self.sync = bool(sync) and R > 1
        self._grad_scale = 1.0
        self._no_local = False   # set after a launch found a replica's workgroups on two XCDs (PERR_PLACE)
        self._fused_done = False  # the last _run_steps ended with the fused replica averaging
        # ps_hook: the persistent plan will push / pull a device parameter server every
        # step inside the launch (attach_param_server), so it keeps the V1 roles
        self.ps_hook = bool(ps_hook)
        self._ps = None
        # row-chain step plan (3 launches, csrc/kernels/rowchain.hip): None ->
        # $ELEPHAS_AMD_ROWCHAIN (default -1: whenever the model is eligible), 0 off, 1 required
        self.rowchain_mode = int(os.environ.get("ELEPHAS_AMD_ROWCHAIN", "-1")) if rowchain is None else int(rowchain)
        # persistent chunk kernel (csrc/kernels/persist.hip): None -> $ELEPHAS_AMD_PERSIST
        # (default -1: whenever eligible), 0 off, 1 required.  It keeps a whole cluster of
        # workgroups per replica resident and waiting on each other
        self.persist_mode = int(os.environ.get("ELEPHAS_AMD_PERSIST", "-1")) if persist is None else int(persist)
        # persist_cus: the persistent grid is sized to this share of the GPU's CUs, so
        # several trainers whose shares sum to at most the CU count run their persistent
        # kernels side by side (async worker groups, ranks sharing one GPU); without it a
        # trainer assumes the whole GPU and its persistent launches are serialised with
        # every other trainer's of the process
        self.persist_cus = int(persist_cus) if persist_cus else 0
        if not plan.native_ok:
            raise ValueError(f"model is not supported by the native engine: {plan.reason}")
        self.dev = torch.device(device) if device is not None else config.get_device()
        if self.dev.type != "cuda":
            raise ValueError("NativeTrainer needs a GPU device")
        if not self.persist_cus:
            share = _shared_cu_share(self.dev)
            if share:
                self.persist_cus = share
                _log.info("ranks share this GPU: persistent grids sized to %d CUs each", share)
        policy = policy or config.get_policy()
        self.bf16 = policy == "mixed_bfloat16"
        self.T = torch.bfloat16 if self.bf16 else torch.float32
        self.seed = int(seed) if seed is not None else int(np.random.randint(1, 2**62))
        self.eval_B = max(int(eval_batch), self.B)
        # every launch of this trainer goes to one HIP stream (shared by several trainers
        # when a caller wants their work serialised on one hardware queue)
        self.stream = stream if stream is not None else torch.cuda.Stream(device=self.dev)
        self.loader = self.C.HostLoader(8 << 20, 3)
        # optimizer
        opt = model.optimizer
        nat = opt.native() if opt is not None else None
        if nat is None:
            raise ValueError(f"optimizer {type(opt).__name__} is not supported by the native engine")
        self.opt_id, self.opt_hp, self.nstate = nat
        if self.loss.native is None:
            raise ValueError(f"loss {self.loss.name} is not supported by the native engine")
        if any(m.native is None for m in self.metrics) or len(self.metrics) > 4:
            raise ValueError("metrics not supported by the native engine")

        L = plan.layers
        self.dims = []
        wsh, wtsh = 0, 0
        for s in L:
            K, N = s.in_dim, s.units
            d = dict(K=K, N=N, Kp=pad8(K), Np=pad8(N), wsh_off=wsh, wtsh_off=wtsh)
            wsh += K * d["Np"]
            wtsh += N * d["Kp"]
            self.dims.append(d)
        self.wsh_total, self.wtsh_total = wsh, wtsh
        self.n = plan.n_params
        self.Kp0 = self.dims[0]["Kp"]
        self.ldy = 1 if self.loss.name == "sparse_categorical_crossentropy" else self.n_out
        dev, R = self.dev, self.R
        with torch.cuda.device(dev):
            self.P = torch.zeros(R, self.n, dtype=torch.float32, device=dev)
            self.S = torch.zeros(R, max(self.nstate, 1), self.n, dtype=torch.float32, device=dev)
            if "state_init" in self.opt_hp:
                self.S.fill_(float(self.opt_hp["state_init"]))
            self.G = torch.zeros(R, self.n, dtype=torch.float32, device=dev)
            self.Wsh = torch.zeros(R, 2, max(wsh, 1), dtype=self.T, device=dev)
            self.WTsh = torch.zeros(R, 2, max(wtsh, 1), dtype=self.T, device=dev)
            self.ctr = torch.zeros(2 + R, dtype=torch.int64, device=dev)
            self.acc = torch.zeros(R, 6, dtype=torch.float64, device=dev)
            self.acc_val = torch.zeros(R, 6, dtype=torch.float64, device=dev)
            self.ws = self._alloc_workspace(self.B)
            self.ws_eval = None
            # empty data shard until set_data
            self.nmax = 1
            self.X = torch.zeros(R, 1, self.Kp0, dtype=self.T, device=dev)
            self.Y = torch.zeros(R, 1, self.ldy, dtype=torch.float32, device=dev)
            self.perm = torch.zeros(R, 1, dtype=torch.int32, device=dev)
            self.ntrain = torch.zeros(R, dtype=torch.int32, device=dev)
            self.vstart = torch.zeros(R, dtype=torch.int32, device=dev)
            self.vcount = torch.zeros(R, dtype=torch.int32, device=dev)
        self.ntrain_h = [0] * R
        self.vcount_h = [0] * R
        self.active = [True] * R
        self.shuffle = True
        self.exe = None
        self.exe_eval = None
        # the weight images (Wsh / WTsh) lag P: set by an averaging that only rewrote the
        # masters (the persistent kernel reads P alone); every other reader of the images
        # refreshes them first (_ensure_images)
        self._images_stale = False
        self._graphs: Dict[tuple, int] = {}
        self._build_executor()
        self.set_weights_flat(flatten_weights(model.get_weights()))

    # ------------------------------------------------------------ workspaces
    def _alloc_workspace(self, B: int) -> dict:
        Bp = pad8(B)
        R, dev, T = self.R, self.dev, self.T
        layers = []
        for d in self.dims:
            N, Np = d["N"], d["Np"]
            layers.append(dict(
                Z=torch.zeros(R, B, N, dtype=torch.float32, device=dev),
                D=torch.zeros(R, B, Np, dtype=T, device=dev),
                DT=torch.zeros(R, N, Bp, dtype=T, device=dev),
                dZ=torch.zeros(R, B, Np, dtype=T, device=dev),
                dZT=torch.zeros(R, N, Bp, dtype=T, device=dev)))
        XT = torch.zeros(R, self.Kp0, Bp, dtype=T, device=dev)
        return dict(B=B, Bp=Bp, layers=layers, XT=XT)

    def _cfg(self, ws: dict) -> dict:
        layers = []
        for s, d, w in zip(self.plan.layers, self.dims, ws["layers"]):
            layers.append(dict(K=d["K"], N=d["N"], Kp=d["Kp"], Np=d["Np"], act=s.act_id,
                               has_bias=int(s.use_bias), rate=float(s.dropout), p_off=s.p_off,
                               Z=w["Z"].data_ptr(), D=w["D"].data_ptr(), DT=w["DT"].data_ptr(),
                               dZ=w["dZ"].data_ptr(), dZT=w["dZT"].data_ptr(),
                               wsh_off=d["wsh_off"], wtsh_off=d["wtsh_off"]))
        # sync: the gradient is the sum over the R replicas (and, with the in-launch rank
        # exchange, over the ranks): the mean
        xw = self._xr["world"] if getattr(self, "_xr", None) else 1
        opt = dict(opt=self.opt_id, s_plane=self.n,
                   grad_scale=self._grad_scale / (self.R * xw if self.sync else 1))
        opt.update({k: v for k, v in self.opt_hp.items() if k != "state_init"})
        return dict(
            R=self.R, B=ws["B"], Bp=ws["Bp"], bf16=int(self.bf16), seed=self.seed,
            force_cfg=int(os.environ.get("ELEPHAS_AMD_GEMM_CFG", "-1")),
            big=int(os.environ.get("ELEPHAS_AMD_BIG", "-1")),
            rc_lean=int(os.environ.get("ELEPHAS_AMD_RC_LEAN", "1")),
            thr_min_k=int(os.environ.get("ELEPHAS_AMD_THR_MIN_K", "64")),
            thr_min_n=int(os.environ.get("ELEPHAS_AMD_THR_MIN_N", "256")),
            rowchain=self.rowchain_mode if ws is self.ws else 0,
            persist=self.persist_mode if ws is self.ws else 0,
            persist_timeout_ms=int(os.environ.get("ELEPHAS_AMD_PERSIST_TIMEOUT_MS", "2000")),
            persist_cus=self.persist_cus,
            persist_v2=0 if self.ps_hook else int(os.environ.get("ELEPHAS_AMD_PERSIST_V2", "-1")),
            persist_local=0 if self._no_local else int(os.environ.get("ELEPHAS_AMD_PERSIST_LOCAL", "-1")),
            persist_sync=int(self.sync) if ws is self.ws else 0,
            deep=int(os.environ.get("ELEPHAS_AMD_DEEP", "-1")),
            rc_split=int(os.environ.get("ELEPHAS_AMD_RC_SPLIT", "0")),
            tail=int(os.environ.get("ELEPHAS_AMD_TAIL", "-1")) if ws is self.ws else 0,
            no_reorder=int(os.environ.get("ELEPHAS_AMD_NO_REORDER", "0")),
            dual=int(os.environ.get("ELEPHAS_AMD_DUAL", "1")),
            layers=layers,
            X=self.X.data_ptr(), sX=self.nmax * self.Kp0, ldx=self.Kp0,
            Y=self.Y.data_ptr(), sY=self.nmax * self.ldy, ldy=self.ldy,
            perm=self.perm.data_ptr(), sPerm=self.nmax,
            ntrain=self.ntrain.data_ptr(), vstart=self.vstart.data_ptr(), vcount=self.vcount.data_ptr(),
            XT=ws["XT"].data_ptr(),
            P=self.P.data_ptr(), sP=self.n, nparams=self.n,
            G=self.G.data_ptr(), sG=self.n,
            S=self.S.data_ptr(), sS=self.S.shape[1] * self.n,
            Wsh=self.Wsh.data_ptr(), sWsh=2 * self.Wsh.shape[2], wsh_par=self.Wsh.shape[2],
            WTsh=self.WTsh.data_ptr(), sWTsh=2 * self.WTsh.shape[2], wtsh_par=self.WTsh.shape[2],
            opt=opt, loss=self.loss.native, metrics=[m.native for m in self.metrics],
            acc=self.acc.data_ptr(), acc_stride=6, ctr=self.ctr.data_ptr())

    def _build_executor(self):
        tag0 = 0
        if self.exe is not None:
            tag0 = self.exe.rank_exchange_steps()
            self.exe.destroy_graphs()
        self._graphs = {}
        self.exe = self.C.Executor(self._cfg(self.ws))
        self._built_persist_mode = self.persist_mode
        why = self.exe.plan_reason()
        if why and why != getattr(self, "_logged_reason", None):
            # a shape cliff: the step runs as several launches instead of one persistent
            # launch per chunk (2-3x the step time) -- say which constraint the model misses
            self._logged_reason = why
            _log.info("no persistent plan for this model (%s): %s", why, self.plan_name())
        self.GRAPH_CHUNK = self.PERSIST_CHUNK if self.exe.persistent() else type(self).GRAPH_CHUNK
        if self._ps is not None and not self.exe.set_param_server(*self._ps):
            self._ps = None   # the rebuilt plan cannot (e.g. the row-chain fallback): host-side exchange
        xr = getattr(self, "_xr", None)
        if xr is not None:
            xr["live"] = bool(self.exe.set_rank_exchange(xr["bases"], xr["world"], xr["rank"], tag0, xr["timeout"]))

    def attach_rank_exchange(self, rank: int, world: int, allgather=None, timeout_s: Optional[float] = None) -> bool:
        """Per-step synchronous DP across ranks INSIDE the persistent launch (reference
        spark_model.py:217-228 with per-batch exchange; SURVEY §2.3 DP-sync 'batch'): a
        sync trainer's replica sum of every weight-gradient tile is exchanged with the
        other ranks through a peer-mapped buffer (HIP IPC, uncached; over xGMI between
        GPUs) and summed in rank order by the owning workgroups -- the same update on every
        rank and replica, no host round trip per step.  Collective: every rank calls it
        with the same shard sizes.  Returns False on every rank (and changes nothing) if
        any rank cannot: the caller keeps its own per-step exchange."""
        from ..parallel import dist as _dist
        from ..parallel.p2p import exchange_handles
        gather = allgather or _dist.all_gather_object
        world = int(world)
        if world <= 1:
            return False
        ok = bool(self.sync and self.exe.persistent() and self._sync_in_launch())
        if not ok:
            _log.warning("rank exchange: this trainer's plan cannot run it (%s)", self.plan_name())
        buf = None
        try:
            if ok:
                devi = self.dev.index if self.dev.index is not None else torch.cuda.current_device()
                if self.exe.persist_variant()[0] == 3:   # the layer pipeline: [2][nw][XT] floats
                    geo = self.exe.deep_geometry()
                    nbytes = 2 * int(geo[0]) * int(geo[5]) * 4
                else:                                    # persist.hip: [2][wgs][PM_XSLOT] floats
                    nbytes = 2 * int(self.exe.persist_geometry()[5]) * 7 * 1024 * 4
                buf = self.C.PeerBuffer(int(rank), world, nbytes, int(devi))
        except Exception as e:  # noqa: BLE001 - voted below
            _log.warning("rank exchange: buffer setup failed: %r", e)
            ok, buf = False, None
        handles = exchange_handles(bytes(buf.handle()) if buf is not None else b"", allgather)
        if ok and all(handles):
            try:
                buf.open(handles)
            except Exception:  # noqa: BLE001
                ok = False
        else:
            ok = False
        # every rank must run the same step sequence (the exchange tags): equal shard sizes
        votes = gather((ok, tuple(self.ntrain_h)))
        if not all(v[0] for v in votes) or len({v[1] for v in votes}) != 1:
            return False
        timeout = float(os.environ.get("ELEPHAS_AMD_P2P_TIMEOUT_S", "60")) if timeout_s is None else float(timeout_s)
        self._xr = dict(buf=buf, bases=list(buf.bases()), world=world, rank=int(rank), timeout=timeout, live=False)
        self._build_executor()   # the grad scale now includes 1 / world
        live = gather(bool(self._xr["live"]))
        if not all(live):
            self._xr = None
            self._build_executor()
            return False
        # numeric self-test before the path is trusted (the first time it crosses xGMI may
        # be a production run): known integer tiles through the very buffers, flags and tags
        # of the exchange, checked against the exact rank sums on every rank, voted; any
        # mismatch or timeout -> every rank detaches and keeps its own per-step exchange
        from ..parallel import fault
        corrupt = 0
        try:
            fault.maybe_inject("xrank_selftest", int(rank))
        except fault.InjectedFault:
            corrupt = 1   # this rank sends a wrong tile: the vote must catch it
        try:
            wrong, late = (int(v) for v in self.exe.rank_exchange_selftest(2, corrupt))
        except Exception as e:  # noqa: BLE001 - voted below
            _log.warning("rank exchange self-test failed to run: %r", e)
            wrong, late = -1, -1
        verdicts = gather((wrong, late))
        self.xr_selftest = dict(votes=[list(v) for v in verdicts], ok=all(v == (0, 0) for v in verdicts))
        if not self.xr_selftest["ok"]:
            _log.warning("rank exchange self-test failed on some rank (%s): using the per-step all-reduce",
                         verdicts)
            self._xr = None
            self._build_executor()
            return False
        return True

    @property
    def rank_exchange(self) -> bool:
        xr = getattr(self, "_xr", None)
        return bool(xr and xr["live"])

    def attach_param_server(self, ps, consistent: bool) -> bool:
        """Per-step parameter-server exchange INSIDE the persistent launch (reference
        worker.py:114-127 frequency='batch': pull, train_on_batch, push): after every
        step each owning workgroup pushes theta_new - theta_pulled of its parameters into
        the sharded device server and pulls its slice for the next step.  The host then
        only pulls theta into P before each chunk.  Returns False when the plan cannot
        (not persistent / V2 roles): the caller keeps the per-step host-side rounds."""
        mode = 2 if consistent else 1
        if not self.exe.persistent() or not self.exe.set_param_server(ps, mode):
            return False
        self._ps = (ps, mode)
        return True

    def detach_param_server(self):
        """Back to the host-side pull / push rounds (ps_mode 0 in the launch)."""
        if self._ps is not None:
            self.exe.set_param_server(self._ps[0], 0)
            self._ps = None

    @property
    def param_server_in_launch(self) -> bool:
        return self._ps is not None

    def _eval_exe(self):
        if self.exe_eval is None:
            # the workspace's zero fill on the executor stream: the eval kernels run there, and a
            # fill on another stream could land after the first validation pass's writes (its
            # padded columns must be zero; reused allocator memory is not) -- seen as a wrong
            # first-epoch val_loss now and then on the Otto shape in a long test process
            with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
                self.ws_eval = self._alloc_workspace(self.eval_B)
            self.exe_eval = self.C.Executor(self._cfg(self.ws_eval))
        return self.exe_eval

    @property
    def s(self) -> int:
        return int(self.stream.cuda_stream)

    def _enter(self):
        self.stream.wait_stream(torch.cuda.current_stream(self.dev))

    def _exit(self):
        torch.cuda.current_stream(self.dev).wait_stream(self.stream)

    # ---------------------------------------------------------------- weights
    def set_weights_flat(self, flat):
        flat = np.asarray(flat, np.float32)
        if flat.ndim == 1:
            flat = np.broadcast_to(flat, (self.R, flat.size))
        self._enter()
        # pinned staging (the caching host allocator keeps it until the copy has run): no
        # pageable-memory DMA, see _host
        src = torch.from_numpy(np.array(flat, dtype=np.float32, copy=True)).pin_memory()
        with torch.cuda.stream(self.stream):
            self.P.copy_(src, non_blocking=True)
            self.exe.refresh_shadows(True, self.s)
        self._exit()
        self._images_stale = False

    def sync_shadows(self):
        """Rebuild the weight images after P was modified on device (all-reduce, PS pull)."""
        with torch.cuda.stream(self.stream):
            self.exe.refresh_shadows(True, self.s)
        self._images_stale = False

    def _ensure_images(self):
        """Before a launch that reads the weight images: rebuild them if an averaging left
        only the masters current (stream-ordered, no host sync)."""
        if self._images_stale:
            self.sync_shadows()

    def get_weights_flat(self):
        return self._host(self.P)

    def average_replicas(self, allreduce=None, n_total: Optional[int] = None, include: bool = True):
        """Reference synchronous averaging (spark_model.py:221-227) on the device, the one
        implementation the bench and ``SparkModel`` share: theta <- (1/n_total) * sum of
        every worker's theta_i.  This rank's R replicas are summed by one kernel (fp64
        accumulation; ``include=False``: a rank without partitions contributes zeros),
        summed over ranks by ``allreduce`` (issued on this trainer's stream, so every
        read of the sum is stream-ordered after it), scaled, and written back into every
        replica's master and both weight-image parities by one kernel.  No host sync.
        Returns the mean as a device tensor; the caller's current stream is ordered after
        it (an event wait), so reading it there needs no explicit synchronisation."""
        n_total = int(n_total or self.R)
        with torch.cuda.stream(self.stream):
            avg = getattr(self, "_avg_buf", None)
            if avg is None or avg.numel() != self.n:
                avg = self._avg_buf = torch.empty(self.n, dtype=torch.float32, device=self.dev)
            if self.exe.persistent() and include:
                # the next training chunk reads only the masters: write the mean into
                # every replica's P (one kernel; after the all-reduce, one broadcast copy)
                # and leave the weight images to whichever reader comes first
                if allreduce is None:
                    self.C.replica_average(self.P.data_ptr(), self.P.stride(0), self.R, self.n, avg.data_ptr(), 1,
                                           self.s, 1.0 / n_total)
                else:
                    self.C.replica_average(self.P.data_ptr(), self.P.stride(0), self.R, self.n, avg.data_ptr(), 0,
                                           self.s, 1.0)
                    allreduce(avg)
                    avg.mul_(1.0 / n_total)
                    self.P.copy_(avg.expand_as(self.P))
                self._images_stale = True
            else:
                if include:
                    scale = 1.0 if allreduce is not None else 1.0 / n_total
                    self.C.replica_average(self.P.data_ptr(), self.P.stride(0), self.R, self.n, avg.data_ptr(), 0,
                                           self.s, scale)
                else:
                    avg.zero_()
                if allreduce is not None:
                    allreduce(avg)
                    avg.mul_(1.0 / n_total)
                self.exe.refresh_from(avg.data_ptr(), 0, self.s)
                self._images_stale = False
        # the caller reads the mean on its own stream (mean.cpu(), checkpoints): join it
        self._exit()
        return avg

    def reset_for_fit(self, flat, seed: Optional[int] = None):
        """Reuse this trainer (buffers, uploaded shards, eval executor) for a new fit the
        way the reference starts every fit with a freshly built worker model: weights =
        ``flat``, zero optimizer state and iterations, a fresh dropout seed (the training
        executor is rebuilt around the same buffers; its graphs are recaptured lazily)."""
        self.seed = int(seed) if seed is not None else int(np.random.randint(1, 2**62))
        if self.persist_mode == self._built_persist_mode:
            # the same plan: only the seed changes (no executor rebuild -- that allocated and
            # zeroed the persistent workspace and synchronised the device on every fit)
            self.exe.set_seed(self.seed)
            self._graphs = {}
        else:
            self._build_executor()
        with torch.cuda.stream(self.stream):
            self.S.fill_(float(self.opt_hp.get("state_init", 0.0)))
            self.ctr.zero_()
        self.set_weights_flat(flat)   # + both weight-image parities

    def reset_optimizer_state(self):
        with torch.cuda.stream(self.stream):
            self.S.fill_(float(self.opt_hp.get("state_init", 0.0)))
            self.ctr.zero_()
            self.exe.refresh_shadows(True, self.s)

    def iterations(self) -> np.ndarray:
        return self._host(self.ctr[2:])

    def get_state_flat(self):
        return self._host(self.S), self.iterations()

    def set_state_flat(self, state, iterations):
        st = torch.from_numpy(np.array(np.broadcast_to(np.asarray(state, np.float32), tuple(self.S.shape)),
                                       dtype=np.float32))
        it = torch.from_numpy(np.array(np.broadcast_to(np.asarray(iterations, np.int64), (self.R,)),
                                       dtype=np.int64))
        self._enter()
        st, it = st.pin_memory(), it.pin_memory()   # pinned staging, as set_weights_flat
        with torch.cuda.stream(self.stream):
            self.S.copy_(st, non_blocking=True)
            self.ctr[2:].copy_(it, non_blocking=True)
            self.exe.refresh_shadows(True, self.s)
        self._exit()

    # ------------------------------------------------------------------- data
    def _upload_rows(self, dst: torch.Tensor, x: np.ndarray, stream: Optional[torch.cuda.Stream] = None):
        """Stream host rows into the rows of a device tensor (fp32 or bf16, row stride
        >= the row) through the native pinned double-buffered loader, on ``stream``
        (default: the trainer's). Asynchronous: the loader packs (and, for a bf16
        destination, converts) each chunk into pinned staging on the host before its
        DMA is queued, so ``x`` may be released as soon as this returns."""
        x = np.asarray(x, dtype=np.float32)
        if x.ndim == 1:
            x = x.reshape(-1, 1)
        if x.strides[1] != 4:
            x = np.ascontiguousarray(x)
        n, k = x.shape
        if n == 0:
            return
        if stream is None:
            self._enter()   # after the caller's pending work on dst (e.g. its zero fill)
        s = int((stream or self.stream).cuda_stream)
        if dst.shape[-1] < k or dst.stride(-1) != 1:
            raise ValueError("destination rows too narrow")
        if dst.dtype == torch.float32:
            self.loader.upload_rows(x.ctypes.data, x.strides[0], dst.data_ptr(), dst.stride(0) * 4, n, k * 4, s)
        elif dst.dtype == torch.bfloat16:
            self.loader.upload_rows_bf16(x.ctypes.data, x.strides[0], dst.data_ptr(), dst.stride(0) * 2, n, k, s)
        else:
            raise TypeError(f"upload into {dst.dtype}")

    def set_data(self, xs, ys, validation_split=0.0, active=None, shuffle=True):
        assert len(xs) == self.R and len(ys) == self.R
        xs = [prepare_features(x, self.in_dim) if len(x) else np.zeros((0, self.in_dim), np.float32) for x in xs]
        ys = [prepare_targets(y, self.n_out, self.loss) if len(y) else np.zeros((0, self.ldy), np.float32)
              for y in ys]
        nmax = max(1, max(len(x) for x in xs))
        self._enter()
        with torch.cuda.stream(self.stream):
            if nmax != self.nmax:
                self.nmax = nmax
                self.X = torch.zeros(self.R, nmax, self.Kp0, dtype=self.T, device=self.dev)
                self.Y = torch.zeros(self.R, nmax, self.ldy, dtype=torch.float32, device=self.dev)
                self.perm = torch.zeros(self.R, nmax, dtype=torch.int32, device=self.dev)
                rebuild = True
            else:
                self.X.zero_()
                self.Y.zero_()
                rebuild = False
            for r in range(self.R):
                self._upload_rows(self.X[r], xs[r])
                self._upload_rows(self.Y[r], ys[r])
        self.active = [True if active is None else bool(active[r]) for r in range(self.R)]
        nt, vs, vc = [], [], []
        for r in range(self.R):
            n = len(xs[r])
            sp = split_point(n, validation_split)
            nt.append(sp if self.active[r] else 0)
            vs.append(sp)
            vc.append(n - sp if self.active[r] else 0)
        self.ntrain_h, self.vcount_h = nt, vc
        # in-launch gradient exchange needs every replica to run the same steps
        self._sync_equal = len(set(nt)) == 1
        with torch.cuda.stream(self.stream):
            # (pinned staging, as set_weights_flat)
            self.ntrain.copy_(torch.tensor(nt, dtype=torch.int32).pin_memory(), non_blocking=True)
            self.vstart.copy_(torch.tensor(vs, dtype=torch.int32).pin_memory(), non_blocking=True)
            self.vcount.copy_(torch.tensor(vc, dtype=torch.int32).pin_memory(), non_blocking=True)
        self.shuffle = shuffle
        if rebuild:
            self._build_executor()
            if self.exe_eval is not None:
                self.exe_eval = None
        self._exit()

    def _new_perm(self, gen: Optional[torch.Generator] = None):
        """This epoch's row order of every replica: one launch of the keyed Feistel
        permutation kernel (csrc/kernels/shuffle.hip). The key is a pure function of the
        trainer seed and an epoch counter (or drawn from ``gen``), so a run is
        reproducible from its seed."""
        if gen is not None:
            key = int(torch.randint(0, 2**31 - 1, (1,), generator=gen, device=gen.device).item())
        else:
            self._perm_epoch = getattr(self, "_perm_epoch", 0) + 1
            key = (self.seed * 0x9E3779B97F4A7C15 + self._perm_epoch * 0xBF58476D1CE4E5B9) >> 17
        self.C.shuffle_perm(self.perm.data_ptr(), self.nmax, self.ntrain.data_ptr(), self.R, self.nmax,
                            key & 0xFFFFFFFF, int(bool(self.shuffle)), self.s)

    # ------------------------------------------------------------------ train
    def steps_per_epoch(self) -> int:
        return int(math.ceil(max(self.ntrain_h) / self.B)) if max(self.ntrain_h) > 0 else 0

    def _graph(self, nsteps: int, mode: int) -> int:
        key = (nsteps, mode)
        if key not in self._graphs:
            self._graphs[key] = self.exe.capture(nsteps, mode, self.s)
        return self._graphs[key]

    def _persist_fence(self) -> bool:
        """Order this trainer's next persistent launch after the device's previous one
        (see _PERSIST_LAST); returns whether the plan is persistent."""
        if not self.exe.persistent():
            return False
        if self.persist_cus:
            return False   # a partitioned grid: co-resident with the other shares by construction
        last = _PERSIST_LAST.get(self.dev.index)
        if last is not None and last[0] != self.s:
            self.stream.wait_event(last[1])
        return True

    def _persist_mark(self):
        ev = torch.cuda.Event()
        ev.record(self.stream)
        _PERSIST_LAST[self.dev.index] = (self.s, ev)

    def run_steps_and_average(self, nsteps: int, allreduce=None, n_total: Optional[int] = None,
                              use_graph: bool = True):
        """run_steps(nsteps) then average_replicas(allreduce, n_total) -- the reference's
        train-then-average (spark_model.py:217-228) -- on a persistent plan with the averaging
        in the last chunk's post node (mode 2: one launch does the flag clear, the counter
        advance and the averaging -- one kernel boundary fewer than post + replica_average),
        or with ELEPHAS_AMD_FUSED_AVG=1 inside the last launch itself (mode 1, persist.hip
        grid_average; measured slower at the bench's 20-step shape -- the write-through
        epilogue it needs costs more).  The replica mean (world 1) or the replica sum for the
        caller's all-reduce lands in the same buffer average_replicas fills.  Returns that
        buffer, as average_replicas does."""
        mode = 1 if os.environ.get("ELEPHAS_AMD_FUSED_AVG", "0") == "1" else 2
        fusable = (nsteps > 0 and self.exe.persistent() and not self.sync and self._ps is None
                   and getattr(self, "_xr", None) is None
                   and (mode == 2 or self.exe.persist_variant()[0] in (1, 2))
                   and os.environ.get("ELEPHAS_AMD_FUSED_AVG", "") != "0")
        if not fusable:
            self.run_steps(nsteps, use_graph=use_graph)
            return self.average_replicas(allreduce, n_total)
        n_total = int(n_total or self.R)
        avg = getattr(self, "_avg_buf", None)
        if avg is None or avg.numel() != self.n:
            with torch.cuda.stream(self.stream):
                avg = self._avg_buf = torch.empty(self.n, dtype=torch.float32, device=self.dev)
        fused = (avg.data_ptr(), 1, 1.0 / n_total, mode) if allreduce is None else (avg.data_ptr(), 0, 1.0, mode)
        if self.persist_cus:
            self._run_steps(nsteps, use_graph, fused)
        else:
            with _persist_lock(self.dev.index):
                self._persist_fence()
                try:
                    self._run_steps(nsteps, use_graph, fused)
                finally:
                    self._persist_mark()
        if not self._fused_done:   # the plan declined (train_chunk_avg false): the separate kernel
            return self.average_replicas(allreduce, n_total)
        with torch.cuda.stream(self.stream):
            if allreduce is not None:
                allreduce(avg)
                avg.mul_(1.0 / n_total)
                self.P.copy_(avg.expand_as(self.P))
            self._images_stale = True
        self._exit()
        return avg

    def run_steps(self, nsteps: int, use_graph: bool = True):
        """Launch nsteps fused training steps on self.stream (asynchronous)."""
        if nsteps <= 0:
            return
        if getattr(self, "_xr", None) is not None and not (self._xr["live"] and self._sync_in_launch()):
            raise RuntimeError("per-step sync across ranks: the rank exchange is attached but this plan / data "
                               "cannot run it inside the launch (every rank must keep equal shard sizes)")
        if self.sync and not self._sync_in_launch():
            # per-step synchronous DP without the in-launch exchange: forward/backward of
            # every replica -> gradient sum over the replicas -> apply (grad_scale 1/R)
            self.run_steps_allreduce(nsteps, _replica_sum, use_graph=use_graph)
            return
        if not self.exe.persistent() or self.persist_cus:
            self._run_steps(nsteps, use_graph)
            return
        with _persist_lock(self.dev.index):
            self._persist_fence()
            try:
                self._run_steps(nsteps, use_graph)
            finally:
                self._persist_mark()

    def _sync_in_launch(self) -> bool:
        return bool(self.exe.persistent() and self.exe.persist_variant()[2] and getattr(self, "_sync_equal", False))

    def _run_steps(self, nsteps: int, use_graph: bool, fused_avg=None):
        self._fused_done = False
        if self.exe.persistent():
            # one persistent launch per chunk of up to PERSIST_CHUNK steps, a remainder
            # included (the kernel takes its step count at launch): a chunk is two
            # stream operations (the kernel, then a 1-block post kernel that clears the
            # hand-off flags and advances the counters), so there is nothing for a graph
            # to save, and every extra launch would pay the kernel's fill / drain
            # (weights, optimizer state, first forward) again
            if not self.exe.persist_images():
                self._images_stale = True   # the kernel updates the masters only (V2)
            while nsteps > 0:
                n = min(nsteps, self.GRAPH_CHUNK)
                if fused_avg is not None and n == nsteps:   # the last chunk ends with the averaging
                    self._fused_done = bool(self.exe.train_chunk_avg(n, self.s, *fused_avg))
                    if not self._fused_done:
                        self.exe.train_chunk(n, self.s)
                else:
                    self.exe.train_chunk(n, self.s)
                nsteps -= n
            return
        self._ensure_images()
        if not use_graph:
            for _ in range(nsteps):
                self.exe.train_step(self.s)
            return
        # fixed chunk shapes (GRAPH_CHUNK and its binary fractions, all captured by
        # prepare_graphs), so no capture lands inside a timed loop whose step count
        # differs from the warmup's; a remainder of r steps is popcount(r) graph
        # launches instead of r (each graph boundary costs a launch gap on the GPU)
        full, rest = divmod(nsteps, self.GRAPH_CHUNK)
        if full:
            self.exe.replay_n(self._graph(self.GRAPH_CHUNK, 0), full, self.s)
        b = self.GRAPH_CHUNK // 2
        while rest:
            if rest >= b:
                self.exe.replay_n(self._graph(b, 0), 1, self.s)
                rest -= b
            b //= 2

    def prepare_graphs(self, allreduce_path: bool = False):
        """Capture (without running) every graph run_steps / run_steps_allreduce use."""
        if self.exe.persistent() and not allreduce_path:
            return   # persistent chunks launch without graphs (_run_steps)
        chunks = []
        b = self.GRAPH_CHUNK
        while b >= 1:
            chunks.append((b, 0))
            b //= 2
        keys = [(1, 1), (1, 2)] if allreduce_path else chunks
        for n, mode in keys:
            self._graph(n, mode)

    def run_steps_allreduce(self, nsteps: int, allreduce, use_graph: bool = True):
        """Per-step gradient all-reduce path: [fwd+bwd -> G] -> allreduce(G) -> [apply]."""
        self._ensure_images()
        for _ in range(nsteps):
            if use_graph:
                self.exe.replay(self._graph(1, 1), self.s)
            else:
                self.exe.forward_backward(self.s)
            with torch.cuda.stream(self.stream):
                allreduce(self.G)
            if use_graph:
                self.exe.replay(self._graph(1, 2), self.s)
            else:
                self.exe.apply(self.s)

    def run_steps_allreduce_graph(self, nsteps: int, channel, algo: int = -1):
        """Per-step gradient all-reduce with the whole step -- forward/backward, the peer
        all-reduce of G over IPC-mapped buffers (parallel/p2p.py graph channel), the
        optimizer apply -- captured as ONE hipGraph of GRAPH_CHUNK steps (and one of 1
        step), so the host launches one graph per 16 steps.  R == 1 (one replica per rank)."""
        self._ensure_images()
        if self.R != 1:
            raise ValueError("run_steps_allreduce_graph: one replica per rank")
        graphs = self._graphs.setdefault(("peer_ar", id(channel)), {})
        full, rest = divmod(nsteps, self.GRAPH_CHUNK)
        for k, reps in ((self.GRAPH_CHUNK, full), (1, rest)):
            if reps == 0:
                continue
            if k not in graphs:
                g = torch.cuda.CUDAGraph()
                self.stream.synchronize()
                with torch.cuda.graph(g, stream=self.stream):
                    for _ in range(k):
                        self.exe.forward_backward(self.s)
                        channel.all_reduce_graph_(self.G[0], algo=algo, stream=self.stream)
                        self.exe.apply(self.s)
                graphs[k] = g
            with torch.cuda.stream(self.stream):
                for _ in range(reps):
                    graphs[k].replay()

    def run_steps_allreduce_overlap(self, nsteps: int, allreduce_bucket, comm_stream=None):
        """Per-step gradient path with the all-reduce bucketed per layer and overlapped
        with the rest of the backward: as soon as the launch that completes layer l's
        dW / db has run, ``allreduce_bucket(G[:, lo:hi])`` is issued on ``comm_stream``
        (RCCL runs it beside the next backward launch); the optimizer apply waits for
        every bucket. Eager launches (the buckets' host calls sit between them)."""
        self._ensure_images()
        comm = comm_stream or getattr(self, "_comm_stream", None)
        if comm is None:
            comm = self._comm_stream = torch.cuda.Stream(device=self.dev)
        nl = self.exe.grad_launches()
        spans = []
        for s in self.plan.layers:
            lo = int(s.p_off)
            spans.append((lo, lo + s.in_dim * s.units + (s.units if s.use_bias else 0)))
        for _ in range(nsteps):
            done = []
            for i in range(nl):
                self.exe.grad_launch(i, self.s)
                layer = self.exe.grad_launch_layer(i)
                if layer < 0:
                    continue
                ev = torch.cuda.Event()
                ev.record(self.stream)
                with torch.cuda.stream(comm):
                    comm.wait_event(ev)
                    lo, hi = spans[layer]
                    allreduce_bucket(self.G[:, lo:hi])
                    d = torch.cuda.Event()
                    d.record(comm)
                    done.append(d)
            for d in done:
                self.stream.wait_event(d)
            self.exe.apply(self.s)

    def begin_epoch(self, gen=None):
        with torch.cuda.stream(self.stream):
            self.exe.reset_epoch(self.s)
            self.acc.zero_()
        self._new_perm(gen)

    def set_grad_scale(self, scale: float):
        """Scale every gradient by ``scale`` before the optimizer (the mean over ranks after
        a sum all-reduce); sync trainers add their 1/R on top."""
        if float(scale) != self._grad_scale:
            self._grad_scale = float(scale)
            self._build_executor()

    def fit(self, epochs, verbose=0, allreduce=None):
        """Keras-style fit of every replica. On the persistent plan the entry state
        (masters, optimizer state, counters, shuffle epoch) is snapshotted on the device
        first: if a persistent launch gives up (GPU shared, grid not resident -- see
        check()), the trainer re-plans onto the row chain, restores the snapshot and
        runs the whole fit again, so the caller sees a slower fit, not an exception."""
        if self.exe.persistent():
            self._enter()   # the snapshot orders after the caller's pending work (e.g. a weight write)
        snap = self._snapshot() if self.exe.persistent() else None
        try:
            return self._fit(epochs, verbose, allreduce)
        except PersistentPlanError:
            if snap is None or getattr(self, "_xr", None) is not None:
                raise
            self._restore(snap)
            return self._fit(epochs, verbose, allreduce)

    def _snapshot(self):
        """The fit-entry state, copied into buffers kept for the trainer's life (stream
        ordered; no allocation per fit)."""
        with torch.cuda.stream(self.stream):
            snap = getattr(self, "_snap", None)
            if snap is None or snap["P"].shape != self.P.shape or snap["S"].shape != self.S.shape:
                snap = self._snap = dict(P=torch.empty_like(self.P), S=torch.empty_like(self.S),
                                         ctr=torch.empty_like(self.ctr))
            snap["P"].copy_(self.P)
            snap["S"].copy_(self.S)
            snap["ctr"].copy_(self.ctr)
            return dict(snap, perm_epoch=getattr(self, "_perm_epoch", 0))

    def _restore(self, snap):
        with torch.cuda.stream(self.stream):
            self.P.copy_(snap["P"])
            self.S.copy_(snap["S"])
            self.ctr.copy_(snap["ctr"])
        self._perm_epoch = snap["perm_epoch"]
        self.sync_shadows()

    def _fit(self, epochs, verbose=0, allreduce=None):
        hist = self.new_history()
        self._enter()
        epochs = int(epochs)
        if verbose or allreduce is not None:
            # per-epoch host reads (progress lines; the all-reduce path is host-driven anyway)
            for epoch in range(epochs):
                self.launch_epoch(allreduce)
                self.collect_epoch(hist, epoch, epochs, verbose)
        else:
            # every epoch enqueued back to back: the epoch-end loss / metric sums and the
            # validation pass land in per-epoch device slots, read with ONE host copy at
            # the end (no host synchronisation -- and no GPU bubble -- per epoch)
            has_val = max(self.vcount_h) > 0
            with torch.cuda.stream(self.stream):
                slots = torch.zeros(epochs, 2, self.R, 6, dtype=torch.float64, device=self.dev)
            for epoch in range(epochs):
                self.launch_epoch()
                with torch.cuda.stream(self.stream):
                    slots[epoch, 0].copy_(self.acc)
                if has_val:
                    self.launch_val(slots[epoch, 1])
            host = self._host(slots)
            for epoch in range(epochs):
                self._append_history(hist, host[epoch, 0] if self.steps_per_epoch() > 0 else None,
                                     host[epoch, 1] if has_val else None, epoch, epochs, 0)
        self._exit()
        return hist

    def new_history(self):
        return [dict() if self.active[r] else None for r in range(self.R)]

    def launch_epoch(self, allreduce=None):
        """Enqueue one epoch (reshuffle + every step) on self.stream; no host sync."""
        self.begin_epoch()
        steps = self.steps_per_epoch()
        if allreduce is None:
            self.run_steps(steps)
        else:
            self.run_steps_allreduce(steps, allreduce)

    def collect_epoch(self, hist, epoch, epochs, verbose=0):
        """Append the launched epoch's loss / metrics and validation pass to ``hist``."""
        sums = self._host(self.acc) if self.steps_per_epoch() > 0 else None
        val = self._val_sums() if max(self.vcount_h) > 0 else None
        return self._append_history(hist, sums, val, epoch, epochs, verbose)

    def _append_history(self, hist, sums, val, epoch, epochs, verbose):
        if sums is None:
            sums = np.zeros((self.R, 6))
        for r in range(self.R):
            if not self.active[r]:
                continue
            h = self._history_from_sums(sums[r]) if self.ntrain_h[r] > 0 else {}
            if val is not None and self.vcount_h[r] > 0:
                h.update(self._history_from_sums(val[r], "val_"))
            for k, v in h.items():
                hist[r].setdefault(k, []).append(v)
            if verbose:
                self.print_epoch(epoch, epochs, h, r)
        return hist

    def launch_val(self, dst: Optional[torch.Tensor] = None):
        """Enqueue the validation pass over the tails of the training shards (per
        replica, dropout off) into acc_val, and a copy of it into ``dst`` (a [R, 6]
        fp64 device tensor) if given; no host synchronisation."""
        exe = self._eval_exe()
        self._ensure_images()
        with torch.cuda.stream(self.stream):
            self.acc_val.zero_()
            nch = int(math.ceil(max(self.vcount_h) / self.eval_B))
            src = dict(X=self.X.data_ptr(), sX=self.nmax * self.Kp0, ldx=self.Kp0,
                       Y=self.Y.data_ptr(), sY=self.nmax * self.ldy, ldy=self.ldy,
                       vstart=self.vstart.data_ptr(), vcount=self.vcount.data_ptr(),
                       acc=self.acc_val.data_ptr())
            for c in range(nch):
                exe.eval_chunk(c, src, self.s)
            if dst is not None:
                dst.copy_(self.acc_val)

    def _val_sums(self):
        """Validation tails of the training shards (per replica), dropout off."""
        self.launch_val()
        return self._host(self.acc_val)

    def _host(self, t: torch.Tensor) -> np.ndarray:
        """Device -> host read ordered after everything queued on the executor stream, through
        a pinned staging tensor on that stream (no pageable-memory DMA: every intermittent
        illegal-address error of the long GPU test runs surfaced at a pageable copy)."""
        out = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        with torch.cuda.stream(self.stream):
            out.copy_(t.detach(), non_blocking=True)
        self.stream.synchronize()
        self.check()
        return out.numpy().copy()

    def check(self):
        """Raise PersistentPlanError if a persistent-plan launch gave up waiting inside the
        kernel (its sticky error word: later launches of that executor did nothing and
        their post kernels did not advance the counters).  Before raising, the error word
        is cleared and the trainer re-planned onto the row chain (logged), so it stays
        usable; fit() restores its snapshot and re-runs."""
        if self.exe is not None and self.exe.persistent():
            e = self.exe.persist_error()
            if e:
                self.exe.persist_clear_error()
                if getattr(self, "_xr", None) is not None:
                    # the in-launch rank exchange cannot move to another plan on this rank
                    # alone (the other ranks keep waiting in their launches until their
                    # exchange timeout): one clear error, no local re-plan, no fit() retry
                    self._xr["live"] = False
                    raise PersistentPlanError(e, rank_exchange=True)
                if e == 12 and not self._no_local:
                    # a replica's workgroups on two XCDs: the XCD-local instance's premise does
                    # not hold on this device -- the write-through instance, same plan
                    _log.warning("persistent step kernel: replica not on one XCD (code 12); using the "
                                 "write-through instance")
                    self._no_local = True
                else:
                    _log.warning("persistent step kernel gave up (code %d%s); falling back to the row-chain plan",
                                 e, ", grid not resident" if e == 9 else "")
                    self.persist_mode = 0
                self._build_executor()
                self._images_stale = True   # P may hold a partial chunk: images from P first
                raise PersistentPlanError(e)

    # ------------------------------------------------------------------- eval
    def _eval_buffers(self, n: int, with_y: bool, want_pred: bool):
        """Device input / target / prediction buffers for ``n`` rows and a pinned host
        buffer for the predictions, grown on demand and kept (HBM is plentiful; a
        pinned allocation per call would cost more than the transfer)."""
        cap = getattr(self, "_ebuf", None)
        need = max(int(n), 1)
        if cap is None or cap["n"] < need:
            n2 = max(need, 2 * cap["n"] if cap else 0)
            with torch.cuda.device(self.dev):
                cap = self._ebuf = dict(n=n2, X=None, Y=None, pred=None, host=None)
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):   # fills ordered before the eval kernels
            if cap["X"] is None:
                cap["X"] = torch.zeros(cap["n"], self.Kp0, dtype=self.T, device=self.dev)
            if with_y and cap["Y"] is None:
                cap["Y"] = torch.zeros(cap["n"], self.ldy, dtype=torch.float32, device=self.dev)
            if want_pred and cap["pred"] is None:
                cap["pred"] = torch.empty(cap["n"], self.n_out, dtype=torch.float32, device=self.dev)
                cap["host"] = torch.empty(cap["n"], self.n_out, dtype=torch.float32, pin_memory=True)
        return cap

    def _copy_streams(self):
        if getattr(self, "_h2d", None) is None:
            self._h2d = torch.cuda.Stream(device=self.dev)
            self._d2h = torch.cuda.Stream(device=self.dev)
        return self._h2d, self._d2h

    def _eval_pipeline(self, x: np.ndarray, y: Optional[np.ndarray], want_pred: bool, r: int,
                       out: Optional[np.ndarray] = None):
        """Inference over host rows as a three-stream pipeline run natively
        (csrc/runtime/host_loader.cpp infer_pipeline): the loader's packing threads fill
        pinned staging for stage s+1 and its DMA runs on a copy stream while the eval
        kernels compute stage s on the trainer's stream and stage s-1's predictions
        stream back into pinned host memory on a second copy stream; events order each
        stage's kernels after its upload and its download after its kernels. Only
        replica ``r`` computes (the others see zero rows). With ``want_pred`` the
        predictions land in ``out`` (a C-contiguous fp32 [n, n_out] array): the packing
        threads copy each finished stage out of pinned memory while later stages are
        still in flight."""
        n = len(x)
        if x.strides[1] != 4 or x.strides[0] % 4:
            x = np.ascontiguousarray(x)
        exe = self._eval_exe()
        self._ensure_images()
        buf = self._eval_buffers(n, y is not None, want_pred)
        h2d, d2h = self._copy_streams()
        cur = torch.cuda.current_stream(self.dev)
        h2d.wait_stream(cur)
        self.stream.wait_stream(cur)
        d2h.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            vcount = torch.zeros(self.R, dtype=torch.int32, device=self.dev)
            vcount[r] = n
            vstart = torch.zeros(self.R, dtype=torch.int32, device=self.dev)
        src = dict(X=buf["X"].data_ptr(), sX=0, ldx=self.Kp0, vstart=vstart.data_ptr(), vcount=vcount.data_ptr(),
                   acc=self.acc_val.data_ptr())
        esz = buf["X"].element_size()
        # ~32 MB of staged input per stage (whole eval chunks): big DMAs, few events
        row_bytes = self.in_dim * esz
        stage = max(1, (4 * self.loader.chunk_bytes // max(row_bytes, 1)) // self.eval_B) * self.eval_B
        a = dict(x=x.ctypes.data, x_ld=x.strides[0] // 4, n=n, k=self.in_dim, dX=buf["X"].data_ptr(),
                 dX_ld=self.Kp0 * esz, x_bf16=int(buf["X"].dtype == torch.bfloat16), stage_rows=stage,
                 B=self.eval_B)
        if a["x_bf16"]:
            st = getattr(self, "_stage32", None)
            if st is None or st.numel() < stage * self.in_dim:
                st = self._stage32 = torch.empty(stage * self.in_dim, dtype=torch.float32, device=self.dev)
            a["dStage"] = st.data_ptr()
        if y is not None:
            y2 = np.asarray(y, dtype=np.float32).reshape(len(y), -1)
            if y2.strides[1] != 4 or y2.strides[0] % 4:
                y2 = np.ascontiguousarray(y2)
            src.update(Y=buf["Y"].data_ptr(), sY=0, ldy=self.ldy)
            a.update(y=y2.ctypes.data, y_ld=y2.strides[0] // 4, ky=y2.shape[1], dY=buf["Y"].data_ptr(),
                     dY_ld=self.ldy)
        if want_pred:
            src.update(pred=buf["pred"].data_ptr(), sPred=0, ldp=self.n_out)
            assert out is not None and out.flags.c_contiguous and out.dtype == np.float32 and out.shape == (n, self.n_out)
            a.update(dPred=buf["pred"].data_ptr(), ldp=self.n_out, hPred=buf["host"].data_ptr(), out=out.ctypes.data)
        self.C.infer_pipeline(exe, self.loader, a, src, int(h2d.cuda_stream), self.s, int(d2h.cuda_stream))
        for t in (vstart, vcount):
            t.record_stream(self.stream)
        self.stream.wait_stream(h2d)
        if want_pred:
            self.stream.wait_stream(d2h)   # the next call's kernels overwrite pred after these copies

    def evaluate_sums(self, x, y, batch_size=None, r: int = 0) -> np.ndarray:
        x = prepare_features(x, self.in_dim)
        y = prepare_targets(y, self.n_out, self.loss)
        self._enter()
        with torch.cuda.stream(self.stream):
            self.acc_val.zero_()
        self._eval_pipeline(x, y, False, r)
        out = self._host(self.acc_val[r])
        self._exit()
        return out

    def evaluate(self, x, y, batch_size=None, r: int = 0):
        s = self.evaluate_sums(x, y, batch_size, r)
        cnt = max(s[1], 1.0)
        return [float(s[0] / cnt)] + [float(s[2 + i] / cnt) for i in range(len(self.metrics))]

    def predict(self, x, batch_size=None, r: int = 0):
        x = prepare_features(x, self.in_dim)
        if len(x) == 0:
            return np.zeros((0, self.n_out), np.float32)
        self._enter()
        out = _OUT_POOL.take((len(x), self.n_out))
        self._eval_pipeline(x, None, True, r, out)
        self.check()
        self._exit()
        return out

    def train_on_batch(self, x, y, r: int = 0):
        """One optimizer step on exactly this batch (rows in order), keras semantics."""
        x = prepare_features(x, self.in_dim)
        self.set_data([x] * self.R, [y] * self.R, 0.0, shuffle=False)
        self.begin_epoch()
        self.run_steps(1, use_graph=False)
        s = self._host(self.acc[r])
        cnt = max(s[1], 1.0)
        return [float(s[0] / cnt)] + [float(s[2 + i] / cnt) for i in range(len(self.metrics))]

    def launch_count(self):
        """Kernel launches per training step of a long run (the persistent plan: the kernel
        and its 1-block post kernel per chunk of up to PERSIST_CHUNK steps)."""
        if self.exe.persistent():
            return 2.0 / self.GRAPH_CHUNK
        return self.exe.launches_per_step()

    def launches_for(self, nsteps: int) -> int:
        """Kernels a run_steps(nsteps) call issues (what a timed region of nsteps holds)."""
        if nsteps <= 0:
            return 0
        if self.exe.persistent():
            return 2 * ((nsteps + self.GRAPH_CHUNK - 1) // self.GRAPH_CHUNK)
        full, rest = divmod(nsteps, self.GRAPH_CHUNK)
        graphs = full + bin(rest).count("1")
        return nsteps * self.exe.launches_per_step() + graphs   # + one counter advance per graph

    @property
    def persist_variant(self) -> int:
        """3: the layer pipeline (deep.hip: deeper / wider stacks), 2: the V2 roles (plain
        SGD, ReLU: L0 Gram corrections, DW workgroups), 1: V1, 0: not persistent."""
        return int(self.exe.persist_variant()[0]) if self.exe.persistent() else 0

    @property
    def persistent(self) -> bool:
        """True when training chunks run the persistent kernel (one launch per chunk)."""
        return bool(self.exe.persistent())

    def plan_name(self) -> str:
        if self.exe.persistent() and self.exe.persist_variant()[0] == 3:
            nw, grid, rt, ks, lds = self.exe.deep_geometry()[:5]
            sy = ", per-step gradient exchange of the replicas inside the launch" if self.exe.persist_variant()[2] else ""
            sy += ", XCD-local hand-offs" if self.exe.persist_variant()[3] else ""
            return (f"persistent layer pipeline{sy} (deep.hip; 1 kernel + 1 post kernel per <= {self.GRAPH_CHUNK}-step "
                    f"chunk; {nw} workgroups of 512 threads per replica owning 16-column tiles of every layer, "
                    f"{rt} row tiles x {ks}-way k split, {lds // 1024} KB LDS; grid {grid})")
        if self.exe.persistent():
            nk0, nc0, kc0, cw, nch, wgs, grid = self.exe.persist_geometry()
            var, nd, sync, local = self.exe.persist_variant()[:4]
            dw = f" + {nd} weight-gradient workgroups" if var == 2 else ""
            sy = ", per-step gradient exchange of the replicas inside the launch" if sync else ""
            sy += {1: ", XCD-local hand-offs", 2: ", replica exchange in the XCD's L2"}.get(local, "")
            return (f"persistent V{var}{sy} (1 kernel + 1 post kernel per <= {self.GRAPH_CHUNK}-step chunk; per "
                    f"replica {nk0}x{nc0} layer-0 tiles of {kc0}x{cw} + {nch} row-chain workgroups{dw}; "
                    f"grid {grid})")
        if self.exe.rowchain():
            return "row-chain (3 launches per step)"
        if self.exe.tailchain():
            return f"tail-chain ({self.exe.launches_per_step()} launches per step)"
        return f"grouped ({self.exe.launches_per_step()} launches per step)"

    @property
    def plan_reason(self) -> str:
        """Why the training step does not run one of the persistent plans ('' when it does)."""
        return str(self.exe.plan_reason())

    @property
    def rowchain(self) -> bool:
        """True when training steps run the 3-launch row-chain plan (csrc/kernels/rowchain.hip)."""
        return bool(self.exe.rowchain())
