"""Workers: what runs per partition (reference elephas/worker.py:11-131).

``SparkWorker``           synchronous mode: train the partition for all epochs
                          with a fresh optimizer, report (weights_before -
                          weights_after, history); skip when n <= batch_size.
``AsynchronousSparkWorker`` asynchronous / hogwild: per epoch (or per batch)
                          pull -> train -> push delta to the parameter server.

Both keep the reference's per-partition ``train(iterator)`` generator API.  On
the MI355X path ``SparkWorker.train_partitions`` trains ALL of a rank's
partitions at once as replicas of one native executor (every grouped launch
covers every local worker), and the async worker moves parameters
device-to-device with the DeviceClient (no host round trip).
"""
from __future__ import annotations

import logging
import math
import os
from typing import List, Optional, Sequence

import numpy as np

from .models import optimizers as O
from .models import model_from_json
from .ops.plan import flatten_weights, unflatten_weights
from .parameter.client import BaseParameterClient, DeviceClient
from .utils.functional_utils import subtract_params

_log = logging.getLogger(__name__)


def _value(parameters):
    return parameters.value if hasattr(parameters, "value") else parameters


def partition_to_numpy(data):
    """A partition's (features, labels) arrays: the views of a columnar partition as
    they are, else stacked from its (x, y) rows."""
    from .data.rdd import ColumnarPartition
    if isinstance(data, ColumnarPartition):
        return np.asarray(data.x), np.asarray(data.y)
    items = list(data)
    if not items:
        return np.zeros((0,)), np.zeros((0,))
    x = np.asarray([xy[0] for xy in items])
    y = np.asarray([xy[1] for xy in items])
    return x, y


def _build_model(json_str, custom_objects, optimizer, loss, metrics, weights):
    model = model_from_json(json_str, custom_objects)
    opt = O.deserialize(optimizer, custom_objects) if isinstance(optimizer, dict) else O.clone(optimizer)
    model.compile(optimizer=opt, loss=loss, metrics=metrics, custom_objects=custom_objects)
    model.set_weights(weights)
    return model


def _frozen(a: np.ndarray) -> bool:
    """True when no one can write a's bytes: a and every array it views are read-only."""
    while isinstance(a, np.ndarray):
        if a.flags.writeable:
            return False
        a = a.base
    return True


class _DataKey:
    """Identity of a rank's partitions for the trainer cache.  Uploaded shards are
    reused only for the very same array objects (held here, so their ids and buffers
    cannot be recycled by the allocator) that are frozen -- read-only down the whole
    view chain, as the columnar partitions ``RDD.repartition`` builds -- so no in-place
    edit can go unseen.  Writable arrays never match: their shards are re-uploaded."""

    __slots__ = ("arrays", "meta", "reusable")

    def __init__(self, xs, ys, vs, active, shuffle):
        self.arrays = tuple(np.asarray(a) for a in list(xs) + list(ys))
        self.meta = (float(vs), tuple(bool(a) for a in active), bool(shuffle))
        self.reusable = all(a.size == 0 or _frozen(a) for a in self.arrays)

    def __eq__(self, other):
        return (isinstance(other, _DataKey) and self.reusable and other.reusable and self.meta == other.meta
                and len(self.arrays) == len(other.arrays)
                and all(a is b for a, b in zip(self.arrays, other.arrays)))

    def __ne__(self, other):
        return not self.__eq__(other)

    __hash__ = None


def _data_key(xs, ys, vs, active, shuffle):
    return _DataKey(xs, ys, vs, active, shuffle)


class _TrainerCache:
    """The last native trainer a SparkWorker built (one per process): a following fit
    of the same model / optimizer / loss / metrics / batch size / replica count reuses its
    device buffers, executor plan and -- for unchanged partitions -- its uploaded shards."""

    def __init__(self):
        self._key, self._entry = None, None

    @staticmethod
    def _key_of(worker, R, engine):
        import json
        from . import config
        bs, _, _, _, _ = worker._cfg()
        enc = lambda o: json.dumps(o, sort_keys=True, default=lambda v: getattr(v, "__name__", repr(v)))
        custom = tuple((k, id(v)) for k, v in sorted((worker.custom_objects or {}).items()))
        return (worker.json, enc(worker.master_optimizer), enc(worker.master_loss), enc(worker.master_metrics),
                custom, int(R), int(bs), config.get_policy(), str(config.get_device()), engine)

    def lookup(self, worker, R, engine):
        if self._entry is None or self._key != self._key_of(worker, R, engine):
            return None
        return self._entry

    def store(self, worker, R, engine, trainer, model, data_key):
        if not hasattr(trainer, "reset_for_fit"):   # only the native engine is reused
            self._key, self._entry = None, None
            return
        self._key, self._entry = self._key_of(worker, R, engine), (trainer, model, data_key)

    def set_data_key(self, data_key):
        if self._entry is not None:
            self._entry = (self._entry[0], self._entry[1], data_key)

    def clear(self):
        self._key, self._entry = None, None


_trainer_cache = _TrainerCache()


class SparkWorker:
    """Synchronous worker (reference worker.py:11-49)."""

    def __init__(self, json, parameters, train_config, master_optimizer, master_loss, master_metrics,
                 custom_objects):
        self.json = json
        self.parameters = parameters
        self.train_config = dict(train_config)
        self.master_optimizer = master_optimizer
        self.master_loss = master_loss
        self.master_metrics = master_metrics
        self.custom_objects = custom_objects or {}
        self.model = None

    def _cfg(self):
        tc = self.train_config
        return (int(tc.get("batch_size", 32)), int(tc.get("epochs", 1)), int(tc.get("verbose", 0)),
                float(tc.get("validation_split", 0.0)), bool(tc.get("shuffle", True)))

    def train(self, data_iterator):
        """Single-partition generator, as the reference's mapPartitions function."""
        self.model = _build_model(self.json, self.custom_objects, self.master_optimizer, self.master_loss,
                                  self.master_metrics, _value(self.parameters))
        x_train, y_train = partition_to_numpy(data_iterator)
        bs, epochs, verbose, vs, shuffle = self._cfg()
        before = self.model.get_weights()
        history = None
        if x_train.shape[0] > bs:
            h = self.model.fit(x_train, y_train, batch_size=bs, epochs=epochs, verbose=verbose,
                               validation_split=vs, shuffle=shuffle)
            history = h.history
        after = self.model.get_weights()
        yield [subtract_params(before, after), history]

    def prepare_partitions(self, partitions: Sequence[list], engine: Optional[str] = None,
                           seed: Optional[int] = None, sync: bool = False):
        """Build the shared executor with one replica per partition and load the
        shards (no training). Returns (trainer, active). ``sync``: the replicas are one
        model trained with per-step synchronous DP (native engine; NativeTrainer sync)."""
        from .ops.engine import make_trainer
        bs, epochs, verbose, vs, shuffle = self._cfg()
        native_kw = {"sync": True} if sync else {}
        base_engine = engine
        if sync:   # a sync trainer is cached apart from an independent-replica one
            engine = f"{engine or ''}|sync"
        xs, ys = [], []
        for p in partitions:
            x, y = partition_to_numpy(p)
            xs.append(x)
            ys.append(y)
        active = [len(x) > bs for x in xs]   # reference worker.py:41 (`if n > batch_size: fit`)
        hit = _trainer_cache.lookup(self, len(partitions), engine)
        if hit is not None:
            # same model / optimizer / shapes as the previous fit: reset the cached native
            # trainer instead of rebuilding it, and keep its device shards if the
            # partitions are the very same arrays (columnar RDDs of an unchanged dataset)
            trainer, model, data_key = hit
            self.model = model
            trainer.reset_for_fit(flatten_weights(list(_value(self.parameters))), seed)
            key = _data_key(xs, ys, vs, active, shuffle)
            if partitions and (key is None or key != data_key):
                trainer.set_data(xs, ys, vs, active=active, shuffle=shuffle)
                _trainer_cache.set_data_key(key)
            return trainer, active
        self.model = _build_model(self.json, self.custom_objects, self.master_optimizer, self.master_loss,
                                  self.master_metrics, _value(self.parameters))
        trainer = make_trainer(self.model, max(1, len(partitions)), bs, engine=base_engine, seed=seed, **native_kw)
        if partitions:
            trainer.set_data(xs, ys, vs, active=active, shuffle=shuffle)
        _trainer_cache.store(self, len(partitions), engine, trainer, self.model,
                             _data_key(xs, ys, vs, active, shuffle) if partitions else None)
        return trainer, active

    def train_partitions(self, partitions: Sequence[list], engine: Optional[str] = None, seed: Optional[int] = None):
        """Batched: train every partition as one replica of a shared executor.

        Returns (trainer, histories, active); the trainer's per-replica weights
        are the workers' final weights (theta_i); delta_i = theta_0 - theta_i.
        """
        from .ops.engine import make_trainer
        self.model = _build_model(self.json, self.custom_objects, self.master_optimizer, self.master_loss,
                                  self.master_metrics, _value(self.parameters))
        bs, epochs, verbose, vs, shuffle = self._cfg()
        xs, ys = [], []
        for p in partitions:
            x, y = partition_to_numpy(p)
            xs.append(x)
            ys.append(y)
        active = [len(x) > bs for x in xs]   # reference worker.py:41 (`if n > batch_size: fit`)
        R = max(1, len(partitions))
        trainer = make_trainer(self.model, R, bs, engine=engine, seed=seed)
        if not partitions:
            return trainer, [], []
        trainer.set_data(xs, ys, vs, active=active, shuffle=shuffle)
        hist = trainer.fit(epochs, verbose=verbose) if any(active) else [None] * R
        hist = [h if a else None for h, a in zip(hist, active)]
        return trainer, hist, active


class AsynchronousSparkWorker:
    """Asynchronous / hogwild worker (reference worker.py:52-131)."""

    def __init__(self, json, parameters, client, train_config, frequency, master_optimizer, master_loss,
                 master_metrics, custom_objects):
        if isinstance(client, BaseParameterClient):
            self.client = client
        else:
            self.client = BaseParameterClient.get_client(client)
        self.train_config = dict(train_config)
        self.frequency = frequency
        self.master_optimizer = master_optimizer
        self.master_loss = master_loss
        self.master_metrics = master_metrics
        self.json = json
        self.parameters = parameters
        self.custom_objects = custom_objects or {}
        self.model = None

    def train(self, data_iterator):
        x_train, y_train = partition_to_numpy(data_iterator)
        if x_train.size == 0:
            return
        self.model = _build_model(self.json, self.custom_objects, self.master_optimizer, self.master_loss,
                                  self.master_metrics, _value(self.parameters))
        epochs = int(self.train_config.get("epochs", 1))
        batch_size = int(self.train_config.get("batch_size", 32))
        verbose = int(self.train_config.get("verbose", 0))
        vs = float(self.train_config.get("validation_split", 0.0))
        if self.frequency not in ("epoch", "batch"):
            raise ValueError("frequency parameter can be `epoch` or `batch, got {}".format(self.frequency))
        from .ops.engine import make_trainer
        trainer = make_trainer(self.model, 1, batch_size)
        native = hasattr(trainer, "exe") and isinstance(self.client, DeviceClient)
        if self.frequency == "epoch":
            trainer.set_data([x_train], [y_train], vs, shuffle=True)
            for _ in range(epochs):
                self._pull(trainer, native)
                if x_train.shape[0] > batch_size:
                    trainer.fit(1, verbose=verbose)
                self._push(trainer, native)
        else:
            if x_train.shape[0] > batch_size:
                trainer.set_data([x_train], [y_train], 0.0, shuffle=False)
                nb = int(math.ceil(x_train.shape[0] / batch_size))
                for _ in range(epochs):
                    if native:
                        trainer.begin_epoch()
                    for b in range(nb):
                        self._pull(trainer, native)
                        if native:
                            trainer.run_steps(1, use_graph=True)
                        else:
                            trainer.train_batch(0, trainer.xs[0][b * batch_size:(b + 1) * batch_size],
                                                trainer.ys[0][b * batch_size:(b + 1) * batch_size])
                        self._push(trainer, native)
        self.model.set_weights(unflatten_weights(trainer.get_weights_flat()[0], self.model.get_weights()))
        yield []

    # --- parameter-server exchange
    def _pull(self, trainer, native):
        from .parallel import dist, fault
        fault.maybe_inject("pull", dist.rank())
        if native:
            import torch
            with torch.cuda.stream(trainer.stream):
                self.client.pull_into(trainer.P.data_ptr(), trainer.s)
                trainer.sync_shadows()
                self._before = trainer.P.clone()
        else:
            w = self.client.get_parameters()
            self._before = flatten_weights(list(w))
            trainer.set_weights_flat(self._before)

    def _push(self, trainer, native):
        from .parallel import dist, fault
        fault.maybe_inject("push", dist.rank())
        if native:
            import torch
            with torch.cuda.stream(trainer.stream):
                delta = self._before - trainer.P   # theta_pulled - theta_after
                self.client.push_from(delta.data_ptr(), trainer.s)
        else:
            after = trainer.get_weights_flat()[0]
            delta = self._before - after
            self.client.update_parameters(unflatten_weights(delta, self.model.get_weights()))


def group_persist_cus(groups: int, device=None) -> int:
    """CU share of each of ``groups`` concurrently running worker groups: their persistent
    chunk kernels (csrc/kernels/persist.hip) need every workgroup resident, so the grids
    are sized to split the GPU between them -- their total never exceeds the CU count,
    so each can always become resident once the transient kernels (parameter-server
    pulls / pushes) beside it finish. (MNIST: 8 groups x 32 CUs = one replica's grid each.)"""
    import torch
    ncu = torch.cuda.get_device_properties(device if device is not None else torch.cuda.current_device()
                                           ).multi_processor_count
    return max(1, ncu // max(1, groups))


class BatchedAsynchronousWorker:
    """GPU path of the asynchronous / hogwild workers for all of a rank's partitions.

    The reference runs one AsynchronousSparkWorker per partition in its own process
    (worker.py:52-131), each progressing on its own against a concurrently served
    parameter server.  Here a rank's partitions are split into ``groups`` (default:
    one per partition) that progress just as independently: every group is its own
    native executor on its own HIP stream, and its exchange with the sharded device
    parameter server (parameter/client.py DeviceClient) is stream-ordered kernels --
    pull (gather theta, chunk-consistent in 'asynchronous' mode) -> refresh every
    replica's weights -> train -> push (fp32 atomic adds of sum_r(P[r] - before)) --
    with no host lock and no host synchronisation.  The host only enqueues, so the
    groups' pulls and pushes interleave on the GPU in whatever order the hardware
    runs them; within a group the replicas move in lockstep and push one summed
    delta.  For frequency='batch' a group's whole pull/step/push is ONE hipGraph
    replay per batch.  Replicas without a batch in a step (shorter partitions) push
    a zero delta, as do partitions with n <= batch_size (reference worker.py:116).
    """

    def __init__(self, json, parameters, client, train_config, frequency, master_optimizer, master_loss,
                 master_metrics, custom_objects, groups: Optional[int] = None):
        self.json, self.parameters, self.client = json, parameters, client
        self.train_config = dict(train_config)
        self.frequency = frequency
        self.master_optimizer, self.master_loss, self.master_metrics = master_optimizer, master_loss, master_metrics
        self.custom_objects = custom_objects or {}
        self.groups = groups
        self.model = None
        self.histories = []

    def _n_groups(self, nparts: int) -> int:
        import os
        g = self.groups if self.groups else int(os.environ.get("ELEPHAS_AMD_ASYNC_GROUPS", "0") or 0)
        return max(1, min(nparts, g if g > 0 else nparts))

    def train_partitions(self, partitions):
        from .ops.engine import make_trainer
        if self.frequency not in ("epoch", "batch"):
            raise ValueError("frequency parameter can be `epoch` or `batch, got {}".format(self.frequency))
        parts = [p for p in partitions if len(p)]
        if not parts:
            return None
        self.model = _build_model(self.json, self.custom_objects, self.master_optimizer, self.master_loss,
                                  self.master_metrics, _value(self.parameters))
        tc = self.train_config
        epochs, bs = int(tc.get("epochs", 1)), int(tc.get("batch_size", 32))
        verbose, vs = int(tc.get("verbose", 0)), float(tc.get("validation_split", 0.0))
        data = [partition_to_numpy(p) for p in parts]
        G = self._n_groups(len(parts))
        bounds = [len(parts) * g // G for g in range(G + 1)]
        groups = []
        for g in range(G):
            xs, ys = zip(*data[bounds[g]:bounds[g + 1]])
            # several groups run concurrently on their own streams: each persistent grid
            # gets its share of the CUs so all of them are resident at once
            kw = {"persist_cus": group_persist_cus(G)} if G > 1 else {}
            if self.frequency == "batch":
                kw["ps_hook"] = True   # the per-batch exchange inside the persistent launch
            t = make_trainer(self.model, len(xs), bs, engine="native", **kw)
            active = [len(x) > bs for x in xs]   # inactive replicas push a zero delta
            if self.frequency == "epoch":
                t.set_data(list(xs), list(ys), vs, active=active, shuffle=True)
            else:
                t.set_data(list(xs), list(ys), 0.0, active=active, shuffle=False)
            grp = _Group(t, active)
            if self.frequency == "batch":
                grp.attach(self.client)
            groups.append(grp)
        if self.frequency == "batch" and len({bool(g.inlaunch) for g in groups}) > 1:
            # one protocol for every writer: in-launch pushes bracket their slices with
            # slice counters, host pushes with chunk counters, and an in-launch pull looks at
            # the slice counters only -- so either every group exchanges inside its launch or
            # none does
            for g in groups:
                g.detach()
        if self.frequency == "epoch":
            for e in range(epochs):
                for g in groups:          # enqueue every group's epoch, then read histories
                    self._pull(g)
                    if any(g.active):
                        g.t.launch_epoch()
                    self._push(g)
                for g in groups:
                    if any(g.active):
                        g.t.collect_epoch(g.hist, e, epochs, verbose)
        else:
            live = [g for g in groups if any(g.active)]
            for g in live:
                g.capture(self)
            for _ in range(epochs):
                for g in live:                 # each group runs its epoch on its own stream
                    g.t.begin_epoch()
                steps = {g.t.steps_per_epoch() for g in live}
                if len(steps) == 1:
                    run_group_rounds(live, self, steps.pop())
                else:
                    for g in live:
                        g.steps(self, g.t.steps_per_epoch())
        for g in groups:
            g.t.stream.synchronize()
        if hasattr(self.client, "check"):
            self.client.check()
        self.histories = [h for g in groups for h in g.hist]
        self.trainers = [g.t for g in groups]
        return groups[0].t

    def _pull(self, g):
        import torch
        from .parallel import dist, fault
        fault.maybe_inject("pull", dist.rank())
        t = g.t
        with torch.cuda.stream(t.stream):
            if hasattr(self.client, "pull_refresh"):
                if getattr(t, "persistent", False) and hasattr(self.client, "pull_into_replicas"):
                    # the persistent kernel reads only the masters: theta straight into
                    # every replica's P by the gather itself, weight images left to their
                    # next reader
                    self.client.pull_into_replicas(g.before.data_ptr(), t.P.data_ptr(), t.P.stride(0), t.R, t.s)
                    t._images_stale = True
                    return
                self.client.pull_refresh(t, g.before.data_ptr())
                return
            self.client.pull_into(t.P[0].data_ptr(), t.s)
            if t.R > 1:
                t.P[1:].copy_(t.P[0].expand(t.R - 1, -1))
            t.sync_shadows()
            g.before.copy_(t.P[0])

    def _push(self, g):
        import torch
        from .parallel import dist, fault
        fault.maybe_inject("push", dist.rank())
        t = g.t
        with torch.cuda.stream(t.stream):
            if hasattr(self.client, "push_replicas"):
                self.client.push_replicas(t.P.data_ptr(), t.P.stride(0), t.R, g.before.data_ptr(), t.s)
                return
            # sum_r (theta_pulled - theta_r), each difference formed before summing (exact
            # for close values; R*before - sum P rounds at ulp(R*|w|) and loses the deltas)
            delta = (g.before.unsqueeze(0) - t.P).sum(0)
            self.client.push_from(delta.data_ptr(), t.s)


def run_group_rounds(groups, worker, n):
    """Enqueue n pull/step/push rounds for every group, each on its own stream.

    Measured, not kept: submitting every group's graph replays from a thread of its own
    (graph replay drops the GIL) -- no change (8 groups, 'batch': 1.87 vs 1.89 M
    samples/s). A round is ~6 kernels per group and the groups' rounds overlap ~2.3x on
    the GPU (profiles/async_batch_trace_r3.txt), so kernel count per round, not host
    submission, bounds frequency='batch'."""
    for g in groups:
        g.steps(worker, n)


class _Group:
    """One independently progressing set of lockstep replicas (BatchedAsynchronousWorker).

    frequency='batch': ``steps(n)`` runs n rounds of pull -> train step -> push on the
    group's own stream, replayed from hipGraphs holding CHUNK rounds and 1 round, so the
    host issues one launch per CHUNK batches per group and the groups' streams run
    side by side on the GPU."""

    CHUNK = 16

    def __init__(self, t, active):
        import torch
        self.t, self.active = t, active
        self.hist = t.new_history()
        self.before = torch.empty(t.P.shape[1], dtype=torch.float32, device=t.P.device)
        self.graphs = {}
        self.capture_error = None   # repr of the exception if hipGraph capture failed

    @property
    def graph(self):
        return bool(self.graphs)

    @property
    def t_inlaunch(self) -> bool:
        """The exchange runs inside the persistent launch NOW: asked of the trainer, not
        cached at attach time (a rebuilt executor -- plan fallback, grad-scale change -- may
        have dropped the hook, and then the host rounds must push the deltas)."""
        return bool(getattr(self, "inlaunch", False) and getattr(self.t, "param_server_in_launch", False))

    def attach(self, client):
        """frequency='batch' on the persistent plan: the server's push / pull per step runs
        inside the launch (NativeTrainer.attach_param_server); the host pulls theta
        into the masters once per chunk. ELEPHAS_AMD_ASYNC_INLAUNCH=0 keeps host rounds."""
        self.inlaunch = False
        ps = getattr(client, "ps", None)
        if (ps is None or os.environ.get("ELEPHAS_AMD_ASYNC_INLAUNCH", "1") == "0"
                or not hasattr(self.t, "attach_param_server")):
            return
        from .parallel import fault
        if fault.injection_active():
            return
        self.inlaunch = bool(self.t.attach_param_server(ps, bool(ps.consistent)))

    def detach(self):
        if getattr(self, "inlaunch", False):
            self.t.detach_param_server()
        self.inlaunch = False

    def capture(self, worker):
        """Capture the CHUNK-round and 1-round graphs; eager launches (logged) if capture fails."""
        import torch
        from .parallel import fault
        if self.t_inlaunch:
            return   # one persistent launch per chunk, exchange inside it
        if os.environ.get("ELEPHAS_AMD_ASYNC_GRAPH", "1") == "0" or fault.injection_active():
            return
        try:
            for k in (self.CHUNK, 1):
                g = torch.cuda.CUDAGraph()
                self.t.stream.synchronize()
                with torch.cuda.graph(g, stream=self.t.stream):
                    for _ in range(k):
                        worker._pull(self)
                        self.t.exe.train_step(self.t.s)
                        worker._push(self)
                self.graphs[k] = g
        except Exception as e:  # noqa: BLE001 - eager launches are equivalent, just slower
            # a capture failure is the first thing a new box / driver shows: say so (once
            # per group, with the cause) instead of silently running every step eagerly;
            # ELEPHAS_AMD_ASYNC_GRAPH=require turns it into an error
            self.graphs = {}
            if os.environ.get("ELEPHAS_AMD_ASYNC_GRAPH") == "require":
                raise RuntimeError(f"async group: hipGraph capture failed: {e!r}") from e
            _log.warning("async worker group: hipGraph capture failed (%r); running its pull/step/push "
                         "rounds as eager launches", e)
            self.capture_error = repr(e)

    def steps(self, worker, n):
        """Enqueue n pull/step/push rounds (no host synchronisation)."""
        import torch
        if self.t_inlaunch:
            # one host pull of theta into every replica's masters per persistent chunk; the
            # kernel pushes each step's delta and pulls the next step's theta itself
            while n > 0:
                k = min(n, self.t.GRAPH_CHUNK)
                worker._pull(self)
                self.t.run_steps(k)
                n -= k
            return
        if self.graphs:
            full, rest = divmod(n, self.CHUNK)
            with torch.cuda.stream(self.t.stream):
                for _ in range(full):
                    self.graphs[self.CHUNK].replay()
                for _ in range(rest):
                    self.graphs[1].replay()
            return
        for _ in range(n):
            worker._pull(self)
            self.t.run_steps(1, use_graph=True)
            worker._push(self)

    def step(self, worker):
        self.steps(worker, 1)
