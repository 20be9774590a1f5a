"""SparkModel / SparkMLlibModel / load_spark_model on MI355X
(reference elephas/spark_model.py:28-389).

Mapping of the reference's distribution:
  * Spark partition -> logical worker.  The partitions of the RDD are split in
    contiguous blocks over the ranks of the job (one process per GPU, launched
    by torchrun); a rank trains all of its partitions as replicas of one native
    executor on its GPU.
  * broadcast(init) -> every rank starts from the same master weights
    (broadcast from rank 0 over RCCL).
  * collect + driver-side averaging (spark_model.py:217-228) -> per-rank sum of
    the replicas' weights on the device + one RCCL all-reduce over xGMI of the
    flat parameter vector; theta <- theta0 - sum_i(delta_i)/N == mean_i(theta_i)
    with N the number of partitions (empty / tiny partitions count, as in the
    reference).
  * parameter server (async / hogwild) -> the flat vector sharded over the GPUs
    ('device' transport: every shard IPC-mapped into every rank; single-kernel
    pulls / atomic pushes on the workers' streams), or the http/socket
    compatibility transports.
  * small all-reduces -> peer-memory kernels over xGMI (parallel/p2p.py), RCCL
    above 64 MB.
  * distributed predict / evaluate -> contiguous shards per rank, ordered
    gather / sample-weighted all-reduce of [sum loss, sum metrics, n].
"""
from __future__ import annotations

import json
import os
import subprocess
import threading
from copy import deepcopy
from pathlib import Path
from typing import Any, Dict, List, Optional, Union
from uuid import uuid4

import numpy as np

from .data.linalg import Matrix, Vector
from .data.rdd import RDD, SparkContext
from .io import h5lite
from .mllib.adapter import from_matrix, from_vector, to_matrix, to_vector
from .models import optimizers as O
from .models import load_model
from .ops.plan import flatten_weights, unflatten_weights
from .parallel import dist, fault
from .profiling import MetricsLogger, PhaseTimer, device_sync, trace_range
from .utils import checkpoint as ckpt
from .parameter.factory import ClientServerFactory
from .utils.functional_utils import divide_by, subtract_params
from .utils.rdd_utils import lp_to_simple_rdd, to_simple_rdd
from .utils.serialization import model_to_dict
from .worker import AsynchronousSparkWorker, BatchedAsynchronousWorker, SparkWorker


def _resolve_ps_mode(mode: Optional[str]) -> str:
    if mode in (None, "auto"):
        import torch
        return "device" if torch.cuda.is_available() else "http"
    return mode


class SparkModel:
    def __init__(self, model, mode="asynchronous", frequency="epoch", parameter_server_mode="auto", num_workers=None,
                 custom_objects=None, batch_size=32, port=4000, *args, **kwargs):
        """SparkModel

        :param model: compiled Keras-compatible model (elephas_amd.models)
        :param mode: 'asynchronous', 'synchronous' or 'hogwild'
        :param frequency: 'epoch' or 'batch' (async / hogwild)
        :param parameter_server_mode: 'device' (HBM-resident, MI355X), 'http', 'socket', or 'auto'
        :param num_workers: number of logical workers (repartition), default: the RDD's partitions
        :param custom_objects: custom activations / losses
        :param batch_size: batch size for inference
        :param port: port of the http/socket parameter servers
        """
        self._training_histories = []
        self._master_network = model
        if not hasattr(model, "loss"):
            raise Exception("Compile your Keras model before initializing an Elephas model with it")
        dist.init_from_env()
        metrics = model.compiled_metrics._metrics
        loss = model.loss
        optimizer = O.serialize(model.optimizer)
        if custom_objects is None:
            custom_objects = {}
        if metrics is None:
            metrics = []
        self.mode = mode
        self.frequency = frequency
        self.num_workers = num_workers
        self.weights = self._master_network.get_weights()
        self.master_optimizer = optimizer
        self.master_loss = loss
        self.master_metrics = metrics
        self.custom_objects = custom_objects
        self.parameter_server_mode = parameter_server_mode
        self.batch_size = batch_size
        self.port = port
        self.kwargs = kwargs
        self.serialized_model = model_to_dict(model)
        # synchronous-mode averaging granularity (an extension):
        #   'fit'   -- the reference: train all epochs locally, average once per fit
        #   'epoch' -- average the workers' weights after every epoch
        #   'batch' -- per-step gradient all-reduce (standard synchronous DP)
        self.sync_granularity = kwargs.get("sync_granularity", "fit")
        if self.sync_granularity not in ("fit", "epoch", "batch"):
            raise ValueError("sync_granularity must be 'fit', 'epoch' or 'batch'")
        self.metrics: Dict[str, Any] = {}
        self.metrics_logger = MetricsLogger(kwargs.get("metrics_path"), rank=dist.rank())
        self.parameter_server = None
        self.client = None
        if self.mode != "synchronous":
            self._ps_type = _resolve_ps_mode(self.parameter_server_mode)
            factory = ClientServerFactory.get_factory(self._ps_type)
            if dist.rank() == 0:
                self.parameter_server = factory.create_server(self.serialized_model, self.port, self.mode,
                                                              custom_objects=self.custom_objects)
            self.client = factory.create_client(self.port)

    # ------------------------------------------------------------- config
    def get_config(self):
        base_config = {
            "parameter_server_mode": self.parameter_server_mode,
            "mode": self.mode,
            "frequency": self.frequency,
            "num_workers": self.num_workers,
            "batch_size": self.batch_size}
        config = base_config.copy()
        config.update(self.kwargs)
        return config

    def save(self, file_name: str, overwrite: bool = False, to_hadoop: bool = False):
        """Keras HDF5 of the master network + root attr ``distributed_config``
        (reference spark_model.py:92-134)."""
        assert file_name[-3:] == ".h5" or file_name[-6:] == ".keras", \
            "File name must end with either '.h5' or '.keras'"
        if dist.rank() != 0:
            return
        if overwrite and not to_hadoop and Path(file_name).exists():
            Path(file_name).unlink()
        if to_hadoop:
            cluster_file_path = deepcopy(file_name)
            file_name = str(uuid4()) + "-temp-model-file." + file_name.split(".")[-1]
        self._master_network.save(file_name)
        f = h5lite.File(file_name, mode="a")
        f.attrs["distributed_config"] = json.dumps({
            "class_name": self.__class__.__name__,
            "config": self.get_config()
        }).encode("utf8")
        f.flush()
        f.close()
        if to_hadoop:
            cli = ["hadoop", "fs", "-moveFromLocal"]
            if overwrite:
                cli.append("-f")
            cli.append(file_name)
            cli.append(cluster_file_path)
            subprocess.run(cli)

    @property
    def training_histories(self):
        return self._training_histories

    @property
    def master_network(self):
        return self._master_network

    @master_network.setter
    def master_network(self, network):
        self._master_network = network

    def start_server(self):
        if self.parameter_server is not None:
            self.parameter_server.start()

    def stop_server(self):
        if self.parameter_server is not None:
            self.parameter_server.stop()

    # ---------------------------------------------------------- inference
    def predict(self, data: Union[RDD, np.ndarray]) -> List[np.ndarray]:
        """Distributed inference; returns one prediction row per input row, in order."""
        if isinstance(data, RDD):
            data = np.asarray(data.collect())
        return self._predict(np.asarray(data))

    def evaluate(self, x_test: np.ndarray, y_test: np.ndarray, **kwargs) -> Union[List[float], float]:
        return self._evaluate(np.asarray(x_test), np.asarray(y_test), **kwargs)

    def _predict(self, x: np.ndarray) -> List[np.ndarray]:
        lo, hi = dist.block_range(len(x))
        local = self._master_network.predict(x[lo:hi]) if hi > lo else \
            np.zeros((0,) + tuple(self._master_network.output_shape[1:]), np.float32)
        out = dist.all_gather_rows(local, len(x))
        return list(out)

    def _evaluate(self, x, y, **kwargs):
        import torch
        lo, hi = dist.block_range(len(x))
        nmet = len(self.master_metrics)
        sums = np.zeros(2 + nmet)
        if hi > lo:
            t = self._master_network._trainer(int(kwargs.get("batch_size") or 32)) \
                if self._master_network._compiled else None
            if t is None:
                raise RuntimeError("master network is not compiled")
            s = np.asarray(t.evaluate_sums(x[lo:hi], y[lo:hi]))
            sums[:2 + nmet] = s[:2 + nmet]
        ts = torch.tensor(sums, dtype=torch.float64)
        dist.all_reduce_sum_(ts)
        sums = ts.numpy()
        n = max(sums[1], 1.0)
        avg_loss = float(sums[0] / n)
        avg_metrics = [float(v / n) for v in sums[2:2 + nmet]]
        return [avg_loss, *avg_metrics] if avg_metrics else avg_loss

    # ------------------------------------------------------------ training
    def fit(self, rdd: RDD, **kwargs):
        """Train on an RDD of (features, label) pairs.

        :param epochs: number of epochs; :param batch_size: per-worker batch size;
        :param verbose: 0/1/2; :param validation_split: tail fraction held out per worker
        :param checkpoint_dir: (extension, synchronous mode) write a resumable
            checkpoint there after every averaging point (each epoch for
            sync_granularity 'epoch'/'batch', the end of fit for 'fit')
        :param resume: continue from the checkpoint in checkpoint_dir if present
        """
        print(">>> Fit model")
        if self.num_workers:
            rdd = rdd.repartition(self.num_workers)
        if self.mode in ["asynchronous", "synchronous", "hogwild"]:
            self._fit(rdd, **kwargs)
        else:
            raise ValueError("Choose from one of the modes: asynchronous, synchronous or hogwild")

    def _broadcast_init(self) -> List[np.ndarray]:
        import torch
        init = self._master_network.get_weights()
        if dist.world_size() > 1:
            flat = torch.from_numpy(flatten_weights(init))
            if dist.backend() == "nccl":
                flat = flat.cuda()
            dist.broadcast_(flat, 0)
            init = unflatten_weights(flat.cpu().numpy(), init)
            self._master_network.set_weights(init)
        return init

    def _fit(self, rdd: RDD, **kwargs):
        self._master_network.compile(optimizer=O.get(self.master_optimizer), loss=self.master_loss,
                                     metrics=self.master_metrics, custom_objects=self.custom_objects)
        train_config = dict(kwargs)
        checkpoint_dir = train_config.pop("checkpoint_dir", None)
        resume = bool(train_config.pop("resume", False))
        train_config.setdefault("epochs", 1)
        train_config.setdefault("batch_size", 32)
        timer = PhaseTimer(sync=device_sync())
        self._timer = timer
        t0 = __import__("time").perf_counter()
        with trace_range("elephas.fit"):
            model_json = self._master_network.to_json()
            with timer.phase("broadcast"):
                init = self._broadcast_init()
            parts = rdd.partitions()
            lo, hi = dist.block_range(len(parts))
            local = parts[lo:hi]
            if self.mode in ["asynchronous", "hogwild"]:
                new_parameters = self._fit_async(model_json, init, local, train_config)
            elif self.mode == "synchronous":
                new_parameters = self._fit_sync(model_json, init, local, len(parts), train_config,
                                                checkpoint_dir, resume)
            else:
                raise ValueError("Unsupported mode {}".format(self.mode))
            self._master_network.set_weights(new_parameters)
        wall = __import__("time").perf_counter() - t0
        rows = sum(len(p) for p in parts)
        epochs = int(train_config.get("epochs", 1))
        vs = float(train_config.get("validation_split", 0.0) or 0.0)
        samples = int(rows * (1.0 - vs)) * epochs
        self.metrics = dict(mode=self.mode, granularity=self.sync_granularity if self.mode == "synchronous" else None,
                            workers=len(parts), world_size=dist.world_size(), epochs=epochs, samples=samples,
                            seconds=round(wall, 6), samples_per_sec=round(samples / wall, 2) if wall > 0 else None,
                            phases=timer.as_dict())
        self.metrics_logger.log("fit", **self.metrics)

    # ------------------------------------------------------ sync averaging
    def _sum_replicas(self, trainer, n):
        """Sum over this rank's replicas of their weights, as a tensor on the
        collective's device (stays in HBM on the native engine)."""
        import torch
        if hasattr(trainer, "P"):                      # native: stays on the device
            trainer.stream.synchronize()
            total = trainer.P.sum(0, dtype=torch.float32)
            return total if dist.backend() == "nccl" else total.cpu()
        w = trainer.get_weights_flat()
        total = torch.from_numpy(w.sum(0).astype(np.float32) if len(w) else np.zeros(n, np.float32))
        return total.cuda() if dist.backend() == "nccl" else total

    def _average_into(self, trainer, n_params, n_parts, active_local):
        """theta <- mean over all N workers of theta_i (reference spark_model.py:221-227:
        theta0 - sum(delta_i)/N), written back into every local replica."""
        fault.maybe_inject("allreduce", dist.rank())
        with self._timer.phase("allreduce"):
            if hasattr(trainer, "average_replicas"):
                # native engine: the bench's device path (NativeTrainer.average_replicas),
                # all-reduce ordered on the trainer's stream
                multi = dist.world_size() > 1
                mean = trainer.average_replicas(dist.all_reduce_sum_ if multi else None, max(n_parts, 1),
                                                include=bool(active_local))
                if multi:
                    trainer.stream.synchronize()
                    from .parallel import p2p
                    peer = p2p.current()
                    if peer is not None:
                        peer.check()   # a timed-out peer wait must not pass as a mean
                return mean
            total = self._sum_replicas(trainer, n_params) if active_local else self._zeros(n_params)
            dist.all_reduce_sum_(total)
            mean = total / float(max(n_parts, 1))
        if active_local:
            trainer.set_weights_flat(mean.cpu().numpy())
        return mean

    def _zeros(self, n):
        import torch
        z = torch.zeros(n, dtype=torch.float32)
        return z.cuda() if dist.backend() == "nccl" else z

    def _grad_allreduce(self, n_parts):
        """Per-step gradient averaging over all workers of the job for [R, n] G blocks."""
        def allreduce(G):
            tot = G.sum(0)
            dist.all_reduce_sum_(tot)
            G.copy_((tot / float(max(n_parts, 1))).expand_as(G))
        return allreduce

    def _fit_sync(self, model_json, init, local, n_parts, train_config, checkpoint_dir=None, resume=False):
        worker = SparkWorker(model_json, init, train_config, self.master_optimizer, self.master_loss,
                             self.master_metrics, self.custom_objects)
        n_params = len(flatten_weights(init))
        gran = self.sync_granularity
        epochs = int(train_config.get("epochs", 1))
        verbose = int(train_config.get("verbose", 0))
        # per-step sync DP on one rank: the partitions are replicas of ONE sync trainer whose
        # gradients are summed every step (inside the persistent launch on the native
        # engine) instead of a host-issued all-reduce per step
        bs = int(train_config.get("batch_size", 32))
        sync_local = (gran == "batch" and dist.world_size() == 1 and len(local) > 1
                      and all(len(p) > bs for p in local))
        # several ranks: the same, with the replica sums exchanged between the ranks inside
        # the launch (attach_rank_exchange), when every rank holds equally many partitions
        # of equal sizes (the exchange needs one step sequence on all ranks)
        cross = False
        if gran == "batch" and dist.world_size() > 1:
            sizes = dist.all_gather_object(tuple(len(p) for p in local))
            cross = (len(set(sizes)) == 1 and len(set(sizes[0])) == 1 and len(local) >= 2
                     and all(n > bs for n in sizes[0]) and self._native_ok())
        with self._timer.phase("setup"):
            trainer, active = worker.prepare_partitions(local, sync=sync_local or cross)
            if cross:
                # collective on every rank (all hold >= 2 equal partitions: sync trainers)
                ok = trainer.attach_rank_exchange(dist.rank(), dist.world_size())
                if not all(dist.all_gather_object(bool(ok))):
                    trainer, active = worker.prepare_partitions(local, sync=False)
        start = 0
        if checkpoint_dir and resume and ckpt.exists(checkpoint_dir):
            with self._timer.phase("checkpoint"):
                start, weights, state = ckpt.load(checkpoint_dir, dist.rank(), len(local))
                if local:
                    trainer.set_weights_flat(weights)
                    if state is not None:
                        trainer.set_state_flat(*state)
            print(f">>> Resuming from epoch {start} of {epochs} ({checkpoint_dir})")
        hist = [dict() if a else None for a in active]
        if gran == "fit":
            # the reference: every worker trains all epochs on its own, one average at the end
            if start < epochs and local and any(active):
                fault.maybe_inject("train", dist.rank())
                with self._timer.phase("train"):
                    h = trainer.fit(epochs - start, verbose=verbose)
                hist = [hh if a else None for hh, a in zip(h, active)]
            mean = self._average_into(trainer, n_params, n_parts, bool(local))
            if checkpoint_dir:
                self._save_checkpoint(checkpoint_dir, epochs, epochs, mean, trainer, local)
        else:
            mean = None
            allreduce = (self._grad_allreduce(n_parts) if gran == "batch" and not getattr(trainer, "sync", False)
                         else None)
            for e in range(start, epochs):
                if local and any(active):
                    fault.maybe_inject("train", dist.rank())
                    with self._timer.phase("train"):
                        h = trainer.fit(1, verbose=verbose, allreduce=allreduce) if allreduce is not None \
                            else trainer.fit(1, verbose=verbose)
                    for r, (hh, a) in enumerate(zip(h, active)):
                        if a and hh:
                            for k, v in hh.items():
                                hist[r].setdefault(k, []).extend(v)
                elif gran == "batch":
                    raise RuntimeError("per-step all-reduce needs at least one partition on every rank")
                mean = self._average_into(trainer, n_params, n_parts, bool(local))
                if checkpoint_dir:
                    self._save_checkpoint(checkpoint_dir, e + 1, epochs, mean, trainer, local)
            if mean is None:
                mean = self._average_into(trainer, n_params, n_parts, bool(local))
        with self._timer.phase("gather_histories"):
            for h in dist.all_gather_object(hist if local else []):
                self._training_histories.extend(h)
        print(">>> Synchronous training complete.")
        return unflatten_weights(mean.cpu().numpy(), init)

    def _save_checkpoint(self, directory, epoch, epochs, mean, trainer, local):
        with self._timer.phase("checkpoint"), trace_range("elephas.checkpoint"):
            state = trainer.get_state_flat() if local else None
            weights = mean.cpu().numpy()
            if dist.rank() == 0:
                self._master_network.set_weights(unflatten_weights(weights, self._master_network.get_weights()))
            ckpt.save(directory, epoch, epochs, self._master_network, weights, state, dist.rank(),
                      dict(class_name=self.__class__.__name__, config=self.get_config()))
            dist.barrier()

    def _native_ok(self) -> bool:
        import torch
        from .ops.engine import native_supported
        from . import config
        if not torch.cuda.is_available() or config.get_engine() == "torch":
            return False
        ok, _ = native_supported(self._master_network)
        return ok

    def _fit_async(self, model_json, init, local, train_config):
        import torch
        ps = self.parameter_server
        if dist.rank() == 0 and ps is not None:
            ps.set_weights(init)     # snapshot at fit time (reference quirk 3 fixed)
            self.start_server()
        client = self.client
        if self._ps_type == "device":
            # collective: every rank allocates its shard of theta and maps the others'
            client.like = init
            client.connect(len(flatten_weights(init)), self.mode, server=ps if dist.rank() == 0 else None)
            if dist.rank() == 0:
                ps.set_weights(init)
        dist.barrier()
        print(">>> Initialize workers")
        errors = []

        def run(part):
            try:
                w = AsynchronousSparkWorker(model_json, init, client, train_config, self.frequency,
                                            self.master_optimizer, self.master_loss, self.master_metrics,
                                            self.custom_objects)
                for _ in w.train(iter(part)):
                    pass
            except BaseException as e:  # propagate worker failures (fail fast)
                errors.append(e)

        print(">>> Distribute load")
        try:
            if self._ps_type == "device" and self._native_ok() and local:
                # MI355X path: the rank's partitions as independently progressing groups of
                # native replicas, each on its own stream, exchanging with the sharded device
                # parameter server through stream-ordered kernels (worker.py)
                try:
                    BatchedAsynchronousWorker(model_json, init, client, train_config, self.frequency,
                                              self.master_optimizer, self.master_loss, self.master_metrics,
                                              self.custom_objects,
                                              groups=self.kwargs.get("async_groups")).train_partitions(local)
                except BaseException as e:  # noqa: BLE001 - voted on below, then raised
                    errors.append(e)
                local = []
            threads = [threading.Thread(target=run, args=(p,)) for p in local]
            for t in threads:
                t.start()
            for t in threads:
                t.join()
            # failure vote instead of a barrier: a healthy rank learns that a peer failed
            # and raises now rather than blocking in the next collective until it times out
            if dist.any_failed(bool(errors)):
                if errors:
                    raise errors[0]
                raise RuntimeError("asynchronous training failed on another rank")
            print(">>> Async training complete.")
            if dist.rank() == 0:
                new_parameters = ps.get_weights()
                flat = flatten_weights(new_parameters)
            else:
                flat = np.zeros(len(flatten_weights(init)), np.float32)
            t = torch.from_numpy(flat.copy())
            if dist.backend() == "nccl":
                t = t.cuda()
            dist.broadcast_(t, 0)
            final = unflatten_weights(t.cpu().numpy(), init)
        finally:
            if dist.rank() == 0:
                self.stop_server()   # always, also when a worker failed
            if self._ps_type == "device":
                # after a completed broadcast every rank has synchronised its pulls and
                # pushes and rank 0 its final pull: the shards can be freed
                if ps is not None:
                    ps.close()
                client.close(release="final" in locals())
        if ps is not None and self._ps_type == "device":
            ps.set_weights(final)    # host copy of the final weights (the shards are gone)
        return final


class SparkMLlibModel(SparkModel):
    def __init__(self, model, mode="asynchronous", frequency="epoch", parameter_server_mode="auto", num_workers=4,
                 elephas_optimizer=None, custom_objects=None, batch_size=32, port=4000, *args, **kwargs):
        """SparkMLlibModel: trains on RDDs of LabeledPoints (reference spark_model.py:311-352)."""
        SparkModel.__init__(self, model=model, mode=mode, frequency=frequency,
                            parameter_server_mode=parameter_server_mode, num_workers=num_workers,
                            custom_objects=custom_objects, batch_size=batch_size, port=port, *args, **kwargs)

    def fit(self, labeled_points: RDD, epochs: int = 10, batch_size: int = 32, verbose: int = 0,
            validation_split: float = 0.1, categorical: bool = False, nb_classes: Optional[int] = None):
        rdd = lp_to_simple_rdd(labeled_points, categorical, nb_classes)
        rdd = rdd.repartition(self.num_workers)
        self._fit(rdd=rdd, epochs=epochs, batch_size=batch_size, verbose=verbose, validation_split=validation_split)

    def predict(self, mllib_data):
        """Predict on an MLlib Matrix (rows) or Vector (one sample), returning the same type."""
        if isinstance(mllib_data, Matrix):
            return to_matrix(self._master_network.predict(from_matrix(mllib_data)))
        elif isinstance(mllib_data, Vector):
            return to_vector(self._master_network.predict(from_vector(mllib_data).reshape(1, -1))[0])
        raise ValueError("Provide either an MLLib matrix or vector, got {}".format(type(mllib_data).__name__))


def load_spark_model(file_name: str, from_hadoop: bool = False) -> Union[SparkModel, SparkMLlibModel]:
    """Load a SparkModel / SparkMLlibModel saved by ``save`` (reference spark_model.py:355-389)."""
    assert file_name[-3:] == ".h5" or file_name[-6:] == ".keras", \
        "File name must end with either '.h5' or '.keras'"
    if from_hadoop:
        temp_file = str(uuid4()) + "-temp-model-file." + file_name.split(".")[-1]
        subprocess.run(["hadoop", "fs", "-copyToLocal", file_name, temp_file])
        file_name = temp_file
    model = load_model(file_name)
    f = h5lite.File(file_name, mode="r")
    raw = f.attrs.get("distributed_config")
    elephas_conf = json.loads(raw.decode("utf8") if isinstance(raw, (bytes, np.bytes_)) else str(raw))
    class_name = elephas_conf.get("class_name")
    config = elephas_conf.get("config")
    if from_hadoop:
        Path(file_name).unlink()
    if class_name == SparkModel.__name__:
        return SparkModel(model=model, **config)
    elif class_name == SparkMLlibModel.__name__:
        return SparkMLlibModel(model=model, **config)
    raise ValueError(f"unknown distributed model class {class_name}")
