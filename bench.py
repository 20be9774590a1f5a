#!/usr/bin/env python
"""Headline benchmark: MNIST-MLP 784-128-128-10 synchronous data-parallel
training throughput (samples/sec, whole node) on MI355X.

Config (BASELINE.json / BASELINE.md, reference examples/mnist_mlp_spark_synchronous.py):
  model 784-128(relu, dropout .2)-128(relu, dropout .2)-10(softmax), SGD lr .1,
  categorical cross-entropy + accuracy, batch 64 per worker, validation_split .1,
  8 workers per node-slot (the reference's ``local[8]``), mode='synchronous'.
Data: synthetic MNIST-shaped (784 features in [0,1], 10 one-hot classes),
  random-init weights (no network access for datasets/checkpoints).

Semantics (``--granularity``):
  fit   (default, the reference's 'synchronous' mode, spark_model.py:217-228):
        every worker trains its own partition; the timed region is K optimizer
        steps of EVERY worker followed by the synchronous parameter averaging
        (device replica sum + RCCL all-reduce over xGMI + divide).
  batch (per-step sync DP): the gradients of all workers are averaged every step
        (local batch 64*workers, RCCL all-reduce of the flat gradient per step).
A "step" = one optimizer step on one batch of 64 rows by every worker; epoch
rollover (reshuffle) happens inside the timed region as it does in fit().

Precision: fp32 by default (the reference trains with Keras's default float32); bf16
MFMA operands with fp32 master weights under --policy mixed_bfloat16.
Scaling (``--scaling``): weak (default) = 8 workers on every GPU; strong = the reference
job (8 partitions in total) split over the GPUs.

Usage: python bench.py --gpus N --steps K --warmup W
  (N>1: launched by torch.distributed.run, or -- without WORLD_SIZE in the environment --
  bench.py starts the N ranks itself as a child torchrun job before touching the GPU)
Prints ONE JSON line on rank 0.

Deadline: ``$ELEPHAS_AMD_BENCH_DEADLINE_S`` (default 900, 0 = none) bounds every rank's
wall time from its process start.  Past it, rank 0 prints the line it has -- the
headline with every sub-measurement still pending recorded as ``{"error": "deadline"}``,
or, before the headline was measured, a line with ``value`` null and ``error`` set --
and every rank exits, so one stalled cross-rank wait cannot cost the record.
"""
from __future__ import annotations

import os

# at least 16 HIP hardware queues per process (ELEPHAS_AMD_HW_QUEUES, 0 = leave the
# runtime's setting; the environment may pin HIP's default of 4): the HIP runtime
# reads this when its library loads (on `import torch`), so it is set before any import
# that could load it (elephas_amd/__init__.py explains the measurements)
_hwq = int(os.environ.get("ELEPHAS_AMD_HW_QUEUES", "16") or 0)
if _hwq > 0 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _hwq:
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, _hwq))

import argparse
import hashlib
import json
import math
import sys
import threading
import time

_T0 = time.monotonic()   # the job-wide deadline counts from the process start

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MODELS = {
    # name: (layers, dropout, classes, rows per worker, lr)
    "mnist": ([784, 128, 128], 0.2, 10, 7500, 0.1),
    "otto": ([93, 512, 512, 512], 0.5, 9, 7735, 0.01),
    "wide": ([4096, 4096, 4096], 0.0, 1000, 16384, 0.01),   # 16 batches of 1024 per epoch
}
NAMES = {"mnist": "MNIST-MLP 784-128-128-10", "otto": "Otto-MLP 93-512-512-512-9",
         "wide": "Wide-MLP 4096-4096-4096-1000"}


# rank 0's line under construction, shared with the deadline watchdog
_REPORT = {"line": None, "subs": None, "pending": [], "printed": False, "out": None, "metric": None}
_REPORT_LOCK = threading.Lock()


def _emit(line, out):
    s = json.dumps(line)
    print(s, flush=True)
    if out:
        with open(out, "a") as f:
            f.write(s + "\n")


def _finish_report(line, out):
    """Normal end: print the line unless the watchdog already did."""
    with _REPORT_LOCK:
        if _REPORT["printed"]:
            return
        _REPORT["printed"] = True
    _emit(line, out)


def _warm_calls(w):
    """Split w warmup steps into up to ELEPHAS_AMD_BENCH_WARM_CALLS calls (default 3), the
    last one the largest: [1, 1, w - 2] for w >= 3."""
    k = max(1, min(int(os.environ.get("ELEPHAS_AMD_BENCH_WARM_CALLS", "3")), w))
    return [1] * (k - 1) + [w - (k - 1)] if w > 0 else []


def _start_deadline(rank, world):
    """Job-wide deadline (module docstring): a daemon thread that, once the process has run
    for $ELEPHAS_AMD_BENCH_DEADLINE_S seconds, prints rank 0's line as far as it got and
    ends the process (os._exit: the main thread may be blocked in a collective or a device
    wait that no signal interrupts)."""
    limit = float(os.environ.get("ELEPHAS_AMD_BENCH_DEADLINE_S", "900") or 0)
    if limit <= 0:
        return

    def fire():
        time.sleep(max(0.0, limit - (time.monotonic() - _T0)))
        with _REPORT_LOCK:
            if rank == 0 and not _REPORT["printed"]:
                _REPORT["printed"] = True
                line = _REPORT["line"]
                if line is not None:
                    for name in _REPORT["pending"]:
                        _REPORT["subs"][name] = {"error": "deadline"}
                    line["config"]["sub_measurements"] = _REPORT["subs"] or None
                else:
                    line = {"metric": _REPORT["metric"], "value": None, "unit": "samples/s", "n_gpus": world,
                            "error": "deadline", "deadline_s": limit}
                line["deadline_s"] = limit
                try:
                    _emit(line, _REPORT["out"])
                except Exception:  # noqa: BLE001 - exiting regardless
                    pass
        sys.stderr.write(f"bench.py: rank {rank} reached the {limit:g} s deadline, exiting\n")
        sys.stderr.flush()
        os._exit(0)

    threading.Thread(target=fire, name="bench-deadline", daemon=True).start()


def build_model(name, optimizer="sgd", lr=None):
    from elephas_amd.models import Sequential, Dense, Activation, Dropout
    dims, drop, classes, _, lr_default = MODELS[name]
    m = Sequential()
    m.add(Dense(dims[1], input_dim=dims[0]))
    m.add(Activation("relu"))
    if drop:
        m.add(Dropout(drop))
    for d in dims[2:]:
        m.add(Dense(d))
        m.add(Activation("relu"))
        if drop:
            m.add(Dropout(drop))
    m.add(Dense(classes))
    m.add(Activation("softmax"))
    m.compile(_optimizer(optimizer, lr, lr_default), "categorical_crossentropy", ["acc"])
    return m


def _optimizer(kind, lr, lr_default):
    """sgd: SGD at the model's rate (the reference examples'); adam: Adam at lr 0.01, the
    Otto notebook's (examples/Spark_ML_Pipeline.ipynb:361)."""
    from elephas_amd.models.optimizers import SGD, Adam
    if kind == "adam":
        return Adam(learning_rate=0.01 if lr is None else lr)
    return SGD(learning_rate=lr_default if lr is None else lr)


def _optimizer_desc(args):
    if args.optimizer == "adam":
        return "Adam(lr=%g)" % (0.01 if args.lr is None else args.lr)
    return "SGD(lr=%g)" % (MODELS[args.model][4] if args.lr is None else args.lr)


def _spawn_ranks(argv, n):
    """--gpus N without a launcher: start N ranks (one process per GPU) as a child
    torchrun job and exit with its status. Runs before anything touches the GPU."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--model", default="mnist", choices=sorted(MODELS))
    ap.add_argument("--dims", default=None,
                    help="e.g. 784,256,128,10: the MNIST recipe (relu, dropout .2, SGD .1, 7500 rows per "
                         "worker) on other Dense widths -- diagnostics for the persistent plans' shape coverage")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --workers-per-gpu workers on every GPU (each GPU is one local[8] node); "
                         "strong: the reference job itself -- 8 partitions in total (examples/"
                         "mnist_mlp_spark_synchronous.py local[8]), 8/N workers per GPU")
    ap.add_argument("--workers-per-gpu", type=int, default=8)
    ap.add_argument("--batch", type=int, default=None,
                    help="rows per worker per step (default: 64 MNIST, 128 Otto -- the reference examples' sizes, "
                         "1024 Wide)")
    ap.add_argument("--policy", default="float32", choices=["mixed_bfloat16", "float32"],
                    help="float32 = the reference's Keras precision (default); mixed_bfloat16 = bf16 MFMA "
                         "operands with fp32 master weights")
    ap.add_argument("--granularity", default="fit", choices=["fit", "batch"])
    ap.add_argument("--validation-split", type=float, default=0.1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--rccl", action="store_true",
                    help="batch granularity: all-reduce through torch.distributed/RCCL (no peer-memory kernels)")
    ap.add_argument("--overlap", action="store_true",
                    help="batch granularity: per-layer gradient buckets all-reduced beside the backward")
    ap.add_argument("--dropout", type=float, default=None, help="override the model's dropout (diagnostics)")
    ap.add_argument("--out", default=None, help="also append the JSON line to this file")
    ap.add_argument("--no-sub", action="store_true",
                    help="skip the extra per-step-sync / strong-split measurements of the headline line")
    ap.add_argument("--async-groups", type=int, default=None,
                    help="async/hogwild: independently progressing worker groups per GPU (default: one per worker)")
    ap.add_argument("--frequency", default="batch", choices=["epoch", "batch"],
                    help="async / hogwild exchange frequency (reference SparkModel frequency: its async "
                         "examples use the default 'epoch')")
    ap.add_argument("--mode", default="synchronous", choices=["synchronous", "asynchronous", "hogwild"],
                    help="asynchronous / hogwild: every worker pulls from and pushes to the HBM "
                         "parameter server around each step (--frequency batch) or epoch (--frequency "
                         "epoch, the reference examples' setting); BASELINE config #3")
    ap.add_argument("--task", default="train", choices=["train", "fit", "predict", "evaluate"],
                    help="predict / evaluate: distributed inference of the master network "
                         "(SparkModel.predict / evaluate path, BASELINE config #5)")
    ap.add_argument("--infer-rows", type=int, default=None, help="rows per GPU for --task predict/evaluate")
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "adam"],
                    help="sgd (default: the reference examples' SGD at the model's rate) or adam (Adam lr 0.01, "
                         "the Otto notebook's optimizer)")
    ap.add_argument("--lr", type=float, default=None, help="override the optimizer's learning rate")
    args = ap.parse_args()

    if args.dims:
        dims = [int(v) for v in args.dims.split(",")]
        MODELS["custom"] = (dims[:-1], 0.2, dims[-1], 7500, 0.1)
        NAMES["custom"] = "MLP " + "-".join(map(str, dims))
        args.model = "custom"
    if args.batch is None:
        args.batch = {"otto": 128, "wide": 1024}.get(args.model, 64)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(sys.argv[1:], args.gpus))

    import torch
    from elephas_amd import config
    from elephas_amd.parallel import dist
    from elephas_amd.ops.plan import build_plan

    dist.init_from_env()
    rank, world = dist.rank(), dist.world_size()
    _REPORT["out"] = args.out
    _REPORT["metric"] = ("samples/sec (whole node) MNIST-MLP 784-128-128-10 sync DP at 1/2/4/8 MI355X"
                         if args.model == "mnist" else f"samples/sec (whole node) {NAMES[args.model]} sync DP")
    _start_deadline(rank, world)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the job has {world} rank(s)")
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    config.set_device(dev)
    config.set_policy(args.policy)
    np.random.seed(1234 + rank)

    if args.dropout is not None:
        d, dr, c, r, lr = MODELS[args.model]
        MODELS[args.model] = (d, args.dropout, c, r, lr)
    model = build_model(args.model, args.optimizer, args.lr)
    if args.task == "fit":
        return bench_fit(args, model, dist, rank, world, dev)
    if args.task != "train":
        return bench_infer(args, model, dist, rank, world, dev)
    if args.mode != "synchronous":
        return bench_async(args, model, dist, rank, world, dev)
    if args.scaling == "strong" and 8 % world:
        raise SystemExit("bench.py --scaling strong: the 8 reference partitions must split evenly over the GPUs")
    W = 8 // world if args.scaling == "strong" else args.workers_per_gpu
    batch_mode = args.granularity == "batch"
    m = measure_train(args, model, dist, rank, world, dev, gpu, W, batch_mode, args.steps, args.warmup)
    provenance = None
    if gpu:
        from elephas_amd.ops import native
        provenance = native.provenance()   # the loaded _C's source digest vs this tree's csrc/
    B, rows, R, samples, dt_max = args.batch, m["rows"], m["R"], m["samples"], m["dt_max"]
    batch_mode, t, state, digests = m["batch_mode"], m["t"], m["state"], m["digests"]
    devices, path, nbytes = m["devices"], m["path"], m["nbytes"]
    subs = {}
    line = None
    if rank == 0:
        value = samples / dt_max
        launches = round(t.launches_for(args.steps) / args.steps, 4) if gpu else None
        names = NAMES
        line = {
            "metric": _REPORT["metric"],
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "bf16" if args.policy == "mixed_bfloat16" else "fp32",
            "data": (f"synthetic {args.model.upper()}-shaped ({MODELS[args.model][0][0]} features, "
                     f"{MODELS[args.model][2]} classes), random-init weights"),
            "config": {
                "model": names[args.model],
                "global_batch": B * W * world,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "ranks": world,
                "backend": dist.backend(),
                "workers_per_gpu": W,
                "workers_total": W * world,
                "batch_per_worker": B,
                "rows_per_worker": rows,
                "sync": m["sync"],
                "allreduce": path,
                "allreduce_bytes": nbytes if world > 1 else None,
                "comm_world_size": dist.world_size(),
                "rank_devices": devices,
                "theta_sha1_16": digests[0],
                "theta_equal_on_all_ranks": all(d == digests[0] for d in digests),
                "optimizer": _optimizer_desc(args),
                "engine": m["engine"],
                "launches_per_step": launches,   # kernels the timed region issued / steps
                "native_provenance": provenance,
                "policy": args.policy,
                "validation_passes_timed": state["val_passes"],
                "sub_measurements": None,
            },
        }
    # extra measurements in the same line (after the headline's timed region, never inside
    # it), so a multi-GPU record also exercises the per-step exchange and the reference
    # job's strong split: per-step sync DP at the same workers per GPU, and 8 // N workers
    # per GPU (only for the default headline invocation; --no-sub skips them).  The headline
    # line exists before they start: the deadline watchdog prints it if one of them stalls.
    todo = []
    if (not args.no_sub and args.model == "mnist" and not batch_mode and args.scaling == "weak"
            and args.workers_per_gpu == 8):
        strong_w = 8 // world if 8 % world == 0 and 8 // world != W else None   # N = 1: the headline itself
        todo = [(name, w_, bm) for name, w_, bm in (("per_step_sync", W, True), ("strong", strong_w, False))
                if w_ is not None]
    with _REPORT_LOCK:
        _REPORT["line"], _REPORT["subs"], _REPORT["pending"] = line, subs, [name for name, _, _ in todo]
    sk, sw = max(1, args.steps), max(1, args.warmup)
    from elephas_amd.parallel import fault
    for name, w_, bm in todo:
        try:
            fault.maybe_inject("bench_sub:" + name, rank)
            r = measure_train(args, model, dist, rank, world, dev, gpu, w_, bm, sk, sw)
            res = {"value": round(r["samples"] / r["dt_max"], 1), "ms_per_step": round(r["dt_max"] / sk * 1e3, 4),
                   "steps": sk, "workers_per_gpu": w_, "sync": r["sync"], "engine": r["engine"],
                   "scaling": "weak" if name != "strong" else "strong",
                   "theta_equal_on_all_ranks": r["theta_equal"], "allreduce": r["path"],
                   "rank_exchange_selftest": r["xr_selftest"]}
        except Exception as e:  # noqa: BLE001 - an extra measurement never costs the headline line
            res = {"error": repr(e)[:300]}
        with _REPORT_LOCK:
            subs[name] = res
            _REPORT["pending"].remove(name)
    if rank == 0:
        line["config"]["sub_measurements"] = subs or None
        _finish_report(line, args.out)
    if dist.is_initialized():
        dist.barrier()
        import torch.distributed as tdist
        from elephas_amd.parallel import p2p
        p2p.shutdown()   # peer buffers freed only after every rank is done with them
        tdist.destroy_process_group()


def measure_train(args, model, dist, rank, world, dev, gpu, W, batch_mode, steps, warmup):
    """One timed training measurement (W workers per GPU, fit or per-step sync
    granularity): warmup steps, then EXACTLY ``steps`` steps (+ the fit averaging) between
    a barrier and device synchronisation on both sides; the max over ranks is returned
    with the evidence fields of the JSON line."""
    import torch
    from elephas_amd.ops.plan import build_plan
    plan = build_plan(model)
    dims, drop, classes, rows, _ = MODELS[args.model]
    B = args.batch
    # per-step sync DP: the W workers are replicas of one sync trainer whose gradients are
    # summed every step inside the persistent launch (native_engine sync), across ranks too
    # (the rank exchange over peer-mapped buffers, attach_rank_exchange); where that
    # cannot run: one replica of the rank's W * B rows and a per-step all-reduce
    sync_local = (batch_mode and gpu and not args.rccl and not args.overlap
                  and (world == 1 or os.environ.get("ELEPHAS_AMD_XRANK", "1") != "0"))

    def make(sync_local):
        R = W if (not batch_mode or sync_local) else 1
        Bloc = B if (not batch_mode or sync_local) else B * W
        # synthetic MNIST-shaped shards, one per worker
        rng = np.random.default_rng(1000 + rank)
        centers = rng.normal(0, 1, size=(classes, dims[0])).astype(np.float32)
        xs, ys = [], []
        for r in range(R):
            n = rows * (W if R == 1 and batch_mode else 1)
            y = rng.integers(0, classes, n)
            x = centers[y] + rng.normal(0, 2.0, size=(n, dims[0])).astype(np.float32)
            x = (x - x.min()) / (x.max() - x.min())
            xs.append(x.astype(np.float32))
            ys.append(np.eye(classes, dtype=np.float32)[y])
        if gpu:
            from elephas_amd.ops.native_engine import NativeTrainer
            t = NativeTrainer(model, plan, R, Bloc, dev, seed=4321 + rank, sync=sync_local)
        else:
            from elephas_amd.ops.torch_engine import TorchTrainer
            t = TorchTrainer(model, plan, R, Bloc, dev, seed=4321 + rank)
        t.set_data(xs, ys, args.validation_split, shuffle=True)
        return t, R, Bloc

    t, R, Bloc = make(sync_local)
    if world > 1:
        # one initial model on every rank (the reference's driver broadcasts the master
        # weights; per-step sync DP never averages, so the ranks must start equal)
        init = torch.from_numpy(np.ascontiguousarray(t.get_weights_flat()[0]))
        dist.broadcast_(init, 0)
        init_np = init.cpu().numpy()
        t.set_weights_flat(init_np)
    xrank = False
    xr_selftest = None
    if sync_local and world > 1:
        xrank = t.attach_rank_exchange(rank, world)   # collective: the same answer on every rank
        xr_selftest = getattr(t, "xr_selftest", None)   # the voted numeric self-test of the path
        if not xrank:
            sync_local = False
            t, R, Bloc = make(False)
            t.set_weights_flat(init_np)
    ntrain = t.ntrain_h[0] if gpu else t.split[0]
    steps_per_epoch = int(math.ceil(ntrain / Bloc))

    def allreduce_grads(G):
        dist.all_reduce_sum_(G)

    if batch_mode and gpu and not sync_local and (world > 1 or args.overlap):
        t.set_grad_scale(1.0 / world)   # mean of the ranks' gradients after the sum all-reduce
    channel = None
    if (batch_mode and gpu and world > 1 and not sync_local and not args.overlap and not args.no_graph
            and not args.rccl):
        from elephas_amd.parallel import p2p   # per-step peer all-reduce captured with the step
        channel = p2p.graph_channel(t.G.numel())

    state = {"step_in_epoch": steps_per_epoch, "epochs": 0, "val_passes": 0}

    def run(k, then_average=False):
        """k optimizer steps with epoch rollover (the epoch-end validation pass of the
        reference's Keras fit runs at every epoch boundary); returns rows per worker.
        then_average: the reference's averaging follows the last step (fit granularity) --
        on the persistent plan it runs fused into the last launch's end
        (NativeTrainer.run_steps_and_average)."""
        done_rows = 0
        while k > 0:
            if state["step_in_epoch"] >= steps_per_epoch:
                if state["epochs"] > 0 and args.validation_split > 0 and gpu:
                    t.launch_val()   # enqueued like fit() does: no host sync at the epoch end
                    state["val_passes"] += 1
                if gpu:
                    t.begin_epoch()
                state["step_in_epoch"] = 0
                state["epochs"] += 1
            n = min(k, steps_per_epoch - state["step_in_epoch"])
            if gpu:
                if channel is not None:
                    t.run_steps_allreduce_graph(n, channel)
                elif batch_mode and args.overlap:
                    t.run_steps_allreduce_overlap(n, dist.all_reduce_sum_)
                elif batch_mode and world > 1 and not sync_local:
                    t.run_steps_allreduce(n, allreduce_grads, use_graph=not args.no_graph)
                elif then_average and not batch_mode and n == k:
                    t.run_steps_and_average(n, dist.all_reduce_sum_ if world > 1 else None, R * world,
                                            use_graph=not args.no_graph)
                    state["averaged"] = True
                else:
                    t.run_steps(n, use_graph=not args.no_graph)
            else:
                t.train_steps(n)
            s0 = state["step_in_epoch"]
            for s in range(s0, s0 + n):
                done_rows += min(Bloc, ntrain - s * Bloc)
            state["step_in_epoch"] += n
            k -= n
        return done_rows

    def average():
        """Reference sync mode: theta <- mean_i theta_i over all workers of the job
        (device replica mean -> RCCL all-reduce -> write-back into every replica); already
        done if run() fused it into its last launch."""
        if batch_mode or state.pop("averaged", False):
            return
        if gpu:
            t.average_replicas(dist.all_reduce_sum_ if world > 1 else None, R * world)
        else:
            w = t.get_weights_flat().sum(0)
            tt = torch.from_numpy(w)
            dist.all_reduce_sum_(tt)
            t.set_weights_flat(tt.numpy() / float(R * world))

    def sync():
        if gpu:
            t.stream.synchronize()
            torch.cuda.synchronize()
        dist.barrier()

    # warmup (includes hipGraph capture of both chunk shapes)
    if gpu and not args.no_graph:
        t.prepare_graphs(allreduce_path=batch_mode and world > 1 and not args.overlap and not sync_local)
    if gpu and args.validation_split > 0:
        t._eval_exe()   # the epoch-end validation executor exists before the timed region
    # the warmup's W steps as a few calls (the timed region's call path -- launch, post node,
    # averaging -- has run more than once before it is timed; measured on the MNIST driver
    # shape: the first call after a single warmup call ran 25-100 us slower than later ones)
    for n in _warm_calls(warmup):
        run(n, then_average=True)
        average()
    sync()
    t0 = time.perf_counter()
    rows_done = run(steps, then_average=True)
    average()
    sync()
    dt = time.perf_counter() - t0
    # diagnostics only (stderr; the reported line keeps the first timed region): the same
    # region timed again ELEPHAS_AMD_BENCH_REPEAT - 1 more times
    for _ in range(int(os.environ.get("ELEPHAS_AMD_BENCH_REPEAT", "1")) - 1):
        ta = time.perf_counter()
        run(steps, then_average=True)
        average()
        sync()
        print(f"bench repeat: {(time.perf_counter() - ta) * 1e6:.1f} us (first {dt * 1e6:.1f})", file=sys.stderr)

    dts = dist.all_gather_object(dt)
    dt_max = max(dts)
    samples = rows_done * R * world
    # evidence for the multi-GPU record, gathered after the timed region: every rank's
    # HIP device, the all-reduce path actually taken, and a bit-exact digest of the
    # averaged theta (equal on every rank iff the all-reduce gave all ranks one result)
    if gpu:
        props = torch.cuda.get_device_properties(dev)
        where = (torch.cuda.current_device(), "%x:%x" % (getattr(props, "pci_bus_id", -1),
                                                        getattr(props, "pci_device_id", -1)))
        theta = t.get_weights_flat()[0]
    else:
        where, theta = None, t.get_weights_flat()[0]
    digest = hashlib.sha1(np.ascontiguousarray(theta, np.float32).tobytes()).hexdigest()[:16]
    devices = dist.all_gather_object(where)
    digests = dist.all_gather_object(digest)
    from elephas_amd.parallel import p2p
    nbytes = (t.G.numel() if batch_mode and gpu else theta.size) * 4
    if xrank:
        kern = "deep_impl.h" if t.persist_variant == 3 else "persist.hip"
        path = f"in-launch rank exchange: per-step weight-gradient tiles through peer-mapped buffers ({kern})"
    elif channel is not None:
        path = "peer-memory kernel captured in the step's hipGraph (dedicated channel)"
    elif gpu and world > 1 and not batch_mode:
        path = p2p.describe(nbytes)
    elif world > 1:
        path = f"torch.distributed {dist.backend()}" if not gpu else p2p.describe(nbytes)
    else:
        path = None
    provenance = None
    if gpu:
        from elephas_amd.ops import native
        provenance = native.provenance()   # the loaded _C's source digest vs this tree's csrc/
    sync_desc = ("reference (one-shot averaging per fit)" if not batch_mode else
                 ("per-step synchronous DP of every worker of the job inside the launch (gradient sum over "
                  "the replicas, then over the ranks, every step)" if xrank else
                  "per-step synchronous DP of the GPU's workers (gradient sum over the replicas every step)")
                 if sync_local else "per-step gradient all-reduce")
    engine = ((("native HIP executor: " if t.persistent else "native HIP executor + hipGraph: ") + t.plan_name())
              if gpu else "torch CPU reference")
    out = dict(t=t, R=R, rows=rows, samples=samples, dt_max=dt_max, state=state, digests=digests, devices=devices,
               path=path, nbytes=nbytes, batch_mode=batch_mode, sync=sync_desc, engine=engine,
               theta_equal=all(d == digests[0] for d in digests), W=W, xr_selftest=xr_selftest)
    return out


def bench_fit(args, model, dist, rank, world, dev):
    """End-to-end fit wall time through the public API -- the reference's measured unit.
    MNIST (default): SparkModel.fit as in examples/mnist_mlp_spark_synchronous.py:47-57
      (60,000 rows in local[8] partitions, 1 epoch, batch 64, validation_split 0.1).
    Otto (--model otto, BASELINE config #4): SparkMLlibModel.fit on an RDD of
      LabeledPoints (reference spark_model.py:311-341; model of examples/ml_pipeline_otto.py
      :57-68: 93-512-512-512-9, Dropout 0.5, batch 128, validation_split 0.15,
      categorical labels, 61,878 rows), 8 partitions, mode='synchronous'.
    RDD partitions -> workers -> native executor -> averaging. A "step" = one whole fit
    call; warmup fits absorb executor construction.
    strong: the reference job split over the GPUs; weak: that job on every GPU."""
    import torch
    from elephas_amd.data import SparkContext
    from elephas_amd.spark_model import SparkMLlibModel, SparkModel
    from elephas_amd.utils.rdd_utils import to_labeled_point, to_simple_rdd
    dims, _, classes, _, _ = MODELS[args.model]
    otto = args.model == "otto"
    base_rows = 61878 if otto else 60000
    parts = 8 if args.scaling == "strong" else 8 * world
    rows = base_rows if args.scaling == "strong" else base_rows * world
    rng = np.random.default_rng(2024)
    centers = rng.normal(0, 1, size=(classes, dims[0])).astype(np.float32)
    y = rng.integers(0, classes, rows)
    x = np.clip(centers[y] * 0.25 + 0.5 + rng.normal(0, 0.25, size=(rows, dims[0])), 0, 1).astype(np.float32)
    yo = np.eye(classes, dtype=np.float32)[y]
    sc = SparkContext(master=f"local[{parts}]")
    if otto:
        x = (x - x.mean(0)) / x.std(0)              # the pipeline's StandardScaler(withMean, withStd)
        data = to_labeled_point(sc, x, y.astype(np.float64))
        sm = SparkMLlibModel(model, mode="synchronous", num_workers=parts)
        vs = 0.15 if args.validation_split == 0.1 else args.validation_split
        kw = dict(epochs=1, batch_size=args.batch, verbose=0, validation_split=vs, categorical=True,
                  nb_classes=classes)
    else:
        data = to_simple_rdd(sc, x, yo)
        sm = SparkModel(model, mode="synchronous")
        kw = dict(epochs=1, batch_size=args.batch, verbose=0, validation_split=args.validation_split)

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.barrier()

    for _ in range(max(args.warmup, 0)):
        sm.fit(data, **kw)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sm.fit(data, **kw)
    sync()
    dt = time.perf_counter() - t0
    dt_max = max(dist.all_gather_object(dt))
    samples = sm.metrics["samples"] * args.steps
    if rank == 0:
        acc = sm.master_network.evaluate(x[:10000], yo[:10000])[1]
        line = {
            "metric": ("samples/sec (whole node) Otto-MLP 93-512-512-512-9 SparkMLlibModel.fit wall (end to end)"
                       if otto else "samples/sec (whole node) MNIST-MLP 784-128-128-10 SparkModel.fit wall (end to end)"),
            "value": round(samples / dt_max, 1), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt_max / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None,
            "dtype": "bf16" if args.policy == "mixed_bfloat16" else "fp32",
            "data": (f"synthetic {args.model.upper()}-shaped, learnable (class centers + noise)"
                     f"{', standardised, LabeledPoint RDD' if otto else ''}, random-init weights"),
            "config": {"model": "Otto-MLP 93-512-512-512-9" if otto else "MNIST-MLP 784-128-128-10",
                       "api": "SparkMLlibModel" if otto else "SparkModel", "rows": rows, "partitions": parts,
                       "epochs": 1, "batch": args.batch, "validation_split": kw["validation_split"],
                       "mode": "synchronous",
                       "seq_len": None, "global_batch": args.batch * parts, "parallelism": f"dp{world}",
                       "phases_ms_last_fit": {k: round(v * 1e3, 3) for k, v in sm.metrics["phases"].items()},
                       "optimizer": _optimizer_desc(args),
                       "train_accuracy_after": round(float(acc), 4)},
        }
        _finish_report(line, args.out)
    if dist.is_initialized():
        dist.barrier()
        import torch.distributed as tdist
        from elephas_amd.parallel import p2p
        p2p.shutdown()   # peer buffers freed only after every rank is done with them
        tdist.destroy_process_group()


def bench_infer(args, model, dist, rank, world, dev):
    """Distributed predict / evaluate of the master network, the SparkModel path
    (spark_model.py _predict / _evaluate): every rank runs its block of the rows through
    the native eval executor; predict gathers the rows with one tensor all-gather
    (RCCL), evaluate all-reduces the loss / metric sums. A "step" = one call over all
    rows; weak scaling (--infer-rows per GPU). Host -> device upload and the
    device -> host result copies are inside the timed region."""
    import torch
    dims, _, classes, _, _ = MODELS[args.model]
    per = args.infer_rows or (16384 if args.model == "wide" else 65536)
    n = per * world
    lo, hi = dist.block_range(n)
    rng = np.random.default_rng(77 + rank)
    x = rng.random((hi - lo, dims[0]), dtype=np.float32)
    y = np.eye(classes, dtype=np.float32)[rng.integers(0, classes, hi - lo)]
    bs = 2048

    def call():
        if args.task == "predict":
            out = dist.all_gather_rows(model.predict(x, batch_size=bs), n)
            assert out.shape == (n, classes)
        else:
            t = model._trainer(bs)
            s = torch.tensor(np.asarray(t.evaluate_sums(x, y), np.float64))
            dist.all_reduce_sum_(s)

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.barrier()

    for _ in range(max(args.warmup, 1)):
        call()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        call()
    sync()
    dt = time.perf_counter() - t0
    dt_max = max(dist.all_gather_object(dt))
    if rank == 0:
        names = NAMES
        line = {
            "metric": f"samples/sec (whole node) {names[args.model]} distributed {args.task}",
            "value": round(n * args.steps / dt_max, 1), "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if args.policy == "mixed_bfloat16" else "fp32",
            "data": "synthetic (uniform features, random labels), random-init weights",
            "config": {"model": names[args.model], "global_batch": n, "seq_len": None,
                       "parallelism": f"dp{world}", "rows_per_gpu": per, "eval_batch": bs,
                       "engine": "native HIP eval executor" if torch.cuda.is_available() else "torch CPU"},
        }
        _finish_report(line, args.out)
    if dist.is_initialized():
        dist.barrier()
        import torch.distributed as tdist
        from elephas_amd.parallel import p2p
        p2p.shutdown()   # peer buffers freed only after every rank is done with them
        tdist.destroy_process_group()


def bench_async(args, model, dist, rank, world, dev):
    """Async / hogwild DP through the sharded device parameter server (reference
    worker.py:102-127, frequency 'batch' or 'epoch'): the W workers of a GPU are split into G
    independently progressing groups (worker.BatchedAsynchronousWorker, one executor +
    HIP stream each); with frequency='batch' every group-step is ONE hipGraph replay of
    pull (gather theta from the shards, chunk-consistent in 'asynchronous') -> refresh ->
    train -> push (fp32 atomic adds into the owners' shards over xGMI); with 'epoch' the
    same pull / push bracket each epoch of graph-replayed training steps.  No host
    lock, no host sync."""
    import torch
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.plan import build_plan, flatten_weights
    from elephas_amd.parameter.client import DeviceClient
    from elephas_amd.worker import BatchedAsynchronousWorker, _Group, group_persist_cus, run_group_rounds
    dims, drop, classes, rows, _ = MODELS[args.model]
    W, B = args.workers_per_gpu, args.batch
    G = max(1, min(W, args.async_groups or W))
    init = flatten_weights(model.get_weights())
    client = DeviceClient().connect(len(init), args.mode)
    if rank == 0:
        src = torch.from_numpy(init).to(dev)
        client.ps.set(src.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    dist.barrier()
    plan = build_plan(model)
    rng = np.random.default_rng(1000 + rank)
    centers = rng.normal(0, 1, size=(classes, dims[0])).astype(np.float32)
    dx, dy = [], []
    for w in range(W):
        y = rng.integers(0, classes, rows)
        x = centers[y] + rng.normal(0, 2.0, size=(rows, dims[0])).astype(np.float32)
        dx.append(((x - x.min()) / (x.max() - x.min())).astype(np.float32))
        dy.append(np.eye(classes, dtype=np.float32)[y])
    bounds = [W * g // G for g in range(G + 1)]
    freq = args.frequency
    worker = BatchedAsynchronousWorker(None, None, client, {}, freq, None, None, None, None)
    groups = []
    for g in range(G):
        lo, hi = bounds[g], bounds[g + 1]
        t = NativeTrainer(model, plan, hi - lo, B, dev, seed=4321 + 97 * rank + g,
                          persist_cus=group_persist_cus(G, dev) if G > 1 else None, ps_hook=freq == "batch")
        t.set_data(dx[lo:hi], dy[lo:hi], args.validation_split, shuffle=True)
        t.begin_epoch()
        grp = _Group(t, [True] * (hi - lo))
        if freq == "batch":
            grp.attach(client)   # push / pull per step inside the persistent launch
        if not args.no_graph:
            if freq == "batch":
                grp.capture(worker)
            else:
                t.prepare_graphs()
        groups.append(grp)
    spe = groups[0].t.steps_per_epoch()
    state = {"pos": 0}

    def run(k):
        if freq == "epoch":
            # reference worker.py:102-113: pull, train the epoch, push the epoch's delta;
            # every call also starts with a pull and ends with a push, so the timed
            # region holds complete exchanges
            for grp in groups:
                worker._pull(grp)
        while k > 0:
            if state["pos"] >= spe:
                for grp in groups:
                    if freq == "epoch":
                        worker._push(grp)
                        worker._pull(grp)
                    grp.t.begin_epoch()
                state["pos"] = 0
            n = min(k, spe - state["pos"])
            if freq == "epoch":
                for grp in groups:        # every group enqueues n steps on its own stream
                    grp.t.run_steps(n, use_graph=not args.no_graph)
            else:
                run_group_rounds(groups, worker, n)
            state["pos"] += n
            k -= n
        if freq == "epoch":
            for grp in groups:
                worker._push(grp)

    def sync():
        for grp in groups:
            grp.t.stream.synchronize()
        torch.cuda.synchronize()
        dist.barrier()

    run(args.warmup)
    sync()
    t0 = time.perf_counter()
    run(args.steps)
    sync()
    dt = time.perf_counter() - t0
    client.check()
    dt_max = max(dist.all_gather_object(dt))
    if rank == 0:
        value = W * B * args.steps * world / dt_max
        line = {
            "metric": f"samples/sec (whole node) {args.model.upper()}-MLP {args.mode} DP (device parameter server)",
            "value": round(value, 1), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt_max / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if args.policy == "mixed_bfloat16" else "fp32",
            "data": "synthetic, random-init weights",
            "config": {"model": args.model, "global_batch": B * W * world, "seq_len": None,
                       "parallelism": f"{args.mode}-dp{world}", "workers_per_gpu": W, "batch_per_worker": B,
                       "frequency": freq, "groups_per_gpu": G,
                       "plan": groups[0].t.plan_name() if hasattr(groups[0].t, "plan_name") else None,
                       "ps": f"sharded over {world} GPU(s), 4096-parameter chunks, IPC-mapped",
                       "exchange": ("pull / push per epoch around hipGraph training chunks" if freq == "epoch"
                                    else "per step inside the persistent launch (push delta, pull theta; "
                                         "host pull per chunk)" if getattr(groups[0], "inlaunch", False)
                                    else "hipGraph per group-step (pull, refresh, train, push)" if groups[0].graph
                                    else "eager launches")},
        }
        _finish_report(line, args.out)
    dist.barrier()
    client.close()
    if dist.is_initialized():
        import torch.distributed as tdist
        from elephas_amd.parallel import p2p
        p2p.shutdown()   # peer buffers freed only after every rank is done with them
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
