"""One rank of the multi-process peer-memory GPU tests (tests/test_peer_gpu.py).

Started as a child process per rank; every rank uses cuda:0 (two processes sharing
one MI355X: HIP IPC maps the other process's buffers exactly as it maps another
GPU's), a gloo process group exchanges the IPC handles.  Prints one JSON line.
Usage: python tests/_peer_worker.py SCENARIO   (RANK / WORLD_SIZE / MASTER_* in env)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _gloo():
    import torch.distributed as dist
    from datetime import timedelta
    dist.init_process_group("gloo", timeout=timedelta(seconds=120))
    return dist


def _allgather(dist):
    def f(obj):
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, obj)
        return out
    return f


def allreduce(dist, rank, world):
    """Every algorithm and size class against the fp32 rank-order sum; outputs of all
    ranks must be bit-identical."""
    import torch
    from elephas_amd.parallel.p2p import PeerAllReduce
    ag = _allgather(dist)
    pa = PeerAllReduce(rank, world, 0, cap_elems=65536, allgather=ag)
    res = {"self_test": pa.ok, "cases": []}
    s = torch.cuda.Stream()
    for n in (1, 5, 1000, 4096, 65536, 118_282, 200_003):
        for algo in (0, 1, -1):
            xs = [torch.from_numpy(np.random.default_rng(1000 * r + n + algo).normal(size=n).astype(np.float32))
                  for r in range(world)]
            want = xs[0].clone()
            for r in range(1, world):
                want += xs[r]
            x = xs[rank].cuda()
            s.wait_stream(torch.cuda.current_stream())
            pa.all_reduce_(x, algo=algo, stream=s)
            s.synchronize()
            got = x.cpu()
            digests = ag(float(got.double().sum()))
            res["cases"].append(dict(n=n, algo=algo, exact=bool(torch.equal(got, want)),
                                     same_on_all_ranks=len(set(digests)) == 1))
    # misaligned view (goes through the aligned bounce buffer)
    base = torch.arange(1001, dtype=torch.float32, device="cuda") * (rank + 1)
    v = base[1:]
    pa.all_reduce_(v)
    torch.cuda.synchronize()
    res["misaligned_ok"] = bool(torch.equal(v.cpu(), torch.arange(1, 1001, dtype=torch.float32)
                                            * sum(r + 1 for r in range(world))))
    # peer barrier: a rank that arrives late holds every other rank in the barrier
    t0 = time.perf_counter()
    if rank == 1:
        time.sleep(0.3)
    pa.barrier()
    res["barrier_waited"] = time.perf_counter() - t0
    res["error"] = int(pa.impl.error())
    return res


def bench(dist, rank, world):
    """us per call of the peer all-reduce vs RCCL-less baseline (two processes on one
    GPU: the peer reads are local HBM reads, so this bounds the kernel's fixed cost,
    not the xGMI transfer time)."""
    import torch
    from elephas_amd.parallel.p2p import PeerAllReduce
    pa = PeerAllReduce(rank, world, 0, allgather=_allgather(dist))
    out = {}
    for nbytes in (473_128, 2_312_228, 16 << 20):
        n = nbytes // 4
        x = torch.ones(n, dtype=torch.float32, device="cuda")
        for algo in (0, 1):
            for _ in range(20):
                pa.all_reduce_(x, algo=algo)
            torch.cuda.synchronize()
            dist.barrier()
            iters = 200
            t0 = time.perf_counter()
            for _ in range(iters):
                pa.all_reduce_(x, algo=algo)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / iters
            out[f"{nbytes}B_{'two' if algo else 'one'}shot_us"] = round(dt * 1e6, 2)
            dist.barrier()
    out["error"] = int(pa.impl.error())
    return out


def ps(dist, rank, world):
    """Both ranks push concurrently into the sharded PS (each owns half the chunks):
    no update is lost and asynchronous pulls are chunk-consistent."""
    import torch
    from elephas_amd.ops import native
    from elephas_amd.parallel.p2p import exchange_handles
    C = native.require()
    n, K = 50_000, 40
    p = C.ShardedParameterServer(rank, world, n, 1, 0, 4096)
    p.open(exchange_handles(p.handle(), _allgather(dist)))
    if rank == 0:
        z = torch.zeros(n, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        p.set(z.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    dist.barrier()
    d = torch.full((n,), -float(rank + 1), dtype=torch.float32, device="cuda")
    snaps = torch.empty(K, n, dtype=torch.float32, device="cuda")
    sp, sq = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for k in range(K):
        p.push_delta(d.data_ptr(), sp.cuda_stream)
        p.pull(snaps[k].data_ptr(), sq.cuda_stream)
    torch.cuda.synchronize()
    dist.barrier()
    fin = torch.empty(n, dtype=torch.float32, device="cuda")
    p.pull(fin.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = float(K * sum(r + 1 for r in range(world)))
    torn = 0
    for c0 in range(0, n, 4096):
        blk = snaps[:, c0:c0 + 4096]
        torn += int((blk != blk[:, :1]).any(1).sum())
    res = dict(final_exact=bool(torch.equal(fin, torch.full_like(fin, want))), torn_chunks=torn,
               shard_begin=[int(p.shard_begin(r)) for r in range(world)], error=int(p.error()))
    dist.barrier()   # nobody frees its shard while a peer may still read it
    return res


def spark_async(dist, rank, world, mode):
    """SparkModel asynchronous / hogwild fit with two ranks sharing the GPU: sharded
    device PS across the two processes, two independent worker groups per rank.
    Learnable synthetic data: accuracy must rise well above chance on every rank and
    the final weights must be identical on both ranks."""
    import torch
    from elephas_amd import config
    from elephas_amd.data import SparkContext
    from elephas_amd.models import Sequential, Dense, Dropout
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.parallel import dist as edist
    from elephas_amd.spark_model import SparkModel
    from elephas_amd.utils.rdd_utils import to_simple_rdd
    config.set_policy("float32")
    rng = np.random.default_rng(5)
    centers = rng.normal(0, 1, size=(10, 64)).astype(np.float32)
    y = rng.integers(0, 10, 4000)
    x = (centers[y] + rng.normal(0, 0.7, size=(4000, 64))).astype(np.float32)
    yo = np.eye(10, dtype=np.float32)[y]
    np.random.seed(0)
    m = Sequential()
    m.add(Dense(64, activation="relu", input_dim=64))
    m.add(Dropout(0.1))
    m.add(Dense(10, activation="softmax"))
    m.compile(SGD(learning_rate=0.05), "categorical_crossentropy", ["acc"])
    acc0 = m.evaluate(x, yo)[1]
    sm = SparkModel(m, mode=mode, frequency="batch", parameter_server_mode="device", num_workers=4,
                    async_groups=2)
    sm.fit(to_simple_rdd(SparkContext.getOrCreate(), x, yo), epochs=2, batch_size=32, verbose=0,
           validation_split=0.0)
    w = np.concatenate([a.ravel() for a in sm.master_network.get_weights()])
    digests = _allgather(dist)(float(np.float64(w).sum()))
    acc = sm.master_network.evaluate(x, yo)[1]
    edist.barrier()
    return dict(acc0=float(acc0), acc=float(acc), finite=bool(np.isfinite(w).all()),
                same_on_all_ranks=len(set(digests)) == 1)


def ps_selftest(dist, rank, world):
    """DeviceClient.connect's collective self-test of the sharded PS, both consistency
    modes; with ELEPHAS_AMD_FAULT_INJECT=rank=1,phase=ps_selftest one rank pushes a
    wrong delta and every rank must raise."""
    from elephas_amd.parameter.client import DeviceClient
    out = {}
    for mode in ("asynchronous", "hogwild"):
        c = DeviceClient()
        try:
            c.connect(70_001, mode, allgather=_allgather(dist), chunk=4096)
            out[mode] = dict(raised=False, votes=c.self_test_result)
        except RuntimeError as e:
            out[mode] = dict(raised=True, msg=str(e)[:300])
        dist.barrier()   # nobody frees its shard while a peer may still read it
    return out


def spark_sync(dist, rank, world, gran):
    """SparkModel(mode='synchronous') at one sync granularity on the native engine with
    the peer all-reduce, then distributed predict / evaluate and ElephasTransformer
    .transform; everything is saved for the test to compare against a single-process
    run of the same scenario (no dropout, no shuffling: every partition's trajectory is
    deterministic, so the only difference is the fp32 summation order of averaging)."""
    import torch
    from elephas_amd import config
    from elephas_amd.data import SparkContext
    from elephas_amd.ml.adapter import to_data_frame
    from elephas_amd.ml_model import ElephasTransformer
    from elephas_amd.models import Sequential, Dense, initializers
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.spark_model import SparkModel
    from elephas_amd.utils.model_utils import ModelType
    from elephas_amd.utils.rdd_utils import to_simple_rdd
    from elephas_amd.parallel import p2p
    from elephas_amd import worker as worker_mod
    config.set_policy("float32")
    persist = gran.endswith("p")   # 'fitp' / 'epochp': a model the persistent plan takes
    gran = gran.rstrip("p")
    rng = np.random.default_rng(21)
    centers = rng.normal(0, 1, size=(5, 30)).astype(np.float32)
    y = rng.integers(0, 5, 1600)
    x = (centers[y] + rng.normal(0, 1.0, size=(1600, 30))).astype(np.float32)
    yo = np.eye(5, dtype=np.float32)[y]
    initializers.set_seed(8)
    if persist:
        m = Sequential([Dense(64, activation="relu", input_dim=30), Dense(64, activation="relu"),
                        Dense(5, activation="softmax")])
    else:
        m = Sequential([Dense(48, activation="relu", input_dim=30), Dense(5, activation="softmax")])
    m.compile(SGD(learning_rate=0.05, momentum=0.5), "categorical_crossentropy", ["acc"])
    sm = SparkModel(m, mode="synchronous", sync_granularity=gran, num_workers=4)
    sm.fit(to_simple_rdd(SparkContext(master="local[4]"), x, yo), epochs=2, batch_size=32, verbose=0,
           validation_split=0.0, shuffle=False)
    preds = np.stack(sm.predict(x[:333]))
    ev = np.asarray(sm.evaluate(x, yo, batch_size=64))
    tr = ElephasTransformer(weights=sm.master_network.get_weights(), model_type=ModelType.CLASSIFICATION)
    tr.set_keras_model_config(sm.master_network.to_json())
    tr.set_inference_batch_size(64)
    df = to_data_frame(SparkContext(master="local[4]"), x[:257], yo[:257], categorical=True)
    trans = np.asarray([r[tr.getOutputCol()] for r in tr.transform(df).collect()])
    w = [np.asarray(a) for a in sm.master_network.get_weights()]
    out_dir = os.environ["ELEPHAS_AMD_TEST_OUT"]
    tag = gran + ("p" if persist else "")
    np.savez(os.path.join(out_dir, f"{tag}_w{world}_r{rank}.npz"), *w, preds=preds, ev=ev, trans=trans)
    entry = worker_mod._trainer_cache._entry
    persistent = bool(entry is not None and getattr(entry[0], "persistent", False))
    peer = p2p.current()
    digests = _allgather(dist)(float(np.float64(np.concatenate([a.ravel() for a in w])).sum()))
    return dict(peer_path=peer is not None, same_on_all_ranks=len(set(digests)) == 1,
                histories=len(sm.training_histories), native=bool(sm._native_ok()), persistent=persistent,
                gpu=bool(torch.cuda.is_available()))


def step_graph(dist, rank, world):
    """Per-step gradient all-reduce captured in the training step's hipGraph (peer
    kernels, device-side epochs) vs the eager path with a gloo all-reduce of the same
    gradients: bit-identical weights after 40 steps (a 2-term fp32 sum is exact in
    either order), identical on both ranks."""
    import torch
    from elephas_amd import config
    from elephas_amd.models import Sequential, Dense
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.parallel.p2p import PeerAllReduce
    from elephas_amd.models import initializers
    config.set_policy("float32")
    initializers.set_seed(3)   # the same initial weights on every rank
    m = Sequential()
    m.add(Dense(48, activation="relu", input_dim=40))
    m.add(Dense(6, activation="softmax"))
    m.compile(SGD(learning_rate=0.1, momentum=0.9), "categorical_crossentropy", ["acc"])
    rng = np.random.default_rng(10 + rank)
    x = rng.normal(size=(640, 40)).astype(np.float32)
    y = np.eye(6, dtype=np.float32)[rng.integers(0, 6, 640)]
    ag = _allgather(dist)
    ts = []
    for _ in range(2):
        t = NativeTrainer(m, build_plan(m), 1, 32, torch.device("cuda"), seed=99)
        t.set_grad_scale(1.0 / world)
        t.set_data([x], [y], 0.0, shuffle=False)
        t.begin_epoch()
        ts.append(t)
    ch = PeerAllReduce(rank, world, 0, cap_elems=ts[0].G.numel(), allgather=ag, verify=False)
    ts[0].run_steps_allreduce_graph(17, ch)          # one 16-step graph + one 1-step graph
    ts[0].run_steps_allreduce_graph(3, ch)

    def gloo_sum(G):
        h = G.detach().cpu()
        dist.all_reduce(h)
        G.copy_(h.to(G.device))
    ts[1].run_steps_allreduce(20, gloo_sum)
    w0, w1 = ts[0].get_weights_flat(), ts[1].get_weights_flat()
    digests = ag(float(np.float64(w0).sum()))
    from elephas_amd.ops.plan import flatten_weights
    init = flatten_weights(m.get_weights())
    return dict(bit_equal=bool(np.array_equal(w0, w1)), max_diff=float(np.abs(w0 - w1).max()),
                moved=float(np.abs(w0 - init).max()), same_on_all_ranks=len(set(digests)) == 1,
                error=int(ch.impl.error()))


def _sync_model(deep, seed):
    """The scenarios' model: the MNIST MLP (persist.hip V1 roles), or with deep=True an
    Otto-like 93-256-256-9 stack on the layer pipeline (tanh: no ReLU kink turns fp32
    summation noise into a different gradient between the two summation orders compared)."""
    from elephas_amd.models import Sequential, Dense, initializers
    from elephas_amd.models.optimizers import SGD
    initializers.set_seed(seed)   # the same initial weights on every rank
    m = Sequential()
    if deep:
        m.add(Dense(256, activation="tanh", input_dim=93))
        m.add(Dense(256, activation="tanh"))
        m.add(Dense(9, activation="softmax"))
        m.compile(SGD(0.05), "categorical_crossentropy", ["acc"])
        return m, 93, 9
    m.add(Dense(128, activation="relu", input_dim=784))
    m.add(Dense(128, activation="relu"))
    m.add(Dense(10, activation="softmax"))
    m.compile(SGD(0.1), "categorical_crossentropy", ["acc"])
    return m, 784, 10


def sync_inlaunch(dist, rank, world, deep=False):
    """Per-step synchronous DP across ranks inside the persistent launch: two ranks x
    two replicas (each rank's grid on half the CUs), the weight-gradient tiles summed
    over the replicas and then over the ranks by the owning workgroups.  Every replica
    of every rank ends bit-identical, and equal (to fp32 summation order) to ONE torch
    model trained on the four workers' batches stacked in rank-major order."""
    import hashlib
    import torch
    from elephas_amd import config
    from elephas_amd.models import Sequential, Dense, initializers
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.torch_engine import TorchTrainer
    config.set_policy("float32")
    m, d, k = _sync_model(deep, 21)
    R, B, steps = 2, 64, 9
    rng = np.random.default_rng(77)   # every rank builds every worker's shard
    xs_all = [rng.random((B * steps, d), dtype=np.float32) for _ in range(world * R)]
    ys_all = [np.eye(k, dtype=np.float32)[rng.integers(0, k, B * steps)] for _ in range(world * R)]
    xs, ys = xs_all[rank * R:(rank + 1) * R], ys_all[rank * R:(rank + 1) * R]
    ag = _allgather(dist)
    t = NativeTrainer(m, build_plan(m), R, B, torch.device("cuda"), seed=5, sync=True, persist_cus=128)
    w0 = t.get_weights_flat()[0].copy()
    t.set_data(xs, ys, 0.0, shuffle=False)
    attached = t.attach_rank_exchange(rank, world, allgather=ag)
    if not attached:
        return dict(attached=False, plan=t.plan_name())
    t.GRAPH_CHUNK = 4   # several launches: the exchange tags continue across them
    t.fit(2)
    w = t.get_weights_flat()
    replicas_equal = all(np.array_equal(w[r], w[0]) for r in range(R))
    dig = hashlib.sha1(w[0].tobytes()).hexdigest()[:16]
    digs = ag(dig)
    xc = np.concatenate([np.concatenate([x[i * B:(i + 1) * B] for x in xs_all]) for i in range(steps)])
    yc = np.concatenate([np.concatenate([y[i * B:(i + 1) * B] for y in ys_all]) for i in range(steps)])
    ref = TorchTrainer(m, build_plan(m), 1, world * R * B, torch.device("cuda"))
    ref.set_data([xc], [yc], 0.0, shuffle=False)
    ref.fit(2)
    wt = ref.get_weights_flat()[0]
    err = float(np.abs(w[0] - wt).max() / np.abs(wt - w0).max())
    return dict(attached=True, plan=t.plan_name(), replicas_equal=replicas_equal,
                same_on_all_ranks=len(set(digs)) == 1, err=err, error=int(t.exe.persist_error()),
                steps_tagged=int(t.exe.rank_exchange_steps()))


def xrank_selftest(dist, rank, world, deep=False):
    """The voted numeric self-test of the in-launch rank exchange (NativeTrainer
    .attach_rank_exchange): without a fault every rank attaches and trains inside the
    launch; with ELEPHAS_AMD_FAULT_INJECT=rank=1,phase=xrank_selftest rank 1 sends a wrong
    tile, every rank detaches, and the per-step all-reduce path it falls back to (one
    replica of the rank's stacked batches, gradient sum over the ranks) still trains to
    the same weights as ONE torch model on every worker's batches."""
    import hashlib
    import torch
    from elephas_amd import config
    from elephas_amd.models import Sequential, Dense, initializers
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.torch_engine import TorchTrainer
    config.set_policy("float32")
    m, d, k = _sync_model(deep, 23)
    R, B, steps = 2, 64, 6
    rng = np.random.default_rng(78)
    xs_all = [rng.random((B * steps, d), dtype=np.float32) for _ in range(world * R)]
    ys_all = [np.eye(k, dtype=np.float32)[rng.integers(0, k, B * steps)] for _ in range(world * R)]
    xs, ys = xs_all[rank * R:(rank + 1) * R], ys_all[rank * R:(rank + 1) * R]
    ag = _allgather(dist)
    t = NativeTrainer(m, build_plan(m), R, B, torch.device("cuda"), seed=5, sync=True, persist_cus=128)
    w0 = t.get_weights_flat()[0].copy()
    t.set_data(xs, ys, 0.0, shuffle=False)
    attached = bool(t.attach_rank_exchange(rank, world, allgather=ag))
    selftest = getattr(t, "xr_selftest", None)
    if attached:
        t.fit(2)
        w = t.get_weights_flat()[0]
    else:
        # the fallback: one replica of the rank's R stacked batches, gradients summed over
        # the ranks every step (gloo here; the peer all-reduce / RCCL in the bench)
        xr = np.concatenate([np.concatenate([x[i * B:(i + 1) * B] for x in xs]) for i in range(steps)])
        yr = np.concatenate([np.concatenate([y[i * B:(i + 1) * B] for y in ys]) for i in range(steps)])
        f = NativeTrainer(m, build_plan(m), 1, R * B, torch.device("cuda"), seed=5)
        f.set_grad_scale(1.0 / world)
        f.set_data([xr], [yr], 0.0, shuffle=False)

        def gloo_sum(G):
            h = G.detach().cpu()
            dist.all_reduce(h)
            G.copy_(h.to(G.device))
        for _ in range(2):
            f.begin_epoch()
            f.run_steps_allreduce(steps, gloo_sum)
        w = f.get_weights_flat()[0]
    digs = ag(hashlib.sha1(np.ascontiguousarray(w).tobytes()).hexdigest()[:16])
    xc = np.concatenate([np.concatenate([x[i * B:(i + 1) * B] for x in xs_all]) for i in range(steps)])
    yc = np.concatenate([np.concatenate([y[i * B:(i + 1) * B] for y in ys_all]) for i in range(steps)])
    ref = TorchTrainer(m, build_plan(m), 1, world * R * B, torch.device("cuda"))
    ref.set_data([xc], [yc], 0.0, shuffle=False)
    ref.fit(2)
    wt = ref.get_weights_flat()[0]
    err = float(np.abs(w - wt).max() / np.abs(wt - w0).max())
    return dict(attached=attached, selftest=selftest, same_on_all_ranks=len(set(digs)) == 1, err=err)


def main():
    scenario = sys.argv[1]
    dist = _gloo()
    rank, world = dist.get_rank(), dist.get_world_size()
    import torch
    torch.cuda.set_device(0)
    if scenario == "allreduce":
        res = allreduce(dist, rank, world)
    elif scenario == "bench":
        res = bench(dist, rank, world)
    elif scenario == "step_graph":
        res = step_graph(dist, rank, world)
    elif scenario == "ps":
        res = ps(dist, rank, world)
    elif scenario == "ps_selftest":
        res = ps_selftest(dist, rank, world)
    elif scenario == "xrank_selftest_deep":
        res = xrank_selftest(dist, rank, world, deep=True)
    elif scenario == "sync_inlaunch_deep":
        res = sync_inlaunch(dist, rank, world, deep=True)
    elif scenario == "xrank_selftest":
        res = xrank_selftest(dist, rank, world)
    elif scenario == "sync_inlaunch":
        res = sync_inlaunch(dist, rank, world)
    elif scenario.startswith("spark_sync_"):  # spark_sync_<fit|epoch|batch>[p]
        res = spark_sync(dist, rank, world, scenario.rsplit("_", 1)[1])
    elif scenario in ("spark_asynchronous", "spark_hogwild"):
        res = spark_async(dist, rank, world, scenario.split("_", 1)[1])
    else:
        raise SystemExit(f"unknown scenario {scenario}")
    print("RESULT " + json.dumps(dict(rank=rank, **res)), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
