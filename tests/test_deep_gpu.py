"""Persistent layer-pipeline kernel (csrc/kernels/deep_impl.h) against the fp32 torch
engine with the same dropout masks and against the multi-launch plans (GPU only).

The kernel runs a whole chunk of steps of a deeper / wider Dense stack in one launch:
every hidden layer's 16-column tiles are owned by the replica's workgroups, which hand
activations, gradients and transposed weight images to each other through flag barriers.
A stale read (a phase that did not wait for its producers, a weight image not rewritten
after an update) shows up as a weight gap far above fp32 rounding; padded widths (not a
multiple of 16), partial batches, replicas that run out of data early and launch
boundaries must behave as in the other plans.  Reference shapes: Otto 93-512-512-512-9
(examples/ml_pipeline_otto.py:57-68), Boston 13-64-64-1 (tests/conftest.py:22-28).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _mlp(in_dim, hidden, out, act="relu", out_act="softmax", dropout=0.0, bias=True):
    from elephas_amd.models import Sequential, Dense, Dropout, Activation
    m = Sequential()
    m.add(Dense(hidden[0], input_dim=in_dim, use_bias=bias))
    m.add(Activation(act))
    if dropout:
        m.add(Dropout(dropout))
    for h in hidden[1:]:
        m.add(Dense(h, activation=act, use_bias=bias))
        if dropout:
            m.add(Dropout(dropout))
    m.add(Dense(out, activation=out_act))
    return m


def _shards(sizes, d, k, seed=0, regression=False):
    rng = np.random.default_rng(seed)
    xs, ys = [], []
    for n in sizes:
        xs.append(rng.random((n, d), dtype=np.float32))
        if regression:
            ys.append(rng.normal(size=(n, k)).astype(np.float32))
        else:
            ys.append(np.eye(k, dtype=np.float32)[rng.integers(0, k, n)])
    return xs, ys


def _native(model, R, B, seed=12345, deep="2", persist=1, monkeypatch=None):
    from elephas_amd import config
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy("float32")
    if monkeypatch is not None:
        monkeypatch.setenv("ELEPHAS_AMD_DEEP", deep)
    return NativeTrainer(model, build_plan(model), R, B, torch.device("cuda"), seed=seed, persist=persist)


@pytest.mark.parametrize("name,in_dim,hidden,out,B,opt,drop,bias", [
    ("l3_sgd", 40, (64, 48), 6, 32, "sgd", 0.3, True),
    ("l3_mom", 40, (64, 48), 6, 32, "sgd_mom", 0.3, True),
    ("l3_adam", 40, (64, 48), 6, 32, "adam", 0.3, True),
    ("l2_pad", 20, (100,), 7, 24, "sgd", 0.2, True),
    ("l4_nobias", 30, (96, 80, 64), 5, 48, "sgd", 0.25, False),
    ("l5", 30, (64, 64, 64, 64), 5, 16, "sgd_mom", 0.0, True),
    ("wide_b128", 93, (256, 256), 9, 128, "sgd", 0.5, True),
    # B <= 32 with an inner hidden layer wider than 64: bw_phase's second DW-partial buffer
    # (the dZ_0^T stripe) must hold [4][64][4] floats, more than 16 x (Bp + 4) at Bp <= 32
    ("b32_wide", 93, (256, 256), 9, 32, "sgd", 0.5, True),
    ("b16_wide", 40, (128, 200), 7, 16, "sgd_mom", 0.2, True),
    ("otto_b32_adam", 93, (512, 512, 512), 9, 32, "adam", 0.5, True),
])
def test_deep_matches_fp32_reference_with_same_masks(monkeypatch, name, in_dim, hidden, out, B, opt, drop, bias):
    """Layer pipeline == fp32 torch autograd with the same dropout masks (2 replicas of
    unequal shard sizes, partial last batches, 2 epochs, every hand-off of every step):
    2..5 layers, widths that are not multiples of 16, biases off, SGD / Nesterov / Adam."""
    from elephas_amd.models import initializers, optimizers as O
    initializers.set_seed(31)
    model = _mlp(in_dim, list(hidden), out, dropout=drop, bias=bias)
    optim = {"sgd": O.SGD(0.2), "sgd_mom": O.SGD(0.05, momentum=0.9, nesterov=True), "adam": O.Adam(0.003)}[opt]
    model.compile(optim, "categorical_crossentropy", ["acc"])
    xs, ys = _shards([3 * B, 2 * B + B // 2], in_dim, out, seed=3)
    nat = _native(model, 2, B, monkeypatch=monkeypatch)
    assert nat.persistent and nat.persist_variant == 3, nat.plan_name()
    _compare_with_torch(nat, model, xs, ys, B, adaptive=opt == "adam")


def _compare_with_torch(nat, model, xs, ys, B, adaptive=False, epochs=2):
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.torch_engine import TorchTrainer
    ref = TorchTrainer(model, build_plan(model), len(xs), B, torch.device("cuda"), hash_dropout_seed=12345)
    w0 = nat.get_weights_flat()[0].copy()
    for t in (nat, ref):
        t.set_data(xs, ys, 0.0, shuffle=False)
    hn = nat.fit(epochs)
    hr = ref.fit(epochs)
    nat.check()
    wn, wr = nat.get_weights_flat(), ref.get_weights_flat()
    if adaptive:   # adaptive rule: near-zero gradients amplify fp32 rounding
        err = np.abs(wn - wr).mean() / np.abs(wr - w0).mean()
        assert err < 1e-3, (err, nat.plan_name())
    else:
        err = np.abs(wn - wr).max() / np.abs(wr - w0).max()
        assert err < 1e-4, (err, nat.plan_name())
    for a, b in zip(hn, hr):
        np.testing.assert_allclose(a["loss"], b["loss"], rtol=1e-4)
        np.testing.assert_allclose(a["acc"], b["acc"], atol=1e-6)


@pytest.mark.parametrize("hidden,B,opt", [
    ((256, 128), 64, "sgd"), ((256, 128), 128, "sgd_mom"),
    ((128,), 64, "sgd"), ((128,), 128, "adam"),
    ((128, 128, 128), 64, "sgd_mom"), ((128, 128, 128), 128, "sgd"),
    ((128, 128), 128, "sgd_mom"),
])
def test_mnist_family_shapes_stay_persistent(monkeypatch, hidden, B, opt):
    """The persistent plans' shape coverage at the default planning (no override): MNIST-
    family widths other than the headline's, B 64 and 128, momentum and Adam -- 8 replicas
    as in the reference's local[8] job -- all run one launch per chunk of steps and train
    as fp32 torch with the same masks."""
    from elephas_amd.models import initializers, optimizers as O
    initializers.set_seed(17)
    model = _mlp(784, list(hidden), 10, dropout=0.2)
    optim = {"sgd": O.SGD(0.1), "sgd_mom": O.SGD(0.05, momentum=0.9), "adam": O.Adam(0.001)}[opt]
    model.compile(optim, "categorical_crossentropy", ["acc"])
    xs, ys = _shards([2 * B] * 7 + [B + B // 3], 784, 10, seed=8)
    nat = _native(model, 8, B, deep="-1", monkeypatch=monkeypatch)
    assert nat.persistent, (nat.plan_name(), nat.plan_reason)
    _compare_with_torch(nat, model, xs, ys, B, adaptive=opt == "adam", epochs=1)


def test_deep_regression_generic_loss(monkeypatch):
    """The generic loss tile (mse, linear output, mae metric) on the Boston shape
    13-64-64-1 at B = 128 (past persist.hip's B <= 64), SGD with momentum (a state plane)."""
    from elephas_amd.models import initializers
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.torch_engine import TorchTrainer
    initializers.set_seed(5)
    model = _mlp(13, [64, 64], 1, out_act="linear")
    model.compile(SGD(0.01, momentum=0.9), "mse", ["mae"])
    xs, ys = _shards([300, 277, 128, 60], 13, 1, seed=4, regression=True)
    nat = _native(model, 4, 128, deep="-1", monkeypatch=monkeypatch)
    assert nat.persistent and nat.persist_variant == 3, nat.plan_name()
    ref = TorchTrainer(model, build_plan(model), 4, 128, torch.device("cuda"))
    w0 = nat.get_weights_flat()[0].copy()
    for t in (nat, ref):
        t.set_data(xs, ys, 0.0, shuffle=False)
    hn, hr = nat.fit(3), ref.fit(3)
    nat.check()
    wn, wr = nat.get_weights_flat(), ref.get_weights_flat()
    err = np.abs(wn - wr).max() / np.abs(wr - w0).max()
    assert err < 1e-4, err
    for a, b in zip(hn, hr):
        np.testing.assert_allclose(a["loss"], b["loss"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(a["mae"], b["mae"], rtol=1e-4, atol=1e-6)


def test_deep_otto_shape_matches_tail_chain_plan(monkeypatch):
    """The Otto shape of BASELINE config #4 (93-512-512-512-9, dropout 0.5, 8 replicas x
    B 128) on the layer pipeline, with shuffling, a validation split and a short last
    shard: the same training as the tail-chain plan within fp32 summation order, and the
    weight images rebuilt after the launch serve evaluation."""
    from elephas_amd.models import initializers
    from elephas_amd.models.optimizers import SGD
    initializers.set_seed(2024)
    model = _mlp(93, [512, 512, 512], 9, dropout=0.5)
    model.compile(SGD(learning_rate=0.01), "categorical_crossentropy", ["acc"])
    xs, ys = _shards([1000] * 7 + [450], 93, 9, seed=11)
    out = []
    for persist in (-1, 0):
        monkeypatch.setenv("ELEPHAS_AMD_DEEP", "-1")
        t = _native(model, 8, 128, seed=7, persist=persist)
        assert t.persistent == (persist != 0), t.plan_name()
        if persist:
            assert t.persist_variant == 3, t.plan_name()
            nw, grid, rt, ks, lds = t.exe.deep_geometry()[:5]
            assert nw == 32 and grid <= torch.cuda.get_device_properties(0).multi_processor_count
        t.set_data(xs, ys, 0.15, shuffle=True)
        torch.manual_seed(5)   # epoch shuffles draw from the global CUDA generator
        h = t.fit(2)
        t.check()
        out.append((t.get_weights_flat(), h, t.evaluate(xs[0], ys[0])))
    (wp, hp, ep), (wr, hr, er) = out
    scale = np.abs(wr).max()
    assert np.abs(wp - wr).max() <= 1e-4 * scale, (np.abs(wp - wr).max(), scale)
    for a, b in zip(hp, hr):
        for key in a:
            np.testing.assert_allclose(a[key], b[key], rtol=5e-4, atol=5e-4)
    np.testing.assert_allclose(ep, er, rtol=1e-4, atol=1e-5)


def test_deep_chunking_is_bit_exact(monkeypatch):
    """37 steps in persistent launches of 16 + 16 + 5 steps == 37 one-step launches, bit
    for bit (every launch re-reads the masters it wrote back, the images are rebuilt from
    them, the optimizer state lives in S)."""
    from elephas_amd.models import initializers
    from elephas_amd.models.optimizers import SGD
    initializers.set_seed(9)
    model = _mlp(93, [256, 128, 64], 9, dropout=0.5)
    model.compile(SGD(0.05, momentum=0.5), "categorical_crossentropy", ["acc"])
    xs, ys = _shards([64 * 40] * 2, 93, 9, seed=2)
    ws = []
    for chunk in (16, 1):
        t = _native(model, 2, 64, seed=99, deep="-1", monkeypatch=monkeypatch)
        assert t.persist_variant == 3, t.plan_name()
        t.set_data(xs, ys, 0.0, shuffle=False)
        t.GRAPH_CHUNK = chunk
        t.begin_epoch()
        t.run_steps(37)
        t.check()
        ws.append((t.get_weights_flat(), t.get_state_flat()[0]))
    assert np.array_equal(ws[0][0], ws[1][0])
    assert np.array_equal(ws[0][1], ws[1][1])


def test_deep_oversubscribed_grid_falls_back(monkeypatch):
    """A layer-pipeline grid that cannot be resident (the CU count overridden upwards): the
    GO-flag wait gives up before touching any state, fit() re-plans onto the multi-launch
    plan and re-runs from its snapshot -- the same result as that plan."""
    from elephas_amd.models import initializers
    from elephas_amd.models.optimizers import SGD
    initializers.set_seed(4)
    model = _mlp(93, [512, 512], 9, dropout=0.5)
    model.compile(SGD(0.01), "categorical_crossentropy", ["acc"])
    xs, ys = _shards([512] * 8, 93, 9, seed=6)
    monkeypatch.setenv("ELEPHAS_AMD_PERSIST_TIMEOUT_MS", "200")
    monkeypatch.setenv("ELEPHAS_AMD_PERSIST_OVERSUBSCRIBE", "4096")
    monkeypatch.setenv("ELEPHAS_AMD_DEEP", "-1")
    t = _native(model, 16, 128, seed=21)
    assert t.persist_variant == 3 and t.exe.deep_geometry()[1] > torch.cuda.get_device_properties(0).multi_processor_count
    xs16, ys16 = xs + xs, ys + ys
    t.set_data(xs16, ys16, 0.0, shuffle=False)
    h = t.fit(1)
    assert not t.persistent, t.plan_name()
    monkeypatch.delenv("ELEPHAS_AMD_PERSIST_OVERSUBSCRIBE")
    ref = _native(model, 16, 128, seed=21, persist=0)
    ref.set_data(xs16, ys16, 0.0, shuffle=False)
    hr = ref.fit(1)
    assert np.array_equal(t.get_weights_flat(), ref.get_weights_flat())
    for a, b in zip(h, hr):
        np.testing.assert_allclose(a["loss"], b["loss"], rtol=1e-6)


@pytest.mark.parametrize("name,in_dim,hidden,out,B,opt", [
    ("otto_like", 93, (256, 256, 128), 9, 128, "sgd"),
    ("mnist_mom", 784, (128, 128), 10, 64, "sgd_mom"),
    ("l2_adam", 40, (100,), 7, 32, "adam"),
])
def test_deep_sync_replicas_match_eager_exchange(monkeypatch, name, in_dim, hidden, out, B, opt):
    """Per-step synchronous DP on the layer pipeline (every workgroup's weight-gradient tile
    summed over the replicas inside the launch -- reduce-scatter in replica order, then
    every replica applies the same sums): the replicas stay bit-identical, and both it and
    the eager per-step path (forward / backward, replica sum of G, apply) equal ONE fp32
    torch model trained on the replicas' batches stacked (no dropout: no masks to match)."""
    from elephas_amd.models import initializers, optimizers as O
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.torch_engine import TorchTrainer
    from elephas_amd import config
    config.set_policy("float32")
    initializers.set_seed(12)
    # tanh: a ReLU kink turns a pre-activation within fp32 summation noise of 0 (one in the
    # otto_like data: |z| < 1e-6, unit 94 of layer 1 -- tools/grad_diag.py) into a different
    # gradient, whichever two summation orders are compared; the exchange is what is tested
    model = _mlp(in_dim, list(hidden), out, act="tanh")
    optim = {"sgd": O.SGD(0.05), "sgd_mom": O.SGD(0.05, momentum=0.9), "adam": O.Adam(0.002)}[opt]
    model.compile(optim, "categorical_crossentropy", ["acc"])
    R, steps = 4, 5
    xs, ys = _shards([B * steps] * R, in_dim, out, seed=13)
    monkeypatch.setenv("ELEPHAS_AMD_DEEP", "2")
    out_w = []
    for persist in (1, 0):
        t = NativeTrainer(model, build_plan(model), R, B, torch.device("cuda"), seed=5, persist=persist, sync=True)
        assert t.persistent == bool(persist)
        if persist:
            assert t.persist_variant == 3 and t.exe.persist_variant()[2] == 1, t.plan_name()
        w0 = t.get_weights_flat()[0].copy()
        t.set_data(xs, ys, 0.0, shuffle=False)
        t.fit(2)
        t.check()
        out_w.append(t.get_weights_flat())
    xc = np.concatenate([np.concatenate([x[i * B:(i + 1) * B] for x in xs]) for i in range(steps)])
    yc = np.concatenate([np.concatenate([y[i * B:(i + 1) * B] for y in ys]) for i in range(steps)])
    ref = TorchTrainer(model, build_plan(model), 1, R * B, torch.device("cuda"))
    ref.set_data([xc], [yc], 0.0, shuffle=False)
    ref.fit(2)
    wt = ref.get_weights_flat()[0]
    for label, w in zip(("in-launch", "eager"), out_w):
        for r in range(1, R):
            assert np.array_equal(w[r], w[0]), (label, r)
        if opt == "adam":
            err = np.abs(w[0] - wt).mean() / np.abs(wt - w0).mean()
            assert err < 1e-3, (label, err)
        else:
            err = np.abs(w[0] - wt).max() / np.abs(wt - w0).max()
            assert err < 1e-3, (label, err)


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_deep_exact_otto_matches_fp32_torch(monkeypatch, opt):
    """The exact Otto configuration of the reference notebook on the layer pipeline
    (93-512-512-512-9, ReLU, Dropout 0.5, 8 replicas x B 128; SGD(0.01) as bench.py's default
    and Adam(lr 0.01) as examples/Spark_ML_Pipeline.ipynb:361) == fp32 torch autograd with the
    same dropout masks, over 2 epochs with a short last shard."""
    from elephas_amd.models import initializers, optimizers as O
    initializers.set_seed(77)
    model = _mlp(93, [512, 512, 512], 9, dropout=0.5)
    model.compile(O.SGD(0.01) if opt == "sgd" else O.Adam(0.01), "categorical_crossentropy", ["acc"])
    xs, ys = _shards([2 * 128] * 7 + [128 + 50], 93, 9, seed=21)
    nat = _native(model, 8, 128, deep="-1", monkeypatch=monkeypatch)
    assert nat.persistent and nat.persist_variant == 3, (nat.plan_name(), nat.plan_reason)
    _compare_with_torch(nat, model, xs, ys, 128, adaptive=opt == "adam")


@pytest.mark.parametrize("mode", ["asynchronous", "hogwild"])
def test_deep_async_inlaunch_single_worker_equals_plain_training(mode):
    """The layer pipeline's in-launch parameter-server hook (frequency='batch', reference
    worker.py:114-127): every step each workgroup pushes theta_new - theta_old of the tiles it
    owns and pulls them back for the next step.  With ONE worker the server always returns
    that worker's own weights, so the run equals plain layer-pipeline training on the same
    batches, across launch boundaries (chunks of 8 steps) -- Otto-like shape, dropout."""
    from elephas_amd.models import initializers
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.plan import build_plan, flatten_weights
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.parameter.client import DeviceClient
    from elephas_amd.worker import BatchedAsynchronousWorker, _Group
    from elephas_amd import config
    config.set_policy("float32")
    initializers.set_seed(43)
    model = _mlp(93, [256, 256, 128], 9, dropout=0.3)
    model.compile(SGD(0.05), "categorical_crossentropy", ["acc"])
    xs, ys = _shards([128 * 20], 93, 9, seed=18)
    init = flatten_weights(model.get_weights())
    client = DeviceClient().connect(len(init), mode, rank=0, world=1, allgather=lambda h: [h])
    th = torch.from_numpy(init).cuda()
    torch.cuda.synchronize()
    client.ps.set(th.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    t = NativeTrainer(model, build_plan(model), 1, 128, torch.device("cuda"), seed=3, ps_hook=True)
    assert t.persistent and t.persist_variant == 3, t.plan_name()
    t.set_data(xs, ys, 0.0, shuffle=False)
    t.GRAPH_CHUNK = 8
    grp = _Group(t, [True])
    grp.attach(client)
    assert grp.inlaunch, "the layer pipeline must take the in-launch PS hook"
    worker = BatchedAsynchronousWorker(None, None, client, {}, "batch", None, None, None, None)
    t.begin_epoch()
    grp.steps(worker, 19)
    torch.cuda.synchronize()
    t.check()
    got = torch.empty(len(init), dtype=torch.float32, device="cuda")
    client.ps.pull(got.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert client.ps.error() == 0
    ref = NativeTrainer(model, build_plan(model), 1, 128, torch.device("cuda"), seed=3, persist=1)
    assert ref.persist_variant == 3
    ref.set_data(xs, ys, 0.0, shuffle=False)
    ref.begin_epoch()
    ref.run_steps(19)
    wr = ref.get_weights_flat()[0]
    step = np.abs(wr - init).max()
    err = np.abs(got.cpu().numpy() - wr).max()
    assert err <= 1e-5 * step + 1e-7, (err, step)


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_deep_xcd_local_instance_is_bit_exact(monkeypatch, opt):
    """The layer pipeline's XCD-local instance (deep_l*_local.hip: a replica's hand-offs
    stored plain and read from its XCD's L2, placement checked at launch) is picked for the
    Otto job's 8 replicas and trains bit for bit as the write-through instance."""
    from elephas_amd.models import initializers, optimizers as O
    initializers.set_seed(52)
    model = _mlp(93, [512, 512, 512], 9, dropout=0.5)
    model.compile(O.SGD(0.01) if opt == "sgd" else O.Adam(0.01), "categorical_crossentropy", ["acc"])
    xs, ys = _shards([128 * 3] * 7 + [128 + 40], 93, 9, seed=23)
    out = []
    for local in ("-1", "0"):
        monkeypatch.setenv("ELEPHAS_AMD_PERSIST_LOCAL", local)
        t = _native(model, 8, 128, deep="-1", monkeypatch=monkeypatch)
        var = t.exe.persist_variant()
        assert t.persistent and var[0] == 3 and var[3] == (1 if local == "-1" else 0), (local, var, t.plan_name())
        t.set_data(xs, ys, 0.15, shuffle=True)
        torch.manual_seed(2)
        h = t.fit(2)
        t.check()
        out.append((t.get_weights_flat(), h))
    (wl, hl), (wg, hg) = out
    assert np.array_equal(wl, wg), np.abs(wl - wg).max()
    for a, b in zip(hl, hg):
        for key in a:
            np.testing.assert_array_equal(a[key], b[key])


def test_deep_post_node_average_equals_separate_kernel(monkeypatch):
    """The layer pipeline's fit-granularity chunk with the replica averaging in its post node
    (run_steps_and_average, default mode) == run_steps + the replica_average kernel, bit for
    bit, over a chunk boundary; the mean is in every replica afterwards."""
    from elephas_amd.models import initializers
    from elephas_amd.models.optimizers import SGD
    initializers.set_seed(19)
    model = _mlp(93, [256, 256], 9, dropout=0.5)
    model.compile(SGD(0.05), "categorical_crossentropy", ["acc"])
    xs, ys = _shards([128 * 9] * 8, 93, 9, seed=23)
    monkeypatch.delenv("ELEPHAS_AMD_FUSED_AVG", raising=False)
    out = []
    for fused in (True, False):
        t = _native(model, 8, 128, seed=6, deep="-1", monkeypatch=monkeypatch)
        assert t.persistent and t.persist_variant == 3, t.plan_name()
        t.set_data(xs, ys, 0.0, shuffle=False)
        t.GRAPH_CHUNK = 4
        t.begin_epoch()
        if fused:
            avg = t.run_steps_and_average(7, None, 8)
            assert t._fused_done, "the layer pipeline must average in its post node"
        else:
            t.run_steps(7)
            avg = t.average_replicas(None, 8)
        torch.cuda.synchronize()
        t.check()
        out.append((t.get_weights_flat(), avg.cpu().numpy().copy()))
    (wf, af), (ws, as_) = out
    assert np.array_equal(af, as_), np.abs(af - as_).max()
    assert np.array_equal(wf, ws), np.abs(wf - ws).max()
    for r in range(1, 8):
        assert np.array_equal(wf[r], wf[0])
