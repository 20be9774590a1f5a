"""Native HIP executor vs. the torch fp32 reference (GPU only).

The native engine must reproduce the reference engine's math: with dropout off
and shuffling off, one optimizer step on the same batch gives the same weights
(fp32 policy: exact-f32 MFMA, tight tolerance; bf16 policy: loose tolerance).
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


def _data(n, d, k, seed=0, onehot=True):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, d)).astype(np.float32)
    y = rng.integers(0, k, n)
    if onehot:
        y = np.eye(k, dtype=np.float32)[y]
    return x, y


def _engines(model, B, policy):
    from elephas_amd import config
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.torch_engine import TorchTrainer
    plan = build_plan(model)
    config.set_policy(policy)
    nat = NativeTrainer(model, plan, 1, B, torch.device("cuda"))
    ref = TorchTrainer(model, plan, 1, B, torch.device("cuda"))
    return nat, ref


@pytest.mark.parametrize("policy,tol", [("float32", 2e-5), ("mixed_bfloat16", 3e-2)])
@pytest.mark.parametrize("opt", ["sgd", "sgd_mom", "adam", "rmsprop", "rmsprop_mom", "adagrad", "adamax"])
def test_one_step_matches_reference(policy, tol, opt):
    from elephas_amd.models import initializers, optimizers as O
    initializers.set_seed(77)   # the initial weights must not depend on which tests ran before
    model = _mlp(784, [128, 128], 10)
    optim = {"sgd": O.SGD(0.1), "sgd_mom": O.SGD(0.01, momentum=0.9, nesterov=True, decay=1e-6),
             "adam": O.Adam(0.001), "rmsprop": O.RMSprop(), "rmsprop_mom": O.RMSprop(momentum=0.5, decay=1e-3),
             "adagrad": O.Adagrad(0.01), "adamax": O.Adamax(0.002)}[opt]
    model.compile(optim, "categorical_crossentropy", ["acc"])
    x, y = _data(64, 784, 10)
    nat, ref = _engines(model, 64, policy)
    for t in (nat, ref):
        t.set_data([x], [y], 0.0, shuffle=False)
        t.fit(2)
    wn, wr = nat.get_weights_flat()[0], ref.get_weights_flat()[0]
    w0 = np.concatenate([w.reshape(-1) for w in model.get_weights()])
    step = np.abs(wr - w0).max()
    assert step > 0
    if policy == "float32" and opt.startswith("sgd"):
        err = np.abs(wn - wr).max() / step
        assert err < 1e-3, err
    elif policy == "float32":
        # adaptive rules normalise by sqrt(state): near-zero gradients amplify f32 rounding
        err = np.abs(wn - wr).mean() / np.abs(wr - w0).mean()
        assert err < 1e-2, err
    else:
        # bf16 operands: adaptive optimizers amplify near-zero-gradient noise
        # (Adam step ~ lr*sign(g)), so compare on average
        err = np.abs(wn - wr).mean() / np.abs(wr - w0).mean()
        assert err < 0.15, err


@pytest.mark.parametrize("loss,act,metrics,out", [
    ("categorical_crossentropy", "softmax", ["acc"], 10),
    ("binary_crossentropy", "sigmoid", ["acc"], 1),
    ("mse", "linear", ["mae", "mean_absolute_percentage_error"], 1),
    ("mae", "linear", ["mse"], 3),
    ("sparse_categorical_crossentropy", "softmax", ["acc"], 7),
    ("logcosh", "tanh", ["mae"], 4),
    ("kld", "softmax", ["acc"], 5),
])
def test_evaluate_predict_match_reference(loss, act, metrics, out):
    from elephas_amd import config
    model = _mlp(20, [32, 16], out, act="tanh", out_act=act)
    model.compile("sgd", loss, metrics)
    x, y = _data(300, 20, out, seed=1, onehot=loss != "sparse_categorical_crossentropy")
    if loss in ("mse", "mae", "logcosh"):
        y = np.random.default_rng(2).normal(size=(300, out)).astype(np.float32)
    if loss == "binary_crossentropy":
        y = (np.random.default_rng(3).random((300, 1)) > 0.5).astype(np.float32)
    nat, ref = _engines(model, 32, "float32")
    en, er = nat.evaluate(x, y), ref.evaluate(x, y)
    assert np.allclose(en, er, rtol=1e-4, atol=1e-5), (en, er)
    pn, pr = nat.predict(x), ref.predict(x)
    assert np.allclose(pn, pr, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("policy", ["float32", "mixed_bfloat16"])
@pytest.mark.parametrize("B", [64, 60])
def test_wide_output_loss_rows_path(policy, B):
    # 200 classes > GEMM tile width: wave-per-row loss kernel (bf16: dZ^T staged in LDS;
    # B = 60 leaves a partial 8-row group and invalid rows in the last batch)
    model = _mlp(64, [96], 200)
    model.compile("sgd", "categorical_crossentropy", ["acc"])
    x, y = _data(250, 64, 200)
    nat, ref = _engines(model, B, policy)
    for t in (nat, ref):
        t.set_data([x], [y], 0.0, shuffle=False)
        t.fit(2)
    wn, wr = nat.get_weights_flat(), ref.get_weights_flat()
    if policy == "float32":
        assert np.allclose(wn, wr, atol=1e-5)
        assert np.allclose(nat.evaluate(x, y), ref.evaluate(x, y), rtol=1e-4)
    else:
        w0 = np.concatenate([w.reshape(-1) for w in model.get_weights()])
        assert np.abs(wn - wr).mean() / np.abs(wr - w0).mean() < 0.05
        assert np.allclose(nat.evaluate(x, y), ref.evaluate(x, y), rtol=2e-2, atol=2e-2)
    from elephas_amd import config
    config.set_policy("float32")


@pytest.mark.parametrize("policy", ["float32", "mixed_bfloat16"])
def test_split_k_wide_last_layer(policy):
    """A wide last layer with a deep reduction (K = 2048 -> 300 classes at batch 256)
    runs as split-K slabs (PK_PARTIAL, 4 slabs) summed with the bias by the loss rows
    kernel; training, evaluation and prediction match the fp32 torch reference."""
    from elephas_amd import config
    model = _mlp(64, [2048], 300)
    model.compile("sgd", "categorical_crossentropy", ["acc"])
    x, y = _data(600, 64, 300, seed=6)
    nat, ref = _engines(model, 256, policy)
    kinds = [p for p in nat.exe.launch_cfgs()]
    for t in (nat, ref):
        t.set_data([x], [y], 0.0, shuffle=False)
        t.fit(2)
    wn, wr = nat.get_weights_flat(), ref.get_weights_flat()
    w0 = np.concatenate([w.reshape(-1) for w in model.get_weights()])
    if policy == "float32":
        assert np.abs(wn - wr).max() <= 1e-4 * np.abs(wr - w0).max() + 1e-6
        assert np.allclose(nat.evaluate(x, y), ref.evaluate(x, y), rtol=1e-4)
        assert np.allclose(nat.predict(x[:100]), ref.predict(x[:100]), rtol=1e-4, atol=1e-6)
    else:
        assert np.abs(wn - wr).mean() / np.abs(wr - w0).mean() < 0.05
        assert np.allclose(nat.evaluate(x, y), ref.evaluate(x, y), rtol=2e-2, atol=2e-2)
    assert kinds  # the plan was built
    config.set_policy("float32")


def test_partial_batches_and_validation():
    model = _mlp(30, [40], 4, dropout=0.0)
    model.compile("sgd", "categorical_crossentropy", ["acc"])
    x, y = _data(203, 30, 4)
    nat, ref = _engines(model, 32, "float32")
    hs = []
    for t in (nat, ref):
        t.set_data([x], [y], 0.2, shuffle=False)
        hs.append(t.fit(3)[0])
    assert np.allclose(nat.get_weights_flat(), ref.get_weights_flat(), atol=2e-5)
    for k in ("loss", "acc", "val_loss", "val_acc"):
        assert np.allclose(hs[0][k], hs[1][k], rtol=1e-4, atol=1e-5), k


def test_replicas_independent_and_dropout_trains():
    # R replicas with different shards == R separate single-replica runs (no dropout)
    from elephas_amd import config
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy("float32")
    model = _mlp(50, [64], 6)
    model.compile("adam", "categorical_crossentropy", ["acc"])
    plan = build_plan(model)
    shards = [_data(n, 50, 6, seed=n) for n in (100, 37, 64, 10)]
    multi = NativeTrainer(model, plan, 4, 16, torch.device("cuda"))
    multi.set_data([s[0] for s in shards], [s[1] for s in shards], 0.0, shuffle=False,
                   active=[True, True, True, False])
    multi.fit(2)
    wm = multi.get_weights_flat()
    w0 = np.concatenate([w.reshape(-1) for w in model.get_weights()])
    assert np.array_equal(wm[3], w0)  # inactive replica untouched
    for r in range(3):
        single = NativeTrainer(model, plan, 1, 16, torch.device("cuda"))
        single.set_data([shards[r][0]], [shards[r][1]], 0.0, shuffle=False)
        single.fit(2)
        assert np.allclose(single.get_weights_flat()[0], wm[r], atol=1e-6)
    # dropout + shuffle + bf16: loss goes down
    config.set_policy("mixed_bfloat16")
    model2 = _mlp(784, [128, 128], 10, dropout=0.2)
    model2.compile("sgd", "categorical_crossentropy", ["acc"])
    from elephas_amd.models.datasets import synthetic_classification
    xx, yy = synthetic_classification(4096, 784, 10, seed=5)
    t = NativeTrainer(model2, build_plan(model2), 1, 64, torch.device("cuda"))
    t.set_data([xx / 10], [np.eye(10, dtype=np.float32)[yy]], 0.1)
    h = t.fit(3)[0]
    assert h["loss"][-1] < h["loss"][0]
    config.set_policy("float32")


def test_graph_replay_equals_eager():
    from elephas_amd import config
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy("float32")
    model = _mlp(100, [64, 32], 5, dropout=0.3)
    model.compile("sgd", "categorical_crossentropy")
    x, y = _data(640, 100, 5)
    ws = []
    for graph in (True, False):
        t = NativeTrainer(model, build_plan(model), 2, 32, torch.device("cuda"), seed=7)
        t.set_data([x, x], [y, y], 0.0, shuffle=False)
        t.begin_epoch()
        t.run_steps(20, use_graph=graph)
        ws.append(t.get_weights_flat())
    assert np.array_equal(ws[0], ws[1])
    assert not np.array_equal(ws[0][0], ws[0][1])  # replicas draw different dropout masks


def _fit_weights(model, policy, B, xs, ys, rowchain, epochs=1, val=0.0, R=None, seed=7, persist=0):
    from elephas_amd import config
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy(policy)
    R = R or len(xs)
    # persist=0: these cases pin the row-chain and grouped plans (the persistent plan has
    # its own file, tests/test_persist_gpu.py)
    t = NativeTrainer(model, build_plan(model), R, B, torch.device("cuda"), seed=seed, rowchain=rowchain,
                      persist=persist)
    t.set_data(xs, ys, val, shuffle=True)
    np.random.seed(3)
    torch.manual_seed(5)   # epoch shuffles draw from the global CUDA generator
    h = t.fit(epochs)
    return t, t.get_weights_flat(), h


def _plan_case(case):
    from elephas_amd.models import initializers
    from elephas_amd.models.optimizers import SGD, Adam, RMSprop
    initializers.set_seed(2024)   # the initial weights must not depend on which tests ran before
    rng = np.random.default_rng(11)
    if case in ("mnist_bf16_dropout", "mnist_f32_dropout"):
        model = _mlp(784, [128, 128], 10, dropout=0.2)
        model.compile(SGD(learning_rate=0.1), "categorical_crossentropy", ["acc"])
        policy, tol = ("mixed_bfloat16", 2e-2) if "bf16" in case else ("float32", 1e-4)
        B, d, k = 64, 784, 10
        sizes = [300, 130, 40]            # third replica runs out of batches early
    elif case == "tanh_f32_adam":
        model = _mlp(30, [64, 48], 5, act="tanh", dropout=0.1)
        model.compile(Adam(learning_rate=0.01), "categorical_crossentropy", ["acc", "mse"])
        policy, B, d, k, tol = "float32", 32, 30, 5, 1e-4
        sizes = [200, 200]
    elif case == "mse_f32":
        model = _mlp(20, [32], 1, out_act="linear")
        model.compile(SGD(learning_rate=0.05, momentum=0.9), "mse", ["mae"])
        policy, B, d, k, tol = "float32", 16, 20, 1, 1e-4
        sizes = [160]
    else:
        model = _mlp(50, [96, 64], 7, dropout=0.3)
        model.compile(RMSprop(learning_rate=0.005), "sparse_categorical_crossentropy", ["acc"])
        policy, B, d, k, tol = "mixed_bfloat16", 48, 50, 7, 3e-2
        sizes = [250, 180]
    xs, ys = [], []
    for n in sizes:
        x = rng.random((n, d), dtype=np.float32)
        if k == 1:
            y = rng.normal(size=(n, 1)).astype(np.float32)
        elif case.startswith("sparse"):
            y = rng.integers(0, k, (n, 1)).astype(np.float32)
        else:
            y = np.eye(k, dtype=np.float32)[rng.integers(0, k, n)]
        xs.append(x)
        ys.append(y)
    tf, wf, hf = _fit_weights(model, policy, B, xs, ys, rowchain=1, epochs=2, val=0.1)
    tg, wg, hg = _fit_weights(model, policy, B, xs, ys, rowchain=0, epochs=2, val=0.1)
    assert tf.rowchain and not tg.rowchain
    assert tf.launch_count() == 3
    if policy == "float32":
        scale = np.abs(wg).max()
        assert np.abs(wf - wg).max() <= tol * scale, (np.abs(wf - wg).max(), scale)
    else:
        # bf16 weight images: the plans sum layer 0 in different orders, and a 1-ulp
        # fp32 difference flips the bf16 rounding of some weight images, which later
        # steps carry on (tools/plan_flake_probe.py: both plans are bit-deterministic,
        # the gap between them depends on the initial weights, 1e-10 .. 0.2 of the mean
        # update after 10 steps at lr 0.1). The fp32 cases pin the plans' equivalence
        # tightly; here the plans must agree within a few bf16 ulps: the mean weight gap
        # below 2^-6 of the mean weight magnitude (worst of 15 initialisations: 4.5e-3;
        # a wrong mask or update rule on any layer is tens of percent)
        err = np.abs(wf - wg).mean() / np.abs(wg).mean()
        assert err < 2.0 ** -6, err
    for a, b in zip(hf, hg):
        if a is None:
            assert b is None
            continue
        for key in a:
            assert np.allclose(a[key], b[key], rtol=5 * tol, atol=5 * tol), (key, a[key], b[key])


@pytest.mark.parametrize("cfg", [0, 1, 2, 4])
@pytest.mark.parametrize("bf16", [1, 0])
@pytest.mark.parametrize("M,N,K", [(64, 128, 784), (64, 10, 128), (785, 128, 64), (300, 200, 136), (512, 512, 512),
                                   (513, 770, 264)])
def test_plain_gemm_matches_torch_fp32(M, N, K, bf16, cfg):
    """Library entry of the MFMA GEMM (LAT / THR / 256x256 tiles) vs. a torch fp32 matmul."""
    from elephas_amd.ops import native
    C = native.require()
    torch.manual_seed(0)
    dt = torch.bfloat16 if bf16 else torch.float32
    A = torch.randn(M, K, device="cuda").to(dt)
    BT = torch.randn(N, K, device="cuda").to(dt)
    out = torch.zeros(M, N, device="cuda")
    C.gemm_nt(A.data_ptr(), BT.data_ptr(), out.data_ptr(), M, N, K, K, K, N, bf16, cfg,
              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = A.float() @ BT.float().t()
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < (1e-4 if not bf16 else 1e-3), err


@pytest.mark.parametrize("cfg", [1, 2])
@pytest.mark.parametrize("M,N,K,ks", [(1024, 1000, 4096, 4), (300, 200, 136, 2), (513, 770, 1000, 3), (64, 10, 128, 5)])
def test_plain_gemm_split_k_matches_torch_fp32(M, N, K, ks, cfg):
    """The GEMM entry with the reduction split over workgroup slabs (PK_PARTIAL) and one
    slab-sum launch -- including more slabs than 64-wide K chunks (empty slabs) -- vs. a
    torch fp32 matmul, bf16 operands."""
    from elephas_amd.ops import native
    C = native.require()
    torch.manual_seed(1)
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    BT = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    out = torch.full((M, N), float("nan"), device="cuda")
    C.gemm_nt(A.data_ptr(), BT.data_ptr(), out.data_ptr(), M, N, K, K, K, N, 1, cfg,
              torch.cuda.current_stream().cuda_stream, 0, 0, ks)
    torch.cuda.synchronize()
    ref = A.float() @ BT.float().t()
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-3, err


def test_plain_gemm_rejects_misaligned_shapes():
    from elephas_amd.ops import native
    C = native.require()
    A = torch.zeros(4, 10, device="cuda")
    with pytest.raises(Exception):
        C.gemm_nt(A.data_ptr(), A.data_ptr(), A.data_ptr(), 4, 4, 10, 10, 10, 4, 0, 0, 0)


@pytest.mark.parametrize("rowchain", [0, 1])
def test_training_is_bit_deterministic(rowchain):
    """Same seeds -> bit-identical weights (no races between the update epilogue
    and the GEMMs that read the weight shadows, no order-dependent reductions)."""
    from elephas_amd.models.optimizers import SGD
    rng = np.random.default_rng(11)
    model = _mlp(784, [128, 128], 10, dropout=0.2)
    model.compile(SGD(learning_rate=0.1), "categorical_crossentropy", ["acc"])
    xs = [rng.random((n, 784), dtype=np.float32) for n in (300, 130, 40)]
    ys = [np.eye(10, dtype=np.float32)[rng.integers(0, 10, len(x))] for x in xs]
    _, w1, _ = _fit_weights(model, "mixed_bfloat16", 64, xs, ys, rowchain=rowchain, epochs=2, val=0.1)
    _, w2, _ = _fit_weights(model, "mixed_bfloat16", 64, xs, ys, rowchain=rowchain, epochs=2, val=0.1)
    assert np.array_equal(w1, w2), np.abs(w1 - w2).max()


@pytest.mark.parametrize("cfg", ["1", "2", "4"])
@pytest.mark.parametrize("policy,tol", [("mixed_bfloat16", 5e-2), ("float32", 1e-3)])
def test_throughput_tiles_match_reference(monkeypatch, policy, tol, cfg):
    """Force the 128x128 THR tiles (LDS-staged glds main loop for bf16) or the
    256x256 8-wave tile (cfg 4: FWD / DX / DW epilogues over two 128-row halves,
    the last layer and the X^T gather on their own launches) on every layer:
    gathered layer-0 rows, the ones row of the bias gradient, K / N / M tails
    (K=100, N=70, B=48 of 64) and the fused SGD update must all match."""
    from elephas_amd.models.optimizers import SGD
    monkeypatch.setenv("ELEPHAS_AMD_GEMM_CFG", cfg)
    model = _mlp(200, [136, 72], 70, dropout=0.0)
    model.compile(SGD(0.05), "categorical_crossentropy", ["acc"])
    x, y = _data(48, 200, 70)
    nat, ref = _engines(model, 48, policy)
    for t in (nat, ref):
        t.set_data([x], [y], 0.0, shuffle=False)
        t.fit(3)
    wn, wr = nat.get_weights_flat()[0], ref.get_weights_flat()[0]
    w0 = np.concatenate([w.reshape(-1) for w in model.get_weights()])
    if policy == "float32":
        err = np.abs(wn - wr).max() / np.abs(wr - w0).max()
    else:  # bf16 operand rounding: compare on average
        err = np.abs(wn - wr).mean() / np.abs(wr - w0).mean()
    assert err < tol, err
    assert np.allclose(nat.evaluate(x, y), ref.evaluate(x, y), rtol=5 * tol, atol=5 * tol)


def test_native_inference_is_batch_invariant():
    """Batched and unbatched inference agree exactly on the MFMA path too
    (reference tests/test_ml_model.py:345-354)."""
    from elephas_amd import config
    config.set_policy("mixed_bfloat16")
    model = _mlp(784, [128, 128], 10, dropout=0.2)
    model.compile("sgd", "categorical_crossentropy", ["acc"])
    x, _ = _data(3000, 784, 10, seed=9)
    full = model.predict(x)
    chunks = np.concatenate([model.predict(x[i:i + 1000]) for i in range(0, 3000, 1000)])
    odd = np.concatenate([model.predict(x[i:i + 37]) for i in range(0, 3000, 37)])
    assert np.array_equal(full, chunks)
    assert np.array_equal(full, odd)
    config.set_policy("float32")


@pytest.mark.parametrize("policy", ["float32", "mixed_bfloat16"])
@pytest.mark.parametrize("opt", ["sgd_mom", "adam"])
def test_allreduce_apply_path_equals_fused_update(policy, opt):
    """Per-step gradient path ([fwd+bwd -> G] -> all-reduce -> tiled apply kernel
    that also rebuilds the W / W^T images) == the fused DW_UPDATE epilogue."""
    from elephas_amd import config
    from elephas_amd.models import optimizers as O
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy(policy)
    model = _mlp(130, [200, 72], 9, dropout=0.25)
    model.compile(O.SGD(0.05, momentum=0.9) if opt == "sgd_mom" else O.Adam(0.002), "categorical_crossentropy")
    x, y = _data(400, 130, 9, seed=4)
    ws = []
    for path in ("fused", "allreduce"):
        t = NativeTrainer(model, build_plan(model), 2, 32, torch.device("cuda"), seed=3)
        t.set_data([x, x[::-1].copy()], [y, y[::-1].copy()], 0.0, shuffle=False)
        t.begin_epoch()
        if path == "fused":
            t.run_steps(12, use_graph=True)
        else:
            t.run_steps_allreduce(12, lambda g: None, use_graph=True)
        ws.append(t.get_weights_flat())
    w0 = np.concatenate([w.reshape(-1) for w in model.get_weights()])
    if policy == "float32" and opt == "adam":
        # the fused path is the layer pipeline here (persistent plan for 130-200-72-9), the
        # all-reduce path the grouped launches: Adam's normalised steps amplify the fp32
        # summation-order differences of near-zero gradients -- compare on average
        err = np.abs(ws[0] - ws[1]).mean() / np.abs(ws[0] - w0).mean()
        assert err < 1e-3, err
    elif policy == "float32":
        err = np.abs(ws[0] - ws[1]).max() / np.abs(ws[0] - w0).max()
        assert err < 1e-4, err
    else:
        # bf16 weight images: a 1-ulp fp32 difference between the two update kernels'
        # instruction schedules can flip the bf16 rounding of a weight, and Adam's
        # normalised steps carry such flips on; compare on average (as the THR test)
        err = np.abs(ws[0] - ws[1]).mean() / np.abs(ws[0] - w0).mean()
        assert err < 2e-2, err
    config.set_policy("float32")


def test_refresh_shadows_round_trip():
    """set_weights -> tiled refresh -> forward uses exactly the new weights."""
    from elephas_amd import config
    config.set_policy("float32")
    model = _mlp(70, [130], 3, out_act="linear")
    model.compile("sgd", "mse")
    x, _ = _data(50, 70, 3)
    p0 = model.predict(x)
    rng = np.random.default_rng(0)
    model.set_weights([rng.normal(size=w.shape).astype(np.float32) for w in model.get_weights()])
    p1 = model.predict(x)
    W = model.get_weights()
    ref = np.maximum(x @ W[0] + W[1], 0) @ W[2] + W[3]
    assert not np.allclose(p0, p1)
    assert np.allclose(p1, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("gran", ["fit", "epoch", "batch"])
def test_spark_model_granularities_native_vs_torch(gran, tmp_path):
    """SparkModel sync modes on the native executor (device replica sums, G
    all-reduce callback, checkpoint state) agree with the torch engine."""
    from elephas_amd import config
    from elephas_amd.data import SparkContext
    from elephas_amd.models.optimizers import Adam
    from elephas_amd.spark_model import SparkModel
    from elephas_amd.models import initializers
    config.set_policy("float32")
    x, y = _data(600, 40, 5, seed=2)
    ws = []
    for engine in ("native", "torch"):
        config.set_engine(engine)
        initializers.set_seed(3)
        m = _mlp(40, [64, 32], 5)
        m.compile(Adam(0.005), "categorical_crossentropy", ["acc"])
        sm = SparkModel(m, mode="synchronous", sync_granularity=gran)
        rdd = SparkContext.getOrCreate().parallelize(list(zip(x, y)), 3)
        sm.fit(rdd, epochs=3, batch_size=32, verbose=0, shuffle=False,
               checkpoint_dir=str(tmp_path / engine))
        ws.append(np.concatenate([w.reshape(-1) for w in sm.master_network.get_weights()]))
    config.set_engine("auto")
    assert np.abs(ws[0] - ws[1]).max() < 2e-4, np.abs(ws[0] - ws[1]).max()


@pytest.mark.parametrize("case", ["mnist_bf16_dropout", "mnist_f32_dropout", "tanh_f32_adam", "mse_f32",
                                  "sparse_bf16_rmsprop"])
def test_rowchain_matches_grouped_path(case):
    """Row-chain plan (3 launches: layer-0 split-K slabs, one row-local chain kernel for
    layers 1..L-1 forward / loss / input gradients, one DW launch for every layer) ==
    the grouped 2L-launch plan: same dropout masks, same update rules, fp32
    accumulation (only the layer-0 summation order differs)."""
    _plan_case(case)


@pytest.mark.parametrize("mode,freq", [("synchronous", "epoch"), ("asynchronous", "epoch"), ("asynchronous", "batch"),
                                       ("hogwild", "epoch"), ("hogwild", "batch")])
def test_spark_model_end_to_end_on_gpu(mode, freq):
    """Reference tests/integration/test_end_to_end.py on the MI355X path: native
    executor workers, device parameter server (HBM, locked / lock-free), and the
    reference's consistency checks (distributed predict == master predict,
    distributed evaluate within 0.01 of the master network's)."""
    from elephas_amd import config
    from elephas_amd.data import SparkContext
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.spark_model import SparkModel
    from elephas_amd.utils.rdd_utils import to_simple_rdd
    config.set_policy("mixed_bfloat16")
    x, y = _data(1000, 784, 10, seed=8)
    x = (x - x.min()) / (x.max() - x.min())
    model = _mlp(784, [128, 128], 10, dropout=0.2)
    model.compile(SGD(learning_rate=0.1), "categorical_crossentropy", ["acc"])
    sm = SparkModel(model, mode=mode, frequency=freq, parameter_server_mode="device", num_workers=2)
    sm.fit(to_simple_rdd(SparkContext.getOrCreate(), x, y), epochs=2, batch_size=64, verbose=0,
           validation_split=0.1)
    preds = np.stack(sm.predict(x[:300]))
    assert np.array_equal(np.argmax(preds, 1), np.argmax(sm.master_network.predict(x[:300]), 1))
    ev = sm.evaluate(x, y)
    ref = sm.master_network.evaluate(x, y)
    assert np.allclose(ev, ref, atol=0.01), (ev, ref)
    assert np.isfinite(ev).all()
    config.set_policy("float32")


def test_overlapped_bucket_allreduce_equals_graph_path():
    """Per-layer gradient buckets issued on a comm stream beside the backward give
    the same weights as the whole-vector all-reduce path."""
    from elephas_amd import config
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy("mixed_bfloat16")
    model = _mlp(784, [128, 128], 10, dropout=0.2)
    model.compile(SGD(0.1, momentum=0.9), "categorical_crossentropy", ["acc"])
    x, y = _data(640, 784, 10, seed=2)
    ws, calls = [], []
    for path in ("graph", "overlap"):
        # both on the grouped plan (the bucketed path issues its launches one by one)
        t = NativeTrainer(model, build_plan(model), 1, 64, torch.device("cuda"), seed=5, rowchain=0)
        t.set_data([x], [y], 0.0, shuffle=False)
        t.begin_epoch()
        if path == "graph":
            t.run_steps_allreduce(8, lambda g: g.mul_(1.0), use_graph=True)
        else:
            t.run_steps_allreduce_overlap(8, lambda g: (calls.append(g.shape[1]), g.mul_(1.0)))
        ws.append(t.get_weights_flat())
    assert np.array_equal(ws[0], ws[1])
    assert sorted(set(calls)) == sorted({785 * 128, 129 * 128, 129 * 10}) and len(calls) == 24
    config.set_policy("float32")


@pytest.mark.parametrize("threads", [1, 4])
def test_host_loader_uploads(threads):
    """Pinned double-buffered loader: contiguous and row-strided uploads (multi-threaded
    packing of each chunk) reproduce the host data exactly, across chunk boundaries."""
    from elephas_amd.ops import native
    C = native.require()
    L = C.HostLoader(1 << 20, 2, threads)
    assert L.threads == threads
    s = torch.cuda.Stream()
    rng = np.random.default_rng(5)
    a = rng.random(3_000_001, dtype=np.float32)          # ~12 MB: 12 chunks + a ragged tail
    d = torch.empty(a.size, dtype=torch.float32, device="cuda")
    s.wait_stream(torch.cuda.current_stream())   # the allocation / fills run on the current stream
    L.upload(a.ctypes.data, d.data_ptr(), a.nbytes, s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(d.cpu().numpy(), a)
    x = rng.random((5000, 781), dtype=np.float32)          # rows padded to 784 on the device
    dx = torch.zeros(5000, 784, dtype=torch.float32, device="cuda")
    s.wait_stream(torch.cuda.current_stream())   # the zero-fill must land before the copy
    L.upload_rows(x.ctypes.data, 781 * 4, dx.data_ptr(), 784 * 4, 5000, 781 * 4, s.cuda_stream)
    assert (L.last_pack_threads > 1) == (threads > 1)   # ~1 MB chunks are packed by up to 4 threads
    s.synchronize()
    got = dx.cpu().numpy()
    np.testing.assert_array_equal(got[:, :781], x)
    assert not got[:, 781:].any()


@pytest.mark.parametrize("consistent", [0, 1])
def test_ps_replica_pull_push(consistent):
    """Sharded device PS (one rank): pull gathers theta exactly; push_replicas applies
    theta += sum_r (P[r] - before) (fp64 reference); push_delta applies theta -= d."""
    from elephas_amd.ops import native
    C = native.require()
    n, R = 118_282, 8
    ps = C.ShardedParameterServer(0, 1, n, consistent, 0)
    assert ps.nchunks == (n + 4095) // 4096
    rng = np.random.default_rng(9)
    theta = torch.from_numpy(rng.normal(size=n).astype(np.float32)).cuda()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    ps.set(theta.data_ptr(), s.cuda_stream)
    before = torch.empty(n, dtype=torch.float32, device="cuda")
    ps.pull(before.data_ptr(), s.cuda_stream)
    s.synchronize()
    assert torch.equal(before, theta)
    P = torch.zeros(R, n + 6, dtype=torch.float32, device="cuda")[:, :n]   # padded row stride
    P.copy_(theta.expand(R, n) + torch.from_numpy(rng.normal(size=(R, n)).astype(np.float32)).cuda() * 1e-2)
    want = (theta.double() + (P.double() - before.double()).sum(0)).float()
    s.wait_stream(torch.cuda.current_stream())   # P is written on the current stream
    ps.push_replicas(P.data_ptr(), P.stride(0), R, before.data_ptr(), s.cuda_stream)
    got = torch.empty(n, dtype=torch.float32, device="cuda")
    ps.pull(got.data_ptr(), s.cuda_stream)
    s.synchronize()
    torch.testing.assert_close(got, want, rtol=0, atol=1e-5)
    d = torch.from_numpy(rng.normal(size=n).astype(np.float32)).cuda()
    s.wait_stream(torch.cuda.current_stream())
    ps.push_delta(d.data_ptr(), s.cuda_stream)
    ps.pull(got.data_ptr(), s.cuda_stream)
    s.synchronize()
    torch.testing.assert_close(got, want - d, rtol=0, atol=1e-5)
    # pull straight into every replica master (the persistent trainers' async pull): the
    # replica rows of an odd-sized vector are only 8-byte aligned, the copy must cope
    for stride in (n, n + 6):
        Q = torch.zeros(R, stride, dtype=torch.float32, device="cuda")
        dst = torch.empty(n, dtype=torch.float32, device="cuda")
        s.wait_stream(torch.cuda.current_stream())
        ps.pull_replicas(dst.data_ptr(), Q.data_ptr(), stride, R, s.cuda_stream)
        s.synchronize()
        assert torch.equal(dst, got)    # the server's theta, as pulled above
        for r in range(R):
            assert torch.equal(Q[r, :n], got), (stride, r)
        if stride > n:
            assert not Q[:, n:].any()   # nothing written past each row
    assert ps.error() == 0


def test_ps_concurrent_streams_lose_no_update():
    """Eight streams push integer deltas into the same chunks concurrently while four
    others pull: every push lands exactly once (fp32 atomics, integers exact) and an
    'asynchronous' pull never sees a chunk with half of a push applied (each push adds
    the same value to every element of the vector, so a consistent chunk is constant)."""
    from elephas_amd.ops import native
    C = native.require()
    n, K = 40_000, 25
    ps = C.ShardedParameterServer(0, 1, n, 1, 0, 4096)
    zero = torch.zeros(n, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ps.set(zero.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ones = torch.full((n,), -1.0, dtype=torch.float32, device="cuda")   # theta -= -1 per push
    pushers = [torch.cuda.Stream() for _ in range(8)]
    pullers = [torch.cuda.Stream() for _ in range(4)]
    snaps = [torch.empty(K, n, dtype=torch.float32, device="cuda") for _ in pullers]
    torch.cuda.synchronize()
    for k in range(K):
        for st in pushers:
            ps.push_delta(ones.data_ptr(), st.cuda_stream)
        for st, sn in zip(pullers, snaps):
            ps.pull(sn[k].data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    assert ps.error() == 0
    final = torch.empty(n, dtype=torch.float32, device="cuda")
    ps.pull(final.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(final, torch.full_like(final, 8.0 * K))
    for sn in snaps:
        for c0 in range(0, n, 4096):
            blk = sn[:, c0:c0 + 4096]
            assert torch.equal(blk, blk[:, :1].expand_as(blk)), "torn chunk in an asynchronous pull"


def test_ps_pull_refresh_then_steps_match_set_weights():
    """DeviceClient.pull_refresh (gather kernel + refresh of every replica's master and
    both weight-image parities) leaves the executor in the same state as uploading the
    same weights with set_weights_flat: the next steps give bit-identical weights."""
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.models import optimizers as O
    from elephas_amd.parameter.client import DeviceClient
    from elephas_amd import config
    config.set_policy("mixed_bfloat16")
    model = _mlp(784, [128, 128], 10, dropout=0.2)
    model.compile(O.SGD(0.1), "categorical_crossentropy", ["acc"])
    R = 4
    x, y = _data(512, 784, 10)
    ts = [NativeTrainer(model, build_plan(model), R, 64, torch.device("cuda"), seed=77) for _ in range(2)]
    n = ts[0].P.shape[1]
    client = DeviceClient().connect(n, "asynchronous", rank=0, world=1, allgather=lambda h: [h])
    theta = torch.from_numpy(np.random.default_rng(3).normal(size=n).astype(np.float32) * 0.05).cuda()
    torch.cuda.synchronize()
    client.ps.set(theta.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    before = torch.empty(n, dtype=torch.float32, device="cuda")
    for i, t in enumerate(ts):
        t.set_data([x] * R, [y] * R, 0.0, shuffle=False)
        t.begin_epoch()
        if i == 0:
            with torch.cuda.stream(t.stream):
                client.pull_refresh(t, before.data_ptr())
        else:
            t.set_weights_flat(theta.cpu().numpy())
        t.stream.synchronize()
        t.run_steps(2, use_graph=False)
    assert torch.equal(before, theta)
    w0, w1 = ts[0].get_weights_flat(), ts[1].get_weights_flat()
    assert np.abs(w0 - theta.cpu().numpy()).max() > 0
    np.testing.assert_array_equal(w0, w1)


@pytest.mark.parametrize("rowchain", [0, 1])
def test_native_dropout_matches_fp32_reference_with_same_masks(rowchain):
    """Native dropout (masks regenerated from the counter hash in the forward AND the
    backward kernels) == the fp32 torch autograd engine drawing the same masks
    (ops/dropout_hash.py): weights and per-step losses agree over several steps of 2
    replicas, on both step plans -- so the masks, their fwd/bwd identity and the
    1 / (1 - rate) scaling are those of tf.nn.dropout (reference conftest.py:13,16)."""
    from elephas_amd import config
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.torch_engine import TorchTrainer
    config.set_policy("float32")
    model = _mlp(40, [48, 32], 6, dropout=0.3)
    model.compile(SGD(0.2), "categorical_crossentropy", ["acc"])
    plan = build_plan(model)
    xs, ys = [], []
    for r in range(2):
        x, y = _data(96, 40, 6, seed=20 + r)
        xs.append(x)
        ys.append(y)
    nat = NativeTrainer(model, plan, 2, 32, torch.device("cuda"), seed=12345, rowchain=rowchain)
    ref = TorchTrainer(model, plan, 2, 32, torch.device("cuda"), hash_dropout_seed=12345)
    w0 = nat.get_weights_flat()[0].copy()
    for t in (nat, ref):
        t.set_data(xs, ys, 0.0, shuffle=False)
    hn = nat.fit(2)
    hr = ref.fit(2)
    wn, wr = nat.get_weights_flat(), ref.get_weights_flat()
    err = np.abs(wn - wr).max() / np.abs(wr - w0).max()
    assert err < 1e-4, err
    for a, b in zip(hn, hr):
        np.testing.assert_allclose(a["loss"], b["loss"], rtol=1e-4)
    # without the shared masks the runs differ: the comparison above has teeth
    free = TorchTrainer(model, plan, 2, 32, torch.device("cuda"), seed=3)
    free.set_data(xs, ys, 0.0, shuffle=False)
    free.fit(2)
    assert np.abs(free.get_weights_flat() - wr).max() / np.abs(wr - w0).max() > 1e-2


def test_spark_model_refit_reuses_trainer_exactly():
    """A second SparkModel.fit of the same model reuses the cached native trainer (same
    object; shards kept for the same columnar RDD, re-uploaded for a new one) and gives
    bit-identical weights to a fit on a freshly built trainer from the same start."""
    from elephas_amd import config, worker
    from elephas_amd.data import SparkContext
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.spark_model import SparkModel
    from elephas_amd.utils.rdd_utils import to_simple_rdd
    config.set_policy("float32")
    x, y = _data(1200, 64, 5, seed=4)
    sc = SparkContext(master="local[4]")
    rdd = to_simple_rdd(sc, x, y)
    kw = dict(epochs=2, batch_size=32, verbose=0, validation_split=0.1, shuffle=False)

    def new_model(weights=None):
        m = _mlp(64, [48, 32], 5)
        m.compile(SGD(learning_rate=0.05, momentum=0.9), "categorical_crossentropy", ["acc"])
        if weights is not None:
            m.set_weights(weights)
        return m
    worker._trainer_cache.clear()
    sm = SparkModel(new_model(), mode="synchronous")
    sm.fit(rdd, **kw)
    first = worker._trainer_cache._entry[0]
    w1 = sm.master_network.get_weights()
    sm.fit(rdd, **kw)                                  # reuses trainer and shards
    assert worker._trainer_cache._entry[0] is first
    w2 = sm.master_network.get_weights()
    worker._trainer_cache.clear()
    fresh = SparkModel(new_model(w1), mode="synchronous")
    fresh.fit(rdd, **kw)
    for a, b in zip(w2, fresh.master_network.get_weights()):
        np.testing.assert_array_equal(a, b)
    # a different dataset through the cached trainer: re-uploaded, same as fresh again
    x2, y2 = _data(1200, 64, 5, seed=9)
    rdd2 = to_simple_rdd(sc, x2, y2)
    w3_start = fresh.master_network.get_weights()
    fresh.fit(rdd2, **kw)
    w3 = fresh.master_network.get_weights()
    worker._trainer_cache.clear()
    ref = SparkModel(new_model(w3_start), mode="synchronous")
    ref.fit(rdd2, **kw)
    for a, b in zip(w3, ref.master_network.get_weights()):
        np.testing.assert_array_equal(a, b)


def test_sparkmodel_averaging_is_the_bench_kernel_bit_for_bit():
    """SparkModel._average_into and the bench's NativeTrainer.average_replicas are one
    implementation: both give fp32(fp64 replica sum * 1/n) bit for bit (3 replicas, so
    1/n is inexact), written back into every replica, with no host synchronisation in
    between (the result is read after the trainer's stream)."""
    from elephas_amd import config
    from elephas_amd.models import Sequential, Dense, initializers
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.spark_model import SparkModel
    from elephas_amd.profiling import PhaseTimer
    config.set_policy("float32")
    initializers.set_seed(4)
    m = Sequential([Dense(40, activation="relu", input_dim=24), Dense(7, activation="softmax")])
    m.compile(SGD(0.1), "categorical_crossentropy", ["acc"])
    n = sum(w.size for w in m.get_weights())
    P = np.random.default_rng(6).normal(size=(3, n)).astype(np.float32)
    want = (P.astype(np.float64).sum(0) * (1.0 / 3)).astype(np.float32)
    outs = []
    for path in ("bench", "spark"):
        t = NativeTrainer(m, build_plan(m), 3, 32, torch.device("cuda"), seed=1)
        t.set_weights_flat(P)
        if path == "bench":
            mean = t.average_replicas(None, 3)
        else:
            sm = SparkModel(m, mode="synchronous")
            sm._timer = PhaseTimer()
            mean = sm._average_into(t, n, 3, True)
        t.stream.synchronize()
        outs.append((mean.cpu().numpy(), t.get_weights_flat()))
    for mean, reps in outs:
        assert np.array_equal(mean, want)
        assert all(np.array_equal(r, want) for r in reps)


@pytest.mark.parametrize("policy", ["float32", "mixed_bfloat16"])
def test_pipelined_inference_multi_chunk(policy):
    """predict / evaluate stream the rows through the three-stream pipeline (chunked
    uploads on a copy stream, eval kernels per chunk, chunked downloads): the result of
    one call over many chunks equals the single-chunk calls, only replica r computes,
    and the bf16 host conversion matches torch's fp32 -> bf16 rounding bit for bit."""
    from elephas_amd import config
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    model = _mlp(50, [64], 7)
    model.compile("sgd", "categorical_crossentropy", ["acc"])
    config.set_policy(policy)
    try:
        t = NativeTrainer(model, build_plan(model), 3, 32, torch.device("cuda"), eval_batch=256)
        x, y = _data(1000, 50, 7, seed=5)
        x[3, 4] = np.nan                     # a quiet NaN stays NaN through the converting pack
        x[5, :] = np.float32(1.0 + 2.0 ** -8)   # a tie: rounds to even
        t.set_weights_flat(np.stack([t.get_weights_flat()[0] * s for s in (1.0, 0.5, 2.0)]))
        full = t.predict(x, r=2)
        parts = np.concatenate([t.predict(x[i:i + 200], r=2) for i in range(0, 1000, 200)])
        assert np.array_equal(np.isnan(full), np.isnan(parts))
        ok = ~np.isnan(full).any(1)
        np.testing.assert_array_equal(full[ok], parts[ok])
        assert not np.allclose(full[ok], t.predict(x, r=0)[ok])   # replica 2 != replica 0
        ev = t.evaluate(x[ok], y[ok], r=1)
        ev_parts = [t.evaluate_sums(x[ok][i:i + 300], y[ok][i:i + 300], r=1) for i in range(0, ok.sum(), 300)]
        s = np.sum(ev_parts, 0)
        assert np.allclose(ev, [s[0] / s[1], s[2] / s[1]], rtol=1e-6)
        if policy == "mixed_bfloat16":
            dev = torch.zeros(4, t.Kp0, dtype=torch.bfloat16, device="cuda")
            t._upload_rows(dev, x[:4])
            t.stream.synchronize()
            want = torch.from_numpy(x[:4]).to(torch.bfloat16)
            got = dev[:, :50].cpu()
            assert torch.equal(got.view(torch.int16)[~torch.isnan(want)], want.view(torch.int16)[~torch.isnan(want)])
            assert torch.isnan(got[3, 4])
    finally:
        config.set_policy("float32")


@pytest.mark.parametrize("hidden,B,policy", [([96, 320, 272], 64, "float32"),   # 512-wide class (NBW 8)
                                             ([300, 120], 48, "float32"),        # 128-wide tail (NBW 2)
                                             ([64, 512], 40, "float32"),         # Otto's widths, partial batch
                                             ([96, 320, 272], 64, "mixed_bfloat16")])
def test_tail_chain_matches_fp32_reference_with_same_masks(hidden, B, policy):
    """Tail-chain plan (rowchain.hip at L = 2 over the last two layers of a deeper stack:
    after the grouped FWD of layer L-2, one row-local kernel recomputes its activation /
    dropout from the stored pre-activations and runs the last layer's forward, the loss
    and both input gradients) == the fp32 torch engine
    drawing the same dropout masks, over several steps of 2 replicas with a partial last
    batch; the plan really is the tail chain (one launch fewer than FWD + BWD per layer)."""
    from elephas_amd import config
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.torch_engine import TorchTrainer
    config.set_policy(policy)
    model = _mlp(40, hidden, 9, dropout=0.3)
    model.compile(SGD(0.1), "categorical_crossentropy", ["acc"])
    plan = build_plan(model)
    xs, ys = [], []
    for r in range(2):
        x, y = _data(3 * B - 7, 40, 9, seed=40 + r)
        xs.append(x)
        ys.append(y)
    # persist=0: these shapes would take the persistent layer pipeline (test_deep_gpu.py)
    nat = NativeTrainer(model, plan, 2, B, torch.device("cuda"), seed=777, persist=0)
    assert nat.exe.tailchain() and not nat.exe.rowchain() and not nat.persistent
    if hidden == [96, 320, 272]:
        # layer 2's DW (321 x 272 x 64: 128x64 tiles) and DX (64 x 320 x 272: 64x32 split-K
        # tiles) share one launch, each on its own tile (gemm_dual)
        assert any(c >= 100 for c in nat.exe.launch_cfgs()), nat.exe.launch_cfgs()
    config.set_policy("float32")
    ref = TorchTrainer(model, plan, 2, B, torch.device("cuda"), hash_dropout_seed=777)
    w0 = nat.get_weights_flat()[0].copy()
    for t in (nat, ref):
        t.set_data(xs, ys, 0.1, shuffle=False)
    hn = nat.fit(2)
    hr = ref.fit(2)
    wn, wr = nat.get_weights_flat(), ref.get_weights_flat()
    if policy == "float32":
        err = np.abs(wn - wr).max() / np.abs(wr - w0).max()
        assert err < 1e-4, err
        for a, b in zip(hn, hr):
            np.testing.assert_allclose(a["loss"], b["loss"], rtol=1e-4)
    else:
        err = np.abs(wn - wr).mean() / np.abs(wr - w0).mean()
        assert err < 0.05, err
    # the grouped plan (tail off) computes the same step
    import os
    os.environ["ELEPHAS_AMD_TAIL"] = "0"
    try:
        config.set_policy(policy)
        grp = NativeTrainer(model, plan, 2, B, torch.device("cuda"), seed=777, persist=0)
    finally:
        del os.environ["ELEPHAS_AMD_TAIL"]
    assert not grp.exe.tailchain()
    assert nat.exe.launches_per_step() < grp.exe.launches_per_step(), (nat.plan_name(), grp.plan_name())
    grp.set_weights_flat(w0)
    grp.set_data(xs, ys, 0.1, shuffle=False)
    hg = grp.fit(2)
    tol = 1e-5 if policy == "float32" else 2e-2
    for a, b in zip(hn, hg):
        np.testing.assert_allclose(a["val_loss"], b["val_loss"], rtol=10 * tol)
    d = np.abs(grp.get_weights_flat() - wn).max() / np.abs(wn - w0).max()
    assert d < tol, d
    config.set_policy("float32")


def test_predict_output_pool_never_aliases_a_live_array():
    """Large predictions come from a pool of pinned host buffers recycled only after the
    previous array (and its views) is gone: arrays the caller holds never share memory,
    and a recycled buffer holds exactly the new call's predictions."""
    import gc
    from elephas_amd import config
    from elephas_amd.ops.native_engine import NativeTrainer, _OUT_POOL
    from elephas_amd.ops.plan import build_plan
    config.set_policy("float32")
    m = _mlp(16, [32], 32, out_act="softmax")
    m.compile("sgd", "categorical_crossentropy", ["acc"])
    t = NativeTrainer(m, build_plan(m), 1, 256, torch.device("cuda"))
    rng = np.random.default_rng(3)
    x1 = rng.random((70000, 16), dtype=np.float32)   # 70000 x 32 fp32 = 9 MB: pooled
    x2 = rng.random((70000, 16), dtype=np.float32)
    a = t.predict(x1)
    b = t.predict(x2)
    c = t.predict(x1)
    assert not np.shares_memory(a, b) and not np.shares_memory(a, c) and not np.shares_memory(b, c)
    assert np.array_equal(a, c) and not np.array_equal(a, b)
    view = b[:10]
    del b
    gc.collect()
    d = t.predict(x1)                          # b's buffer is still referenced by the view
    assert not np.shares_memory(d, view) and np.array_equal(d, a)
    ref_b = view.copy()
    del a, c, d
    gc.collect()
    e = t.predict(x2)                          # may reuse a recycled buffer
    assert np.array_equal(e[:10], ref_b) and np.array_equal(view, ref_b)
    assert sum(len(v) for v in _OUT_POOL._free.values()) <= _OUT_POOL.KEEP
