"""Per-epoch shuffle: keyed Feistel permutation (csrc/kernels/shuffle.hip).

``feistel_perm`` is a numpy transcription of the kernel. The CPU tests pin its
properties (a permutation of the training rows, the validation tail left in place,
position statistics close to uniform); the GPU test checks the kernel against it
bit for bit and that NativeTrainer's epochs draw different orders.
"""
import numpy as np
import pytest

M32 = 0xFFFFFFFF


def fmix32(h):
    h = np.asarray(h, np.uint64) & M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def feistel_perm(n, nmax, key, r, shuffle=True, rounds=6):
    out = np.arange(nmax, dtype=np.int64)
    if not shuffle or n <= 1:
        return out
    b = int(n - 1).bit_length()
    h = (b + 1) >> 1
    mask = (1 << h) - 1
    kr = int(fmix32((key ^ ((0x85EBCA6B * (r + 1)) & M32)) & M32))
    x = np.arange(n, dtype=np.uint64)
    todo = np.ones(n, bool)
    while todo.any():
        l, rr = x[todo] >> np.uint64(h), x[todo] & np.uint64(mask)
        for q in range(rounds):
            f = fmix32(rr ^ np.uint64((kr + 0x9E3779B9 * (q + 1)) & M32)) & np.uint64(mask)
            l, rr = rr, l ^ f
        x[todo] = (l << np.uint64(h)) | rr
        todo = x >= n
    out[:n] = x.astype(np.int64)
    return out


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 1000, 6750, 65537])
def test_feistel_is_permutation(n):
    p = feistel_perm(n, n + 5, 12345, 0)
    assert sorted(p[:n].tolist()) == list(range(n))
    assert p[n:].tolist() == list(range(n, n + 5))


def test_feistel_keys_and_replicas_differ():
    a = feistel_perm(1000, 1000, 1, 0)
    assert not np.array_equal(a, feistel_perm(1000, 1000, 2, 0))
    assert not np.array_equal(a, feistel_perm(1000, 1000, 1, 1))
    assert np.array_equal(feistel_perm(1000, 1000, 7, 0, shuffle=False), np.arange(1000))


def test_feistel_positions_near_uniform():
    # where row 0 lands over many keys: chi-square over 10 positions
    n, trials = 10, 4000
    counts = np.bincount([feistel_perm(n, n, k, 0)[0] for k in range(trials)], minlength=n)
    chi2 = ((counts - trials / n) ** 2 / (trials / n)).sum()
    assert chi2 < 40, counts    # 9 dof: p ~ 1e-5
    # adjacent rows stay adjacent no more often than chance
    p = feistel_perm(6750, 6750, 99, 3)
    assert (np.abs(np.diff(p)) == 1).mean() < 0.01


@pytest.mark.gpu
def test_shuffle_kernel_matches_numpy():
    import torch
    from elephas_amd.ops import native
    C = native.require()
    nt = [6750, 1, 0, 300]
    R, nmax = len(nt), 7000
    perm = torch.full((R, nmax), -1, dtype=torch.int32, device="cuda")
    ntr = torch.tensor(nt, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    for key, shuf in ((0xDEADBEEF, 1), (17, 1), (5, 0)):
        C.shuffle_perm(perm.data_ptr(), nmax, ntr.data_ptr(), R, nmax, key, shuf, s.cuda_stream)
        got = perm.cpu().numpy()
        for r in range(R):
            np.testing.assert_array_equal(got[r], feistel_perm(nt[r], nmax, key, r, bool(shuf)))


@pytest.mark.gpu
def test_trainer_epochs_draw_new_orders():
    import torch
    from elephas_amd.models import Sequential, Dense
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.plan import build_plan
    m = Sequential()
    m.add(Dense(10, input_dim=8, activation="softmax"))
    m.compile(SGD(0.1), "categorical_crossentropy", ["acc"])
    t = NativeTrainer(m, build_plan(m), 2, 16, torch.device("cuda", 0), seed=3)
    rng = np.random.default_rng(0)
    x = rng.random((500, 8), dtype=np.float32)
    y = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 500)]
    t.set_data([x, x[:300]], [y, y[:300]], 0.1)
    orders = []
    for _ in range(3):
        t.begin_epoch()
        p = t._host(t.perm)
        assert sorted(p[0, :450].tolist()) == list(range(450))
        assert sorted(p[1, :270].tolist()) == list(range(270))
        assert p[1, 270:300].tolist() == list(range(270, 300))
        orders.append(p[0, :450].copy())
    assert not np.array_equal(orders[0], orders[1]) and not np.array_equal(orders[1], orders[2])
