"""Statistics of the native engine's counter-based dropout masks (host port,
elephas_amd/ops/dropout_hash.py): keep rate, independence across the hash inputs,
and the 1/(1-p) scaling of the torch reference path that draws the same masks.
Reference dropout rates: tests/conftest.py:13,16 (0.2), Otto example (0.5)."""
import numpy as np
import pytest

from elephas_amd.ops import dropout_hash as H


@pytest.mark.parametrize("rate", [0.2, 0.5])
def test_keep_rate_within_3_sigma(rate):
    n = 0
    kept = 0
    for it in range(8):
        for layer in range(2):
            m = H.keep_mask(1234, 3, layer, it, 64, 128, rate)
            kept += int(m.sum())
            n += m.size
    p = 1.0 - rate
    sigma = np.sqrt(n * p * (1 - p))
    assert abs(kept - n * p) < 3 * sigma, (kept, n * p, sigma)


def test_masks_differ_across_hash_inputs():
    base = H.keep_mask(7, 0, 0, 0, 64, 128, 0.5)
    for other in (H.keep_mask(8, 0, 0, 0, 64, 128, 0.5), H.keep_mask(7, 1, 0, 0, 64, 128, 0.5),
                  H.keep_mask(7, 0, 1, 0, 64, 128, 0.5), H.keep_mask(7, 0, 0, 1, 64, 128, 0.5)):
        agree = float((base == other).mean())
        assert 0.4 < agree < 0.6, agree   # independent masks agree on ~half the elements
    np.testing.assert_array_equal(base, H.keep_mask(7, 0, 0, 0, 64, 128, 0.5))  # pure function


def test_uniforms_are_16_bit_grid_and_pairs_share_a_hash():
    u = H.keep_uniforms(99, 2, 1, 5, 16, 32)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert np.all(np.round(u * 65536) == u * 65536)
    # columns 2j and 2j+1 come from one fmix32: recompute one by hand
    base = H.dropout_base(99, 2, 1, 5)
    h = int(H.fmix32(np.uint64(int(base) ^ ((3 << 16) | 5))))
    assert u[3, 10] == np.float32((h & 0xFFFF) / 65536.0) and u[3, 11] == np.float32((h >> 16) / 65536.0)


def test_torch_hash_dropout_scales_kept_units():
    """The torch reference engine with hash masks: dropped units are exactly 0, kept
    units are scaled by 1 / (1 - rate) (inverted dropout)."""
    import torch
    from elephas_amd.models import Sequential, Dense, Dropout
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.torch_engine import TorchTrainer
    m = Sequential()
    m.add(Dense(32, activation="linear", input_dim=8, kernel_initializer="ones", bias_initializer="zeros"))
    m.add(Dropout(0.25))
    m.add(Dense(4, activation="softmax"))
    m.compile("sgd", "categorical_crossentropy")
    t = TorchTrainer(m, build_plan(m), 1, 16, hash_dropout_seed=11)
    x = torch.ones(16, 8)
    ps = t.params[0]
    h = x @ ps[0] + ps[1]   # 8.0 everywhere
    keep = H.keep_mask(11, 0, 0, 0, 16, 32, 0.25)
    expect = np.where(keep, 8.0 / 0.75, 0.0)
    # the dropout output is the second Dense's input: recover it through a probe weight
    with torch.no_grad():
        ps[2].copy_(torch.eye(32, 4))
        ps[3].zero_()
    _, logits = t.forward(0, x, True)
    np.testing.assert_allclose(logits.numpy(), expect[:, :4], rtol=1e-6)
