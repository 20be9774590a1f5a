"""Host port of the native engine's counter-based dropout masks (csrc/kernels/common.h
``dropout_base`` / ``dropout_u8`` and rowchain.hip ``dropout_u1``).

A keep-uniform is a pure function of (seed, replica, layer, optimizer iteration,
batch row, column): one murmur3 fmix32 per column pair gives two 16-bit uniforms
(u = h & 0xFFFF for even columns, h >> 16 for odd ones, scaled by 2^-16), and an
element is kept iff u >= rate (tf.nn.dropout semantics; kept values scaled by
1 / (1 - rate)). Forward and backward regenerate the same mask instead of storing
it. Batch rows must be < 65536 (the row occupies the hash input's high half).

The torch reference engine uses this port (``TorchTrainer(hash_dropout_seed=...)``)
so native-with-dropout can be checked against an fp32 autograd run drawing the
same masks (tests/test_native_gpu.py), and the keep statistics can be checked on
the host (tests/test_dropout_hash.py).
"""
from __future__ import annotations

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def fmix32(h):
    h = np.asarray(h, np.uint64) & M32
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & M32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & M32
    h ^= h >> np.uint64(16)
    return h


def dropout_base(seed: int, replica: int, layer: int, iteration: int) -> np.uint64:
    seed, it = int(seed) & 0xFFFFFFFFFFFFFFFF, int(iteration) & 0xFFFFFFFFFFFFFFFF
    inner = ((it & 0xFFFFFFFF) * 0x9E3779B1) & 0xFFFFFFFF
    inner ^= (it >> 32) & 0xFFFFFFFF
    inner ^= (int(layer) << 24) & 0xFFFFFFFF
    inner ^= (int(replica) * 0x27D4EB2F) & 0xFFFFFFFF
    inner ^= (seed >> 32) & 0xFFFFFFFF
    return fmix32(np.uint64((seed & 0xFFFFFFFF) ^ int(fmix32(np.uint64(inner)))))


def keep_uniforms(seed: int, replica: int, layer: int, iteration: int, rows: int, cols: int) -> np.ndarray:
    """[rows, cols] float32 uniforms in [0, 1) exactly as the kernels draw them."""
    if rows >= 65536:
        raise ValueError("dropout hash supports batch rows < 65536")
    base = dropout_base(seed, replica, layer, iteration)
    r = np.arange(rows, dtype=np.uint64)[:, None]
    c = np.arange(cols, dtype=np.uint64)[None, :]
    h = fmix32(base ^ ((r << np.uint64(16)) | (c >> np.uint64(1))))
    u = np.where((c & np.uint64(1)) == 1, h >> np.uint64(16), h & np.uint64(0xFFFF))
    return (u.astype(np.float32) * np.float32(1.0 / 65536.0)).astype(np.float32)


def keep_mask(seed: int, replica: int, layer: int, iteration: int, rows: int, cols: int, rate: float) -> np.ndarray:
    return keep_uniforms(seed, replica, layer, iteration, rows, cols) >= np.float32(rate)
