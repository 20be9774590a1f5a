"""Which path is nondeterministic? Repeat grouped and fused fits of the same
config in ONE process and report per-replica max |dw| against the first run."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_native_gpu import _mlp, _fit_weights
from elephas_amd.models.optimizers import RMSprop, SGD
rng = np.random.default_rng(11)
case = sys.argv[1] if len(sys.argv) > 1 else "sparse"
if case == "sparse":
    model = _mlp(50, [96, 64], 7, dropout=0.3)
    model.compile(RMSprop(learning_rate=0.005), "sparse_categorical_crossentropy", ["acc"])
    B, d, k, sizes = 48, 50, 7, [250, 180]
    xs = [rng.random((n, d), dtype=np.float32) for n in sizes]
    ys = [rng.integers(0, k, (n, 1)).astype(np.float32) for n in sizes]
else:
    model = _mlp(784, [128, 128], 10, dropout=0.2)
    model.compile(SGD(learning_rate=0.1), "categorical_crossentropy", ["acc"])
    B, sizes = 64, [300, 130, 40]
    xs = [rng.random((n, 784), dtype=np.float32) for n in sizes]
    ys = [np.eye(10, dtype=np.float32)[rng.integers(0, 10, n)] for n in sizes]
from elephas_amd.ops import native
Cm = native.require()
NAN = 0x7FC07FC0
poison = os.environ.get("POISON", "")
if "alloc" in poison:   # poison the caching allocator's free blocks
    big = torch.full((1 << 28,), float("nan"), device="cuda"); del big
for fused in (0, 1):
    ref = None
    for rep in range(4):
        if "lds" in poison:
            Cm.poison_lds(NAN if rep % 2 else 0x3F803F80, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        _, w, _ = _fit_weights(model, "mixed_bfloat16", B, xs, ys, fused=fused, epochs=2, val=0.1)
        print(f"fused={fused} rep={rep} nan={bool(np.isnan(w).any())}", flush=True)
        if ref is None:
            ref = w
            continue
        print(f"fused={fused} rep={rep} per-replica max|dw| vs rep0:", [float(np.abs(w[r] - ref[r]).max()) for r in range(len(w))], flush=True)
