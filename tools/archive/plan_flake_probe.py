"""Determinism probe for the row-chain vs grouped comparison (tests/test_native_gpu.py
_plan_case): repeats the bf16 / fp32 MNIST cases in one process and prints the error
metric of every repetition, plus whether each plan's weights are bit-identical across
repetitions (a race would show as run-to-run variation)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_native_gpu as T  # noqa: E402
from elephas_amd.models.layers import clear_session  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
LR = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
for case, policy in (("mnist_bf16_dropout", "mixed_bfloat16"), ("mnist_f32_dropout", "float32")):
    first = {}
    errs, rel, var = [], [], {0: 0, 1: 0}
    for i in range(reps):
        clear_session()
        from elephas_amd.models import initializers
        initializers.set_seed(100 + i)
        rng = np.random.default_rng(11)
        model = T._mlp(784, [128, 128], 10, dropout=0.2)
        from elephas_amd.models.optimizers import SGD
        model.compile(SGD(learning_rate=LR), "categorical_crossentropy", ["acc"])
        xs, ys = [], []
        for n in [300, 130, 40]:
            xs.append(rng.random((n, 784), dtype=np.float32))
            ys.append(np.eye(10, dtype=np.float32)[rng.integers(0, 10, n)])
        w0 = np.concatenate([w.reshape(-1) for w in model.get_weights()])
        _, wf, _ = T._fit_weights(model, policy, 64, xs, ys, rowchain=1, epochs=2, val=0.1)
        _, wg, _ = T._fit_weights(model, policy, 64, xs, ys, rowchain=0, epochs=2, val=0.1)
        _, wf2, _ = T._fit_weights(model, policy, 64, xs, ys, rowchain=1, epochs=2, val=0.1)
        _, wg2, _ = T._fit_weights(model, policy, 64, xs, ys, rowchain=0, epochs=2, val=0.1)
        var[1] += int(not np.array_equal(wf, wf2))   # same init, same plan: must be bit-identical
        var[0] += int(not np.array_equal(wg, wg2))
        errs.append(float(np.abs(wf - wg).mean() / np.abs(wg - w0).mean()))
        rel.append(float(np.abs(wf - wg).mean() / np.abs(wg).mean()))
    print(case, "errs", [f"{e:.1e}" for e in errs])
    print(case, "gap / mean |w| (test bound 2^-9 = 1.95e-3): max", max(rel))
    print(case, "err min/max", min(errs), max(errs), "repeat mismatches (race): rowchain", var[1],
          "grouped", var[0], flush=True)
