"""mixed_bfloat16 on the persistent V2 plan vs the bf16 row chain and both vs fp32: mean
|w - w_ref| / mean |w_ref - w0| after 2 epochs of the headline shape (diagnostics)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from elephas_amd.models import Sequential, Dense, Dropout, initializers
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    drop = float(sys.argv[1]) if len(sys.argv) > 1 else 0.2
    initializers.set_seed(15)
    m = Sequential([Dense(128, activation="relu", input_dim=784)] + ([Dropout(drop)] if drop else []) +
                   [Dense(128, activation="relu")] + ([Dropout(drop)] if drop else []) +
                   [Dense(10, activation="softmax")])
    m.compile(SGD(0.1), "categorical_crossentropy", ["acc"])
    rng = np.random.default_rng(19)
    xs = [rng.random((640, 784), dtype=np.float32) for _ in range(8)]
    ys = [np.eye(10, dtype=np.float32)[rng.integers(0, 10, 640)] for _ in range(8)]
    res = {}
    for name, persist, pol in (("v2_bf16", 1, "mixed_bfloat16"), ("rc_bf16", 0, "mixed_bfloat16"),
                               ("v2_f32", 1, "float32"), ("rc_f32", 0, "float32")):
        t = NativeTrainer(m, build_plan(m), 8, 64, torch.device("cuda"), seed=9, persist=persist,
                          rowchain=None if persist else 1, policy=pol)
        w0 = t.get_weights_flat()
        t.set_data(xs, ys, 0.1, shuffle=False)
        h = t.fit(2)
        res[name] = (t.get_weights_flat(), h[0]["loss"], t.plan_name()[:40])
    for a, b in (("v2_bf16", "rc_bf16"), ("v2_bf16", "v2_f32"), ("rc_bf16", "rc_f32"), ("v2_f32", "rc_f32")):
        wa, wb = res[a][0], res[b][0]
        print(f"dropout {drop} {a} vs {b}: rel {np.abs(wa - wb).mean() / np.abs(wb - w0).mean():.4f}  "
              f"loss {res[a][1]} vs {res[b][1]}")


if __name__ == "__main__":
    main()
