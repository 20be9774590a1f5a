"""Diagnosis: the Otto-shape layer-pipeline fit vs the tail-chain plan, per replica and
history key (tests/test_deep_gpu.py::test_deep_otto_shape_matches_tail_chain_plan), with
the XCD-local instance on and off (ELEPHAS_AMD_PERSIST_LOCAL)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    from test_deep_gpu import _mlp, _shards, _native
    from elephas_amd.models import initializers
    from elephas_amd.models.optimizers import SGD
    initializers.set_seed(2024)
    model = _mlp(93, [512, 512, 512], 9, dropout=0.5)
    model.compile(SGD(learning_rate=0.01), "categorical_crossentropy", ["acc"])
    xs, ys = _shards([1000] * 7 + [450], 93, 9, seed=11)
    out = {}
    os.environ["ELEPHAS_AMD_DEEP"] = "-1"
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    runs = [(f"deep_local{i}", -1, "-1") for i in range(reps)] + [(f"deep_wt{i}", -1, "0") for i in range(reps)]
    for name, persist, local in runs + [("tail", 0, "0")]:
        os.environ["ELEPHAS_AMD_PERSIST_LOCAL"] = local
        t = _native(model, 8, 128, seed=7, persist=persist)
        print(name, t.plan_name()[:90])
        t.set_data(xs, ys, 0.15, shuffle=True)
        torch.manual_seed(5)
        h = t.fit(2)
        t.check()
        out[name] = (t.get_weights_flat(), h)
    for name, _, _ in runs:
        w, h = out[name]
        wr, hr = out["tail"]
        print(name, "weights max diff", float(np.abs(w - wr).max()))
        for r, (a, b) in enumerate(zip(h, hr)):
            for key in a:
                d = np.abs(np.asarray(a[key]) - np.asarray(b[key]))
                if d.max() > 5e-4:
                    print(f"  replica {r} {key}: {a[key]} vs {b[key]}")
        print(f"  {name}: per-replica loss epoch 1", [round(float(hh['loss'][0]), 4) for hh in h])


if __name__ == "__main__":
    main()
