"""Localise the eager per-step sync deviation (row-chain plan, 4 layers, B 128): per-layer
weight error vs the stacked torch model after 1..5 steps, for the eager path and the
in-launch path; also the eager path on ONE replica (no exchange) vs torch on that replica."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    from test_deep_gpu import _mlp, _shards
    from elephas_amd import config
    from elephas_amd.models import initializers, optimizers as O
    from elephas_amd.ops.plan import build_plan, unflatten_weights
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.torch_engine import TorchTrainer
    config.set_policy("float32")
    initializers.set_seed(12)
    in_dim, hidden, out, B = 93, (256, 256, 128), 9, 128
    model = _mlp(in_dim, list(hidden), out)
    model.compile(O.SGD(0.05), "categorical_crossentropy", ["acc"])
    like = model.get_weights()
    R, steps = 4, 5
    xs, ys = _shards([B * steps] * R, in_dim, out, seed=13)
    xc = np.concatenate([np.concatenate([x[i * B:(i + 1) * B] for x in xs]) for i in range(steps)])
    yc = np.concatenate([np.concatenate([y[i * B:(i + 1) * B] for y in ys]) for i in range(steps)])

    def layer_err(w, wt, w0):
        out = []
        for a, b, c in zip(unflatten_weights(w, like), unflatten_weights(wt, like), unflatten_weights(w0, like)):
            out.append(float(np.abs(a - b).max() / (np.abs(b - c).max() + 1e-30)))
        return np.round(out, 6).tolist()

    for nst in (1, 2, 5):
        ref = TorchTrainer(model, build_plan(model), 1, R * B, torch.device("cuda"))
        w0 = ref.get_weights_flat()[0].copy()
        ref.set_data([xc], [yc], 0.0, shuffle=False)
        ref.begin_epoch() if hasattr(ref, "begin_epoch") else None
        ref.train_steps(nst)
        wt = ref.get_weights_flat()[0]
        for label, persist, env in (("eager", 0, "-1"), ("eager_norc", 0, "0"), ("in-launch", 1, "-1")):
            os.environ["ELEPHAS_AMD_ROWCHAIN"] = env
            os.environ["ELEPHAS_AMD_DEEP"] = "2"
            t = NativeTrainer(model, build_plan(model), R, B, torch.device("cuda"), seed=5, persist=persist, sync=True)
            t.set_data(xs, ys, 0.0, shuffle=False)
            t.begin_epoch()
            t.run_steps(nst)
            t.check()
            w = t.get_weights_flat()
            print(f"steps {nst} {label:10s} {t.plan_name()[:40]!r} per-layer err {layer_err(w[0], wt, w0)}", flush=True)


if __name__ == "__main__":
    main()
