"""Eager-path localisation: the grad path (forward_backward -> G -> apply) of ONE replica
(R = 1, no exchange) and the fused fit path (R = 4 independent replicas) on the sync test's
data vs torch per replica, per layer, after 1 step."""
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
    if len(sys.argv) > 1:
        hidden = tuple(int(v) for v in sys.argv[1].split(","))
    model = _mlp(in_dim, list(hidden), out)
    model.compile(O.SGD(0.05), "categorical_crossentropy", ["acc"])
    like = model.get_weights()
    R, steps = 4, 5
    xs, ys = _shards([B * steps] * R, in_dim, out, seed=13)

    def layer_err(w, wt, w0):
        return np.round([float(np.abs(a - b).max() / (np.abs(b - c).max() + 1e-30)) for a, b, c in
                         zip(unflatten_weights(w, like), unflatten_weights(wt, like), unflatten_weights(w0, like))],
                        6).tolist()

    ref = TorchTrainer(model, build_plan(model), R, B, torch.device("cuda"))
    w0 = ref.get_weights_flat()[0].copy()
    ref.set_data(xs, ys, 0.0, shuffle=False)
    ref.train_steps(1)
    wt = ref.get_weights_flat()
    for env in ("-1", "0"):
        os.environ["ELEPHAS_AMD_ROWCHAIN"] = env
        # grad path, one replica per trainer (replica r's data)
        errs = []
        for r in range(R):
            t = NativeTrainer(model, build_plan(model), 1, B, torch.device("cuda"), seed=5, persist=0)
            t.set_data([xs[r]], [ys[r]], 0.0, shuffle=False)
            t.begin_epoch()
            t.run_steps_allreduce(1, lambda G: None)
            errs.append(layer_err(t.get_weights_flat()[0], wt[r], w0))
        print(f"rowchain={env} grad path R=1 {t.plan_name()[:30]!r}: per replica per-layer err {errs}", flush=True)
        t = NativeTrainer(model, build_plan(model), R, B, torch.device("cuda"), seed=5, persist=0)
        t.set_data(xs, ys, 0.0, shuffle=False)
        t.begin_epoch()
        t.run_steps(1)
        w = t.get_weights_flat()
        print(f"rowchain={env} fused fit path R=4 {t.plan_name()[:30]!r}: "
              f"{[layer_err(w[r], wt[r], w0) for r in range(R)]}", flush=True)
        t = NativeTrainer(model, build_plan(model), R, B, torch.device("cuda"), seed=5, persist=0)
        t.set_data(xs, ys, 0.0, shuffle=False)
        t.begin_epoch()
        t.run_steps_allreduce(1, lambda G: None)
        w = t.get_weights_flat()
        print(f"rowchain={env} grad path R=4 no exchange: {[layer_err(w[r], wt[r], w0) for r in range(R)]}",
              flush=True)


if __name__ == "__main__":
    main()
