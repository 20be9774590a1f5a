"""The deep sync test's exact setup (tests/test_deep_gpu.py otto_like): the eager per-step
exchange run three times (bitwise repeatable?) and the in-launch one, each against the
stacked-batch torch model, per epoch."""
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
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.torch_engine import TorchTrainer
    config.set_policy("float32")
    initializers.set_seed(12)
    in_dim, hidden, out, B = 93, (256, 256, 128), 9, 128
    model = _mlp(in_dim, list(hidden), out)
    model.compile(O.SGD(0.05), "categorical_crossentropy", ["acc"])
    R, steps = 4, 5
    xs, ys = _shards([B * steps] * R, in_dim, out, seed=13)
    xc = np.concatenate([np.concatenate([x[i * B:(i + 1) * B] for x in xs]) for i in range(steps)])
    yc = np.concatenate([np.concatenate([y[i * B:(i + 1) * B] for y in ys]) for i in range(steps)])
    refs = []
    ref = TorchTrainer(model, build_plan(model), 1, R * B, torch.device("cuda"))
    w0 = ref.get_weights_flat()[0].copy()
    ref.set_data([xc], [yc], 0.0, shuffle=False)
    for ep in range(2):
        ref.fit(1)
        refs.append(ref.get_weights_flat()[0].copy())
    os.environ["ELEPHAS_AMD_DEEP"] = "2"
    for label, persist in (("eager#1", 0), ("in-launch", 1), ("eager#2", 0), ("eager#3", 0)):
        t = NativeTrainer(model, build_plan(model), R, B, torch.device("cuda"), seed=5, persist=persist, sync=True)
        t.set_data(xs, ys, 0.0, shuffle=False)
        errs = []
        for ep in range(2):
            t.fit(1)
            w = t.get_weights_flat()
            errs.append(float(np.abs(w[0] - refs[ep]).max() / np.abs(refs[ep] - w0).max()))
        same = all(np.array_equal(w[r], w[0]) for r in range(R))
        print(f"{label:10s} plan={t.plan_name()[:50]!r} identical={same} err/epoch={errs} "
              f"digest={hash(w[0].tobytes()) & 0xffffffff:08x}", flush=True)


if __name__ == "__main__":
    main()
