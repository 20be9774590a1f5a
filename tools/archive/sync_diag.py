"""Per-step sync (eager exchange, persist=0) vs one stacked-batch fp32 torch model on a
4-layer shape, under the multi-launch plans (tail chain / grouped) -- which plan deviates."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from elephas_amd import config
    from elephas_amd.models import initializers, Sequential, Dense, Activation
    from elephas_amd.models.optimizers import SGD
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    from elephas_amd.ops.torch_engine import TorchTrainer
    config.set_policy("float32")
    dims = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "93,256,256,128,9").split(",")]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    R, steps = 4, 5
    initializers.set_seed(12)
    m = Sequential()
    m.add(Dense(dims[1], input_dim=dims[0]))
    m.add(Activation("relu"))
    for d in dims[2:-1]:
        m.add(Dense(d, activation="relu"))
    m.add(Dense(dims[-1], activation="softmax"))
    m.compile(SGD(0.05), "categorical_crossentropy", ["acc"])
    rng = np.random.default_rng(13)
    xs = [rng.random((B * steps, dims[0]), dtype=np.float32) for _ in range(R)]
    ys = [np.eye(dims[-1], dtype=np.float32)[rng.integers(0, dims[-1], B * steps)] for _ in range(R)]
    xc = np.concatenate([np.concatenate([x[i * B:(i + 1) * B] for x in xs]) for i in range(steps)])
    yc = np.concatenate([np.concatenate([y[i * B:(i + 1) * B] for y in ys]) for i in range(steps)])
    ref = TorchTrainer(m, build_plan(m), 1, R * B, torch.device("cuda"))
    w0 = ref.get_weights_flat()[0].copy()
    ref.set_data([xc], [yc], 0.0, shuffle=False)
    ref.fit(2)
    wt = ref.get_weights_flat()[0]
    step = np.abs(wt - w0).max()
    for label, env in (("deep in-launch", {"ELEPHAS_AMD_DEEP": "2"}), ("eager tail", {"ELEPHAS_AMD_TAIL": "1"}),
                       ("eager grouped", {"ELEPHAS_AMD_TAIL": "0"}), ("eager default", {})):
        saved = {k: os.environ.get(k) for k in ("ELEPHAS_AMD_DEEP", "ELEPHAS_AMD_TAIL")}
        for k in saved:
            os.environ.pop(k, None)
        os.environ.update(env)
        persist = 1 if "deep" in label else 0
        t = NativeTrainer(m, build_plan(m), R, B, torch.device("cuda"), seed=5, persist=persist, sync=True)
        t.set_data(xs, ys, 0.0, shuffle=False)
        t.fit(2)
        w = t.get_weights_flat()
        same = all(np.array_equal(w[r], w[0]) for r in range(R))
        print(f"{label:15s} plan={t.plan_name()[:60]!r} replicas identical={same} "
              f"err vs stacked torch={np.abs(w[0] - wt).max() / step:.2e}", flush=True)
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v


if __name__ == "__main__":
    main()
