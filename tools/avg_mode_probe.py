"""Host-side timing of the bench's timed region (run_steps_and_average of 20 steps + sync)
with the averaging as a separate kernel (ELEPHAS_AMD_FUSED_AVG=0) or in the chunk's post node
(default): median submit time (host returns) and wall time to the stream's completion.

  python tools/avg_mode_probe.py [steps] [reps] [modes]     (modes: "02" = both, interleaved)
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    modes = sys.argv[3] if len(sys.argv) > 3 else "02"
    import bench
    from elephas_amd import config
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy("float32")
    m = bench.build_model("mnist")
    t = NativeTrainer(m, build_plan(m), 8, 64, torch.device("cuda"), seed=4321)
    rng = np.random.default_rng(0)
    xs = [rng.random((7500, 784), dtype=np.float32) for _ in range(8)]
    ys = [np.eye(10, dtype=np.float32)[rng.integers(0, 10, 7500)] for _ in range(8)]
    t.set_data(xs, ys, 0.1, shuffle=True)
    print("plan", t.plan_name())
    res = {}
    for rep in range(reps):
        for mode in modes:
            os.environ["ELEPHAS_AMD_FUSED_AVG"] = mode
            t.begin_epoch()
            t.run_steps_and_average(5, None, 8)
            t.stream.synchronize()
            torch.cuda.synchronize()
            a = time.perf_counter()
            t.run_steps_and_average(steps, None, 8)
            b = time.perf_counter()
            t.stream.synchronize()
            torch.cuda.synchronize()
            c = time.perf_counter()
            res.setdefault(mode, []).append(((b - a) * 1e6, (c - a) * 1e6))
    for mode, v in res.items():
        v = np.array(v)
        print(f"FUSED_AVG={mode}: submit median {np.median(v[:, 0]):.1f} us, wall median {np.median(v[:, 1]):.1f} us "
              f"({np.median(v[:, 1]) / steps:.2f} us/step), min wall {v[:, 1].min():.1f}; walls in order "
              + " ".join(f"{w:.0f}" for w in v[:8, 1]))
    t.check()


if __name__ == "__main__":
    main()
