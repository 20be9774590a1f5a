"""Wall time of the bench's timed region (run_steps_and_average of N steps + device sync) with
the host waiting by stream.synchronize() (blocking) or by spinning on an event query, in
alternation, same process:  python tools/sync_probe.py [steps] [reps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
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
    res = {"block": [], "spin": []}
    ev = torch.cuda.Event()
    for rep in range(reps):
        for mode in ("block", "spin"):
            t.begin_epoch()
            for _ in range(3):
                t.run_steps_and_average(1, None, 8)
            torch.cuda.synchronize()
            a = time.perf_counter()
            t.run_steps_and_average(steps, None, 8)
            b = time.perf_counter()
            if mode == "block":
                t.stream.synchronize()
            else:
                ev.record(t.stream)
                while not ev.query():
                    pass
            torch.cuda.synchronize()
            c = time.perf_counter()
            res[mode].append(((b - a) * 1e6, (c - a) * 1e6))
    for mode, v in res.items():
        v = np.array(v)
        print(f"{mode}: submit median {np.median(v[:, 0]):.1f} us, wall median {np.median(v[:, 1]):.1f} us "
              f"({np.median(v[:, 1]) / steps:.2f} us/step), first {v[0, 1]:.0f}, min {v[:, 1].min():.1f}")
    t.check()


if __name__ == "__main__":
    main()
