"""Host-side cost of the bench's timed region at the driver shape (MNIST 784-128-128-10,
8 workers x 64, 20 steps + the fit averaging): how long run_steps / average_replicas take
to return on the host, how long the device works (events), and the wall the bench would
time (barrier-free: synchronize, t0, run, average, synchronize).

  python tools/host_overhead.py [steps] [reps]
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
    import bench
    from elephas_amd import config
    from elephas_amd.ops.plan import build_plan
    from elephas_amd.ops.native_engine import NativeTrainer
    config.set_policy("float32")
    m = bench.build_model("mnist")
    R, B = 8, 64
    t = NativeTrainer(m, build_plan(m), R, B, torch.device("cuda"), seed=1)
    rng = np.random.default_rng(0)
    xs = [rng.random((7500, 784), dtype=np.float32) for _ in range(R)]
    ys = [np.eye(10, dtype=np.float32)[rng.integers(0, 10, 7500)] for _ in range(R)]
    t.set_data(xs, ys, 0.0)
    print("plan", t.plan_name())
    t.begin_epoch()
    t.run_steps(50)
    t.average_replicas(None, R)
    torch.cuda.synchronize()
    rows = {k: [] for k in ("submit_run", "submit_avg", "sync_wait", "wall", "gpu_chunk", "gpu_total")}
    for i in range(reps):
        if (i + 1) * steps > 100:
            t.begin_epoch()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        torch.cuda.synchronize()
        a = time.perf_counter()
        e0.record(t.stream)
        t.run_steps(steps)
        e1.record(t.stream)
        b = time.perf_counter()
        t.average_replicas(None, R)
        e2.record(t.stream)
        c = time.perf_counter()
        t.stream.synchronize()
        torch.cuda.synchronize()
        d = time.perf_counter()
        rows["submit_run"].append((b - a) * 1e6)
        rows["submit_avg"].append((c - b) * 1e6)
        rows["sync_wait"].append((d - c) * 1e6)
        rows["wall"].append((d - a) * 1e6)
        rows["gpu_chunk"].append(e0.elapsed_time(e1) * 1e3)
        rows["gpu_total"].append(e0.elapsed_time(e2) * 1e3)
    for k, v in rows.items():
        print(f"{k:11s} median {np.median(v):8.1f} us  min {np.min(v):8.1f}  max {np.max(v):8.1f}")
    print(f"per step: wall {np.median(rows['wall']) / steps:.2f} us, device chunk {np.median(rows['gpu_chunk']) / steps:.2f} us")


if __name__ == "__main__":
    main()
