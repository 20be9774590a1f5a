"""Do independent executors on separate HIP streams of ONE process overlap on the GPU?
MNIST fp32, 8 workers: one executor (R=8) vs two (R=4 each) on two streams, hipGraph
and eager launches. Prints us per step."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from elephas_amd import config  # noqa: E402
from elephas_amd.ops.native_engine import NativeTrainer  # noqa: E402
from elephas_amd.ops.plan import build_plan  # noqa: E402

config.set_policy("float32")
m = bench.build_model("mnist")
plan = build_plan(m)
rng = np.random.default_rng(0)
xs = [rng.random((7500, 784), dtype=np.float32) for _ in range(8)]
ys = [np.eye(10, dtype=np.float32)[rng.integers(0, 10, 7500)] for _ in range(8)]


def make(G):
    ts = []
    for g in range(G):
        lo, hi = 8 * g // G, 8 * (g + 1) // G
        t = NativeTrainer(m, plan, hi - lo, 64, torch.device("cuda"), seed=5 + g)
        t.set_data(xs[lo:hi], ys[lo:hi], 0.0, shuffle=True)
        t.begin_epoch()
        ts.append(t)
    return ts


for G in (1, 2, 4):
    for graph in (True, False):
        ts = make(G)
        for t in ts:
            t.run_steps(32, use_graph=graph)
        torch.cuda.synchronize()
        n = 96
        t0 = time.perf_counter()
        for c in range(n // 16):
            for t in ts:
                t.run_steps(16, use_graph=graph)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n * 1e6
        print(f"G={G} graph={graph}: {dt:.1f} us per step of all 8 workers", flush=True)
