"""Do executors on separate HIP streams of ONE process overlap on the GPU?
MNIST fp32, 8 workers split into G executors (R = 8 / G) on G streams; every group
replays its own graphs. Prints us per step of all 8 workers for G = 1, 2, 4, 8.
Usage: stream_probe.py [G ...]  (env ELEPHAS_AMD_PERSIST / GPU_MAX_HW_QUEUES apply)"""
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
ROWS = 40000   # >= 576 steps of 64 rows: no epoch rollover inside the run
xs = [rng.random((ROWS, 784), dtype=np.float32) for _ in range(8)]
ys = [np.eye(10, dtype=np.float32)[rng.integers(0, 10, ROWS)] for _ in range(8)]
Gs = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
graph = os.environ.get("PROBE_GRAPH", "1") == "1"
def run_g(G):
    ts = []
    for g in range(G):
        lo, hi = 8 * g // G, 8 * (g + 1) // G
        t = NativeTrainer(m, plan, hi - lo, 64, torch.device("cuda"), seed=5 + g)
        t.set_data(xs[lo:hi], ys[lo:hi], 0.0, shuffle=True)
        t.begin_epoch()
        t.prepare_graphs()
        ts.append(t)
    for t in ts:
        t.run_steps(64, use_graph=graph)
    torch.cuda.synchronize()
    n = 512
    t0 = time.perf_counter()
    for c in range(n // 64):
        for t in ts:
            t.run_steps(64, use_graph=graph)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e6
    for t in ts:
        t.check()
    print(f"G={G} R={8 // G} graph={graph} plan={ts[0].plan_name()[:40]}: {dt:.1f} us per step of all 8 workers",
          flush=True)


for G in Gs:
    try:
        run_g(G)
    except RuntimeError as e:
        print(f"G={G}: FAILED {e}", flush=True)
        break
