"""Throughput of E concurrent executors (streams) splitting R replicas (diagnostics):
each launch of the small-MLP step is latency-bound and fills few CUs, so
independent replica groups on separate streams can overlap on the GPU."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from elephas_amd import config
from elephas_amd.ops.plan import build_plan
from elephas_amd.ops.native_engine import NativeTrainer

config.set_policy("mixed_bfloat16")
MODEL = sys.argv[1] if len(sys.argv) > 1 else "mnist"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
din, dout = bench.MODELS[MODEL][0][0], bench.MODELS[MODEL][2]
rng = np.random.default_rng(0)
for R, E in [(8, 1), (8, 2), (8, 4), (8, 8), (16, 1), (16, 2), (16, 4)]:
    m = bench.build_model(MODEL)
    ts = [NativeTrainer(m, build_plan(m), R // E, B, torch.device("cuda")) for _ in range(E)]
    for t in ts:
        xs = [rng.random((6000, din), dtype=np.float32) for _ in range(R // E)]
        ys = [np.eye(dout, dtype=np.float32)[rng.integers(0, dout, 6000)] for _ in range(R // E)]
        t.set_data(xs, ys, 0.0)
        t.begin_epoch()
        t.run_steps(32)
    torch.cuda.synchronize()
    K = 64  # steps per epoch = 93; stay inside one epoch
    for t in ts:
        t.begin_epoch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(4):
        for t in ts:
            t.run_steps(K // 4)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{MODEL} R={R} E={E}: {dt / K * 1e6:.1f} us/step  {R * B * K / dt / 1e6:.2f} M samples/s", flush=True)
