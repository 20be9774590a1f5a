"""In-kernel phase stamps for each launch of one training step (diagnostics)."""
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from elephas_amd import config
from elephas_amd.ops.plan import build_plan
from elephas_amd.ops.native_engine import NativeTrainer
# usage: stamps.py [replicas] [model] [batch] [policy]
config.set_policy(sys.argv[4] if len(sys.argv) > 4 else "float32")
MODEL = sys.argv[2] if len(sys.argv) > 2 else "mnist"
BATCH = int(sys.argv[3]) if len(sys.argv) > 3 else 64
m = bench.build_model(MODEL)
R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
t = NativeTrainer(m, build_plan(m), R, BATCH, torch.device("cuda"))
rng = np.random.default_rng(0)
din, dout = bench.MODELS[MODEL][0][0], bench.MODELS[MODEL][2]
xs = [rng.random((7500, din), dtype=np.float32) for _ in range(R)]
ys = [np.eye(dout, dtype=np.float32)[rng.integers(0, dout, 7500)] for _ in range(R)]
t.set_data(xs, ys, 0.1)
t.begin_epoch()
t.run_steps(30)
t.begin_epoch()   # the stamped launches run step 0 of an epoch (no skipped updates)
blocks = t.exe.launch_blocks()
buf = torch.zeros(max(blocks) * 16, dtype=torch.int64, device="cuda")
t.exe.set_stamps(buf.data_ptr())
names = ["start", "setup", "mainloop", "reduce", "end", "e5", "e6", "e7", "e8"]
cfgs = t.exe.launch_cfgs()
for rep in range(2):
    for i, nb in enumerate(blocks):
        if cfgs[i] == -1:  # row chain: stamps 0..15 per block (rowchain.hip rstamp)
            buf.zero_()
            torch.cuda.synchronize()
            t.exe.train_launch(i, t.s)
            t.stream.synchronize()
            st = buf[:nb * 16].view(nb, 16).cpu().numpy().astype(np.int64)
            if rep == 1:
                t0 = st[:, 0].min()
                rel = np.where(st > 0, (st - t0) * 10.0, np.nan)
                med = np.nanmedian(rel, axis=0)
                print(f"launch {i} row chain blocks {nb}: median(ns) " +
                      " ".join(f"{k}:{v:.0f}" for k, v in enumerate(med) if v == v), flush=True)
            continue
        buf.zero_()
        torch.cuda.synchronize()
        t.exe.train_launch(i, t.s)
        t.stream.synchronize()
        st = buf[:nb * 16].view(nb, 16)[:, :9].cpu().numpy().astype(np.int64)
        t0 = st[:, 0].min()
        rel = np.where(st > 0, (st - t0) * 10.0, np.nan)  # ns
        med = np.nanmedian(rel, axis=0)
        mx = np.nanmax(rel, axis=0)
        clk = buf[:nb * 16].view(nb, 16).cpu().numpy().astype(np.int64)
        ok = (clk[:, 11] > 0) & (clk[:, 10] > 0)
        mhz = np.median((clk[ok, 11] - clk[ok, 10]) / ((clk[ok, 4] - clk[ok, 0]) * 10e-3))
        if rep == 1:
            print(f"  est. s_memtime MHz {mhz:.0f}", flush=True)
            print(f"launch {i} blocks {nb}: median(ns) " + " ".join(f"{n}={v:.0f}" for n, v in zip(names, med)) +
                  f" | max end {mx[4]:.0f} | start spread {mx[0]:.0f}", flush=True)
            begins = list(t.exe.table_begins(i)) if hasattr(t.exe, "table_begins") else []
            for pi, b0 in enumerate(begins):
                b1 = begins[pi + 1] if pi + 1 < len(begins) else nb
                sub = rel[b0:b1]
                print(f"    problem {pi} blocks [{b0},{b1}): median " +
                      " ".join(f"{n}={v:.0f}" for n, v in zip(names, np.nanmedian(sub, axis=0))) +
                      f" | p90 end {np.nanpercentile(sub[:, 4], 90):.0f} max end {np.nanmax(sub[:, 4]):.0f}", flush=True)
t.exe.set_stamps(0)
