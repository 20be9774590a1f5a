"""Does an XCD's L2 keep lines across kernel boundaries? Run the row-chain launch
(B) several times back to back: if its weight/slab reads hit L2 after the first run,
phase 0 (stamp 1) and the forward (stamp 2) get shorter on the repeats."""
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from elephas_amd import config
from elephas_amd.ops.plan import build_plan
from elephas_amd.ops.native_engine import NativeTrainer
config.set_policy("float32")
m = bench.build_model("mnist")
R = 8
t = NativeTrainer(m, build_plan(m), R, 64, torch.device("cuda"))
rng = np.random.default_rng(0)
t.set_data([rng.random((7500, 784), dtype=np.float32) for _ in range(R)],
           [np.eye(10, dtype=np.float32)[rng.integers(0, 10, 7500)] for _ in range(R)], 0.1)
t.begin_epoch()
t.run_steps(30)
nb = t.exe.launch_blocks()[1]
buf = torch.zeros(max(t.exe.launch_blocks()) * 16, dtype=torch.int64, device="cuda")
t.exe.set_stamps(buf.data_ptr())
for trial in range(2):
    torch.cuda.synchronize()
    res = []
    for rep in range(4):
        buf.zero_()
        if rep == 0:
            t.exe.train_launch(2, t.s)      # DW launch: rewrites the weight images
            t.exe.train_launch(0, t.s)      # layer-0 slabs
        buf.zero_()
        t.exe.train_launch(1, t.s)
        t.stream.synchronize()
        st = buf[:nb * 16].view(nb, 16).cpu().numpy().astype(np.int64)
        t0 = st[:, 0].min()
        rel = np.where(st > 0, (st - t0) * 10.0, np.nan)
        med = np.nanmedian(rel, axis=0)
        res.append(" ".join(f"{k}:{v:.0f}" for k, v in enumerate(med[:16]) if v == v))
    for i, r_ in enumerate(res):
        print(f"trial {trial} rep {i}: {r_}", flush=True)
t.exe.set_stamps(0)
