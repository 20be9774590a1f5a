"""Wide predict timeline probe: predict with a fresh output array vs a reused (already
faulted-in) one, and the native pipeline call alone, 16,384 rows, bf16 policy."""
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

config.set_policy("mixed_bfloat16")
m = bench.build_model("wide")
t = NativeTrainer(m, build_plan(m), 1, 1024, torch.device("cuda"))
rows = 16384
x = np.random.default_rng(0).random((rows, 4096), dtype=np.float32)


def ms(f, n=5):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return f"{np.median(ts):.2f} ms (min {min(ts):.2f})"


out = np.empty((rows, t.n_out), np.float32)
out[:] = 0


def reuse():
    t._enter()
    t._eval_pipeline(x, None, True, 0, out)
    t._exit()


def fresh_alloc():
    o = np.empty((rows, t.n_out), np.float32)
    return o


def fresh_touch():
    o = np.empty((rows, t.n_out), np.float32)
    o[::1024] = 0
    o[:] = 1
    return o


print("predict (fresh out)", ms(lambda: t.predict(x)), flush=True)
print("pipeline into a reused out", ms(reuse), flush=True)
print("predict again (pooled, prefaulted outputs)", ms(lambda: t.predict(x)), flush=True)
print("np.empty + full write of 65 MB", ms(fresh_touch), flush=True)
cr = torch.cuda.cudart()
o = np.empty((rows, t.n_out), np.float32)
t0 = time.perf_counter()
cr.cudaHostRegister(o.ctypes.data, o.nbytes, 0)
print(f"hipHostRegister of a fresh 65 MB array {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
cr.cudaHostUnregister(o.ctypes.data)
for th in (1, 4):
    os.environ["ELEPHAS_AMD_LOADER_THREADS"] = str(th)
for k in ("predict_only_x_upload",):
    buf = t._eval_buffers(rows, False, True)
    h2d, _ = t._copy_streams()

    def up():
        t._upload_rows(buf["X"][:rows], x, h2d)
        h2d.synchronize()
    print("upload alone", ms(up), flush=True)
