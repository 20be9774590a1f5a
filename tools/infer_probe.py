"""Where does predict time go? MNIST fp32 (65536 rows) and Wide bf16 (16384 rows):
whole predict, the H2D upload alone (one loader call), the eval kernels alone on
resident rows, and the host pack alone (loader into a host-visible buffer is not
possible, so: upload with 1 vs default packing threads)."""
import math
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


def ms(f, n=5):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


pin = torch.empty(256 << 20, dtype=torch.uint8, pin_memory=True)
devb = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
t_dma = ms(lambda: devb.copy_(pin, non_blocking=True))
t_d2h = ms(lambda: pin.copy_(devb, non_blocking=True))
print(f"raw pinned DMA 256 MB: H2D {0.268 / t_dma * 1e3:.1f} GB/s, D2H {0.268 / t_d2h * 1e3:.1f} GB/s", flush=True)
del pin, devb
try:
    cr = torch.cuda.cudart()
    big = np.random.default_rng(1).random((65536, 784), dtype=np.float32)
    t0 = time.perf_counter()
    cr.cudaHostRegister(big.ctypes.data, big.nbytes, 0)
    t1 = time.perf_counter()
    cr.cudaHostUnregister(big.ctypes.data)
    t2 = time.perf_counter()
    print(f"hipHostRegister of {big.nbytes / 1e6:.0f} MB: {1e3 * (t1 - t0):.2f} ms (unregister {1e3 * (t2 - t1):.2f} ms)",
          flush=True)
except Exception as e:  # noqa: BLE001
    print("host register probe failed:", repr(e))

for name, policy, rows in (("mnist", "float32", 65536), ("wide", "mixed_bfloat16", 16384)):
    config.set_policy(policy)
    m = bench.build_model(name)
    t = NativeTrainer(m, build_plan(m), 1, 64 if name == "mnist" else 1024, torch.device("cuda"))
    din = bench.MODELS[name][0][0]
    x = np.random.default_rng(0).random((rows, din), dtype=np.float32)
    buf = t._eval_buffers(rows, False, True)
    h2d, _ = t._copy_streams()
    exe = t._eval_exe()
    vst = torch.zeros(1, dtype=torch.int32, device="cuda")
    vcn = torch.full((1,), rows, dtype=torch.int32, device="cuda")
    src = dict(X=buf["X"].data_ptr(), sX=0, ldx=t.Kp0, vstart=vst.data_ptr(), vcount=vcn.data_ptr(),
               acc=t.acc_val.data_ptr(), pred=buf["pred"].data_ptr(), sPred=0, ldp=t.n_out)
    nch = math.ceil(rows / t.eval_B)

    def upload():
        t._upload_rows(buf["X"][:rows], x, h2d)
        h2d.synchronize()

    def kernels():
        for c in range(nch):
            exe.eval_chunk(c, src, t.s)
        t.stream.synchronize()

    def d2h():
        buf["host"][:rows].copy_(buf["pred"][:rows], non_blocking=True)
        torch.cuda.synchronize()

    res = dict(predict=ms(lambda: t.predict(x)), upload=ms(upload), kernels=ms(kernels), d2h=ms(d2h))
    gb = x.nbytes / (2 if policy == "mixed_bfloat16" else 1) / 1e9
    print(f"{name} {policy} rows {rows}: " + ", ".join(f"{k} {v:.2f} ms" for k, v in res.items()) +
          f" | upload {gb / res['upload'] * 1e3:.1f} GB/s over PCIe | predict {rows / res['predict'] / 1e3:.2f} M rows/s"
          f" | loader threads {t.loader.threads}", flush=True)
