"""Schedule variants of the 8-phase 256x256 tile (gemm_big.h V): cfg 4 = the production
schedule (V1: A copies one phase earlier), 5 = V5 (V6 with the fragment-read wait behind the
barrier), 6 = V6 (copies in the MFMA ticks), 7 = V0 (the round-3 schedule). Checks them
against torch and times all (one order: use tools/big_ab.py for A/B)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elephas_amd.ops import native  # noqa: E402

C = native.require()
dev = "cuda"
s = torch.cuda.current_stream().cuda_stream
torch.manual_seed(0)
ok = True
for (M, N, K) in [(1024, 1024, 1024), (513, 770, 264), (4097, 4096, 1024)]:
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    BT = torch.randn(N, K, device=dev).to(torch.bfloat16)
    ref = A.float() @ BT.float().t()
    for cfg in (4, 5, 6, 7):
        Cm = torch.zeros(M, N, device=dev)
        C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, 1, cfg, s)
        torch.cuda.synchronize()
        err = (Cm - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        print(f"M={M} N={N} K={K} cfg={cfg} relerr={err:.2e}", flush=True)
        ok &= err < 1e-2
for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 8192), (4096, 4096, 1024), (1024, 4096, 4096)]:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    BT = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Cm = torch.zeros(M, N, device=dev)
    res = []
    for cfg in (1, 4, 5, 6, 7, "torch"):
        def f():
            if cfg == "torch":
                torch.matmul(A, BT.t())
            else:
                C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, 1, cfg, s)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t = time.perf_counter()
        n = 10 if M < 8192 else 4
        for _ in range(n):
            f()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / n
        res.append(f"{cfg}: {dt * 1e6:.0f} us {2 * M * N * K / dt / 1e12:.0f} TF")
    print(f"M={M} N={N} K={K}:", " | ".join(res), flush=True)
print("OK" if ok else "FAIL")
sys.exit(0 if ok else 1)
