"""Timing of the 256x256 GEMM tile (cfg 4) against the THR tiles and hipBLASLt on
the 4096^3 / 8192^3 / Wide-MLP shapes (random bf16, numerics checked)."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elephas_amd.ops import native
C = native.require()
s = torch.cuda.current_stream().cuda_stream
v = os.environ.get("ELEPHAS_AMD_BIG_V", "0")
cfgs = [4] if v != "0" else [1, 2, 4, "torch"]
for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 8192), (4097, 4096, 1024), (1024, 4096, 4096)]:
    torch.manual_seed(0)
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    BT = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    out = torch.zeros(M, N, device="cuda")
    ref = None
    res = []
    for cfg in cfgs:
        def f():
            if cfg == "torch":
                torch.matmul(A, BT.t())
            else:
                C.gemm_nt(A.data_ptr(), BT.data_ptr(), out.data_ptr(), M, N, K, K, K, N, 1, cfg, s)
        f(); torch.cuda.synchronize()
        if cfg == 4 and M <= 4097:
            ref = A.float() @ BT.float().t()
            err = ((out - ref).abs().max() / ref.abs().max()).item()
            res.append(f"err {err:.1e}")
        n = 10 if M >= 8192 else 30
        torch.cuda.synchronize(); t = time.time()
        for _ in range(n): f()
        torch.cuda.synchronize(); dt = (time.time() - t) / n
        res.append(f"{cfg}: {dt*1e6:.0f} us {2*M*N*K/dt/1e12:.0f} TF")
    print(f"V={v} {M}x{N}x{K}:", " | ".join(res), flush=True)

