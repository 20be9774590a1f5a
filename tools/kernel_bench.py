"""Per-kernel timing of the grouped GEMM in isolation (run under rocprofv3)."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elephas_amd.ops import native
C = native.require()
dev = 'cuda'
s = torch.cuda.current_stream().cuda_stream
for (M, N, K) in [(64, 128, 128), (64, 128, 784), (785, 128, 64), (64, 32, 128)]:
    for bf16 in (1, 0):
        dt = torch.bfloat16 if bf16 else torch.float32
        A = torch.randn(M, K, device=dev).to(dt); BT = torch.randn(N, K, device=dev).to(dt)
        Cm = torch.zeros(M, N, device=dev)
        for _ in range(20):
            C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, bf16, 0, s)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(200):
            C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, bf16, 0, s)
        torch.cuda.synchronize()
        print(f"plain M={M} N={N} K={K} bf16={bf16}: {(time.perf_counter()-t)/200*1e6:.1f} us/launch (eager)", flush=True)
# empty torch op for reference
x = torch.zeros(16, device=dev)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(200): x.add_(1)
torch.cuda.synchronize(); print(f"torch add_: {(time.perf_counter()-t)/200*1e6:.1f} us/launch", flush=True)
