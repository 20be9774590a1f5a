"""Target program for PMC passes over the THR GEMM (cfg 1 = 128x128, cfg 2 = 128x64):
4096^3 and the wide-MLP forward shape, random bf16 operands, a few launches each."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elephas_amd.ops import native
C = native.require()
s = torch.cuda.current_stream().cuda_stream
for (M, N, K), cfg in [((4096, 4096, 4096), 1), ((1024, 4096, 4096), 2)]:
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    BT = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    out = torch.zeros(M, N, device="cuda")
    for _ in range(5):
        C.gemm_nt(A.data_ptr(), BT.data_ptr(), out.data_ptr(), M, N, K, K, K, N, 1, cfg, s)
    torch.cuda.synchronize()
print("done", flush=True)
