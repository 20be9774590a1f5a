"""Same-process A/B of the 256x256 tile's production launch (cfg 4) and the variant
launcher (cfg 5 / 6 / 7), interleaved A B A B ... with per-config best and median over
rounds -- so order, clocks and L2 state do not favour either side."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elephas_amd.ops import native  # noqa: E402

C = native.require()
dev = "cuda"
s = torch.cuda.current_stream().cuda_stream
cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "4,7,5").split(",")]
for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 8192), (4096, 4096, 1024)]:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    BT = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Cb = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    n = 10 if M < 8192 else 4
    res = {c: [] for c in cfgs}
    for rnd in range(6):
        order = cfgs if rnd % 2 == 0 else cfgs[::-1]
        for cfg in order:
            for _ in range(2):
                C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cb.data_ptr(), M, N, K, K, K, N, 1, cfg, s, 0, 1)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(n):
                C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cb.data_ptr(), M, N, K, K, K, N, 1, cfg, s, 0, 1)
            torch.cuda.synchronize()
            res[cfg].append((time.perf_counter() - t) / n)
    print(f"M={M} N={N} K={K} bf16 C:", " | ".join(
        f"cfg {c}: best {2 * M * N * K / min(v) / 1e12:.0f} TF median {2 * M * N * K / np.median(v) / 1e12:.0f} TF"
        for c, v in res.items()), flush=True)
