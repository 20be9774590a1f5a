"""Where a GEMM launch's time goes, per workgroup, from the kernels' s_memrealtime stamps
(gemm_impl.h stamp(): 0 block start, 1 setup done, 2 main loop done, 3 epilogue start,
4 block end; 10 ns ticks): medians over the grid relative to the earliest block start,
for the 256x256 tile (cfg 4) and the THR tile (cfg 1) on the Wide / square shapes.

  python tools/gemm_stamps.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elephas_amd.ops import native  # noqa: E402

C = native.require()
dev = "cuda"
s = torch.cuda.current_stream().cuda_stream
for (M, N, K) in [(4096, 4096, 4096), (4096, 4096, 1024), (4097, 4096, 1024), (1024, 4096, 4096)]:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    BT = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Cm = torch.zeros(M, N, device=dev)
    Cb = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    for cfg, ob in ((4, 0), (4, 1), (1, 0)):
        out = Cb if ob else Cm
        tm, tn = C.tile_shape(cfg)
        nb = ((M + tm - 1) // tm) * ((N + tn - 1) // tn)
        st = torch.zeros(nb * 16, dtype=torch.int64, device=dev)
        for _ in range(3):
            C.gemm_nt(A.data_ptr(), BT.data_ptr(), out.data_ptr(), M, N, K, K, K, N, 1, cfg, s, 0, ob)
        torch.cuda.synchronize()
        C.gemm_nt(A.data_ptr(), BT.data_ptr(), out.data_ptr(), M, N, K, K, K, N, 1, cfg, s, st.data_ptr(), ob)
        torch.cuda.synchronize()
        v = st.view(nb, 16).cpu().numpy().astype(np.int64)
        t0 = v[:, 0].min()
        rel = (v[:, :5] - t0) / 100.0
        med = np.median(rel, axis=0)
        span = (v[:, 4].max() - t0) / 100.0
        setup = np.median(rel[:, 1] - rel[:, 0])
        loop = np.median(rel[:, 2] - rel[:, 1])
        epi = np.median(rel[:, 4] - rel[:, 2])
        print(f"M={M} N={N} K={K} cfg={cfg}{' bf16-out' if ob else ''} blocks={nb}: span {span:.1f} us; per block median setup {setup:.2f} "
              f"main loop {loop:.2f} epilogue {epi:.2f} us; start spread {np.median(rel[:, 0]):.2f}/"
              f"{rel[:, 0].max():.2f}; stamps {np.round(med, 2)}", flush=True)
