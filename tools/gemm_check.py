"""Quick numerics check of the native NT GEMM against torch fp32 (GPU only)."""
import importlib.util, sys, os, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, 'elephas_amd', '_C.cpython-310-x86_64-linux-gnu.so')
print("module:", SO, flush=True)
spec = importlib.util.spec_from_file_location('_C', SO)
C = importlib.util.module_from_spec(spec); spec.loader.exec_module(C)
dev = 'cuda'
torch.manual_seed(0)
ok = True
for (M, N, K) in [(64, 128, 784), (64, 10, 128), (785, 128, 64), (300, 200, 136), (1024, 1024, 1024), (513, 770, 264), (4097, 4096, 1024)]:
    for bf16 in (1, 0):
        for cfg in ((0, 1, 4) if bf16 else (0, 1)):
            dt = torch.bfloat16 if bf16 else torch.float32
            A = torch.randn(M, K, device=dev).to(dt)
            BT = torch.randn(N, K, device=dev).to(dt)
            Cm = torch.zeros(M, N, device=dev)
            s = torch.cuda.current_stream().cuda_stream
            C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, bf16, cfg, s)
            torch.cuda.synchronize()
            ref = A.float() @ BT.float().t()
            err = (Cm - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
            print(f"M={M} N={N} K={K} bf16={bf16} cfg={cfg} relerr={err:.2e}", flush=True)
            if err > 1e-2:
                ok = False
            if bf16 and N % 8 == 0:   # bf16 C: the fp32 result rounded once
                Cb = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
                C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cb.data_ptr(), M, N, K, K, K, N, bf16, cfg, s, 0, 1)
                torch.cuda.synchronize()
                ok &= bool(torch.equal(Cb, Cm.to(torch.bfloat16)))
# split-K entry (PK_PARTIAL slabs + one slab-sum launch): numerics
for (M, N, K, ks) in [(1024, 1000, 4096, 4), (300, 200, 136, 2), (513, 770, 1000, 3)]:
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    BT = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for cfg in (1, 2):
        Cm = torch.zeros(M, N, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, 1, cfg, s, 0, 0, ks)
        torch.cuda.synchronize()
        ref = A.float() @ BT.float().t()
        err = (Cm - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        print(f"M={M} N={N} K={K} bf16=1 cfg={cfg} splitk={ks} relerr={err:.2e}", flush=True)
        if err > 1e-2:
            ok = False
# timing of the wide-MLP shapes: FWD/DX (M=batch 1024) and DW (K=batch)
s = torch.cuda.current_stream().cuda_stream
for (M, N, K) in [(4096, 4096, 4096), (1024, 4096, 4096), (4096, 4096, 1024), (1024, 1000, 4096)]:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    BT = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    Cm = torch.zeros(M, N, device=dev)
    Cb = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    res = []
    # "4b": the 256x256 tile writing bf16 C, as hipBLASLt's bf16 matmul does (fp32 C doubles
    # the epilogue's HBM writes)
    # "2k4" / "1k2": the split-K entry (4 / 2 slabs on the 128x64 / 128x128 tile, + slab sum)
    for cfg in (1, 2, 4, "4b", "2k4", "2k2", "1k2", "torch"):
        def f():
            if cfg == "torch":
                torch.matmul(A, BT.t())
            elif isinstance(cfg, str) and "k" in cfg:
                c, ks = (int(v) for v in cfg.split("k"))
                C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, 1, c, s, 0, 0, ks)
            elif cfg == "4b":
                C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cb.data_ptr(), M, N, K, K, K, N, 1, 4, s, 0, 1)
            else:
                C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, 1, cfg, s)
        # steady state: a 10-call warm-up (clocks, caches), then the best of 3 rounds of 20
        for _ in range(10): f()
        dt = 1e9
        for _ in range(3):
            torch.cuda.synchronize(); t = time.time()
            for _ in range(20): f()
            torch.cuda.synchronize(); dt = min(dt, (time.time() - t) / 20)
        res.append(f"{cfg}: {dt*1e6:.0f} us {2*M*N*K/dt/1e12:.0f} TF")
    print(f"M={M} N={N} K={K} bf16 random:", " | ".join(res), flush=True)
print("OK" if ok else "FAIL")
sys.exit(0 if ok else 1)
