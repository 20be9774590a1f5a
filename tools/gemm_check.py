"""Quick numerics check of the native NT GEMM against torch fp32 (GPU only)."""
import importlib.util, sys, os, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location('_C', os.path.join(ROOT, 'elephas_amd', '_C.cpython-310-x86_64-linux-gnu.so'))
C = importlib.util.module_from_spec(spec); spec.loader.exec_module(C)
dev = 'cuda'
torch.manual_seed(0)
ok = True
for (M, N, K) in [(64, 128, 784), (64, 10, 128), (785, 128, 64), (300, 200, 136), (1024, 1024, 1024)]:
    for bf16 in (1, 0):
        for cfg in (0, 1):
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
# timing of the big one
M = N = K = 4096
A = torch.randn(M, K, device=dev).to(torch.bfloat16); BT = torch.randn(N, K, device=dev).to(torch.bfloat16)
Cm = torch.zeros(M, N, device=dev); s = torch.cuda.current_stream().cuda_stream
for cfg in (0, 1):
    for _ in range(3): C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, 1, cfg, s)
    torch.cuda.synchronize(); t = time.time()
    for _ in range(10): C.gemm_nt(A.data_ptr(), BT.data_ptr(), Cm.data_ptr(), M, N, K, K, K, N, 1, cfg, s)
    torch.cuda.synchronize(); dt = (time.time() - t) / 10
    print(f"4096^3 bf16 cfg={cfg}: {dt*1e3:.3f} ms  {2*M*N*K/dt/1e12:.1f} TFLOP/s", flush=True)
for _ in range(3): torch.matmul(A, BT.t())
torch.cuda.synchronize(); t = time.time()
for _ in range(10): torch.matmul(A, BT.t())
torch.cuda.synchronize(); dt = (time.time() - t) / 10
print(f"4096^3 bf16 torch.matmul (hipBLASLt): {dt*1e3:.3f} ms  {2*M*N*K/dt/1e12:.1f} TFLOP/s", flush=True)
print("OK" if ok else "FAIL")
sys.exit(0 if ok else 1)
