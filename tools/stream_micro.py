"""Do kernels on different HIP streams of one process run concurrently at all?
torch.cuda._sleep spin kernels (one workgroup each) on S streams, eager and inside
per-stream hipGraphs; prints the wall time relative to one stream doing 1/S of the work."""
import time

import torch

CYC = 200000   # ~80 us per kernel
K = 32         # kernels per stream


def run(S, graph):
    streams = [torch.cuda.Stream() for _ in range(S)]
    graphs = []
    if graph:
        for s in streams:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(K):
                    torch.cuda._sleep(CYC)
            graphs.append(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, s in enumerate(streams):
        with torch.cuda.stream(s):
            if graph:
                graphs[i].replay()
            else:
                for _ in range(K):
                    torch.cuda._sleep(CYC)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


run(1, False)
base = run(1, False)
print(f"1 stream: {K} kernels {base * 1e3:.2f} ms ({base / K * 1e6:.1f} us each)", flush=True)
for graph in (False, True):
    for S in (2, 4, 8):
        run(S, graph)
        dt = run(S, graph)
        print(f"{S} streams graph={graph}: {dt * 1e3:.2f} ms = {dt / base:.2f}x one stream "
              f"(1.00 = fully concurrent, {S:.2f} = serialised)", flush=True)
