// Kernarg access latency (gfx950): a 1 KiB by-value struct whose fields are read
// in dependent order, one cache line apart; eager vs hipGraph launches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Big { long long v[128]; };  // 1 KiB = 16 lines

__global__ void kern(Big b, long long* out) {
  long long t[9];
  long long idx = 0;
  t[0] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    // dependent chain through kernarg lines: idx selects within the next line (0..7)
    long long x = b.v[(q + 1) * 16 - 16 + (idx & 7)];
    idx += x;
    asm volatile("" : "+s"(idx));
    t[q + 1] = __builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    for (int q = 0; q < 8; ++q) out[q] = t[q + 1] - t[q];
    out[8] = idx;
  }
}

int main() {
  Big b;
  for (int i = 0; i < 128; ++i) b.v[i] = 0;
  long long* d; CK(hipMalloc(&d, 128));
  long long h[9];
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int mode = 0; mode < 2; ++mode) {
    std::vector<double> per;
    hipGraphExec_t ge = nullptr;
    if (mode == 1) {
      hipGraph_t g;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
      hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, s, b, d);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    for (int rep = 0; rep < 7; ++rep) {
      if (mode == 0) hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, s, b, d);
      else CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(h, d, 72, hipMemcpyDeviceToHost));
      for (int q = 1; q < 8; ++q) per.push_back(h[q] * 10.0);
      if (rep == 6) { printf("%s last rep per-line:", mode ? "graph" : "eager"); for (int q = 0; q < 8; ++q) printf(" %lld", h[q] * 10); printf(" ns\n"); }
    }
    std::sort(per.begin(), per.end());
    printf("%s: dependent kernarg line access median %.0f ns\n", mode ? "graph" : "eager", per[per.size() / 2]);
  }
  return 0;
}
