// Latency microbenchmarks on MI355X (gfx950): dependent global-load chains and
// kernel-to-kernel gaps in a hipGraph, timed with s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void chase(const unsigned* __restrict__ next, int steps, unsigned start, long long* out) {
  unsigned i = start;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < steps; ++s) i = __builtin_nontemporal_load(&next[i]) ^ 0u, i = next[i];
  long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}

__global__ void chase_plain(const unsigned* next, int steps, unsigned start, long long* out) {
  unsigned i = start;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < steps; ++s) i = next[i];
  long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}

__global__ void writer(unsigned* buf, int n, unsigned salt) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) buf[i] = buf[i] ^ salt ^ salt;
}

__global__ void stamp_kernel(long long* st, int k) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    st[2 * k] = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) st[2 * k + 1] = __builtin_amdgcn_s_memrealtime();
}

int main() {
  const int steps = 64;
  long long* dout; CK(hipMalloc(&dout, 64));
  long long hout[2];
  auto run_chase = [&](const char* name, unsigned* d, unsigned start, int pre_write, int n) {
    std::vector<double> v;
    for (int rep = 0; rep < 5; ++rep) {
      if (pre_write) { hipLaunchKernelGGL(writer, dim3(256), dim3(256), 0, 0, d, n, 12345u); }
      hipLaunchKernelGGL(chase_plain, dim3(1), dim3(64), 0, 0, d, steps, start, dout);
      CK(hipMemcpy(hout, dout, 16, hipMemcpyDeviceToHost));
      v.push_back(hout[0] * 10.0 / steps);
    }
    std::sort(v.begin(), v.end());
    printf("%-48s %8.1f ns/load (median of 5)\n", name, v[2]);
  };
  // small ring (L2 resident after first lap): 64 entries spaced 256 B
  {
    const int n = 1 << 14;
    std::vector<unsigned> h(n);
    for (int i = 0; i < 64; ++i) h[i * 64] = ((i + 1) % 64) * 64;
    unsigned* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    run_chase("ring 64 lines (L2 hot after lap 1)", d, 0, 0, n);
    run_chase("ring 64 lines, rewritten by previous kernel", d, 0, 1, n);
    CK(hipFree(d));
  }
  // large random ring (HBM): 1 GiB, 4096-B stride random permutation
  {
    const long long n = 1ll << 28;
    const int nodes = 1 << 16;
    std::vector<unsigned> perm(nodes);
    for (int i = 0; i < nodes; ++i) perm[i] = i;
    srand(1);
    for (int i = nodes - 1; i > 0; --i) std::swap(perm[i], perm[rand() % (i + 1)]);
    std::vector<unsigned> h(n, 0);
    const unsigned stride = (unsigned)(n / nodes);
    for (int i = 0; i < nodes; ++i) h[(size_t)perm[i] * stride] = perm[(i + 1) % nodes] * stride;
    unsigned* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    run_chase("random 1 GiB ring (HBM / MALL miss)", d, perm[0] * stride, 0, 0);
    CK(hipFree(d));
  }
  // kernel-to-kernel gaps: 20 tiny kernels, eager and in a hipGraph
  {
    const int K = 20;
    long long* st; CK(hipMalloc(&st, 2 * K * 8));
    std::vector<long long> hs(2 * K);
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int mode = 0; mode < 2; ++mode) {
      hipGraph_t g; hipGraphExec_t ge;
      if (mode == 1) {
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        for (int k = 0; k < K; ++k) hipLaunchKernelGGL(stamp_kernel, dim3(256), dim3(256), 0, s, st, k);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      }
      std::vector<double> gaps;
      for (int rep = 0; rep < 5; ++rep) {
        if (mode == 0) for (int k = 0; k < K; ++k) hipLaunchKernelGGL(stamp_kernel, dim3(256), dim3(256), 0, s, st, k);
        else CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(hs.data(), st, 2 * K * 8, hipMemcpyDeviceToHost));
        for (int k = 1; k < K; ++k) gaps.push_back((hs[2 * k] - hs[2 * k - 1]) * 10.0);
      }
      std::sort(gaps.begin(), gaps.end());
      printf("%-48s %8.1f ns (median), p10 %.0f p90 %.0f\n", mode ? "kernel gap in hipGraph (256 blocks)" : "kernel gap eager (256 blocks)",
             gaps[gaps.size() / 2], gaps[gaps.size() / 10], gaps[gaps.size() * 9 / 10]);
    }
  }
  return 0;
}
