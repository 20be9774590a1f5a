// Cold-latency and grid-barrier microbenchmarks (gfx950), s_memrealtime = 100 MHz.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void chase(const unsigned* next, int steps, unsigned start, long long* out) {
  unsigned i = start;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < steps; ++s) i = next[i];
  long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}

// first-touch phases of a fresh kernel: kernarg pointer -> value -> dependent value
__global__ void first_touch(const long long* a, const long long* b, long long* out) {
  long long t0 = __builtin_amdgcn_s_memrealtime();
  long long v = a[0];
  long long t1 = __builtin_amdgcn_s_memrealtime() + (v & 0);  // use v
  asm volatile("" :: "s"(t1));
  long long w = b[v & 7];
  long long t2 = __builtin_amdgcn_s_memrealtime() + (w & 0);
  if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = t1 - t0; out[1] = t2 - t1; out[2] = w; }
}
__global__ void bump(long long* a, long long* b) { if (threadIdx.x == 0) { a[0] = (a[0] + 1) & 3; b[blockIdx.x & 7] += 1; } }

// grid barrier: every block arrives (atomicAdd) and spins on a generation word
__global__ void gridbar(unsigned* bar, int rounds, long long* out) {
  long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < rounds; ++r) {
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned gen = __hip_atomic_load(bar + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      unsigned prev = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == gridDim.x - 1) {
        __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(bar + 1, gen + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        while (__hip_atomic_load(bar + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen) __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
  }
  long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
}

int main() {
  long long* dout; CK(hipMalloc(&dout, 64));
  long long hout[4];
  // cold random chase over 4 GiB: 2^20 nodes at 4 KiB stride, a fresh segment per rep
  {
    const long long n = 1ll << 30;  // unsigned elements (4 GiB)
    const int nodes = 1 << 20;
    std::vector<unsigned> perm(nodes);
    for (int i = 0; i < nodes; ++i) perm[i] = i;
    srand(1);
    for (int i = nodes - 1; i > 0; --i) std::swap(perm[i], perm[rand() % (i + 1)]);
    unsigned* d; CK(hipMalloc(&d, n * 4));
    std::vector<unsigned> h(1 << 20);
    const long long stride = n / nodes;
    // build on device in pieces: next[perm[i]*stride] = perm[i+1]*stride
    CK(hipMemset(d, 0, n * 4));
    for (int i = 0; i < nodes; ++i) {
      unsigned v = (unsigned)(perm[(i + 1) % nodes] * stride);
      CK(hipMemcpy(d + (size_t)perm[i] * stride, &v, 4, hipMemcpyHostToDevice));
      if (i > 20000) break;  // only the first 20000 hops are used
    }
    // evict caches: touch 1 GiB elsewhere
    unsigned* junk; CK(hipMalloc(&junk, 1ll << 30)); CK(hipMemset(junk, 1, 1ll << 30));
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, 256, (unsigned)(perm[rep * 1000] * stride), dout);
      CK(hipMemcpy(hout, dout, 16, hipMemcpyDeviceToHost));
      printf("cold 4GiB random chase rep %d: %.1f ns/load\n", rep, hout[0] * 10.0 / 256);
    }
    CK(hipFree(junk)); CK(hipFree(d));
  }
  // first touch in a fresh kernel after another kernel wrote the data
  {
    long long *a, *b; CK(hipMalloc(&a, 64)); CK(hipMalloc(&b, 4096)); CK(hipMemset(a, 0, 64)); CK(hipMemset(b, 0, 4096));
    std::vector<double> x, y;
    for (int rep = 0; rep < 9; ++rep) {
      hipLaunchKernelGGL(bump, dim3(64), dim3(64), 0, 0, a, b);
      hipLaunchKernelGGL(first_touch, dim3(64), dim3(256), 0, 0, a, b, dout);
      CK(hipMemcpy(hout, dout, 24, hipMemcpyDeviceToHost));
      x.push_back(hout[0] * 10.0); y.push_back(hout[1] * 10.0);
    }
    std::sort(x.begin(), x.end()); std::sort(y.begin(), y.end());
    printf("first load after writer kernel: %.0f ns; dependent second load: %.0f ns (medians)\n", x[4], y[4]);
  }
  // grid barrier cost for 64 / 256 / 512 blocks
  for (int nb : {8, 64, 256, 512}) {
    unsigned* bar; CK(hipMalloc(&bar, 64)); CK(hipMemset(bar, 0, 64));
    std::vector<double> v;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(gridbar, dim3(nb), dim3(256), 0, 0, bar, 100, dout);
      CK(hipMemcpy(hout, dout, 8, hipMemcpyDeviceToHost));
      v.push_back(hout[0] * 10.0 / 100);
    }
    std::sort(v.begin(), v.end());
    printf("grid barrier, %d blocks: %.0f ns per barrier (median)\n", nb, v[2]);
    CK(hipFree(bar));
  }
  return 0;
}
