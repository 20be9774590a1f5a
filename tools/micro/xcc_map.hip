// Block -> XCD placement of a grid on MI355X (gfx950): how often does block b run on XCD
// b % 8 (HW_REG_XCC_ID)?  Idle GPU, and while a spinning kernel occupies part of the CUs on
// another stream.  The XCD-local persistent instance (persist.hip EA_PLOCAL) relies on it
// and checks it in every launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)); }

__global__ void probe(unsigned* out, int threads_busy_ns) {
  if (threadIdx.x == 0) out[blockIdx.x] = xcc_id() | (__smid() << 8);
  if (threads_busy_ns > 0) {
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < threads_busy_ns / 10) __builtin_amdgcn_s_sleep(1);
  }
}

__global__ void spin(int ticks) {
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

// blocks whose XCD differs from block b % 8's (the round-robin may start on any XCD)
static int mismatches(const std::vector<unsigned>& h, int n, int* first) {
  int bad = 0;
  *first = -1;
  for (int b = 0; b < n; ++b)
    if ((h[b] & 0xff) != (h[b % 8] & 0xff)) {
      if (*first < 0) *first = b;
      ++bad;
    }
  return bad;
}

int main() {
  unsigned* d;
  CK(hipMalloc(&d, 4096 * 4));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  std::vector<unsigned> h(4096);
  for (int n : {64, 256, 1024}) {
    for (int busy : {0, 50000}) {
      int tot = 0, first = -1;
      for (int rep = 0; rep < 20; ++rep) {
        hipLaunchKernelGGL(probe, dim3(n), dim3(256), 0, s1, d, busy);
        CK(hipStreamSynchronize(s1));
        CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
        int f;
        const int m = mismatches(h, n, &f);
        tot += m;
        if (m && first < 0) first = f;
      }
      printf("idle GPU          grid %4d, blocks held %5d ns: %6d of %d blocks off their b %% 8 class (first at %d)\n", n, busy, tot,
             20 * n, first);
    }
  }
  // with a kernel of k blocks spinning 2 ms on another stream, launched first
  for (int k : {1, 13, 100, 200}) {
    for (int n : {256}) {
      int tot = 0, first = -1, bad_reps = 0;
      for (int rep = 0; rep < 20; ++rep) {
        hipLaunchKernelGGL(spin, dim3(k), dim3(64), 0, s2, 200000);
        hipLaunchKernelGGL(probe, dim3(n), dim3(256), 0, s1, d, 50000);
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
        CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
        int f;
        const int m = mismatches(h, n, &f);
        tot += m;
        bad_reps += m > 0;
        if (rep == 0) {
          printf("  rep 0: xcc of blocks 0..11:");
          for (int b = 0; b < 12; ++b) printf(" %u", h[b] & 0xff);
          printf("\n");
        }
        if (m && first < 0) {
          first = f;
          printf("  e.g. rep %d: xcc of blocks 0..23:", rep);
          for (int b = 0; b < 24; ++b) printf(" %u", h[b] & 0xff);
          printf("\n");
        }
      }
      printf("busy (%3d blocks spinning) grid %4d: %6d of %d blocks off their b %% 8 class in %d of 20 launches\n", k, n, tot, 20 * n,
             bad_reps);
    }
  }
  return 0;
}
