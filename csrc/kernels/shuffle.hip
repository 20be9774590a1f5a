// Per-epoch shuffle of every replica's training rows (reference: Keras
// `fit(shuffle=True)` inside elephas/worker.py:41-42 draws a fresh permutation of
// the partition each epoch).
//
// No sort: row i of replica r goes to position pi_r(i) where pi_r is a keyed
// Feistel bijection on the smallest even-bit power-of-two domain 2^(2h) >= n,
// cycle-walked until the image falls inside [0, n) (a bijection restricted to a
// subset by cycle walking is still a bijection of that subset; the domain is < 4n,
// so the expected walk is < 4 rounds of the network). Every element is computed
// independently: one launch of R * ceil(nmax / 256) workgroups, no LDS, no
// inter-workgroup traffic -- versus the radix sort of random keys it replaces
// (3-4 rocprim launches + torch rand/where/argsort/copy per epoch).
//
// Rows at or past ntrain[r] (the validation tail, padding) keep their position.
// tests/test_shuffle.py holds a numpy transcription of the same network and
// checks the kernel bit for bit.
#include "common.h"

namespace ea {

constexpr int SHUF_ROUNDS = 6;

__device__ __forceinline__ uint32_t feistel(uint32_t x, int h, uint32_t mask, uint32_t key) {
  uint32_t l = x >> h, r = x & mask;
#pragma unroll
  for (int q = 0; q < SHUF_ROUNDS; ++q) {
    const uint32_t f = fmix32(r ^ (key + 0x9E3779B9u * (uint32_t)(q + 1))) & mask;
    const uint32_t nl = r;
    r = l ^ f;
    l = nl;
  }
  return (l << h) | r;
}

__global__ __launch_bounds__(256) void shuffle_perm_kernel(int* __restrict__ perm, long long sPerm,
                                                           const int* __restrict__ ntrain, int nmax, uint32_t key,
                                                           int shuffle) {
  const int r = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nmax) return;
  const int n = ntrain[r];
  int out = i;
  if (shuffle && i < n && n > 1) {
    const int b = 32 - __builtin_clz((uint32_t)(n - 1));  // bits of n - 1
    const int h = (b + 1) >> 1;
    const uint32_t mask = (1u << h) - 1u;
    const uint32_t kr = fmix32(key ^ (0x85EBCA6Bu * (uint32_t)(r + 1)));
    uint32_t x = (uint32_t)i;
    do {
      x = feistel(x, h, mask, kr);
    } while (x >= (uint32_t)n);
    out = (int)x;
  }
  perm[(long long)r * sPerm + i] = out;
}

extern "C" hipError_t ea_shuffle_perm(int* perm, long long sPerm, const int* ntrain, int R, int nmax, uint32_t key,
                                      int shuffle, hipStream_t s) {
  if (R <= 0 || nmax <= 0) return hipSuccess;
  hipLaunchKernelGGL(shuffle_perm_kernel, dim3((nmax + 255) / 256, R), dim3(256), 0, s, perm, sPerm, ntrain, nmax,
                     key, shuffle);
  return hipGetLastError();
}

}  // namespace ea
