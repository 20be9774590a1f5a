// wave128_regs.hip plus the two-half LDS epilogue (acc of the second half live
// across the first half's epilogue): 36 B of scratch with this trivial epilogue; with
// the fused Dense epilogues and block setup of gemm_big.h the 4-wave kernel spilled
// ~1.2 KB -- the accumulators around the epilogue (profiles/README.md).
#include <hip/hip_runtime.h>
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <int OFF> __device__ __forceinline__ void rd(u32x4& v, unsigned a) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
}
__device__ __forceinline__ void mma(f32x4& c, const u32x4& a, const u32x4& b) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <int I> struct IC { static constexpr int v = I; };
__device__ __forceinline__ void glds16(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
__global__ __launch_bounds__(256) void k(float* out, int ns, const __bf16* const* rows, int K) {
  extern __shared__ char sm[];
  const unsigned base = (unsigned)(size_t)((__attribute__((address_space(3))) char*)sm) + threadIdx.x * 16;
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  u32x4 fa[2][8], fb[2][8];
  typedef unsigned long long u64;
  u64 bs[8];
  unsigned mov = 0;
  for (int u = 0; u < 8; ++u) { bs[u] = (u64)rows[threadIdx.x * 8 + u]; mov |= bs[u] ? 1u << u : 0u; }
  const int c8 = ((threadIdx.x & 3) ^ ((threadIdx.x >> 4) & 3)) * 8;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto stage1 = [&](int s, int u) {
    const int kk = s * 32 + c8;
    const u64 a = bs[u] + (((mov >> u) & 1u) ? (u64)kk * 2u : 0u);
    char* d = sm + (s % 4) * 32768 + (u >> 2) * 16384 + (wave * 4 + (u & 3)) * 1024;
    glds16((const void*)(kk < K ? a : (u64)rows), d);
  };
  auto rdall = [&](unsigned sb, u32x4 (&a)[8], u32x4 (&b)[8]) {
    rd<0>(a[0], sb); rd<1024>(a[1], sb); rd<2048>(a[2], sb); rd<3072>(a[3], sb);
    rd<4096>(a[4], sb); rd<5120>(a[5], sb); rd<6144>(a[6], sb); rd<7168>(a[7], sb);
    rd<8192>(b[0], sb); rd<9216>(b[1], sb); rd<10240>(b[2], sb); rd<11264>(b[3], sb);
    rd<12288>(b[4], sb); rd<13312>(b[5], sb); rd<14336>(b[6], sb); rd<15360>(b[7], sb);
  };
  rdall(base, fa[0], fb[0]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  auto body = [&](int t, u32x4 (&ca)[8], u32x4 (&cb)[8], u32x4 (&na)[8], u32x4 (&nb)[8]) {
    rdall(base + (unsigned)((t & 3) * 32768), na, nb);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      stage1(t + 4, i);
#pragma unroll
      for (int j = 0; j < 8; ++j) mma(acc[i][j], ca[i], cb[j]);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  for (int t = 0; t < ns; t += 2) {
    body(t, fa[0], fb[0], fa[1], fb[1]);
    body(t + 1, fa[1], fb[1], fa[0], fb[0]);
  }
  float* smf = reinterpret_cast<float*>(sm);
  const int wm = (threadIdx.x >> 6) >> 1, wn = (threadIdx.x >> 6) & 1, g = (threadIdx.x & 63) >> 4, i16 = threadIdx.x & 15;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) smf[(i * 16 + g * 4 + q) * 260 + wn * 128 + j * 16 + i16] = acc[i][j][q];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 128 * 256; e += 256) out[h * 32768 + e] = smf[(e / 256) * 260 + e % 256];
    __syncthreads();
  }
}
