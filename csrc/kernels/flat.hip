// Flat-buffer kernels over the packed parameter vector (Keras weight order,
// reference utils/functional_utils.py:6-43 and spark_model.py:221-227):
//   * fused optimizer apply after a gradient all-reduce (sync per-step DP path)
//   * shadow refresh (fp32 master -> compute-dtype W and W^T images)
//   * replica averaging (reference sync mode: theta <- theta0 - mean(delta_i))
//   * parameter-server updates (theta <- theta - delta; lock-free hogwild variant
//     with fp32 global atomics) and generic axpby.
// All loads/stores are 16-byte vectorised where the layout allows.
#include <type_traits>
#include "common.h"

namespace ea {

// Segment lookup with compile-time indices only (dynamic indexing of the
// kernarg segment table would make hipcc copy FlatArgs to scratch per lane).
struct SegV {
  long long p_off, wsh_off, ldwsh, wtsh_off, ldwtsh;
  int K, N;
};

__device__ __forceinline__ SegV find_seg(const FlatArgs& a, long long i) {
  SegV v{a.seg[0].p_off, a.seg[0].wsh_off, a.seg[0].ldwsh, a.seg[0].wtsh_off, a.seg[0].ldwtsh, a.seg[0].K, a.seg[0].N};
#pragma unroll
  for (int q = 1; q < MAX_SEG; ++q) {
    if (q < a.nseg && i >= a.seg[q].p_off) {
      v = SegV{a.seg[q].p_off, a.seg[q].wsh_off, a.seg[q].ldwsh, a.seg[q].wtsh_off, a.seg[q].ldwtsh, a.seg[q].K,
               a.seg[q].N};
    }
  }
  return v;
}

template <typename T>
__device__ __forceinline__ void write_shadow(const FlatArgs& a, int r, long long i, float w, long long par) {
  const SegV g = find_seg(a, i);
  const long long rel = i - g.p_off;
  if (rel < 0) return;
  if (rel >= (long long)g.K * g.N) return;  // bias: no image (read from the fp32 master)
  const long long k = rel / g.N, nn = rel % g.N;
  if (a.Wsh)
    reinterpret_cast<T*>(a.Wsh)[(long long)r * a.sWsh + par * a.wsh_par + g.wsh_off + k * g.ldwsh + nn] = from_f<T>(w);
  if (a.WTsh)
    reinterpret_cast<T*>(a.WTsh)[(long long)r * a.sWTsh + par * a.wtsh_par + g.wtsh_off + nn * g.ldwtsh + k] = from_f<T>(w);
}

// Move the step-counter base by n steps (one block; see GroupArgs::step_off).
__global__ __launch_bounds__(64) void advance_kernel(long long* ctr, const int* ntrain, int R, int B, int n) {
  const long long s0 = ctr[0];
  for (int r = threadIdx.x; r < R; r += 64) {
    const long long nb = ((long long)ntrain[r] + B - 1) / B;
    long long d = nb - s0;
    ctr[2 + r] += d < 0 ? 0 : (d > n ? n : d);
  }
  __syncthreads();
  if (threadIdx.x == 0) ctr[0] = s0 + n;
}

// After a persistent chunk (persist.hip): clear the launch's flag block for the next
// launch and advance the step counters -- one node instead of a flag memset ahead of
// the next launch plus advance_kernel (one block; the flag block is a few thousand words)
__device__ __forceinline__ void persist_post_block(unsigned* flags, int nflags, long long* ctr, const int* ntrain,
                                                   int R, int B, int n, const unsigned* err) {
  for (int e = threadIdx.x; e < nflags; e += 256) flags[e] = 0u;
  // a launch that gave up (sticky error word) did not run its steps: the counters stay
  // (the host re-plans and re-runs them, native_engine.py NativeTrainer.check)
  if (*err != 0u) return;
  const long long s0 = ctr[0];
  for (int r = threadIdx.x; r < R; r += 256) {
    const long long nb = ((long long)ntrain[r] + B - 1) / B;
    const long long d = nb - s0;
    ctr[2 + r] += d < 0 ? 0 : (d > n ? n : d);
  }
  __syncthreads();
  if (threadIdx.x == 0) ctr[0] = s0 + n;
}
__global__ __launch_bounds__(256) void persist_post_kernel(unsigned* flags, int nflags, long long* ctr, const int* ntrain,
                                                           int R, int B, int n, const unsigned* err) {
  persist_post_block(flags, nflags, ctr, ntrain, R, B, n, err);
}

// grid: total_blocks over R*n elements
template <typename T>
__global__ __launch_bounds__(256) void apply_update_kernel(FlatArgs a) {
  const long long total = (long long)a.R * a.n;
  const long long step = a.ctr[0];
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int r = (int)(e / a.n);
    const long long i = e % a.n;
    if ((long long)a.ntrain[r] - step * a.B <= 0) continue;  // replica has no batch this step
    const long long iter = a.ctr[2 + r];
    const float g = a.G[(long long)r * a.sG + i] * a.op.grad_scale;
    float* S = a.S ? a.S + (long long)r * a.sS : nullptr;
    const float w = opt_update(a.op, a.P[(long long)r * a.sP + i], g, S, i, iter);
    a.P[(long long)r * a.sP + i] = w;
    write_shadow<T>(a, r, i, w, (iter + 1) & 1);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void refresh_shadows_kernel(FlatArgs a) {
  const long long total = (long long)a.R * a.n;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int r = (int)(e / a.n);
    const long long i = e % a.n;
    const float w = a.P[(long long)r * a.sP + i];
    if (a.both_parities) {
      write_shadow<T>(a, r, i, w, 0);
      write_shadow<T>(a, r, i, w, 1);
    } else {
      write_shadow<T>(a, r, i, w, a.ctr[2 + r] & 1);
    }
  }
}

// ---- tiled shadow writers: one 64x64 tile of one layer's kernel [K][N] per
// block. P / G / S rows are read coalesced, the row-major W image is written
// coalesced, and W^T goes through an LDS transpose so its stores are coalesced
// too (the element-wise writer above scatters W^T with a stride of Kp elements:
// 0.82 ms for the 37.7 M-parameter wide MLP). UPDATE additionally applies the
// optimizer (per-step all-reduce path); bias rows ride with the k-tile 0 blocks.
struct TileV {
  long long p_off, wsh_off, ldwsh, wtsh_off, ldwtsh;
  int K, N, has_bias, tk, tn;
};

__device__ __forceinline__ TileV find_tile(const FlatArgs& a, int t, int& lt) {
  TileV v{};
  int base = 0;
  lt = t;
#pragma unroll
  for (int q = 0; q < MAX_SEG; ++q) {
    if (q < a.nseg) {
      const int tk = (a.seg[q].K + 63) / 64, tn = (a.seg[q].N + 63) / 64;
      if (t >= base) {
        v = TileV{a.seg[q].p_off, a.seg[q].wsh_off, a.seg[q].ldwsh, a.seg[q].wtsh_off, a.seg[q].ldwtsh,
                  a.seg[q].K, a.seg[q].N, a.seg[q].has_bias, tk, tn};
        lt = t - base;
      }
      base += tk * tn;
    }
  }
  return v;
}

template <typename T, bool UPDATE>
__global__ __launch_bounds__(256) void shadow_tiles_kernel(FlatArgs a, int tiles_per_replica) {
  __shared__ float tile[64][65];
  const int r = __builtin_amdgcn_readfirstlane(blockIdx.x % a.R);  // replica-minor (XCD affinity, gemm_impl.h)
  int lt;
  const TileV g = find_tile(a, __builtin_amdgcn_readfirstlane(blockIdx.x / a.R), lt);
  const int k0 = (lt / g.tn) * 64, n0 = (lt % g.tn) * 64;
  long long iter = a.ctr[2 + r];
  if (UPDATE && (long long)a.ntrain[r] - a.ctr[0] * a.B <= 0) return;  // replica has no batch this step
  const int p0 = UPDATE ? (int)((iter + 1) & 1) : (a.both_parities ? 0 : (int)(iter & 1));
  const int p1 = UPDATE ? p0 : (a.both_parities ? 1 : p0);
  float* P = a.P + (long long)r * a.sP;
  float* S = a.S ? a.S + (long long)r * a.sS : nullptr;
  const int tid = threadIdx.x, nn = tid & 63;
  T* W = a.Wsh ? reinterpret_cast<T*>(a.Wsh) + (long long)r * a.sWsh + g.wsh_off : nullptr;
  T* WT = a.WTsh ? reinterpret_cast<T*>(a.WTsh) + (long long)r * a.sWTsh + g.wtsh_off : nullptr;
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int kk = (tid >> 6) + 4 * i, k = k0 + kk, n = n0 + nn;
    float w = 0.f;
    if (k < g.K && n < g.N) {
      const long long pi = g.p_off + (long long)k * g.N + n;
      if (!UPDATE && a.src) {
        w = a.src[pi];
        P[pi] = w;
        if (r == 0 && a.src_copy) a.src_copy[pi] = w;
      } else {
        w = P[pi];
      }
      if (UPDATE) {
        w = opt_update(a.op, w, a.G[(long long)r * a.sG + pi] * a.op.grad_scale, S, pi, iter);
        P[pi] = w;
      }
      if (W) {
        W[p0 * a.wsh_par + (long long)k * g.ldwsh + n] = from_f<T>(w);
        if (p1 != p0) W[p1 * a.wsh_par + (long long)k * g.ldwsh + n] = from_f<T>(w);
      }
    }
    tile[kk][nn] = w;
  }
  if (k0 == 0 && g.has_bias && tid < 64 && n0 + tid < g.N) {
    const long long pi = g.p_off + (long long)g.K * g.N + n0 + tid;
    float w;
    if (!UPDATE && a.src) {
      w = a.src[pi];
      P[pi] = w;
      if (r == 0 && a.src_copy) a.src_copy[pi] = w;
    } else {
      w = P[pi];
    }
    if (UPDATE) {
      w = opt_update(a.op, w, a.G[(long long)r * a.sG + pi] * a.op.grad_scale, S, pi, iter);
      P[pi] = w;
    }
  }
  if (!WT) return;
  __syncthreads();
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int nl = (tid >> 6) + 4 * i, kl = tid & 63, k = k0 + kl, n = n0 + nl;
    if (k < g.K && n < g.N) {
      const T v = from_f<T>(tile[kl][nl]);
      WT[p0 * a.wtsh_par + (long long)n * g.ldwtsh + k] = v;
      if (p1 != p0) WT[p1 * a.wtsh_par + (long long)n * g.ldwtsh + k] = v;
    }
  }
}

static int shadow_tiles(const FlatArgs& a) {
  int t = 0;
  for (int q = 0; q < a.nseg; ++q) t += ((a.seg[q].K + 63) / 64) * ((a.seg[q].N + 63) / 64);
  return t;
}

// scale * sum over R replicas of P[r][i] (fp64 accumulation; scale 1/R = the mean);
// result written to every replica if write_back (and to out if given)
// theta <- scale * sum_r P_r: fp64 sums in replica order; every replica's loads of a chunk of
// 8 replicas are in flight together (the loop-carried sum otherwise serialised them: one
// memory latency per replica); VEC: 4 elements per lane (16-byte rows, n4 = n / 4 of them)
template <bool VEC>
__device__ __forceinline__ void replica_average_blocks(float* P, long long sP, int R, long long n, float* out,
                                                       int write_back, double scale, int blk, int nblk) {
  constexpr int W = VEC ? 4 : 1;
  using V = typename std::conditional<VEC, float4, float>::type;
  const long long nv = n / W;
  for (long long i = (long long)blk * 256 + threadIdx.x; i < nv; i += (long long)nblk * 256) {
    double s[W];
#pragma unroll
    for (int w = 0; w < W; ++w) s[w] = 0.0;
    for (int r0 = 0; r0 < R; r0 += 8) {
      V x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = r0 + k < R ? r0 + k : r0;
        x[k] = reinterpret_cast<const V*>(P + (long long)r * sP)[i];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (r0 + k >= R) break;
        const float* f = reinterpret_cast<const float*>(&x[k]);
#pragma unroll
        for (int w = 0; w < W; ++w) s[w] += f[w];
      }
    }
    V m;
    float* mf = reinterpret_cast<float*>(&m);
#pragma unroll
    for (int w = 0; w < W; ++w) mf[w] = (float)(s[w] * scale);
    if (out) reinterpret_cast<V*>(out)[i] = m;
    if (write_back)
      for (int r = 0; r < R; ++r) reinterpret_cast<V*>(P + (long long)r * sP)[i] = m;
  }
  if (VEC) {   // the n % 4 tail elements
    const long long t = nv * W + (long long)blk * 256 + threadIdx.x;
    if (t < n) {
      double s = 0.0;
      for (int r = 0; r < R; ++r) s += P[(long long)r * sP + t];
      const float m = (float)(s * scale);
      if (out) out[t] = m;
      if (write_back)
        for (int r = 0; r < R; ++r) P[(long long)r * sP + t] = m;
    }
  }
}
template <bool VEC>
__global__ __launch_bounds__(256) void replica_average_kernel(float* P, long long sP, int R, long long n,
                                                              float* out, int write_back, double scale) {
  replica_average_blocks<VEC>(P, sP, R, n, out, write_back, scale, blockIdx.x, gridDim.x);
}

// The post node of a persistent chunk that ends a fit (train-then-average, reference
// spark_model.py:217-228) with the replica averaging in the same launch: the last block
// clears the flags and advances the counters (persist_post_kernel), the others average.
// One kernel boundary fewer than post + replica_average (measured at the MNIST bench's
// 20-step shape: the post node 4.8 us, then 7.6 us to the average kernel's start).
template <bool VEC>
__global__ __launch_bounds__(256) void persist_post_average_kernel(unsigned* flags, int nflags, long long* ctr,
                                                                   const int* ntrain, int R, int B, int n,
                                                                   const unsigned* err, float* P, long long sP,
                                                                   long long np, float* out, int write_back,
                                                                   double scale) {
  if (blockIdx.x == gridDim.x - 1) {
    persist_post_block(flags, nflags, ctr, ntrain, R, B, n, err);
    return;
  }
  replica_average_blocks<VEC>(P, sP, R, np, out, write_back, scale, blockIdx.x, gridDim.x - 1);
}

// C[m][n] = sum over the ks split-K slabs S[k][m][n] (fp32, slab order): the reduction
// step of the split-K GEMM entry (gemm_nt splitk > 1); VEC: 4 columns per lane
template <bool VEC>
__global__ __launch_bounds__(256) void sum_slabs_kernel(const float* S, int ks, long long slab, int M, int N,
                                                        float* C, long long ldc) {
  constexpr int W = VEC ? 4 : 1;
  const int nw = N / W;
  const long long tot = (long long)M * nw;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < tot; e += (long long)gridDim.x * 256) {
    const int m = (int)(e / nw), c = (int)(e - (long long)m * nw) * W;
    if constexpr (VEC) {
      float4 acc = *reinterpret_cast<const float4*>(S + (long long)m * N + c);
      for (int k = 1; k < ks; ++k) {
        const float4 v = *reinterpret_cast<const float4*>(S + k * slab + (long long)m * N + c);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      *reinterpret_cast<float4*>(C + (long long)m * ldc + c) = acc;
    } else {
      float acc = S[(long long)m * N + c];
      for (int k = 1; k < ks; ++k) acc += S[k * slab + (long long)m * N + c];
      C[(long long)m * ldc + c] = acc;
    }
  }
}

// y = alpha*x + beta*y   (vectorised, n multiple handled with tail)
__global__ __launch_bounds__(256) void axpby_kernel(const float* x, float* y, long long n, float alpha, float beta) {
  const long long n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float4* y4 = reinterpret_cast<float4*>(y);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 a = x4[i], b = y4[i];
    y4[i] = make_float4(alpha * a.x + beta * b.x, alpha * a.y + beta * b.y, alpha * a.z + beta * b.z,
                        alpha * a.w + beta * b.w);
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    y[i] = alpha * x[i] + beta * y[i];
}

// parameter server apply: p -= scale * delta  (plain RMW: serialised by the
// caller's lock in 'asynchronous' mode, racy by design in 'hogwild' mode)
__global__ __launch_bounds__(256) void ps_sub_kernel(float* p, const float* d, long long n, float scale) {
  const long long n4 = n / 4;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* d4 = reinterpret_cast<const float4*>(d);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 a = p4[i], b = d4[i];
    p4[i] = make_float4(a.x - scale * b.x, a.y - scale * b.y, a.z - scale * b.z, a.w - scale * b.w);
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    p[i] -= scale * d[i];
}

// lock-free hogwild apply with fp32 global atomics: no update is lost, order is arbitrary
__global__ __launch_bounds__(256) void ps_sub_atomic_kernel(float* p, const float* d, long long n, float scale) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    atomicAdd(p + i, -scale * d[i]);
}

// delta = a - b
__global__ __launch_bounds__(256) void sub_kernel(const float* a, const float* b, float* out, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    out[i] = a[i] - b[i];
}

static inline int grid_for(long long n) {
  long long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace ea

using namespace ea;

extern "C" hipError_t ea_apply_update(FlatArgs* a, int bf16, hipStream_t s) {
  const int tiles = shadow_tiles(*a);
  a->total_blocks = a->R * tiles;
  if (a->total_blocks <= 0) return hipSuccess;
  if (bf16) hipLaunchKernelGGL((shadow_tiles_kernel<__bf16, true>), dim3(a->total_blocks), dim3(256), 0, s, *a, tiles);
  else hipLaunchKernelGGL((shadow_tiles_kernel<float, true>), dim3(a->total_blocks), dim3(256), 0, s, *a, tiles);
  return hipGetLastError();
}

extern "C" hipError_t ea_persist_post(unsigned* flags, int nflags, long long* ctr, const int* ntrain, int R, int B, int n,
                                      const unsigned* err, hipStream_t s) {
  hipLaunchKernelGGL(persist_post_kernel, dim3(1), dim3(256), 0, s, flags, nflags, ctr, ntrain, R, B, n, err);
  return hipGetLastError();
}

extern "C" hipError_t ea_persist_post_average(unsigned* flags, int nflags, long long* ctr, const int* ntrain, int R,
                                              int B, int n, const unsigned* err, float* P, long long sP, long long np,
                                              float* out, int write_back, double scale, hipStream_t s) {
  const bool vec = sP % 4 == 0 && (reinterpret_cast<uintptr_t>(P) & 15) == 0 &&
                   (out == nullptr || (reinterpret_cast<uintptr_t>(out) & 15) == 0);
  const int g = grid_for(vec ? (np + 3) / 4 : np) + 1;
  if (vec)
    hipLaunchKernelGGL(persist_post_average_kernel<true>, dim3(g), dim3(256), 0, s, flags, nflags, ctr, ntrain, R, B,
                       n, err, P, sP, np, out, write_back, scale);
  else
    hipLaunchKernelGGL(persist_post_average_kernel<false>, dim3(g), dim3(256), 0, s, flags, nflags, ctr, ntrain, R, B,
                       n, err, P, sP, np, out, write_back, scale);
  return hipGetLastError();
}

extern "C" hipError_t ea_advance(long long* ctr, const int* ntrain, int R, int B, int n, hipStream_t s) {
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64), 0, s, ctr, ntrain, R, B, n);
  return hipGetLastError();
}

extern "C" hipError_t ea_refresh_shadows(FlatArgs* a, int bf16, hipStream_t s) {
  const int tiles = shadow_tiles(*a);
  a->total_blocks = a->R * tiles;
  if (a->total_blocks <= 0) return hipSuccess;
  if (bf16) hipLaunchKernelGGL((shadow_tiles_kernel<__bf16, false>), dim3(a->total_blocks), dim3(256), 0, s, *a, tiles);
  else hipLaunchKernelGGL((shadow_tiles_kernel<float, false>), dim3(a->total_blocks), dim3(256), 0, s, *a, tiles);
  return hipGetLastError();
}

extern "C" hipError_t ea_replica_average(float* P, long long sP, int R, long long n, float* out, int write_back,
                                         double scale, hipStream_t s) {
  const bool vec = sP % 4 == 0 && (reinterpret_cast<uintptr_t>(P) & 15) == 0 &&
                   (out == nullptr || (reinterpret_cast<uintptr_t>(out) & 15) == 0);
  if (vec)
    hipLaunchKernelGGL(replica_average_kernel<true>, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, P, sP, R, n, out,
                       write_back, scale);
  else
    hipLaunchKernelGGL(replica_average_kernel<false>, dim3(grid_for(n)), dim3(256), 0, s, P, sP, R, n, out, write_back,
                       scale);
  return hipGetLastError();
}

extern "C" hipError_t ea_sum_slabs(const float* S, int ks, int M, int N, float* C, long long ldc, hipStream_t s) {
  const long long slab = (long long)M * N;
  const bool vec = N % 4 == 0 && ldc % 4 == 0 && (reinterpret_cast<uintptr_t>(S) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(C) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(sum_slabs_kernel<true>, dim3(grid_for(slab / 4)), dim3(256), 0, s, S, ks, slab, M, N, C, ldc);
  else
    hipLaunchKernelGGL(sum_slabs_kernel<false>, dim3(grid_for(slab)), dim3(256), 0, s, S, ks, slab, M, N, C, ldc);
  return hipGetLastError();
}

extern "C" hipError_t ea_axpby(const float* x, float* y, long long n, float alpha, float beta, hipStream_t s) {
  hipLaunchKernelGGL(axpby_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, x, y, n, alpha, beta);
  return hipGetLastError();
}

extern "C" hipError_t ea_ps_sub(float* p, const float* d, long long n, float scale, int atomic, hipStream_t s) {
  if (atomic) hipLaunchKernelGGL(ps_sub_atomic_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, d, n, scale);
  else hipLaunchKernelGGL(ps_sub_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, p, d, n, scale);
  return hipGetLastError();
}

extern "C" hipError_t ea_sub(const float* a, const float* b, float* out, long long n, hipStream_t s) {
  hipLaunchKernelGGL(sub_kernel, dim3(grid_for(n)), dim3(256), 0, s, a, b, out, n);
  return hipGetLastError();
}

// fp32 rows -> bf16 rows on the device (inference uploads of bf16 executors:
// the rows are DMA'd as fp32 straight from pinned host memory and converted here)
__global__ __launch_bounds__(256) void cvt_rows_bf16_kernel(const float* __restrict__ src, long long src_ld,
                                                            __bf16* __restrict__ dst, long long dst_ld, long long nr,
                                                            long long k) {
  const long long total = nr * k;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long r = e / k, c = e % k;
    dst[r * dst_ld + c] = from_f<__bf16>(src[r * src_ld + c]);
  }
}

extern "C" hipError_t ea_cvt_rows_bf16(const float* src, long long src_ld, void* dst, long long dst_ld, long long nr,
                                       long long k, hipStream_t s) {
  if (nr <= 0 || k <= 0) return hipSuccess;
  hipLaunchKernelGGL(cvt_rows_bf16_kernel, dim3(grid_for(nr * k)), dim3(256), 0, s, src, src_ld,
                     reinterpret_cast<__bf16*>(dst), dst_ld, nr, k);
  return hipGetLastError();
}

// Diagnostics: fill every CU's LDS with a pattern (e.g. NaN) so a kernel that
// reads LDS it never wrote shows it deterministically instead of inheriting
// whatever the previous workgroup on that CU left there.
__global__ __launch_bounds__(256) void poison_lds_kernel(unsigned pattern, int bytes) {
  extern __shared__ __attribute__((aligned(16))) unsigned lds_words[];
  for (int i = threadIdx.x; i < bytes / 4; i += 256) lds_words[i] = pattern;
  __syncthreads();
  if (threadIdx.x == 0 && lds_words[(blockIdx.x * 97) % (bytes / 4)] != pattern) lds_words[0] = 0u;  // keep the stores live
}

extern "C" hipError_t ea_poison_lds(unsigned pattern, hipStream_t s) {
  const int bytes = 160 * 1024;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&poison_lds_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  hipLaunchKernelGGL(poison_lds_kernel, dim3(4096), dim3(256), bytes, s, pattern, bytes);
  return hipGetLastError();
}

