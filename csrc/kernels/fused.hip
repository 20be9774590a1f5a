// Fused small-MLP training step tail (MI355X / gfx950).
//
// One workgroup (4 waves) per replica runs, for layers 1..L-1 of a small MLP,
//   forward (MFMA GEMM + bias + activation + dropout), the loss/metrics, and the
//   backward pass with every weight update (DW GEMM + optimizer + shadow images)
//   and the input gradients (DX GEMM + act'/dropout),
// and hands dZ_0^T to the layer-0 weight update. All activations, gradient
// factors and logits live in LDS (<= 160 KB); weights stream from L2/HBM as
// MFMA B fragments. This replaces 2(L-1) grouped launches per step by one, which
// matters because the small layers are latency-bound: each launch costs ~1.6 us
// of graph-node gap plus ~2 us of block spin-up and counter reads on MI355X
// (tools/micro/latency*.hip, profiles/README.md).
//
// Reference behaviour being executed: one Keras `fit` step of a Dense stack
// (reference elephas/worker.py:41-42 SparkWorker.train -> model.fit).
//
// Same numerics as the grouped path: bf16 (or fp32) operands, fp32 accumulate,
// fp32 logits/loss, Philox dropout masks as a pure function of
// (seed, replica, layer, iteration, row, column/4), fp32 master weights.
#include "common.h"
#include "mfma.h"
#include "loss_tile.h"

namespace ea {

namespace {

constexpr int FB = 64;  // batch rows per replica tile (B <= 64)

__device__ __forceinline__ uint4 zero4() { return make_uint4(0u, 0u, 0u, 0u); }

// Walks (row, chunk) = divmod(e, cpr) for e = tid, tid + 256, ... without a
// per-step integer division (one division at construction).
struct RowIter {
  int m, c, dq, dr, cpr;
  __device__ RowIter(int e0, int cpr_) : cpr(cpr_) {
    m = e0 / cpr_;
    c = e0 - m * cpr_;
    dq = 256 / cpr_;
    dr = 256 - dq * cpr_;
  }
  __device__ void next() {
    m += dq;
    c += dr;
    if (c >= cpr) { c -= cpr; ++m; }
  }
};

// EPL elements of one operand column stored with stride `stride` (transposed read)
template <typename T>
__device__ __forceinline__ uint4 lds_gather(const T* p, int stride) {
  if constexpr (sizeof(T) == 2) {
    const unsigned short* q = reinterpret_cast<const unsigned short*>(p);
    unsigned v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = q[i * stride];
    return make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
  } else {
    return make_uint4(__float_as_uint(p[0]), __float_as_uint(p[stride]), __float_as_uint(p[2 * stride]),
                      __float_as_uint(p[3 * stride]));
  }
}

// 8 consecutive compute-dtype values <-> floats
template <typename T> __device__ __forceinline__ void ld8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
template <typename T> __device__ __forceinline__ void st8v(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    unsigned w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned lo = __builtin_bit_cast(unsigned short, from_f<__bf16>(v[2 * i]));
      const unsigned hi = __builtin_bit_cast(unsigned short, from_f<__bf16>(v[2 * i + 1]));
      w[i] = lo | (hi << 16);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// C[64][N] = A[64][Kd] . BT[N][Kd]^T.  A in LDS (row stride lda), BT in global
// (row stride ldb, K-contiguous). Wave w owns the 16-column tiles w, w+4, w+8,
// w+12 (acc[mt][s] = rows 16mt.., tile w+4s). B fragments are prefetched PF
// k-steps ahead through a static register ring.
// Column tiles nt = nt0 + ntstep * (w + 4 s) (ntstep > 1: the workgroup owns a
// strided subset of the output columns).
template <typename T>
__device__ __forceinline__ void gemm64(const T* A, int lda, const T* __restrict__ BT, long long ldb, int Kd, int N,
                                       f32x4 (&acc)[4][4], int w, int lane, int nt0 = 0, int ntstep = 1) {
  constexpr int EPL = KT<T>::EPL, KC = KT<T>::KC, PF = 4;
  const int row = lane & 15, kg = lane >> 4;
  const int ntt = (N + 15) >> 4;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[mt][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  const T* bp[4];
  bool bv[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int col = (nt0 + ntstep * (w + 4 * s)) * 16 + row;
    bv[s] = col < N;
    bp[s] = BT + (long long)(bv[s] ? col : 0) * ldb;
  }
  const int nks = (Kd + KC - 1) / KC;
  uint4 bq[PF][4];
  auto loadB = [&](int ks, uint4(&dst)[4]) {
    const int kk = ks * KC + kg * EPL;
    const bool kin = kk < Kd;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (nt0 + ntstep * (w + 4 * s) < ntt) {
        const uint4 v = *reinterpret_cast<const uint4*>(bp[s] + (kin ? kk : 0));
        dst[s] = (kin && bv[s]) ? v : zero4();
      } else {
        dst[s] = zero4();
      }
    }
  };
#pragma unroll
  for (int i = 0; i < PF; ++i)
    if (i < nks) loadB(i, bq[i]);
  for (int ks0 = 0; ks0 < nks; ks0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int ks = ks0 + u;
      if (ks < nks) {
        uint4 b[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s] = bq[u][s];
        if (ks + PF < nks) loadB(ks + PF, bq[u]);
        const int kk = ks * KC + kg * EPL;
        const bool kin = kk < Kd;
        uint4 a[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const uint4 v = *reinterpret_cast<const uint4*>(A + (mt * 16 + row) * lda + (kin ? kk : 0));
          a[mt] = kin ? v : zero4();
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (nt0 + ntstep * (w + 4 * s) < ntt)
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) mma16<T>(acc[mt][s], a[mt], b[s]);
      }
    }
  }
}

typedef short v4s __attribute__((ext_vector_type(4)));

// MFMA operand fragment holding 8 consecutive rows m0 .. m0+7 of column
// col0 + (lane & 15) of a row-major LDS tile X[m][ld] (a column of X, i.e. a
// transposed read): bf16 via two gfx950 ds_read_b64_tr_b16 (lane 4q+p of each
// 16-lane group addresses row q, columns 4p..4p+3 of a 4x16 block and receives
// column (lane & 15)); fp32 via 4 strided ds_read_b32. EXEC must be full.
template <typename T>
__device__ __forceinline__ uint4 frag_col(const T* X, int ld, int m0, int col0, int lane) {
  if constexpr (sizeof(T) == 2) {
    const int i = lane & 15;
    const T* p = X + (m0 + (i >> 2)) * ld + col0 + 4 * (i & 3);
    typedef __attribute__((address_space(3))) v4s* lds_v4s;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s)(p));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s)(p + 4 * ld));
    const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
    return make_uint4(l2.x, l2.y, h2.x, h2.y);
  } else {
    return lds_gather<T>(X + m0 * ld + col0 + (lane & 15), ld);
  }
}

// Per-wave tile set of one layer's weight update: dW^T tiles (n-tile, k-tile)
// over N x (K + has_bias) (row K of the flat layout = bias; the D tile carries
// a ones column at index K). Workgroup `sp` of S owns tiles t = sp + S*u, wave w
// the local indices u = w + 4j.
struct DwTiles {
  int ntt, ktt, total, sp, S, w;
  __device__ int tile(int j) const { return sp + S * (w + 4 * j); }
  __device__ bool valid(int j) const { return tile(j) < total; }
};

constexpr int DWG = 8;  // tiles per wave per pass

// prefetch P / S of up to DWG tiles (dW^T layout: lane owns n = nt*16 + 4(lane>>4) + q, k = kt*16 + (lane&15))
__device__ __forceinline__ void dw_prefetch(const FusedLayer& ly, const DwTiles& dt, int j0, const float* __restrict__ P,
                                            const float* __restrict__ S, long long splane, int np, int lane,
                                            float (&wv)[DWG * 4], float (&s0)[DWG * 4], float (&s1)[DWG * 4]) {
  const int Keff = ly.K + ly.has_bias;
#pragma unroll
  for (int j = 0; j < DWG; ++j) {
    const int t = dt.tile(j0 + j);  // wave-uniform (scalar)
    if (t >= dt.total) {
#pragma unroll
      for (int q = 0; q < 4; ++q) wv[j * 4 + q] = s0[j * 4 + q] = s1[j * 4 + q] = 0.f;
      continue;
    }
    const int kt = t / dt.ntt, nt = t - kt * dt.ntt;
    const int k = kt * 16 + (lane & 15), n0 = nt * 16 + (lane >> 4) * 4;
    const bool tv = k < Keff;
    if (ly.pvec) {
      const bool in = tv && n0 < ly.N;
      const int pi = (int)ly.p_off + (in ? k * ly.N + n0 : 0);
      const float4 x = *reinterpret_cast<const float4*>(P + pi);
      wv[j * 4 + 0] = x.x; wv[j * 4 + 1] = x.y; wv[j * 4 + 2] = x.z; wv[j * 4 + 3] = x.w;
      if (np > 0) {
        const float4 y = *reinterpret_cast<const float4*>(S + pi);
        s0[j * 4 + 0] = y.x; s0[j * 4 + 1] = y.y; s0[j * 4 + 2] = y.z; s0[j * 4 + 3] = y.w;
      }
      if (np > 1) {
        const float4 y = *reinterpret_cast<const float4*>(S + splane + pi);
        s1[j * 4 + 0] = y.x; s1[j * 4 + 1] = y.y; s1[j * 4 + 2] = y.z; s1[j * 4 + 3] = y.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool in = tv && n0 + q < ly.N;
        const int pi = (int)ly.p_off + (in ? k * ly.N + n0 + q : 0);
        wv[j * 4 + q] = P[pi];
        if (np > 0) s0[j * 4 + q] = S[pi];
        if (np > 1) s1[j * 4 + q] = S[splane + pi];
      }
    }
    if (np < 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) s0[j * 4 + q] = 0.f;
    }
    if (np < 2) {
#pragma unroll
      for (int q = 0; q < 4; ++q) s1[j * 4 + q] = 0.f;
    }
  }
}

// dW^T = dZ^T . D (sum over the 64 batch rows) for up to DWG tiles, then the
// optimizer update of the fp32 master (+ state) and the next-parity W / W^T images.
template <typename T>
__device__ __forceinline__ void dw_pass(const FusedArgs& a, const FusedLayer& ly, const DwTiles& dt, int j0, const T* D,
                                        int ldd, const T* dZ, int ldz, float* __restrict__ P, float* __restrict__ S,
                                        long long splane, int np, T* __restrict__ Wn, T* __restrict__ WTn,
                                        long long iter, int lane, float (&wv)[DWG * 4], float (&s0)[DWG * 4],
                                        float (&s1)[DWG * 4]) {
  constexpr int EPL = KT<T>::EPL, KC = KT<T>::KC;
  const int g = lane >> 4;
  f32x4 acc[DWG];
#pragma unroll
  for (int j = 0; j < DWG; ++j) {
    acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int t = dt.tile(j0 + j);
    if (t < dt.total) {  // wave-uniform: EXEC stays full for the transposed reads
      const int kt = t / dt.ntt, nt = t - kt * dt.ntt;
#pragma unroll
      for (int ks = 0; ks < FB / KC; ++ks) {
        const int m0 = ks * KC + g * EPL;
        const uint4 x = frag_col<T>(dZ, ldz, m0, nt * 16, lane);  // A: rows n
        const uint4 y = frag_col<T>(D, ldd, m0, kt * 16, lane);   // B: cols k
        mma16<T>(acc[j], x, y);
      }
    }
  }
  // one optimizer dispatch for the whole pass (values of absent tiles are discarded)
  const float gs = a.op.grad_scale;
  float gv[DWG * 4];
#pragma unroll
  for (int j = 0; j < DWG; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) gv[j * 4 + q] = acc[j][q] * gs;
  opt_update_v<DWG * 4>(a.op, wv, gv, s0, s1, iter);
  const int Keff = ly.K + ly.has_bias;
#pragma unroll
  for (int j = 0; j < DWG; ++j) {
    const int t = dt.tile(j0 + j);
    if (t >= dt.total) continue;
    const int kt = t / dt.ntt, nt = t - kt * dt.ntt;
    const int k = kt * 16 + (lane & 15), n0 = nt * 16 + g * 4;
    if (k >= Keff || n0 >= ly.N) continue;
    float nw[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) nw[q] = wv[j * 4 + q];
    const int pi = (int)ly.p_off + k * ly.N + n0;
    if (ly.pvec) {
      *reinterpret_cast<float4*>(P + pi) = make_float4(nw[0], nw[1], nw[2], nw[3]);
      if (np > 0) *reinterpret_cast<float4*>(S + pi) = make_float4(s0[j * 4 + 0], s0[j * 4 + 1], s0[j * 4 + 2], s0[j * 4 + 3]);
      if (np > 1) *reinterpret_cast<float4*>(S + splane + pi) = make_float4(s1[j * 4 + 0], s1[j * 4 + 1], s1[j * 4 + 2], s1[j * 4 + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (n0 + q < ly.N) {
          P[pi + q] = nw[q];
          if (np > 0) S[pi + q] = s0[j * 4 + q];
          if (np > 1) S[splane + pi + q] = s1[j * 4 + q];
        }
    }
    if (k == ly.K && a.Bsh) {  // bias row: next-parity fp32 bias image
      float* bn = a.Bsh + (long long)blockIdx.x / a.nsplit * a.sBsh + ((iter + 1) & 1) * a.bsh_par + pi;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (n0 + q < ly.N) bn[q] = nw[q];
    }
    if (k < ly.K) {  // weight images (no image for the bias row)
      T* wrow = Wn + ((int)ly.wsh_off + k * ly.Np + n0);  // 4 consecutive n (Np % 8 == 0)
      if constexpr (sizeof(T) == 2) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = n0 + q < ly.N ? nw[q] : 0.f;
        const unsigned lo = __builtin_bit_cast(unsigned short, from_f<__bf16>(v[0])) |
                            ((unsigned)__builtin_bit_cast(unsigned short, from_f<__bf16>(v[1])) << 16);
        const unsigned hi = __builtin_bit_cast(unsigned short, from_f<__bf16>(v[2])) |
                            ((unsigned)__builtin_bit_cast(unsigned short, from_f<__bf16>(v[3])) << 16);
        *reinterpret_cast<uint2*>(wrow) = make_uint2(lo, hi);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) wrow[q] = n0 + q < ly.N ? nw[q] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (n0 + q < ly.N) WTn[(int)ly.wtsh_off + (n0 + q) * ly.Kp + k] = from_f<T>(nw[q]);
    }
  }
}

__device__ __forceinline__ void fstamp(const FusedArgs& a, int k) {
  if (a.stamps && threadIdx.x == 0) a.stamps[(long long)blockIdx.x * 32 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}

}  // namespace

template <typename T>
__global__ __launch_bounds__(256) void fused_tail_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  fstamp(a, 0);
  const int r = blockIdx.x / a.nsplit, sp = blockIdx.x - r * a.nsplit;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: tile math stays scalar
  const long long s0 = a.ctr[0];
  const long long step = s0 + a.step_off;
  const long long iter = iter_at(a.ctr, a.ntrain, a.B, r, s0, a.step_off);
  const long long cnt = (long long)a.ntrain[r] - step * a.B;
  const int valid = (int)(cnt < 0 ? 0 : (cnt > a.B ? a.B : cnt));
  if (valid == 0) return;  // replica has no batch this step (no update, like DW_UPDATE's skip)
  const long long rpar = iter & 1, wpar = (iter + 1) & 1;
  const int L = a.L;
  const FusedLayer* __restrict__ LY = a.ly;
  const T* Wcur = reinterpret_cast<const T*>(a.Wsh) + (long long)r * a.sWsh + rpar * a.wsh_par;
  const T* WTcur = reinterpret_cast<const T*>(a.WTsh) + (long long)r * a.sWTsh + rpar * a.wtsh_par;
  T* Wnext = reinterpret_cast<T*>(a.Wsh) + (long long)r * a.sWsh + wpar * a.wsh_par;
  T* WTnext = reinterpret_cast<T*>(a.WTsh) + (long long)r * a.sWTsh + wpar * a.wtsh_par;
  float* P = a.P + (long long)r * a.sP;
  float* S = a.S ? a.S + (long long)r * a.sS : nullptr;
  const int np = S ? opt_planes(a.op) : 0;
  const long long splane = a.op.s_plane;
  float* Ys = reinterpret_cast<float*>(smem + a.offY);
  int* srow = reinterpret_cast<int*>(smem + a.offSrow);

  // ---- phase 0: targets; D_0 (+ ones column for layer 1's bias) and
  //      G_0 = act'(Z_0) * dropout_0 / (1 - rate); all loads issued before use
  {
    const int ldy = (int)a.ldy;
    const float* Yb = a.Y + (long long)r * a.sY;
    const int* pr = a.perm + (long long)r * a.sPerm + step * a.B;
    int prow[8];
    const int jy = tid & 31, my = tid >> 5;  // row my + 8 i, column jy
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = my + 8 * i;
      prow[i] = pr[m < valid ? m : 0];
    }
    float yv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool in = my + 8 * i < valid && jy < ldy;
      const float v = Yb[in ? prow[i] * ldy + jy : 0];
      yv[i] = in ? v : 0.f;
    }
    const FusedLayer l0 = LY[0];
    const bool ones = LY[1].has_bias;
    T* D0s = reinterpret_cast<T*>(smem + l0.offD);
    float* G0 = reinterpret_cast<float*>(smem + l0.offG);
    const T* D0g = reinterpret_cast<const T*>(a.D0) + (long long)r * a.sD0;
    const float* Z0g = a.Z0 + (long long)r * a.sZ0;
    const float keep_scale = l0.rate > 0.f ? 1.f / (1.f - l0.rate) : 1.f;
    const uint32_t dbase = dropout_base(a.seed, r, 0, iter);
    const int cpr = l0.Np >> 3, items = FB * cpr;
    const bool zvec = (l0.N & 3) == 0;
    RowIter it(tid, cpr);
    for (int b0 = 0; b0 < items; b0 += 1024) {
      float dv[4][8], z[4][8];
      int mi[4], ci[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        mi[i] = it.m;
        ci[i] = it.c * 8;
        it.next();
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mi[i], c0 = ci[i];
        const bool rv = m < valid;  // rows >= 64 (past the tile) are never valid
        const int ms = rv ? m : 0, cs = rv ? c0 : 0;
        ld8<T>(D0g + (ms * l0.Np + cs), dv[i]);
        if (zvec) {
          const float* zp = Z0g + (ms * l0.N + (cs + 8 <= l0.N ? cs : 0));
          const float4 x = *reinterpret_cast<const float4*>(zp), y = *reinterpret_cast<const float4*>(zp + 4);
          z[i][0] = x.x; z[i][1] = x.y; z[i][2] = x.z; z[i][3] = x.w;
          z[i][4] = y.x; z[i][5] = y.y; z[i][6] = y.z; z[i][7] = y.w;
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) z[i][q] = Z0g[ms * l0.N + (cs + q < l0.N ? cs + q : 0)];
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mi[i], c0 = ci[i];
        if (m >= FB) continue;
        const bool rv = m < valid;
        float u[8], g[8], d[8];
        if (rv && l0.rate > 0.f) {
          dropout_u8(dbase, m, c0, u);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) u[q] = 1.f;
        }
        float ag[8];
        act_g_v<8>(l0.act, z[i], ag);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int c = c0 + q;
          g[q] = (rv && c < l0.N && u[q] >= l0.rate) ? ag[q] * keep_scale : 0.f;
          d[q] = rv ? (c < l0.N ? dv[i][q] : ((ones && c == l0.N) ? 1.f : 0.f)) : 0.f;
        }
        st8v<T>(D0s + m * l0.ldA + c0, d);
        *reinterpret_cast<float4*>(G0 + m * l0.ldG + c0) = make_float4(g[0], g[1], g[2], g[3]);
        *reinterpret_cast<float4*>(G0 + m * l0.ldG + c0 + 4) = make_float4(g[4], g[5], g[6], g[7]);
      }
    }
    if (ones && l0.N == l0.Np && tid < FB) D0s[tid * l0.ldA + l0.N] = from_f<T>(tid < valid ? 1.f : 0.f);
#pragma unroll
    for (int i = 0; i < 8; ++i) Ys[tid + 256 * i] = yv[i];
    if (tid < FB) srow[tid] = tid < valid ? 1 : -1;
  }
  __syncthreads();
  fstamp(a, 1);

  // ---- phase 1: forward through layers 1..L-1 (+ loss); every workgroup of the
  //      replica runs it (cheap, latency-bound), only sp == 0 reports metrics
  for (int l = 1; l < L; ++l) {
    const FusedLayer ly = LY[l], pv = LY[l - 1];
    const T* A = reinterpret_cast<const T*>(smem + pv.offD);
    f32x4 acc[4][4];
    gemm64<T>(A, pv.ldA, WTcur + ly.wtsh_off, ly.Kp, ly.Kp, ly.N, acc, w, lane);
    const bool last = l == L - 1;
    float* Zs = reinterpret_cast<float*>(smem + (last ? a.offLg : ly.offG));
    const int ldz = last ? a.ldLg : ly.ldG;
    // bias from this step's parity image: P's bias row may already hold the
    // update written by another workgroup of this replica
    // (without split workgroups -- nsplit == 1 -- nothing else writes this replica's P
    //  during the launch and the fp32 master is read directly)
    const float* bias = a.Bsh ? a.Bsh + (long long)r * a.sBsh + rpar * a.bsh_par + ly.p_off + (long long)ly.K * ly.N
                              : P + ly.p_off + (long long)ly.K * ly.N;
    const int ntt = (ly.N + 15) >> 4;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int nt = w + 4 * s;
      if (nt >= ntt) continue;
      const int col = nt * 16 + (lane & 15);
      const bool cv = col < ly.N;
      const float bv = bias[cv ? col : 0];
      const float b = (ly.has_bias && cv) ? bv : 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = mt * 16 + (lane >> 4) * 4 + q;
          Zs[m * ldz + col] = cv ? acc[mt][s][q] + b : 0.f;
        }
    }
    __syncthreads();
    fstamp(a, 2 + 3 * l);
    if (!last) {
      // D_l = act(z) * dropout / (1 - rate) (+ ones column for layer l+1's bias);
      // G_l = act'(z) * dropout / (1 - rate), in place of z
      T* Dl = reinterpret_cast<T*>(smem + ly.offD);
      float* Gl = Zs;
      const bool ones = LY[l + 1].has_bias;
      const float keep_scale = ly.rate > 0.f ? 1.f / (1.f - ly.rate) : 1.f;
      const uint32_t dbase = dropout_base(a.seed, r, l, iter);
      const int cpr = ly.Np >> 3;
      for (RowIter it(tid, cpr); it.m < FB; it.next()) {
        const int m = it.m, c0 = it.c * 8;
        const bool rv = m < valid;
        float z[8], o[8], g[8], u[8];
        const float4 za = *reinterpret_cast<const float4*>(Gl + m * ldz + c0);
        const float4 zb = *reinterpret_cast<const float4*>(Gl + m * ldz + c0 + 4);
        z[0] = za.x; z[1] = za.y; z[2] = za.z; z[3] = za.w; z[4] = zb.x; z[5] = zb.y; z[6] = zb.z; z[7] = zb.w;
        if (rv && ly.rate > 0.f) {
          dropout_u8(dbase, m, c0, u);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) u[q] = 1.f;
        }
        float ao[8], ag[8];
        act_fg_v<8>(ly.act, z, ao, ag);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int c = c0 + q;
          const bool keep = rv && c < ly.N && u[q] >= ly.rate;
          o[q] = keep ? ao[q] * keep_scale : ((rv && ones && c == ly.N) ? 1.f : 0.f);
          g[q] = keep ? ag[q] * keep_scale : 0.f;
        }
        st8v<T>(Dl + m * ly.ldA + c0, o);
        *reinterpret_cast<float4*>(Gl + m * ldz + c0) = make_float4(g[0], g[1], g[2], g[3]);
        *reinterpret_cast<float4*>(Gl + m * ldz + c0 + 4) = make_float4(g[4], g[5], g[6], g[7]);
      }
      if (ones && ly.N == ly.Np && tid < FB) Dl[tid * ly.ldA + ly.N] = from_f<T>(tid < valid ? 1.f : 0.f);
    } else {
      // loss + metrics + dL/dz (in place, scaled by 1/valid)
      Prob q;
      q.N = ly.N;
      q.act = ly.act;
      q.loss = a.loss;
      q.nmet = a.nmet;
#pragma unroll
      for (int i = 0; i < 4; ++i) q.met[i] = a.met[i];
      q.Y = a.Y;
      q.pred = nullptr;
      q.sPred = 0;
      q.ldp = 0;
      q.chunk = 0;
      q.B = a.B;
      const float inv_valid = 1.f / (float)valid;
      float sums[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (softmax_cce_fast(q)) {
        if (ly.N <= 16) loss_tile_cce<4, FB, 36, 32>(q, r, 0, Zs, Ys, srow, true, inv_valid, sums);
        else loss_tile_cce<8, FB, 36, 32>(q, r, 0, Zs, Ys, srow, true, inv_valid, sums);
      } else {
        loss_tile_lds<FB, 36, 32>(q, r, 0, Zs, Ys, srow, true, inv_valid, sums);
      }
      if (a.acc && sp == 0) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          if (i < 2 + a.nmet) {
            const float sv = row_sum<64>(sums[i]);
            if (lane == 0 && sv != 0.f) atomicAdd(a.acc + (long long)r * a.acc_stride + i, (double)sv);
          }
        }
      }
      __syncthreads();
      // dZ_{L-1} -> compute dtype, zero-padded to 16-column tiles
      T* dZ = reinterpret_cast<T*>(smem + a.offdZ0);
      const int ncol = ((ly.N + 15) >> 4) * 16;
      for (RowIter it(tid, ncol); it.m < FB; it.next())
        dZ[it.m * a.lddZ + it.c] = from_f<T>(it.c < ly.N ? Zs[it.m * ldz + it.c] : 0.f);
    }
    __syncthreads();
    fstamp(a, 3 + 3 * l);
  }

  // ---- phase 2: backward through layers L-1..1. Per layer: prefetch this
  //      wave's P/S tiles, DX (full, or this workgroup's dZ_0 column tiles),
  //      then the weight update from LDS (stores last: later loads would wait on them)
  int cur = 0;
  for (int l = L - 1; l >= 1; --l) {
    const FusedLayer ly = LY[l], pv = LY[l - 1];
    const T* dZ = reinterpret_cast<const T*>(smem + (cur ? a.offdZ1 : a.offdZ0));
    const T* Dp = reinterpret_cast<const T*>(smem + pv.offD);
    DwTiles dt;
    dt.ntt = (ly.N + 15) >> 4;
    dt.ktt = (ly.K + ly.has_bias + 15) >> 4;
    dt.total = dt.ntt * dt.ktt;
    dt.sp = sp;
    dt.S = a.nsplit;
    dt.w = w;
    float wv[DWG * 4], sa[DWG * 4], sb[DWG * 4];
    const bool deferred = l == 1 && a.dZ1T;  // layer-1 update runs in the next grouped launch
    if (!deferred) dw_prefetch(ly, dt, 0, P, S, splane, np, lane, wv, sa, sb);
    // DX: dD_{l-1} = dZ_l . W_l^T  (current-parity W images, untouched by the update)
    f32x4 acc[4][4];
    const bool first = l == 1;
    gemm64<T>(dZ, a.lddZ, Wcur + ly.wsh_off, ly.Np, ly.Np, ly.K, acc, w, lane, first ? sp : 0, first ? a.nsplit : 1);
    const float* Gp = reinterpret_cast<const float*>(smem + pv.offG);
    const int ntt = (ly.K + 15) >> 4;
    if (!first) {
      T* dZn = reinterpret_cast<T*>(smem + (cur ? a.offdZ0 : a.offdZ1));
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int nt = w + 4 * s;
        if (nt >= ntt) continue;
        const int col = nt * 16 + (lane & 15);
        const bool cv = col < pv.N;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int m = mt * 16 + (lane >> 4) * 4 + q;
            const float gq = Gp[m * pv.ldG + (cv ? col : 0)];
            dZn[m * a.lddZ + col] = from_f<T>(cv ? acc[mt][s][q] * gq : 0.f);
          }
      }
    } else {
      // dZ_0^T [N0][Bp] for the layer-0 weight update (4 consecutive rows per lane)
      T* out = reinterpret_cast<T*>(a.dZ0T) + (long long)r * a.sdZ0T;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int nt = sp + a.nsplit * (w + 4 * s);
        if (nt >= ntt) continue;
        const int col = nt * 16 + (lane & 15);
        if (col >= pv.N) continue;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int m0 = mt * 16 + (lane >> 4) * 4;
          if (m0 >= a.Bp) continue;
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = acc[mt][s][q] * Gp[(m0 + q) * pv.ldG + col];
          T* dst = out + (long long)col * a.Bp + m0;
          if constexpr (sizeof(T) == 2) {
            const unsigned lo = __builtin_bit_cast(unsigned short, from_f<__bf16>(v[0])) |
                                ((unsigned)__builtin_bit_cast(unsigned short, from_f<__bf16>(v[1])) << 16);
            const unsigned hi = __builtin_bit_cast(unsigned short, from_f<__bf16>(v[2])) |
                                ((unsigned)__builtin_bit_cast(unsigned short, from_f<__bf16>(v[3])) << 16);
            *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
          } else {
            *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    }
    fstamp(a, 14 + 3 * (L - 1 - l));
    if (deferred) {
      // deferred layer-1 update: publish dZ_1^T [N1][Bp] for the grouped DW_UPDATE launch
      T* out = reinterpret_cast<T*>(a.dZ1T) + (long long)r * a.sdZ1T;
      for (int e = tid; e < ly.N * a.Bp; e += 256) {
        const int n = e / a.Bp, m = e - n * a.Bp;
        out[(long long)n * a.Bp + m] = dZ[m * a.lddZ + n];
      }
    }
    // weight update of layer l from LDS (D_{l-1} with its ones column, dZ_l)
    for (int j0 = 0; !deferred && dt.valid(j0); j0 += DWG) {
      if (j0 > 0) dw_prefetch(ly, dt, j0, P, S, splane, np, lane, wv, sa, sb);
      dw_pass<T>(a, ly, dt, j0, Dp, pv.ldA, dZ, a.lddZ, P, S, splane, np, Wnext, WTnext, iter, lane, wv, sa, sb);
    }
    fstamp(a, 15 + 3 * (L - 1 - l));
    if (!first) cur ^= 1;
    __syncthreads();
  }
  fstamp(a, 31);
}

}  // namespace ea

using namespace ea;

extern "C" void ea_fused_init() {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_tail_kernel<__bf16>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_tail_kernel<float>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

extern "C" hipError_t ea_fused_tail(const FusedArgs* a, int bf16, hipStream_t s) {
  if (a->lds_bytes > 160 * 1024 || a->B > 64 || a->L < 2 || a->L > FUSED_MAX_L || a->nsplit < 1) return hipErrorInvalidValue;
  const dim3 grid(a->R * a->nsplit);
  if (bf16) hipLaunchKernelGGL(fused_tail_kernel<__bf16>, grid, dim3(256), a->lds_bytes, s, *a);
  else hipLaunchKernelGGL(fused_tail_kernel<float>, grid, dim3(256), a->lds_bytes, s, *a);
  return hipGetLastError();
}
