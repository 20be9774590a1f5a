// Grouped NT GEMM on CDNA4 MFMA with fused Dense-layer epilogues.
//
//   C[m][n] = sum_k A[m][k] * BT[n][k]      (both operands K-contiguous)
//
// Every Dense-layer product of a training step is expressed in this one form by
// keeping each operand in the layout its consumer wants (the producer epilogues
// write both D and D^T):
//   FWD  : Z   = D_{l-1} . W_l        A = D_{l-1} [B x K]   BT = W_l^T  [N x K]
//   DX   : dD  = dZ_l . W_l^T         A = dZ_l    [B x N]   BT = W_l    [K x N]
//   DW   : dW  = D_{l-1}^T . dZ_l     A = D^T     [K x B]   BT = dZ^T   [N x B]
// (reference hot loop: elephas/worker.py:41-42 -> keras fit -> Dense fwd/bwd)
//
// Fragments are loaded straight from L2 into VGPRs with 16-byte loads (K is
// contiguous for both operands), so the main loop needs no LDS; LDS is used once
// per tile for the split-K reduction and for the epilogue (which needs whole
// rows for softmax/loss and a transposed write for D^T / dZ^T).
//
// Two tile configs:
//   LAT : 64x32 tile, the 4 waves split K      (latency-bound small layers)
//   THR : 128x128 tile, 2x2 waves, no split-K   (MFMA-bound wide layers)
//
// Several independent problems (e.g. DW_l and DX_l of the same layer) run in one
// grouped launch; blockIdx.x selects the problem.
#include "common.h"

namespace ea {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ int batch_valid(const Prob& p, int r, long long step) {
  if (p.eval_mode) {
    long long c = (long long)p.vcount[r] - p.chunk * p.B;
    return (int)(c < 0 ? 0 : (c > p.B ? p.B : c));
  }
  long long c = (long long)p.ntrain[r] - step * p.B;
  return (int)(c < 0 ? 0 : (c > p.B ? p.B : c));
}

// absolute data row for batch row m of replica r
__device__ __forceinline__ long long batch_row(const Prob& p, int r, long long step, int m) {
  if (p.eval_mode) return (long long)p.vstart[r] + p.chunk * p.B + m;
  return (long long)p.perm[(long long)r * p.sPerm + step * p.B + m];
}

template <typename T> struct KT;
template <> struct KT<__bf16> { static constexpr int EPL = 8, KC = 32; };
template <> struct KT<float> { static constexpr int EPL = 4, KC = 16; };

template <typename T>
__device__ __forceinline__ void mma16(f32x4& acc, const uint4& a, const uint4& b) {
  if constexpr (sizeof(T) == 2) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  } else {
    // lane group g holds k = 4g..4g+3 of this 16-deep chunk; MFMA t consumes element t.
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
}

template <typename T> __device__ __forceinline__ uint4 ones_frag() {
  if constexpr (sizeof(T) == 2) {
    const unsigned o = 0x3F803F80u;  // two bf16 1.0
    return make_uint4(o, o, o, o);
  } else {
    const unsigned o = 0x3F800000u;
    return make_uint4(o, o, o, o);
  }
}

template <typename T> __device__ __forceinline__ void st(void* base, long long idx, float v) {
  reinterpret_cast<T*>(base)[idx] = from_f<T>(v);
}

// ------------------------------------------------------- gather-transpose
template <typename T>
__device__ void gather_transpose_block(const GroupArgs& ga, const Prob& p, int lb, float* sm) {
  // one block = 64 batch rows x 64 features; output XT[k][m] (ld = lddt)
  // tiles_m: batch blocks, tiles_n: feature blocks
  const int per_r = p.tiles_m * p.tiles_n;
  const int r = lb / per_r;
  const int t = lb % per_r;
  const int b0 = (t / p.tiles_n) * 64;
  const int k0 = (t % p.tiles_n) * 64;
  const long long step = ga.ctr[0];
  const int valid = batch_valid(p, r, step);
  const T* A = reinterpret_cast<const T*>(p.A) + (long long)r * p.sA;
  T* XT = reinterpret_cast<T*>(p.DT) + (long long)r * p.sDT;
  const int tid = threadIdx.x;
  for (int e = tid; e < 64 * 64; e += 256) {
    const int m = e / 64, k = e % 64;
    float v = 0.f;
    if (b0 + m < valid && k0 + k < p.K) {
      const long long row = batch_row(p, r, step, b0 + m);
      v = to_f<T>(A[row * p.lda + k0 + k]);
    }
    sm[m * 65 + k] = v;
  }
  __syncthreads();
  for (int e = tid; e < 64 * 64; e += 256) {
    const int k = e / 64, m = e % 64;
    if (k0 + k < p.K && b0 + m < p.B) XT[(long long)(k0 + k) * p.lddt + b0 + m] = from_f<T>(sm[m * 65 + k]);
  }
}

// ----------------------------------------------------------- wide loss rows
// Final layers wider than one GEMM tile (e.g. 1000 classes): the FWD GEMM writes
// the logits Z, then one wave per row runs the same row_loss math as the fused
// epilogue with wave-wide reductions.
template <typename T>
__device__ void loss_rows_block(const GroupArgs& ga, const Prob& p, int lb) {
  const int r = lb / p.tiles_m;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = (lb % p.tiles_m) * 4 + wave;
  if (row >= p.M) return;
  const long long step = ga.ctr[0];
  const int valid = batch_valid(p, r, step);
  const bool train = !p.eval_mode && p.D;
  const float inv_valid = valid > 0 ? 1.f / (float)valid : 0.f;
  if (row >= valid) {
    if (train) {
      for (int j = lane; j < p.N; j += 64) {
        st<T>(p.D, (long long)r * p.sD + (long long)row * p.ldd + j, 0.f);
        if (p.DT) st<T>(p.DT, (long long)r * p.sDT + (long long)j * p.lddt + row, 0.f);
      }
    }
    return;
  }
  const float* zrow = p.Z + (long long)r * p.sZ + (long long)row * p.ldz;
  float* prow = p.pred ? p.pred + (long long)r * p.sPred + (p.chunk * p.B + row) * p.ldp : nullptr;
  if (!p.Y) {  // predict only
    if (prow) row_predict<64>(lane, p.N, p.act, [&](int j) { return zrow[j]; }, [&](int j, float v) { prow[j] = v; });
    return;
  }
  const long long drow = batch_row(p, r, step, row);
  const float* yrow = p.Y + (long long)r * p.sY + drow * p.ldy;
  RowOut ro;
  ro.loss = 0.f;
  for (int q = 0; q < 4; ++q) ro.metric[q] = 0.f;
  row_loss<64>(lane, p.N, p.act, p.loss, p.met, p.nmet,
               [&](int j) { return zrow[j]; },
               [&](int j) { return yrow[j]; },
               train,
               [&](int j, float v) {
                 st<T>(p.D, (long long)r * p.sD + (long long)row * p.ldd + j, v * inv_valid);
                 if (p.DT) st<T>(p.DT, (long long)r * p.sDT + (long long)j * p.lddt + row, v * inv_valid);
               },
               prow != nullptr, [&](int j, float v) { prow[j] = v; }, ro);
  if (p.acc && lane == 0) {
    double* a = p.acc + (long long)r * p.acc_stride;
    atomicAdd(a + 0, (double)ro.loss);
    atomicAdd(a + 1, 1.0);
    for (int q = 0; q < p.nmet; ++q) atomicAdd(a + 2 + q, (double)ro.metric[q]);
  }
}

// --------------------------------------------------------------- the kernel
template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT>
__global__ __launch_bounds__(256) void gemm_grouped(GroupArgs ga) {
  static_assert(WAVES_M * WAVES_N * KSPLIT == 4, "4 waves per block");
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  constexpr int LDC = BN + 1;
  constexpr int EPL = KT<T>::EPL, KC = KT<T>::KC;
  extern __shared__ __attribute__((aligned(16))) float smem[];

  int bid = blockIdx.x;
  const int pi = (ga.nprob > 1 && bid >= ga.p[1].block_begin) ? 1 : 0;
  const Prob& p = ga.p[pi];
  const int lb = bid - p.block_begin;

  if (p.kind == PK_GATHER_T) {
    gather_transpose_block<T>(ga, p, lb, smem);
  } else if (p.kind == PK_LOSS_ROWS) {
    loss_rows_block<T>(ga, p, lb);
  } else {
    const int per_r = p.tiles_m * p.tiles_n;
    const int r = lb / per_r;
    const int t = lb % per_r;
    const int tm = t / p.tiles_n, tn = t % p.tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const long long step = ga.ctr[0];
    const long long iter = ga.ctr[2 + r];
    const int valid = (p.kind == PK_PLAIN) ? p.M : batch_valid(p, r, step);
    const bool skip_update = (p.kind == PK_DW_UPDATE) && valid == 0;

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wk = wave % KSPLIT;
    const int wsp = wave / KSPLIT;
    const int wm = wsp / WAVES_N, wn = wsp % WAVES_N;
    const int g = lane >> 4, i16 = lane & 15;

    f32x4 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (!skip_update) {
      const T* A = reinterpret_cast<const T*>(p.A) + (long long)r * p.sA;
      const T* BTp = reinterpret_cast<const T*>(p.BT) + (long long)r * p.sB +
                     (p.bt_shadow ? (iter & 1) * p.bt_par : 0);
      const T* arow[WM];
      bool aones[WM];
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const int m = m0 + wm * WM * 16 + i * 16 + i16;
        aones[i] = (m == p.ones_row);
        arow[i] = nullptr;
        if (m < p.M && !aones[i]) {
          if (p.a_gather) {
            if (m < valid) arow[i] = A + batch_row(p, r, step, m) * p.lda;
          } else {
            arow[i] = A + (long long)m * p.lda;
          }
        }
      }
      const T* bcol[WN];
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int n = n0 + wn * WN * 16 + j * 16 + i16;
        bcol[j] = (n < p.N) ? BTp + (long long)n * p.ldb : nullptr;
      }
      const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
      const uint4 one = ones_frag<T>();
      auto load_frags = [&](int kc, uint4 (&a)[WM], uint4 (&b)[WN]) {
        const int kk = kc + g * EPL;
        const bool kin = kk < p.K;
#pragma unroll
        for (int i = 0; i < WM; ++i)
          a[i] = (kin && arow[i]) ? *reinterpret_cast<const uint4*>(arow[i] + kk) : ((kin && aones[i]) ? one : zero);
#pragma unroll
        for (int j = 0; j < WN; ++j)
          b[j] = (kin && bcol[j]) ? *reinterpret_cast<const uint4*>(bcol[j] + kk) : zero;
      };
      constexpr int KSTEP = KSPLIT * KC;
      int kc = wk * KC;
      uint4 a0[WM], b0[WN], a1[WM], b1[WN];
      if (kc < p.K) load_frags(kc, a0, b0);
      while (kc < p.K) {
        const int kn = kc + KSTEP;
        if (kn < p.K) load_frags(kn, a1, b1);
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) mma16<T>(acc[i][j], a0[i], b0[j]);
        if (kn >= p.K) break;
        const int kn2 = kn + KSTEP;
        if (kn2 < p.K) load_frags(kn2, a0, b0);
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) mma16<T>(acc[i][j], a1[i], b1[j]);
        kc = kn2;
      }
    }

    // ---- accumulators -> LDS (one region per k-split wave)
    float* region = smem + wk * BM * LDC;
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = wm * WM * 16 + i * 16 + g * 4 + q;
          const int col = wn * WN * 16 + j * 16 + i16;
          region[row * LDC + col] = acc[i][j][q];
        }
    __syncthreads();
    if constexpr (KSPLIT > 1) {
      for (int e = threadIdx.x; e < BM * BN; e += 256) {
        const int row = e / BN, col = e % BN;
        float s = smem[row * LDC + col];
#pragma unroll
        for (int w = 1; w < KSPLIT; ++w) s += smem[w * BM * LDC + row * LDC + col];
        smem[row * LDC + col] = s;
      }
      __syncthreads();
    }
    float* C = smem;  // final tile [BM][LDC]

    // ---- epilogues
    switch (p.kind) {
      case PK_PLAIN: {
        float* out = reinterpret_cast<float*>(p.D) + (long long)r * p.sD;
        for (int e = threadIdx.x; e < BM * BN; e += 256) {
          const int row = e / BN, col = e % BN, gm = m0 + row, gn = n0 + col;
          if (gm < p.M && gn < p.N) out[(long long)gm * p.ldd + gn] = C[row * LDC + col];
        }
        break;
      }
      case PK_FWD:
      case PK_DX: {
        const bool fwd = p.kind == PK_FWD;
        const float* bias = fwd && p.bias ? p.bias + (long long)r * p.sBias : nullptr;
        float* Z = p.Z ? p.Z + (long long)r * p.sZ : nullptr;
        const float keep_scale = p.rate > 0.f ? 1.f / (1.f - p.rate) : 1.f;
        const bool drop = p.rate > 0.f && !p.eval_mode;
        for (int e = threadIdx.x; e < BM * BN; e += 256) {
          const int row = e / BN, col = e % BN, gm = m0 + row, gn = n0 + col;
          if (gm >= p.M || gn >= p.N) continue;
          float v = C[row * LDC + col];
          float out = 0.f;
          if (gm < valid) {
            bool keep = true;
            if (drop) keep = dropout_uniform(ga.seed, r, p.layer, iter, (long long)gm * p.N + gn) >= p.rate;
            if (fwd) {
              const float z = v + (bias ? bias[gn] : 0.f);
              if (Z) Z[(long long)gm * p.ldz + gn] = z;
              out = keep ? act_fwd(p.act, z) * keep_scale : 0.f;
            } else {
              const float z = Z[(long long)gm * p.ldz + gn];
              out = keep ? v * act_grad(p.act, z) * keep_scale : 0.f;
            }
          } else if (fwd && Z) {
            Z[(long long)gm * p.ldz + gn] = 0.f;
          }
          if (p.D) st<T>(p.D, (long long)r * p.sD + (long long)gm * p.ldd + gn, out);
          C[row * LDC + col] = out;
        }
        if (p.DT) {
          __syncthreads();
          for (int e = threadIdx.x; e < BM * BN; e += 256) {
            const int col = e / BM, row = e % BM, gm = m0 + row, gn = n0 + col;
            if (gm < p.M && gn < p.N) st<T>(p.DT, (long long)r * p.sDT + (long long)gn * p.lddt + gm, C[row * LDC + col]);
          }
        }
        break;
      }
      case PK_FWD_LOSS: {
        // whole rows live in this tile (N <= BN, tiles_n == 1)
        const float* bias = p.bias ? p.bias + (long long)r * p.sBias : nullptr;
        for (int e = threadIdx.x; e < BM * BN; e += 256) {
          const int row = e / BN, col = e % BN;
          if (col < p.N) C[row * LDC + col] += bias ? bias[col] : 0.f;
        }
        __syncthreads();
        const int row = threadIdx.x;  // rows 0..BM-1 handled by the first BM threads
        RowOut ro;
        ro.loss = 0.f;
        for (int q = 0; q < 4; ++q) ro.metric[q] = 0.f;
        const int gm = m0 + row;
        const bool rvalid = row < BM && gm < p.M && gm < valid;
        const bool train = !p.eval_mode && p.D;
        const float inv_valid = valid > 0 ? 1.f / (float)valid : 0.f;
        if (rvalid && !p.Y) {  // predict only
          float* zrow = C + row * LDC;
          float* prow = p.pred ? p.pred + (long long)r * p.sPred + (p.chunk * p.B + gm) * p.ldp : nullptr;
          if (prow) row_predict<1>(0, p.N, p.act, [&](int j) { return zrow[j]; }, [&](int j, float v) { prow[j] = v; });
        } else if (rvalid) {
          const long long drow = batch_row(p, r, step, gm);
          const float* yrow = p.Y + (long long)r * p.sY + drow * p.ldy;
          float* zrow = C + row * LDC;
          float* prow = p.pred ? p.pred + (long long)r * p.sPred + (p.chunk * p.B + gm) * p.ldp : nullptr;
          // The gradient pass is row_loss's last pass and, for every j, reads z_j before
          // it writes dz_j, so dz can overwrite the logits in place in LDS.
          row_loss<1>(0, p.N, p.act, p.loss, p.met, p.nmet,
                      [&](int j) { return zrow[j]; },
                      [&](int j) { return yrow[j]; },
                      train, [&](int j, float v) { zrow[j] = v * inv_valid; },
                      prow != nullptr, [&](int j, float v) { prow[j] = v; }, ro);
        } else if (row < BM) {
          for (int j = 0; j < p.N; ++j) C[row * LDC + j] = 0.f;
        }
        // accumulate loss / metrics (wave 0 holds rows 0..63)
        if (p.acc && p.Y && threadIdx.x < 64 * ((BM + 63) / 64)) {
          float vals[6];
          vals[0] = rvalid ? ro.loss : 0.f;
          vals[1] = rvalid ? 1.f : 0.f;
          for (int q = 0; q < 4; ++q) vals[2 + q] = rvalid ? ro.metric[q] : 0.f;
          for (int q = 0; q < 2 + p.nmet; ++q) {
            float s = row_sum<64>(vals[q]);
            if ((threadIdx.x & 63) == 0 && s != 0.f)
              atomicAdd(p.acc + (long long)r * p.acc_stride + q, (double)s);
          }
        }
        if (train) {
          __syncthreads();  // dz rows were produced by one thread per row
          for (int e = threadIdx.x; e < BM * BN; e += 256) {
            const int rr = e / BN, col = e % BN, gmm = m0 + rr;
            if (gmm < p.M && col < p.N) st<T>(p.D, (long long)r * p.sD + (long long)gmm * p.ldd + col, C[rr * LDC + col]);
          }
          if (p.DT) {
            for (int e = threadIdx.x; e < BM * BN; e += 256) {
              const int col = e / BM, rr = e % BM, gmm = m0 + rr;
              if (gmm < p.M && col < p.N)
                st<T>(p.DT, (long long)r * p.sDT + (long long)col * p.lddt + gmm, C[rr * LDC + col]);
            }
          }
        }
        break;
      }
      case PK_DW_UPDATE:
      case PK_DW_GRAD: {
        if (skip_update) break;
        const bool upd = p.kind == PK_DW_UPDATE;
        float* P = p.P + (long long)r * p.sP;
        float* S = p.S ? p.S + (long long)r * p.sS : nullptr;
        float* G = p.G ? p.G + (long long)r * p.sG : nullptr;
        const long long wpar = ((iter + 1) & 1);
        for (int e = threadIdx.x; e < BM * BN; e += 256) {
          const int row = e / BN, col = e % BN, gm = m0 + row, gn = n0 + col;
          if (gm >= p.M || gn >= p.N) continue;
          const float gval = C[row * LDC + col] * p.op.grad_scale;
          const long long pidx = p.p_off + (long long)gm * p.N + gn;
          if (!upd) {
            if (valid > 0) G[pidx] = gval; else G[pidx] = 0.f;
            continue;
          }
          const float w = opt_update(p.op, P[pidx], gval, S, pidx, iter);
          P[pidx] = w;
          C[row * LDC + col] = w;
          if (gm < p.ones_row || p.ones_row < 0) {  // kernel row (not bias): refresh shadows
            if (p.Wsh) st<T>(p.Wsh, (long long)r * p.sWsh + wpar * p.wsh_par + (long long)gm * p.ldwsh + gn, w);
          }
        }
        if (upd && p.WTsh) {
          __syncthreads();
          for (int e = threadIdx.x; e < BM * BN; e += 256) {
            const int col = e / BM, row = e % BM, gm = m0 + row, gn = n0 + col;
            const int krows = p.ones_row >= 0 ? p.ones_row : p.M;
            if (gm < krows && gn < p.N)
              st<T>(p.WTsh, (long long)r * p.sWTsh + wpar * p.wtsh_par + (long long)gn * p.ldwtsh + gm, C[row * LDC + col]);
          }
        }
        break;
      }
    }
  }

  // ---- end-of-step counter advance (last arriving block)
  if (ga.advance) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      unsigned long long prev = atomicAdd(reinterpret_cast<unsigned long long*>(ga.ctr + 1), 1ull);
      if (prev == (unsigned long long)(ga.total_blocks - 1)) {
        const long long s = ga.ctr[0];
        for (int r = 0; r < ga.adv_R; ++r) {
          long long c = (long long)ga.adv_ntrain[r] - s * ga.adv_B;
          if (c > 0) ga.ctr[2 + r] += 1;
        }
        ga.ctr[0] = s + 1;
        ga.ctr[1] = 0;
        __threadfence();
      }
    }
  }
}

// ------------------------------------------------------------- host side
template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT>
static size_t lds_bytes() {
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  size_t lds = (size_t)KSPLIT * BM * (BN + 1) * sizeof(float);
  if (lds < 64 * 65 * sizeof(float)) lds = 64 * 65 * sizeof(float);  // gather-transpose
  return lds;
}

template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT>
static void set_attr() {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_grouped<T, WM, WN, WAVES_M, WAVES_N, KSPLIT>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_bytes<T, WM, WN, WAVES_M, WAVES_N, KSPLIT>());
}

template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT>
static hipError_t launch_cfg(const GroupArgs& ga, hipStream_t s) {
  if (ga.total_blocks <= 0) return hipSuccess;
  const size_t lds = lds_bytes<T, WM, WN, WAVES_M, WAVES_N, KSPLIT>();
  hipLaunchKernelGGL((gemm_grouped<T, WM, WN, WAVES_M, WAVES_N, KSPLIT>), dim3(ga.total_blocks), dim3(256), lds, s,
                     ga);
  return hipGetLastError();
}

}  // namespace ea

// cfg: 0 = LAT (64x32, split-K 4), 1 = THR (128x128)
extern "C" hipError_t ea_gemm_grouped(const ea::GroupArgs* ga, int bf16, int cfg, hipStream_t s) {
  using namespace ea;
  if (bf16) {
    if (cfg == 0) return launch_cfg<__bf16, 4, 2, 1, 1, 4>(*ga, s);
    return launch_cfg<__bf16, 4, 4, 2, 2, 1>(*ga, s);
  } else {
    if (cfg == 0) return launch_cfg<float, 4, 2, 1, 1, 4>(*ga, s);
    return launch_cfg<float, 4, 4, 2, 2, 1>(*ga, s);
  }
}

extern "C" void ea_gemm_init() {
  using namespace ea;
  static bool done = false;
  if (done) return;
  set_attr<__bf16, 4, 2, 1, 1, 4>();
  set_attr<__bf16, 4, 4, 2, 2, 1>();
  set_attr<float, 4, 2, 1, 1, 4>();
  set_attr<float, 4, 4, 2, 2, 1>();
  done = true;
}

extern "C" int ea_gemm_tile_m(int cfg) { return cfg == 0 ? 64 : 128; }
extern "C" int ea_gemm_tile_n(int cfg) { return cfg == 0 ? 32 : 128; }
extern "C" int ea_gather_tile() { return 64; }
