// Row-chain MLP training step (MI355X / gfx950): layers 1..L-1 of a small MLP
// for 16 batch rows per workgroup.
//
// The grouped plan runs a step of an L-layer Dense stack as 2L dependent
// launches (executor.cpp); every one of them is latency-bound at the MNIST/Boston
// sizes (profiles/README.md: 6 launches of 9-23 us, ~0.4 us of MFMA each). The
// row-chain plan cuts the step to three launches:
//
//   A  layer-0 forward as split-K partial slabs (many workgroups: layer 0's wide
//      K = 784 is the only large reduction) + the X^T gather of the batch
//   B  THIS KERNEL: for its 16 rows a workgroup sums the slabs (+ bias, act,
//      dropout), then runs every later layer's forward, the loss/metrics, and the
//      input gradients back down to dZ_0 -- all row-local work (a row's forward
//      and its dL/dz never need another row), so no inter-workgroup sync
//   C  the weight gradients of every layer (+ fused optimizer update) in one
//      grouped launch over the transposed operands B wrote
//
// Per layer the 16 x N output tile is split over the 4 waves by 16-column
// blocks (wave w owns blocks w, w+4, ...); the activation gradient factor
// G_l = act'(z) * keep / (1 - rate) stays in the registers of the lane that owns
// the element in the forward, because the input-gradient GEMM of the backward
// produces the same element in the same lane. Activations live in LDS as MFMA A
// operands; weights stream from L2 into a register ring started before the data
// they multiply is ready (layer 1's ring is issued at kernel entry, under the
// slab loads).
//
// Reference behaviour executed: one Keras `fit` step of a Dense stack
// (reference elephas/worker.py:41-42 -> model.fit), dropout masks identical to
// the grouped path (common.h dropout_u8), fp32 accumulation.
#include "common.h"
#include "mfma.h"
#include "loss_tile.h"

namespace ea {

namespace {

constexpr int RB = RC_ROWS;  // rows per workgroup

__device__ __forceinline__ uint4 zero4() { return make_uint4(0u, 0u, 0u, 0u); }

// keep-uniform of one column: the per-pair hash of dropout_u8 (common.h), so the
// grouped and row-chain plans draw identical masks
__device__ __forceinline__ float dropout_u1(uint32_t base, int row, int c) {
  const uint32_t h = fmix32(base ^ (((uint32_t)row << 16) | (uint32_t)(c >> 1)));
  return (float)((c & 1) ? (h >> 16) : (h & 0xFFFFu)) * (1.0f / 65536.0f);
}

// B-operand register ring of a 16-row GEMM C[16][N] = A[16][Kd] . BT[N][Kd]^T:
// the wave's column blocks w + 4j (j < NBW), PF reduction chunks in flight.
template <typename T, int NBW, int PF>
struct Ring {
  uint4 b[PF][NBW];
  const T* bp[NBW];
  int nks, Kd, nb;
};

template <typename T, int NBW, int PF>
__device__ __forceinline__ void ring_load(Ring<T, NBW, PF>& R, int slot, int ks, int w, int lane) {
  constexpr int EPL = KT<T>::EPL, KC = KT<T>::KC;
  const int kk = ks * KC + (lane >> 4) * EPL;
  const bool kin = kk < R.Kd;
  // raw values: the k-range mask is applied when the slot is consumed (ring_run), so
  // no wait is forced on a load right after it is issued
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    if (w + 4 * j < R.nb)  // wave-uniform
      R.b[slot][j] = *reinterpret_cast<const uint4*>(R.bp[j] + (kin ? kk : 0));
  }
}

// BT rows past N read row 0 and are never used (their blocks' columns are dropped)
template <typename T, int NBW, int PF>
__device__ __forceinline__ void ring_start(Ring<T, NBW, PF>& R, const T* BT, long long ldb, int Kd, int N, int w,
                                           int lane) {
  constexpr int KC = KT<T>::KC;
  R.Kd = Kd;
  R.nks = (Kd + KC - 1) / KC;
  R.nb = (N + 15) >> 4;
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const int col = (w + 4 * j) * 16 + (lane & 15);
    R.bp[j] = BT + (long long)(col < N ? col : 0) * ldb;
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < R.nks) ring_load(R, u, u, w, lane);
}

// consume the ring: acc[j] = A . BT over the whole reduction (A: LDS rows, stride
// lda). NKMAX = the most reduction chunks any layer of this instantiation has
// (compile-time, so the chunk loop unrolls and every ring slot index is a constant:
// with a runtime trip count hipcc shuttled the accumulators through AGPRs around
// every MFMA group)
template <typename T, int NBW, int PF, int NKMAX>
__device__ __forceinline__ void ring_run(Ring<T, NBW, PF>& R, const T* A, int lda, f32x4 (&acc)[NBW], int w,
                                         int lane) {
  constexpr int EPL = KT<T>::EPL, KC = KT<T>::KC;
#pragma unroll
  for (int j = 0; j < NBW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const T* arow = A + (lane & 15) * lda + (lane >> 4) * EPL;
  const int kg = (lane >> 4) * EPL;
#pragma unroll
  for (int ks = 0; ks < NKMAX; ++ks) {
    if (ks < R.nks) {
      const int slot = ks % PF;
      const bool kin = ks * KC + kg < R.Kd;
      uint4 b[NBW];
#pragma unroll
      for (int j = 0; j < NBW; ++j) b[j] = kin ? R.b[slot][j] : zero4();
      if (NKMAX > PF && ks + PF < R.nks) ring_load(R, slot, ks + PF, w, lane);
      const uint4 av = *reinterpret_cast<const uint4*>(arow + (kin ? ks * KC : 0));
      const uint4 a = kin ? av : zero4();
#pragma unroll
      for (int j = 0; j < NBW; ++j)
        if (w + 4 * j < R.nb) mma16<T>(acc[j], a, b[j]);
    }
  }
}

// 4 consecutive rows (4g..4g+3 of the tile) of one column of a transposed [N][Bp]
// output: one 16-byte (fp32) or 8-byte (bf16) store
template <typename T>
__device__ __forceinline__ void st4t(T* dst, const float (&v)[4]) {
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

// Workgroup barrier for LDS hand-offs only: __syncthreads() also waits for every
// outstanding global load (vmcnt(0)), which would drain the weight ring issued just
// before it and expose the latency the ring exists to hide.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void rstamp(const RcArgs& a, int k) {
  if (a.stamps && threadIdx.x == 0)
    a.stamps[((long long)blockIdx.y * gridDim.x + blockIdx.x) * 16 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}

}  // namespace

// T: compute dtype; L: Dense layers (2..4); NBW: 16-column blocks per wave of the
// widest hidden layer (2: widths <= 128, 4: <= 256, 8: <= 512 -- the tail chain of a
// deeper stack, L = 2 only: its layer 0 is the stack's second-to-last layer, whose
// pre-activations the grouped FWD launch before it wrote); GEN: the generic loss path
// (every Keras loss / activation / metric pairing, ~20k instructions) instead of
// the softmax + (sparse) categorical cross-entropy one -- picked on the host
template <typename T, int L, int NBW, bool GEN>
__global__ __launch_bounds__(256) void rowchain_kernel(RcArgs a) {
  constexpr int EPL = KT<T>::EPL, KC = KT<T>::KC;
  constexpr int NKMAX = NBW * 64 / KC;  // reduction chunks of the widest layer
  constexpr int PF = NKMAX < 8 ? NKMAX : 8;      // NBW 2: the whole reduction in flight
  constexpr int LD = NBW * 64 + (sizeof(T) == 2 ? 8 : 4);  // LDS row stride: conflict-free fragment reads
  constexpr int LDG = NBW * 64 + 4;                         // fp32 rows of G_0
  constexpr int NH = L - 1;                                 // activations D_0 .. D_{L-2} kept in LDS
  constexpr int NKF = (NKMAX + 3) / 4;                      // last-layer forward chunks per wave (K split 4 ways)
  constexpr int NKL = (32 + KC - 1) / KC;                   // last-layer input-gradient chunks (Np_last <= 32)
  constexpr int CPT = NBW * 4;                              // phase 0: columns per thread (16 threads per row)
  constexpr bool ZONLY = NBW >= 8;                          // the 512-wide tail reads z_0, never slabs
  constexpr int CPP = (CPT > 16 && !ZONLY) ? 16 : CPT;      // ... in passes of CPP columns
  constexpr int NPS = CPT / CPP;
  constexpr int MSPLIT = ZONLY ? 1 : RC_MAXSPLIT;           // slabs in flight
  static_assert(NBW < 8 || L == 2, "the 512-wide chain is the two-layer tail only");
  __shared__ __attribute__((aligned(16))) T sD[NH][RB * LD];
  __shared__ __attribute__((aligned(16))) T sdZ[L > 2 ? 2 : 1][RB * LD];
  __shared__ __attribute__((aligned(16))) float sG0[RB * LDG];
  __shared__ __attribute__((aligned(16))) float sRed[4][RB * 32];
  __shared__ __attribute__((aligned(16))) float sLg[RB * 36];
  __shared__ __attribute__((aligned(16))) float sY[RB * 32];
  __shared__ int sRow[RB];

  rstamp(a, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i16 = lane & 15, g = lane >> 4;
  // grid (R, row blocks), x fastest: a replica's row blocks share one XCD and the
  // replica index is a scalar register (uniform loads indexed by it stay scalar)
  const int r = blockIdx.x;
  const int m0 = blockIdx.y * RB;
  const float* Pr = a.P + (long long)r * a.sP;
  // layer-0 slabs and bias FIRST, before the step counter is read: none of their
  // addresses depend on it, so their round trip overlaps the counter's instead of
  // following it (phase 0 waits only for these; the wait counter drains in issue order)
  const int row = tid >> 4, c0 = (tid & 15) * CPT;
  const int m = m0 + row;
  float4 sv[MSPLIT][CPP / 4];
  float z[CPP];
  // pass ps of phase 0: this thread's columns c0 + ps * CPP + [0, CPP) of every slab + bias
  auto load_pass = [&](int ps) {
    const RcLayer l0 = a.ly[0];
    const float* Zr = a.Zp + (long long)r * a.sZp + (long long)(m < a.B ? m : 0) * l0.Np;
    const float* bias = Pr + l0.p_off + (long long)l0.K * l0.N;
    const int cb = c0 + ps * CPP;
    if (ZONLY || a.Zsrc) {  // tail chain: z_0 (bias included) as the grouped FWD launch stored it
      const float* zr = a.Zsrc + (long long)r * a.B * a.ldzs + (long long)(m < a.B ? m : 0) * a.ldzs;
      const bool vec = (a.ldzs & 3) == 0;  // 16-byte rows: cb is a multiple of 4
#pragma unroll
      for (int v = 0; v < CPP / 4; ++v) {
        const int c = cb + 4 * v;
        if (vec && c + 4 <= l0.N) {
          const float4 q = *reinterpret_cast<const float4*>(zr + c);
          z[4 * v] = q.x; z[4 * v + 1] = q.y; z[4 * v + 2] = q.z; z[4 * v + 3] = q.w;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float e = zr[c + k < l0.N ? c + k : 0];
            z[4 * v + k] = c + k < l0.N ? e : 0.f;
          }
        }
      }
      return;
    }
#pragma unroll
    for (int kc = 0; kc < MSPLIT; ++kc) {
      const float* slab = Zr + (long long)(kc < a.nsplitk ? kc : 0) * a.sZpk;
#pragma unroll
      for (int v = 0; v < CPP / 4; ++v) {
        const int c = cb + 4 * v;
        sv[kc][v] = *reinterpret_cast<const float4*>(slab + (c < l0.Np ? c : 0));
      }
    }
#pragma unroll
    for (int i = 0; i < CPP; ++i) {
      const int c = cb + i;
      const bool cv = c < l0.N && l0.has_bias;
      const float bv = bias[cv ? c : 0];
      z[i] = cv ? bv : 0.f;
    }
  };
  load_pass(0);
  const long long s0 = ld_inv(a.ctr);
  const long long step = s0 + a.step_off;
  const long long cnt = (long long)ld_inv(a.ntrain + r) - step * a.B;
  const int valid = (int)(cnt < 0 ? 0 : (cnt > a.B ? a.B : cnt));
  if (valid == 0) return;  // no batch for this replica this step: DW skips its update too
  const long long iter = iter_at(a.ctr, a.ntrain, a.B, r, s0, a.step_off);
  const long long rpar = iter & 1;
  const T* Wcur = reinterpret_cast<const T*>(a.Wsh) + (long long)r * a.sWsh + rpar * a.wsh_par;
  const T* WTcur = reinterpret_cast<const T*>(a.WTsh) + (long long)r * a.sWTsh + rpar * a.wtsh_par;
  const RcLayer LL = a.ly[L - 1];
  const bool rv = m < valid;

  // ---- everything that does not depend on this step's data is requested up front,
  //      under the slab loads: the batch rows' targets, the first hidden layer's
  //      weight ring, the last layer's forward and input-gradient fragments, biases
  int prow[2];
  {
    const int* pr = a.perm + (long long)r * a.sPerm + step * a.B + m0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (tid >> 5) + 8 * i;
      const bool in = m0 + row < valid;
      const int v = pr[in ? row : 0];
      prow[i] = in ? v : -1;
    }
  }
  Ring<T, NBW, PF> ring;
  if constexpr (L > 2) ring_start(ring, WTcur + a.ly[1].wtsh_off, a.ly[1].Kp, a.ly[1].Kp, a.ly[1].N, w, lane);
  uint4 wl[NKF][2];  // last layer forward: B^T rows = its <= 32 outputs, chunks w + 4i
  {
    const T* BT = WTcur + LL.wtsh_off;
#pragma unroll
    for (int i = 0; i < NKF; ++i) {
      const int kk = (w + 4 * i) * KC + g * EPL;
      const bool kin = kk < LL.Kp;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = j * 16 + i16;
        const uint4 v = *reinterpret_cast<const uint4*>(BT + (long long)(col < LL.N ? col : 0) * LL.Kp + (kin ? kk : 0));
        wl[i][j] = (kin && col < LL.N) ? v : zero4();
      }
    }
  }
  uint4 xl[NKL][NBW];  // last layer input gradient: B^T rows = its K inputs, reduction over Np_last
  {
    const T* BT = Wcur + LL.wsh_off;
#pragma unroll
    for (int i = 0; i < NKL; ++i) {
      const int kk = i * KC + g * EPL;
      const bool kin = kk < LL.Np;
#pragma unroll
      for (int j = 0; j < NBW; ++j) {
        const int col = (w + 4 * j) * 16 + i16;
        const uint4 v = *reinterpret_cast<const uint4*>(BT + (long long)(col < LL.K ? col : 0) * LL.Np + (kin ? kk : 0));
        xl[i][j] = (kin && col < LL.K) ? v : zero4();
      }
    }
  }
  float hb[L][NBW];  // hidden-layer biases in the lanes that own the columns
#pragma unroll
  for (int l = 1; l < L - 1; ++l) {
    const RcLayer ly = a.ly[l];
    const float* bias = Pr + ly.p_off + (long long)ly.K * ly.N;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const int col = (w + 4 * j) * 16 + i16;
      const bool cv = col < ly.N && ly.has_bias;
      const float v = bias[cv ? col : 0];
      hb[l][j] = cv ? v : 0.f;
    }
  }
  float lastb;
  {
    const int c = tid & 31;
    const bool cv = c < LL.N && LL.has_bias;
    const float v = Pr[LL.p_off + (long long)LL.K * LL.N + (cv ? c : 0)];
    lastb = cv ? v : 0.f;
  }

  float yv[2];  // this thread's two target values (rows (tid >> 5) + 8i, column tid & 31)

  // G_l (l >= 1) = act'(z_l) * keep / (1 - rate), owned by the lane that owns the
  // element in both the forward and the input-gradient GEMM; G_0 goes through LDS
  float G[L][NBW][4];

  // ---- phase 0: z_0 = sum of the split-K slabs + bias -> D_0 (LDS) and G_0 (LDS);
  //      one row and CPT consecutive columns per thread: 16-byte slab loads, all
  //      issued before the first add
  {
    const RcLayer l0 = a.ly[0];
    // the targets of this workgroup's rows (perm rows requested at entry): loaded now,
    // stored to LDS only before the loss, so nothing waits for this second round trip
    {
      const int ldy = (int)a.ldy;
      const float* Yb = a.Y + (long long)r * a.sY;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + 256 * i, j = e & 31;
        const bool in = prow[i] >= 0 && j < ldy;
        yv[i] = Yb[in ? (long long)prow[i] * ldy + j : 0];
        if (!in) prow[i] = -1;
      }
      if (tid < RB) sRow[tid] = m0 + tid < valid ? 1 : -1;
    }
    const float keep_scale = l0.rate > 0.f ? 1.f / (1.f - l0.rate) : 1.f;
    const uint32_t dbase = dropout_base(a.seed, r, a.l0, iter);
#pragma unroll
    for (int ps = 0; ps < NPS; ++ps) {
      if (ps > 0) load_pass(ps);
      const int cb = c0 + ps * CPP;
#pragma unroll
      for (int kc = 0; kc < MSPLIT; ++kc) {
        if (kc >= a.nsplitk) break;  // uniform; every load above is already in flight
#pragma unroll
        for (int v = 0; v < CPP / 4; ++v) {
          z[4 * v + 0] += sv[kc][v].x;
          z[4 * v + 1] += sv[kc][v].y;
          z[4 * v + 2] += sv[kc][v].z;
          z[4 * v + 3] += sv[kc][v].w;
        }
      }
      if (ps == 0) rstamp(a, 12);  // slabs summed
      float o[CPP], gg[CPP], dv[CPP], gv[CPP];
      act_fg_v<CPP>(l0.act, z, o, gg);
#pragma unroll
      for (int i = 0; i < CPP; ++i) {
        const int c = cb + i;
        const bool live = c < l0.N && rv;
        const float u = (live && l0.rate > 0.f) ? dropout_u1(dbase, m, c) : 1.f;
        const bool keep = live && u >= l0.rate;
        dv[i] = keep ? o[i] * keep_scale : 0.f;
        gv[i] = keep ? gg[i] * keep_scale : 0.f;
      }
#pragma unroll
      for (int i = 0; i < CPP; i += 4) {
        if (cb + i < NBW * 64) {
          *reinterpret_cast<float4*>(sG0 + row * LDG + cb + i) = make_float4(gv[i], gv[i + 1], gv[i + 2], gv[i + 3]);
#pragma unroll
          for (int k = 0; k < 4; ++k) sD[0][row * LD + cb + i + k] = from_f<T>(dv[i + k]);
        }
      }
    }
  }
  rstamp(a, 13);  // D_0 / G_0 in LDS
  lds_barrier();
  rstamp(a, 14);
  // D_0^T (layer 1's weight-gradient operand) from the LDS tile: 4 rows per store
  // (the tail chain's grouped FWD launch already stored it)
  if (!a.Zsrc) {
    const RcLayer l0 = a.ly[0];
    T* DT0 = reinterpret_cast<T*>(l0.DT) + (long long)r * l0.N * a.Bp;
    for (int e = tid; e < l0.N * (RB / 4); e += 256) {
      const int c = e / (RB / 4), rq = (e - c * (RB / 4)) * 4;
      if (m0 + rq >= a.Bp) continue;
      float v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = to_f<T>(sD[0][(rq + k) * LD + c]);
      st4t<T>(DT0 + (long long)c * a.Bp + m0 + rq, v);
    }
  }
  rstamp(a, 1);

  // ---- forward through the hidden layers 1 .. L-2
#pragma unroll
  for (int l = 1; l < L - 1; ++l) {
    const RcLayer ly = a.ly[l];
    f32x4 acc[NBW];
    ring_run<T, NBW, PF, NKMAX>(ring, sD[l - 1], LD, acc, w, lane);
    rstamp(a, 2);
    // the ring's next weights stream in under this epilogue and the loss: the next
    // hidden layer's W^T, or after the last one the row-major W_{L-2} of the backward
    if (l + 1 < L - 1)
      ring_start(ring, WTcur + a.ly[l + 1].wtsh_off, a.ly[l + 1].Kp, a.ly[l + 1].Kp, a.ly[l + 1].N, w, lane);
    else
      ring_start(ring, Wcur + a.ly[L - 2].wsh_off, a.ly[L - 2].Np, a.ly[L - 2].Np, a.ly[L - 2].K, w, lane);
    const int nb = (ly.N + 15) >> 4;
    float z[NBW * 4], o[NBW * 4], gg[NBW * 4];
#pragma unroll
    for (int j = 0; j < NBW; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) z[j * 4 + q] = acc[j][q] + hb[l][j];
    act_fg_v<NBW * 4>(ly.act, z, o, gg);
    const float keep_scale = ly.rate > 0.f ? 1.f / (1.f - ly.rate) : 1.f;
    const uint32_t dbase = dropout_base(a.seed, r, a.l0 + l, iter);
    T* DTl = reinterpret_cast<T*>(ly.DT) + (long long)r * ly.N * a.Bp;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      if (w + 4 * j >= nb) continue;
      const int col = (w + 4 * j) * 16 + i16;
      float dv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + 4 * g + q;
        const bool live = col < ly.N && m < valid;
        const float u = (live && ly.rate > 0.f) ? dropout_u1(dbase, m, col) : 1.f;
        const bool keep = live && u >= ly.rate;
        dv[q] = keep ? o[j * 4 + q] * keep_scale : 0.f;
        G[l][j][q] = keep ? gg[j * 4 + q] * keep_scale : 0.f;
        sD[l][(4 * g + q) * LD + col] = from_f<T>(dv[q]);
      }
      if (col < ly.N && m0 + 4 * g < a.Bp) st4t<T>(DTl + (long long)col * a.Bp + m0 + 4 * g, dv);
    }
    lds_barrier();
  }
  rstamp(a, 3);

  // ---- last layer (N <= 32): the 4 waves split the reduction over their
  //      preloaded fragments, partial tiles summed through LDS, then the loss
  {
#pragma unroll
    for (int i = 0; i < 2; ++i) sY[tid + 256 * i] = prow[i] >= 0 ? yv[i] : 0.f;
    const RcLayer ly = LL;
    const int nks = (ly.Kp + KC - 1) / KC;
    const int nb = (ly.N + 15) >> 4;  // 1 or 2
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const T* arow = sD[L - 2] + i16 * LD + g * EPL;
#pragma unroll
    for (int i = 0; i < NKF; ++i) {
      const int ks = w + 4 * i;
      if (ks < nks) {
        const bool kin = ks * KC + g * EPL < ly.Kp;
        const uint4 av = *reinterpret_cast<const uint4*>(arow + (kin ? ks * KC : 0));
        const uint4 a0 = kin ? av : zero4();
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (j < nb) mma16<T>(acc[j], a0, wl[i][j]);
      }
    }
    rstamp(a, 4);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) sRed[w][(4 * g + q) * 32 + j * 16 + i16] = acc[j][q];
    lds_barrier();
    for (int e = tid; e < RB * 32; e += 256) {  // column e & 31 == tid & 31: lastb
      const int row = e >> 5, c = e & 31;
      const float v = sRed[0][e] + sRed[1][e] + sRed[2][e] + sRed[3][e];
      sLg[row * 36 + c] = (c < ly.N) ? v + lastb : 0.f;
    }
    lds_barrier();
    rstamp(a, 5);
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
    constexpr bool fast = !GEN;
    if constexpr (GEN) {
      loss_tile_lds<RB, 36, 32>(q, r, m0, sLg, sY, sRow, true, inv_valid, sums);
    } else if (w == 0) {  // one quad per row: the 16 rows are wave 0
      if (ly.N <= 16) loss_tile_cce<4, RB, 36, 32>(q, r, m0, sLg, sY, sRow, true, inv_valid, sums);
      else loss_tile_cce<8, RB, 36, 32>(q, r, m0, sLg, sY, sRow, true, inv_valid, sums);
    }
    rstamp(a, 6);
    if (a.acc && (!fast || w == 0)) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        if (i < 2 + a.nmet) {
          const float sv = row_sum<64>(sums[i]);
          if (lane == 0 && sv != 0.f) atomicAdd(a.acc + (long long)r * a.acc_stride + i, (double)sv);
        }
      }
    }
    lds_barrier();
    // dZ_{L-1}: A operand of the first input-gradient GEMM (LDS, zero-padded to the
    // 16-column tile) and the B^T operand of its weight gradient ([N][Bp] global)
    T* dZT = reinterpret_cast<T*>(ly.dZT) + (long long)r * ly.N * a.Bp;
    for (int e = tid; e < RB * 32; e += 256) {
      const int row = e >> 5, c = e & 31;
      sdZ[0][row * LD + c] = from_f<T>(c < ly.N ? sLg[row * 36 + c] : 0.f);
    }
    for (int e = tid; e < ly.N * (RB / 4); e += 256) {
      const int c = e / (RB / 4), rq = (e - c * (RB / 4)) * 4;
      if (m0 + rq >= a.Bp) continue;
      float v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = sLg[(rq + k) * 36 + c];
      st4t<T>(dZT + (long long)c * a.Bp + m0 + rq, v);
    }
    lds_barrier();
  }
  rstamp(a, 7);

  // ---- backward: dZ_{l-1} = (dZ_l . W_l^T) * G_{l-1} for l = L-1 .. 1; the last
  //      layer's fragments were loaded at entry, the others stream through the ring
  int cur = 0;
#pragma unroll
  for (int l = L - 1; l >= 1; --l) {
    const RcLayer ly = a.ly[l];
    const RcLayer pv = a.ly[l - 1];
    f32x4 acc[NBW];
    if (l == L - 1) {
#pragma unroll
      for (int j = 0; j < NBW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const T* arow = sdZ[cur] + i16 * LD + g * EPL;
      const int nb = (ly.K + 15) >> 4;
#pragma unroll
      for (int i = 0; i < NKL; ++i) {
        const bool kin = i * KC + g * EPL < ly.Np;
        const uint4 av = *reinterpret_cast<const uint4*>(arow + (kin ? i * KC : 0));
        const uint4 a0 = kin ? av : zero4();
#pragma unroll
        for (int j = 0; j < NBW; ++j)
          if (w + 4 * j < nb) mma16<T>(acc[j], a0, xl[i][j]);
      }
    } else {
      ring_run<T, NBW, PF, NKMAX>(ring, sdZ[cur], LD, acc, w, lane);
      if (l > 1) ring_start(ring, Wcur + a.ly[l - 1].wsh_off, a.ly[l - 1].Np, a.ly[l - 1].Np, a.ly[l - 1].K, w, lane);
    }
    rstamp(a, 8 + 2 * (L - 1 - l));
    const int nb = (ly.K + 15) >> 4;
    T* dZT = reinterpret_cast<T*>(pv.dZT) + (long long)r * pv.N * a.Bp;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      if (w + 4 * j >= nb) continue;
      const int col = (w + 4 * j) * 16 + i16;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gq = (l - 1 >= 1) ? G[l - 1][j][q] : sG0[(4 * g + q) * LDG + (col < NBW * 64 ? col : 0)];
        v[q] = col < pv.N ? acc[j][q] * gq : 0.f;
        if (l > 1) sdZ[cur ^ 1][(4 * g + q) * LD + col] = from_f<T>(v[q]);
      }
      if (col < pv.N && m0 + 4 * g < a.Bp) st4t<T>(dZT + (long long)col * a.Bp + m0 + 4 * g, v);
      if (l == 1 && a.dZ0 && col < pv.Np) {  // tail chain: row-major dZ_0 (zero past N)
        T* d = reinterpret_cast<T*>(a.dZ0) + (long long)r * a.B * a.ldz0 + col;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (m0 + 4 * g + q < a.B) d[(long long)(m0 + 4 * g + q) * a.ldz0] = from_f<T>(v[q]);
      }
    }
    cur ^= 1;
    if (l > 1) lds_barrier();
    rstamp(a, 9 + 2 * (L - 1 - l));
  }
}

}  // namespace ea

using namespace ea;

namespace {
// one instantiation per (dtype, width class, loss path); the 512-wide class exists for
// the two-layer tail only
template <typename TT, int NB, bool GN>
void launch_rc(const RcArgs* a, dim3 grid, hipStream_t s) {
  if constexpr (NB == 8) {
    hipLaunchKernelGGL((rowchain_kernel<TT, 2, NB, GN>), grid, dim3(256), 0, s, *a);
  } else {
    switch (a->L) {
      case 2: hipLaunchKernelGGL((rowchain_kernel<TT, 2, NB, GN>), grid, dim3(256), 0, s, *a); break;
      case 3: hipLaunchKernelGGL((rowchain_kernel<TT, 3, NB, GN>), grid, dim3(256), 0, s, *a); break;
      default: hipLaunchKernelGGL((rowchain_kernel<TT, 4, NB, GN>), grid, dim3(256), 0, s, *a); break;
    }
  }
}
template <typename TT, int NB>
void launch_rc_g(const RcArgs* a, bool fast, dim3 grid, hipStream_t s) {
  if (fast) launch_rc<TT, NB, false>(a, grid, s);
  else launch_rc<TT, NB, true>(a, grid, s);
}
}  // namespace

// grid: (R, ceil(B / 16)) workgroups of 256 threads
extern "C" hipError_t ea_rowchain(const RcArgs* a, int bf16, int nbw, hipStream_t s) {
  if (a->L < 2 || a->L > RC_MAXL || (nbw != 2 && nbw != 4 && nbw != 8)) return hipErrorInvalidValue;
  if (nbw == 8 && (a->L != 2 || !a->Zsrc || a->nsplitk != 0)) return hipErrorInvalidValue;
  const dim3 grid(a->R, (a->B + RC_ROWS - 1) / RC_ROWS);
  // the loss_tile_cce path: softmax + (sparse) CCE with accuracy / CCE metrics
  bool fast = a->ly[a->L - 1].act == ACT_SOFTMAX && (a->loss == LOSS_CCE || a->loss == LOSS_SPARSE_CCE) &&
              a->ly[a->L - 1].N <= 32;
  for (int i = 0; i < a->nmet; ++i)
    fast = fast && (a->met[i] == MET_ACC_CAT || a->met[i] == MET_ACC_SPARSE || a->met[i] == LOSS_CCE ||
                    a->met[i] == LOSS_SPARSE_CCE);
  if (bf16) {
    if (nbw == 2) launch_rc_g<__bf16, 2>(a, fast, grid, s);
    else if (nbw == 4) launch_rc_g<__bf16, 4>(a, fast, grid, s);
    else launch_rc_g<__bf16, 8>(a, fast, grid, s);
  } else {
    if (nbw == 2) launch_rc_g<float, 2>(a, fast, grid, s);
    else if (nbw == 4) launch_rc_g<float, 4>(a, fast, grid, s);
    else launch_rc_g<float, 8>(a, fast, grid, s);
  }
  return hipGetLastError();
}
