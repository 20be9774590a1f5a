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
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    if (w + 4 * j < R.nb) {  // wave-uniform
      const uint4 v = *reinterpret_cast<const uint4*>(R.bp[j] + (kin ? kk : 0));
      R.b[slot][j] = kin ? v : zero4();
    }
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
      uint4 b[NBW];
#pragma unroll
      for (int j = 0; j < NBW; ++j) b[j] = R.b[slot][j];
      if (NKMAX > PF && ks + PF < R.nks) ring_load(R, slot, ks + PF, w, lane);
      const bool kin = ks * KC + kg < R.Kd;
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

// the generic loss (every Keras loss / activation / metric pairing) is a call, not
// inlined: it is ~20k instructions that the softmax + CCE path never executes
__device__ __attribute__((noinline)) void rc_loss_generic(const Prob& q, int r, int m0, float* sLg, const float* sY,
                                                          const int* sRow, float inv_valid, float (&sums)[6]) {
  loss_tile_lds<RB, 36, 32>(q, r, m0, sLg, sY, sRow, true, inv_valid, sums);
}

__device__ __forceinline__ void rstamp(const RcArgs& a, int k) {
  if (a.stamps && threadIdx.x == 0) a.stamps[(long long)blockIdx.x * 16 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}

}  // namespace

// T: compute dtype; L: Dense layers (2..4); NBW: 16-column blocks per wave of the
// widest hidden layer (2: widths <= 128, 4: <= 256)
template <typename T, int L, int NBW>
__global__ __launch_bounds__(256) void rowchain_kernel(RcArgs a) {
  constexpr int NKMAX = NBW * 64 / KT<T>::KC;  // reduction chunks of the widest layer
  constexpr int PF = NKMAX < 8 ? NKMAX : 8;      // NBW 2: the whole reduction in flight
  constexpr int LD = NBW * 64 + (sizeof(T) == 2 ? 8 : 4);  // LDS row stride: conflict-free fragment reads
  constexpr int NH = L - 1;                                 // activations D_0 .. D_{L-2} kept in LDS
  __shared__ __attribute__((aligned(16))) T sD[NH][RB * LD];
  __shared__ __attribute__((aligned(16))) T sdZ[2][RB * LD];
  __shared__ __attribute__((aligned(16))) float sRed[4][RB * 32];
  __shared__ __attribute__((aligned(16))) float sLg[RB * 36];
  __shared__ __attribute__((aligned(16))) float sY[RB * 32];
  __shared__ int sRow[RB];

  rstamp(a, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i16 = lane & 15, g = lane >> 4;
  const int tiles = (a.B + RB - 1) / RB;
  (void)tiles;
  const int r = blockIdx.x % a.R;  // replica-minor: a replica's row blocks share one XCD
  const int m0 = (blockIdx.x / a.R) * RB;
  const long long s0 = ld_inv(a.ctr);
  const long long step = s0 + a.step_off;
  const long long cnt = (long long)ld_inv(a.ntrain + r) - step * a.B;
  const int valid = (int)(cnt < 0 ? 0 : (cnt > a.B ? a.B : cnt));
  if (valid == 0) return;  // no batch for this replica this step: DW skips its update too
  const long long iter = iter_at(a.ctr, a.ntrain, a.B, r, s0, a.step_off);
  const long long rpar = iter & 1;
  const T* Wcur = reinterpret_cast<const T*>(a.Wsh) + (long long)r * a.sWsh + rpar * a.wsh_par;
  const T* WTcur = reinterpret_cast<const T*>(a.WTsh) + (long long)r * a.sWTsh + rpar * a.wtsh_par;
  const float* Pr = a.P + (long long)r * a.sP;

  // layer 1's weights start streaming now, under the slab loads below (the last
  // layer has a K-split loop of its own)
  Ring<T, NBW, PF> ring;
  if constexpr (L > 2) ring_start(ring, WTcur + a.ly[1].wtsh_off, a.ly[1].Kp, a.ly[1].Kp, a.ly[1].N, w, lane);

  // G_l = act'(z_l) * keep / (1 - rate), owned by the lane that owns the element
  float G[NH][NBW][4];

  // biases of layers 1 .. L-1 (fp32 master), loaded now: nothing below waits a memory
  // round trip for them
  float hb[L][NBW];
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
    const RcLayer ly = a.ly[L - 1];
    const int c = tid & 31;
    const bool cv = c < ly.N && ly.has_bias;
    const float v = Pr[ly.p_off + (long long)ly.K * ly.N + (cv ? c : 0)];
    lastb = cv ? v : 0.f;
  }

  // ---- phase 0: z_0 = sum of the split-K slabs + bias -> D_0 (LDS), D_0^T, G_0;
  //      the targets of this workgroup's rows
  {
    const RcLayer l0 = a.ly[0];
    const float* Zr = a.Zp + (long long)r * a.sZp;
    const float* bias = Pr + l0.p_off + (long long)l0.K * l0.N;
    const int nb = (l0.N + 15) >> 4;
    float z[NBW * 4];
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const int col = (w + 4 * j) * 16 + i16;
      const bool cv = (w + 4 * j < nb) && col < l0.N;
      const float bv = (cv && l0.has_bias) ? bias[col] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) z[j * 4 + q] = bv;
      if (w + 4 * j < nb) {
        // every slab load is issued before the first add (a data-dependent loop exit
        // would serialise one memory round trip per slab)
        float sv[RC_MAXSPLIT][4];
#pragma unroll
        for (int kc = 0; kc < RC_MAXSPLIT; ++kc) {
          const float* slab = Zr + (long long)(kc < a.nsplitk ? kc : 0) * a.sZpk;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int m = m0 + 4 * g + q;
            const bool in = cv && m < valid;
            sv[kc][q] = slab[in ? (long long)m * l0.N + col : 0];
          }
        }
#pragma unroll
        for (int kc = 0; kc < RC_MAXSPLIT; ++kc)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const bool in = cv && m0 + 4 * g + q < valid && kc < a.nsplitk;
            z[j * 4 + q] += in ? sv[kc][q] : 0.f;
          }
      }
    }
    // targets (rows in epoch order through perm) and the row-valid map
    {
      const int ldy = (int)a.ldy;
      const float* Yb = a.Y + (long long)r * a.sY;
      const int* pr = a.perm + (long long)r * a.sPerm + step * a.B + m0;
      for (int e = tid; e < RB * 32; e += 256) {
        const int row = e >> 5, j = e & 31;
        const bool in = m0 + row < valid && j < ldy;
        const int dr = in ? pr[row] : 0;
        sY[e] = in ? Yb[(long long)dr * ldy + j] : 0.f;
      }
      if (tid < RB) sRow[tid] = m0 + tid < valid ? 1 : -1;
    }
    float o[NBW * 4], gg[NBW * 4];
    act_fg_v<NBW * 4>(l0.act, z, o, gg);
    const float keep_scale = l0.rate > 0.f ? 1.f / (1.f - l0.rate) : 1.f;
    const uint32_t dbase = dropout_base(a.seed, r, 0, iter);
    T* DT0 = reinterpret_cast<T*>(l0.DT) + (long long)r * l0.N * a.Bp;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      if (w + 4 * j >= nb) continue;
      const int col = (w + 4 * j) * 16 + i16;
      float dv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + 4 * g + q;
        const bool live = col < l0.N && m < valid;
        const float u = (live && l0.rate > 0.f) ? dropout_u1(dbase, m, col) : 1.f;
        const bool keep = live && u >= l0.rate;
        dv[q] = keep ? o[j * 4 + q] * keep_scale : 0.f;
        G[0][j][q] = keep ? gg[j * 4 + q] * keep_scale : 0.f;
        sD[0][(4 * g + q) * LD + col] = from_f<T>(dv[q]);
      }
      if (col < l0.N && m0 + 4 * g < a.Bp) st4t<T>(DT0 + (long long)col * a.Bp + m0 + 4 * g, dv);
    }
  }
  lds_barrier();
  rstamp(a, 1);

  // ---- forward through the hidden layers 1 .. L-2
#pragma unroll
  for (int l = 1; l < L - 1; ++l) {
    const RcLayer ly = a.ly[l];
    f32x4 acc[NBW];
    ring_run<T, NBW, PF, NKMAX>(ring, sD[l - 1], LD, acc, w, lane);
    rstamp(a, 2);
    // the next hidden layer's weights stream in under this epilogue
    if (l + 1 < L - 1)
      ring_start(ring, WTcur + a.ly[l + 1].wtsh_off, a.ly[l + 1].Kp, a.ly[l + 1].Kp, a.ly[l + 1].N, w, lane);
    const int nb = (ly.N + 15) >> 4;
    float z[NBW * 4], o[NBW * 4], gg[NBW * 4];
#pragma unroll
    for (int j = 0; j < NBW; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) z[j * 4 + q] = acc[j][q] + hb[l][j];
    act_fg_v<NBW * 4>(ly.act, z, o, gg);
    const float keep_scale = ly.rate > 0.f ? 1.f / (1.f - ly.rate) : 1.f;
    const uint32_t dbase = dropout_base(a.seed, r, l, iter);
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

  // ---- last layer (N <= 32): the 4 waves split the reduction, partial tiles
  //      summed through LDS, then the loss over whole rows
  {
    constexpr int l = L - 1;
    const RcLayer ly = a.ly[l];
    constexpr int EPL = KT<T>::EPL, KC = KT<T>::KC;
    const T* BT = WTcur + ly.wtsh_off;
    const int nks = (ly.Kp + KC - 1) / KC;
    const int nb = (ly.N + 15) >> 4;  // 1 or 2
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const T* bp[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = j * 16 + i16;
      bp[j] = BT + (long long)(col < ly.N ? col : 0) * ly.Kp;
    }
    const T* arow = sD[l - 1] + i16 * LD + g * EPL;
    for (int ks = w; ks < nks; ks += 4) {
      const int kk = ks * KC + g * EPL;
      const bool kin = kk < ly.Kp;
      uint4 b[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint4 v = *reinterpret_cast<const uint4*>(bp[j] + (kin ? kk : 0));
        b[j] = (kin && j < nb) ? v : zero4();
      }
      const uint4 av = *reinterpret_cast<const uint4*>(arow + (kin ? ks * KC : 0));
      const uint4 av0 = kin ? av : zero4();
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (j < nb) mma16<T>(acc[j], av0, b[j]);
    }
    rstamp(a, 4);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) sRed[w][(4 * g + q) * 32 + j * 16 + i16] = acc[j][q];
    // the backward's first weights (layer L-1, row-major image) stream in now
    ring_start(ring, Wcur + ly.wsh_off, ly.Np, ly.Np, ly.K, w, lane);
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
    if (softmax_cce_fast(q)) {
      if (ly.N <= 16) loss_tile_cce<4, RB, 36, 32>(q, r, m0, sLg, sY, sRow, true, inv_valid, sums);
      else loss_tile_cce<8, RB, 36, 32>(q, r, m0, sLg, sY, sRow, true, inv_valid, sums);
    } else {
      rc_loss_generic(q, r, m0, sLg, sY, sRow, inv_valid, sums);
    }
    rstamp(a, 6);
    if (a.acc) {
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

  // ---- backward: dZ_{l-1} = (dZ_l . W_l^T) * G_{l-1} for l = L-1 .. 1
  int cur = 0;
#pragma unroll
  for (int l = L - 1; l >= 1; --l) {
    const RcLayer ly = a.ly[l];
    const RcLayer pv = a.ly[l - 1];
    f32x4 acc[NBW];
    ring_run<T, NBW, PF, NKMAX>(ring, sdZ[cur], LD, acc, w, lane);
    rstamp(a, 8 + 2 * (L - 1 - l));
    if (l > 1) ring_start(ring, Wcur + a.ly[l - 1].wsh_off, a.ly[l - 1].Np, a.ly[l - 1].Np, a.ly[l - 1].K, w, lane);
    const int nb = (ly.K + 15) >> 4;
    T* dZT = reinterpret_cast<T*>(pv.dZT) + (long long)r * pv.N * a.Bp;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      if (w + 4 * j >= nb) continue;
      const int col = (w + 4 * j) * 16 + i16;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = col < pv.N ? acc[j][q] * G[l - 1][j][q] : 0.f;
        if (l > 1) sdZ[cur ^ 1][(4 * g + q) * LD + col] = from_f<T>(v[q]);
      }
      if (col < pv.N && m0 + 4 * g < a.Bp) st4t<T>(dZT + (long long)col * a.Bp + m0 + 4 * g, v);
    }
    cur ^= 1;
    if (l > 1) lds_barrier();
    rstamp(a, 9 + 2 * (L - 1 - l));
  }
}

}  // namespace ea

using namespace ea;

// grid: R x ceil(B / 16) workgroups of 256 threads
extern "C" hipError_t ea_rowchain(const RcArgs* a, int bf16, int nbw, hipStream_t s) {
  if (a->L < 2 || a->L > RC_MAXL || (nbw != 2 && nbw != 4)) return hipErrorInvalidValue;
  const dim3 grid(a->R * ((a->B + RC_ROWS - 1) / RC_ROWS));
#define EA_RC(TT, LL, NB) hipLaunchKernelGGL((rowchain_kernel<TT, LL, NB>), grid, dim3(256), 0, s, *a)
#define EA_RC_L(TT, NB)   \
  switch (a->L) {         \
    case 2: EA_RC(TT, 2, NB); break; \
    case 3: EA_RC(TT, 3, NB); break; \
    default: EA_RC(TT, 4, NB); break; \
  }
  if (bf16) {
    if (nbw == 2) { EA_RC_L(__bf16, 2) } else { EA_RC_L(__bf16, 4) }
  } else {
    if (nbw == 2) { EA_RC_L(float, 2) } else { EA_RC_L(float, 4) }
  }
#undef EA_RC_L
#undef EA_RC
  return hipGetLastError();
}
