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
// grouped launch; blockIdx.y (the tile) selects the problem, blockIdx.x is the replica.
//
// This header holds the kernel templates; each tile config is instantiated in a
// translation unit of its own (gemm_cfg*.hip, compiled in parallel) and
// gemm.hip dispatches between them.
#pragma once
#include "common.h"
#include "mfma.h"
#include "loss_tile.h"

#include <algorithm>
#include <cstdlib>

namespace ea {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ int batch_valid(const Prob& p, int r, long long step) {
  if (p.eval_mode) {
    long long c = (long long)ld_inv(p.vcount + r) - p.chunk * p.B;
    return (int)(c < 0 ? 0 : (c > p.B ? p.B : c));
  }
  long long c = (long long)ld_inv(p.ntrain + r) - step * p.B;
  return (int)(c < 0 ? 0 : (c > p.B ? p.B : c));
}

// absolute data row for batch row m of replica r
__device__ __forceinline__ long long batch_row(const Prob& p, int r, long long step, int m) {
  if (p.eval_mode) return (long long)ld_inv(p.vstart + r) + p.chunk * p.B + m;
  return (long long)p.perm[(long long)r * p.sPerm + step * p.B + m];
}

template <typename T> __device__ __forceinline__ void st(void* base, long long idx, float v) {
  reinterpret_cast<T*>(base)[idx] = from_f<T>(v);
}

// ------------------------------------------------------- gather-transpose
template <typename T, typename GA>
__device__ __forceinline__ void gather_transpose_block(const GA& ga, const Prob& p, int r, int t, float* sm) {
  // one block = 64 batch rows x 64 features; output XT[k][m] (ld = lddt)
  // tiles_m: batch blocks, tiles_n: feature blocks
  const int b0 = (t / p.tiles_n) * 64;
  const int k0 = (t % p.tiles_n) * 64;
  const long long step = ld_inv(ga.ctr) + ga.step_off;
  const int valid = batch_valid(p, r, step);
  const T* A = reinterpret_cast<const T*>(p.A) + (long long)r * p.sA;
  T* XT = reinterpret_cast<T*>(p.DT) + (long long)r * p.sDT;
  const int tid = threadIdx.x;
  // thread: column k = tid % 64 of rows tid / 64 + 4 i; every perm load, then every
  // row load, is issued before the first use (one memory round trip each instead of
  // one per row)
  const int k = tid & 63, mb = tid >> 6;
  int rows[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = mb + 4 * i;
    rows[i] = (b0 + m < valid) ? (int)batch_row(p, r, step, b0 + m) : -1;
  }
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const bool in = rows[i] >= 0 && k0 + k < p.K;
    const T x = A[(in ? (long long)rows[i] * p.lda + k0 + k : 0)];
    v[i] = in ? to_f<T>(x) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) sm[(mb + 4 * i) * 65 + k] = v[i];
  __syncthreads();
  for (int e = tid; e < 64 * 64; e += 256) {
    const int k = e / 64, m = e % 64;
    if (k0 + k < p.K && b0 + m < p.B) XT[(long long)(k0 + k) * p.lddt + b0 + m] = from_f<T>(sm[m * 65 + k]);
  }
}

// ----------------------------------------------------------- wide loss rows
// Final layers wider than one GEMM tile (e.g. 1000 classes): the FWD GEMM writes
// the logits Z, then each wave runs the same row_loss math as the fused epilogue
// with wave-wide reductions over LOSS_RPB / 4 rows. dZ^T (the B^T operand of the
// last layer's weight update) is staged in LDS as [N][LOSS_RPB] and written with
// one 16-byte store per class column instead of one scattered 2-byte store per
// element (66 us -> see profiles/kernels_wide_b1024.txt for 1024 x 1000 bf16).
constexpr int LOSS_LDS_MAX_N = 64 * 65 * 4 / (LOSS_RPB * 2);  // fits the smallest launch's LDS (LAT)

// Wide softmax + CCE row (one wave, NV values per lane in registers): the same
// math as loss_tile_cce / row_loss's logits path (loss = -sum y (z - lse),
// dL/dz = softmax(z) * sum(y) - y, accuracy = argmax z == argmax y, first index
// on ties), with every global load of the row issued up front.
__device__ __forceinline__ bool softmax_cce_wide(const Prob& p) {
  if (p.act != ACT_SOFTMAX || !(p.loss == LOSS_CCE || p.loss == LOSS_SPARSE_CCE)) return false;
  bool ok = true;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < p.nmet)
      ok = ok && (p.met[q] == MET_ACC_CAT || p.met[q] == MET_ACC_SPARSE || p.met[q] == LOSS_CCE ||
                  p.met[q] == LOSS_SPARSE_CCE);
  return ok;
}

template <int NV, typename ZL, typename DZ>
__device__ __forceinline__ void row_softmax_cce_reg(const Prob& p, int lane, ZL zload, const float* yrow,
                                                    bool train, DZ dz, RowOut& ro) {
  const int N = p.N;
  const bool sparse = p.loss == LOSS_SPARSE_CCE;
  const int ycls = sparse ? (int)yrow[0] : -1;
  float z[NV], y[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = lane + 64 * i;
    z[i] = j < N ? zload(j) : -INFINITY;
    y[i] = sparse ? (j == ycls ? 1.f : 0.f) : (j < N ? yrow[j] : 0.f);
  }
  float zmax = -INFINITY, bz = -INFINITY, by = -INFINITY;
  int iz = 0x7fffffff, iy = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = lane + 64 * i;
    zmax = fmaxf(zmax, z[i]);
    if (j < N && z[i] > bz) { bz = z[i]; iz = j; }
    if (j < N && y[i] > by) { by = y[i]; iy = j; }
  }
  zmax = row_max<64>(zmax);
  row_argmax<64>(bz, iz);
  row_argmax<64>(by, iy);
  float se = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (lane + 64 * i < N) se += __expf(z[i] - zmax);
  se = row_sum<64>(se);
  const float lse = zmax + logf(se);
  float l = 0.f, ysum = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (lane + 64 * i < N) {
      l += -y[i] * (z[i] - lse);
      ysum += y[i];
    }
  l = row_sum<64>(l);
  ysum = row_sum<64>(ysum);
  ro.loss = l;
  if (sparse) iy = ycls;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < p.nmet) ro.metric[q] = (p.met[q] == MET_ACC_CAT || p.met[q] == MET_ACC_SPARSE) ? (iz == iy ? 1.f : 0.f) : l;
  if (train) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int j = lane + 64 * i;
      if (j < N) dz(0, j, __expf(z[i] - lse) * ysum - y[i]);
    }
  }
}

template <typename T>
__device__ __forceinline__ void loss_rows_block(const GroupArgs& ga, const Prob& p, int r, int lb, float* smem) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = lb * LOSS_RPB;
  const long long step = ld_inv(ga.ctr) + ga.step_off;
  const int valid = batch_valid(p, r, step);
  const bool train = !p.eval_mode && p.D;
  // LDS-staged transposed store (bf16 only: 8 rows x 2 B = one 16-byte store)
  const bool stage_t = train && p.DT && sizeof(T) == 2 && p.N <= LOSS_LDS_MAX_N;
  unsigned short* sdt = reinterpret_cast<unsigned short*>(smem);
  const float inv_valid = valid > 0 ? 1.f / (float)valid : 0.f;
  float wsum[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int rr = 0; rr < LOSS_RPB / 4; ++rr) {
    const int lr = wave * (LOSS_RPB / 4) + rr, row = row0 + lr;
    auto put_t = [&](int j, float v) {
      if (stage_t) sdt[j * LOSS_RPB + lr] = __builtin_bit_cast(unsigned short, from_f<__bf16>(v));
      else if (p.DT) st<T>(p.DT, (long long)r * p.sDT + (long long)j * p.lddt + row, v);
    };
    if (row >= p.M || row >= valid) {
      if (train && row < p.M) {
        for (int j = lane; j < p.N; j += 64) {
          st<T>(p.D, (long long)r * p.sD + (long long)row * p.ldd + j, 0.f);
          put_t(j, 0.f);
        }
      } else if (stage_t) {
        for (int j = lane; j < p.N; j += 64) sdt[j * LOSS_RPB + lr] = 0;
      }
      continue;
    }
    const float* zrow = p.Z + (long long)r * p.sZ + (long long)row * p.ldz;
    // logits: Z, or (split-K last layer) the sum of the tiles_k fp32 slabs + bias
    // (at most LOSS_MAX_SPLIT slabs; unconditional loads with clamped slab indices so
    // every load of a row is in flight at once -- no branch between them)
    const int nsl = p.tiles_k > 1 ? p.tiles_k : 1;
    auto zat = [&](int j) {
      if (nsl == 1) return zrow[j];
      float v = p.bias ? p.bias[(long long)r * p.sBias + j] : 0.f;
#pragma unroll
      for (int k = 0; k < LOSS_MAX_SPLIT; ++k) {
        const float x = zrow[(long long)(k < nsl ? k : 0) * p.sPart + j];
        v += k < nsl ? x : 0.f;
      }
      return v;
    };
    float* prow = p.pred ? p.pred + (long long)r * p.sPred + (p.chunk * p.B + row) * p.ldp : nullptr;
    if (!p.Y) {  // predict only
      if (prow) row_predict<64, 0>(lane, p.N, p.act, [&](int, int j) { return zat(j); }, [&](int, int j, float v) { prow[j] = v; });
      continue;
    }
    const long long drow = batch_row(p, r, step, row);
    const float* yrow = p.Y + (long long)r * p.sY + drow * p.ldy;
    RowOut ro;
    ro.loss = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) ro.metric[q] = 0.f;
    auto dz = [&](int, int j, float v) {
      st<T>(p.D, (long long)r * p.sD + (long long)row * p.ldd + j, v * inv_valid);
      put_t(j, v * inv_valid);
    };
    auto pw = [&](int, int j, float v) { prow[j] = v; };
    if (p.N <= 16 * 64 && softmax_cce_wide(p)) {
      // softmax + (sparse) categorical cross-entropy: the row lives in registers
      // (16 values per lane, all loads in flight at once); the generic loop below
      // re-reads global memory once per pass and per 64-column chunk, one
      // dependent round trip each (66 us for 1024 x 1000)
      row_softmax_cce_reg<16>(p, lane, zat, yrow, train, dz, ro);
    } else {
      row_loss<64, 0>(lane, p.N, p.act, p.loss, p.met, p.nmet, [&](int, int j) { return zat(j); },
                      [&](int, int j) { return yrow[j]; }, yrow[0], train, dz, prow != nullptr, pw, ro);
    }
    // per-wave partial sums; one set of atomics per workgroup below (same-address
    // fp64 atomics serialise: one per row was ~60 ns x rows x counters)
    wsum[0] += ro.loss;
    wsum[1] += 1.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) wsum[2 + q] += ro.metric[q];
  }
  if (p.acc) {
    float* red = smem + (stage_t ? (LOSS_RPB * p.N * 2 + 15) / 16 * 4 : 0);  // past the dZ^T stage
    __syncthreads();
    if (lane == 0)
#pragma unroll
      for (int q = 0; q < 6; ++q) red[wave * 6 + q] = wsum[q];
    __syncthreads();
    if (threadIdx.x < 2 + p.nmet) {
      const float v = red[threadIdx.x] + red[6 + threadIdx.x] + red[12 + threadIdx.x] + red[18 + threadIdx.x];
      if (v != 0.f) atomicAdd(p.acc + (long long)r * p.acc_stride + threadIdx.x, (double)v);
    }
  }
  if (stage_t) {
    __syncthreads();
    // rows row0 .. row0+LOSS_RPB-1 of dZ^T column j: one 8-byte store (row0 % 4 == 0, lddt % 8 == 0)
    static_assert(LOSS_RPB == 4, "one uint2 per column");
    unsigned short* out = reinterpret_cast<unsigned short*>(p.DT) + (long long)r * p.sDT + row0;
    for (int j = threadIdx.x; j < p.N; j += 256)
      if (row0 + LOSS_RPB <= p.lddt)
        *reinterpret_cast<uint2*>(out + (long long)j * p.lddt) = *reinterpret_cast<const uint2*>(sdt + j * LOSS_RPB);
  }
}


__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8f(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void zero8(float (&v)[8]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = 0.f;
}

// 8 contiguous outputs -> one 16-byte (bf16) or two 16-byte (fp32) stores.
// Callers guarantee 16-byte alignment (row strides and column chunks are multiples of 8).
template <typename T>
__device__ __forceinline__ void st8(void* base, long long idx, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    auto pk2 = [](float a, float b) -> unsigned {
      const unsigned lo = __builtin_bit_cast(unsigned short, (__bf16)a);
      const unsigned hi = __builtin_bit_cast(unsigned short, (__bf16)b);
      return lo | (hi << 16);
    };
    *reinterpret_cast<uint4*>(reinterpret_cast<__bf16*>(base) + idx) =
        make_uint4(pk2(v[0], v[1]), pk2(v[2], v[3]), pk2(v[4], v[5]), pk2(v[6], v[7]));
  } else {
    float* f = reinterpret_cast<float*>(base) + idx;
    *reinterpret_cast<float4*>(f) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(f + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// Fused loss over the tile's rows: groups of W lanes own one row each
// (W = 16/32/64 by output width), reductions are W-lane shuffles.
// diagnostics: wall-clock stamps (100 MHz s_memrealtime) of block-relative phases
template <typename GA> __device__ __forceinline__ void stamp(const GA& ga, int k) {
  if (ga.stamps && threadIdx.x == 0)
    ga.stamps[((long long)blockIdx.y * gridDim.x + blockIdx.x) * 16 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}
// shader-clock counter (slots 10..15) to estimate the SCLK the kernel runs at
template <typename GA> __device__ __forceinline__ void stamp_clk(const GA& ga, int k) {
  if (ga.stamps && threadIdx.x == 0)
    ga.stamps[((long long)blockIdx.y * gridDim.x + blockIdx.x) * 16 + k] = (long long)__builtin_amdgcn_s_memtime();
}

// ------------------------------------------------------- LDS-staged main loop
// THR tile (128x128, 2x2 waves of 64x64, bf16): both operand tiles [128][64] are
// staged global -> LDS with 16-byte global_load_lds (no VGPR round trip), double
// buffered so the copy of k-tile t+1 overlaps the MFMAs of tile t, and shared by
// the block's 4 waves (the register-direct loop loads every operand twice).
// LDS image per operand: row-major [128][64] bf16 (128-byte rows) whose 16-byte
// chunk c of row r lives in slot c ^ (r & 7): glds writes lane-linear, so the
// swizzle is applied to the per-lane SOURCE address and undone on the ds_read
// (the 16 lanes of a fragment read then spread over 8 slots: <= 2-way conflicts).
constexpr int THR_BK = 64;

// Masking happens on the SOURCE of each staged chunk: a row past M (or past the
// valid batch rows), a B^T row past N and any chunk past K copy 16 zero bytes,
// and the bias "ones row" copies 16 bytes of bf16 1.0 -- so the LDS image is
// exactly the operand tile and the fragment reads need no per-element selects.
static __device__ __attribute__((aligned(16))) const unsigned short g_thr_zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
static __device__ __attribute__((aligned(16))) const unsigned short g_thr_ones[8] = {0x3F80, 0x3F80, 0x3F80, 0x3F80,
                                                                             0x3F80, 0x3F80, 0x3F80, 0x3F80};

__device__ __forceinline__ void ds_read16(uint4& v, unsigned lds_addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr) : "memory");
}

__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Stage / fragment geometry for a 128 x BN tile (BN = 128 or 64), 2 x 2 waves of
// 64 x (BN/2): every lane stages AR = 4 rows of the A tile and BR = BN/32 rows of
// the B^T tile per k-tile (one 16-byte chunk each).
template <int BN> struct ThrGeom {
  static constexpr int AR = 4, BR = BN / 32, WNF = BN / 32;  // WNF: 16-col fragments per wave
  static constexpr int A_BYTES = 128 * THR_BK * 2, B_BYTES = BN * THR_BK * 2, STAGE = A_BYTES + B_BYTES;
  static constexpr int GLDS = AR + BR;  // glds per wave per k-tile
  // ring depth 2: a 4-deep ring (1 workgroup per CU) measured 603 vs 837 TF at
  // 4096^3, and a 3-deep ring for 128x64 600 vs 613 TF at 1024x4096x4096 -- the
  // k-step waits are not the global-load latency (profiles/pmc_gemm_thr.txt)
  static constexpr int NS = 2;
};

// arow_ld/bcol_ld: per lane, the rows it stages (nullptr = zero row);
// aones: bit t set when staged A row t is the bias ones row.
template <int BN>
__device__ __forceinline__ void thr_lds_mainloop(const __bf16* const (&arow_ld)[4],
                                                 const __bf16* const (&bcol_ld)[ThrGeom<BN>::BR], unsigned aones, int K,
                                                 int wm, int wn, f32x4 (&acc)[4][ThrGeom<BN>::WNF], char* sbase) {
  using G = ThrGeom<BN>;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i16 = lane & 15, g = lane >> 4;
  const int c8 = ((lane & 7) ^ ((lane >> 3) & 7)) * 8;  // element offset of this lane's staged chunk
  const int nk = (K + THR_BK - 1) / THR_BK;
  const unsigned lds_base = (unsigned)(size_t)((__attribute__((address_space(3))) char*)sbase);
  // 64-bit source addresses selected arithmetically (v_cndmask, no branches: a
  // divergent branch would split each glds into several exec-masked copies and
  // break the per-tile glds count the counted waits rely on)
  typedef unsigned long long u64;
  const u64 zp = (u64)(const void*)g_thr_zero, op = (u64)(const void*)g_thr_ones;
  u64 abase[G::AR], bbase[G::BR];
  unsigned amov = 0, bmov = 0;  // bit t: staged row t advances with k (a real operand row)
#pragma unroll
  for (int t = 0; t < G::AR; ++t) {
    const bool ar = arow_ld[t] != nullptr;
    abase[t] = ((aones >> t) & 1u) ? op : (ar ? (u64)arow_ld[t] : zp);
    amov |= (ar && !((aones >> t) & 1u)) ? 1u << t : 0u;
  }
#pragma unroll
  for (int t = 0; t < G::BR; ++t) {
    const bool br = bcol_ld[t] != nullptr;
    bbase[t] = br ? (u64)bcol_ld[t] : zp;
    bmov |= br ? 1u << t : 0u;
  }
  auto stage = [&](int kt, int buf) {
    const int kk = kt * THR_BK + c8;
    const bool kin = kk < K;
    const u64 koff = (u64)kk * 2u;
    char* dA = sbase + buf * G::STAGE + wave * 1024;
    char* dB = sbase + buf * G::STAGE + G::A_BYTES + wave * 1024;
#pragma unroll
    for (int t = 0; t < G::AR; ++t) {
      const u64 a = abase[t] + (((amov >> t) & 1u) ? koff : 0u);
      glds16((const void*)(kin ? a : zp), dA + t * 4096);
    }
#pragma unroll
    for (int t = 0; t < G::BR; ++t) {
      const u64 b = bbase[t] + (((bmov >> t) & 1u) ? koff : 0u);
      glds16((const void*)(kin ? b : zp), dB + t * 4096);
    }
  };
#pragma unroll
  for (int s = 0; s < G::NS - 1; ++s)
    if (s < nk) stage(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    // counted wait: the copies of the tiles issued after kt may stay in flight
    const int ahead = (kt + G::NS - 2 < nk - 1 ? kt + G::NS - 2 : nk - 1) - kt;
    static_assert(G::NS <= 3 && (G::GLDS == 8 || G::GLDS == 6), "vmcnt immediates below");
    if (ahead >= 2) {
      if constexpr (G::GLDS == 8) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    } else if (ahead == 1) {
      if constexpr (G::GLDS == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot refilled below
    __builtin_amdgcn_s_barrier();                        // tile kt landed for every wave; slot kt-1 is free
    asm volatile("" ::: "memory");
    if (kt + G::NS - 1 < nk) stage(kt + G::NS - 1, (kt + G::NS - 1) % G::NS);
    // Fragment reads are inline-asm ds_read_b128: for compiler-visible LDS loads
    // hipcc cannot tell the slot being read from the slot the glds above is
    // filling and waits vmcnt(0) before the first read (draining the prefetch,
    // so every k-step paid a full HBM round trip). The waits for these reads are
    // explicit lgkmcnt + sched_barrier (the MFMAs must not be hoisted above them).
    const unsigned bA = lds_base + (unsigned)((kt % G::NS) * G::STAGE);
    const unsigned bB = bA + G::A_BYTES;
    uint4 fa[2][4], fb[2][G::WNF];
#pragma unroll
    for (int u = 0; u < THR_BK / 32; ++u) {
      const unsigned slot = (unsigned)(((u * 4 + g) ^ (i16 & 7)) * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) ds_read16(fa[u][i], bA + (unsigned)((wm * 64 + i * 16 + i16) * 128) + slot);
#pragma unroll
      for (int j = 0; j < G::WNF; ++j)
        ds_read16(fb[u][j], bB + (unsigned)((wn * (BN / 2) + j * 16 + i16) * 128) + slot);
    }
    if constexpr (G::WNF == 4) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // substep 0 landed
    else asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < G::WNF; ++j) mma16<__bf16>(acc[i][j], fa[0][i], fb[0][j]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < G::WNF; ++j) mma16<__bf16>(acc[i][j], fa[1][i], fb[1][j]);
  }
  __syncthreads();  // the epilogue reuses the staging LDS
}

// KM: bit k set = problem kind k can occur in this instantiation; the other
// kinds' epilogues are compiled out (smaller code per launch, see launch_cfg).
constexpr unsigned KM_ALL = 0x1ffu;  // every ProbKind (0..8, args.h)
constexpr unsigned KB(int k) { return 1u << k; }
// the executor's launches: {FWD, X^T gather}, {FWD_LOSS}, {DW update or grad, DX}
constexpr unsigned KM_NONE = 0u;
constexpr unsigned KM_FWD = KB(PK_FWD), KM_GATHER = KB(PK_GATHER_T);
constexpr unsigned KM_LOSS = KB(PK_FWD_LOSS);
constexpr unsigned KM_DW = KB(PK_DW_UPDATE) | KB(PK_DW_GRAD), KM_DX = KB(PK_DX);
constexpr unsigned KM_PARTIAL = KB(PK_PARTIAL);

// ------------------------------------------------------------- epilogues
// The fused Dense-layer epilogues over a finished fp32 C tile [BM][BN + 4] in LDS
// (tile rows m0.., columns n0.. of problem p), run by NT threads: each thread owns
// 8 contiguous columns of one row per pass. Shared by the 256-thread tiles of
// run_prob and the 512-thread 256x256 tile (gemm_big.h, two 128-row halves).
// PFP / DW_PF: optimizer operands the caller prefetched before its main loop.
template <typename T, int BM, int BN, int NT, unsigned KM, int PFP, bool DW_PF, typename GA>
__device__ __forceinline__ void tile_epilogue(const GA& ga, const Prob& p, const int r, const int m0, const int n0,
                                              const int kch, const int valid, const long long iter,
                                              const long long step, const bool skip_update, float* smem,
                                              const bool (&pf_vec)[PFP], const float (&pf_w)[PFP][8],
                                              const float (&pf_s0)[PFP][8], const float (&pf_s1)[PFP][8]) {
  constexpr int LDC = BN + 4;
  constexpr int CPR = BN / 8;   // 8-column chunks per row
  constexpr int RPP = NT / CPR; // rows per pass
  constexpr int PASSES = BM / RPP;
  static_assert(PASSES * RPP == BM, "epilogue passes");
  // the 256x256 tile runs the epilogue with the other half's accumulators still live
  // (gemm_big.h): passes stay rolled so the epilogue fits the remaining registers
  constexpr int EUNR = (NT == 256 && BM * BN <= 128 * 128) ? PASSES : 1;
  const int t_row = threadIdx.x / CPR, t_c0 = (threadIdx.x % CPR) * 8;
  (void)step; (void)kch; (void)valid; (void)iter; (void)skip_update; (void)pf_vec;
  float* C = smem;  // final tile [BM][LDC]
  stamp(ga, 3);

  // Epilogue thread mapping: each thread owns 8 contiguous columns of one row
  // per pass and issues all of its global loads before any store, so the
  // loads of a pass overlap instead of serialising behind possibly-aliasing
  // stores.
  auto lds8 = [&](int row, int c0, float (&v)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(C + row * LDC + c0);
    const float4 b = *reinterpret_cast<const float4*>(C + row * LDC + c0 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  };
  auto sts8 = [&](int row, int c0, const float (&v)[8]) {
    *reinterpret_cast<float4*>(C + row * LDC + c0) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(C + row * LDC + c0 + 4) = make_float4(v[4], v[5], v[6], v[7]);
  };
  // transposed store of the tile (D^T, dZ^T, W^T): each thread moves 8 consecutive
  // rows of one column (8 LDS reads -> one 16-byte bf16 store, or two for fp32);
  // the BM/8 threads of a column are consecutive, so a column's rows are one
  // contiguous run in memory. Every destination here has ld % 8 == 0 and an
  // 8-element-aligned base (Bp / Kp padding), checked on the host.
  auto store_transposed = [&](void* base, long long off, long long ld, int nrows) {
    constexpr int RC = BM / 8;  // 8-row chunks per column
    for (int e = threadIdx.x; e < RC * BN; e += NT) {
      const int rc = e % RC, col = e / RC, row = rc * 8, gm = m0 + row, gn = n0 + col;
      if (gn >= p.N || gm >= nrows) continue;
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = C[(row + q) * LDC + col];
      const long long idx = off + (long long)gn * ld + gm;
      if (gm + 8 <= nrows) {
        st8<T>(base, idx, v);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (gm + q < nrows) st<T>(base, idx + q, v[q]);
      }
    }
  };

  switch (p.kind) {
    case PK_PARTIAL: {
      if constexpr (!(KM & KB(PK_PARTIAL))) break;
      // raw fp32 slab of this K chunk; rows past the valid batch are zero (masked A)
      float* out = reinterpret_cast<float*>(p.D) + (long long)r * p.sD + (long long)kch * p.sPart;
#pragma unroll EUNR
      for (int ps = 0; ps < PASSES; ++ps) {
        const int row = ps * RPP + t_row, gm = m0 + row, gn0 = n0 + t_c0;
        if (gm >= p.M || gn0 >= p.N) continue;
        float v[8];
        lds8(row, t_c0, v);
        if (gn0 + 8 <= p.N && (p.ldd & 3) == 0) {
          st8f(out + (long long)gm * p.ldd + gn0, v);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (gn0 + q < p.N) out[(long long)gm * p.ldd + gn0 + q] = v[q];
        }
      }
      break;
    }
    case PK_PLAIN: {
      if constexpr (!(KM & KB(PK_PLAIN))) break;
      // 8 contiguous columns per thread: one 32-byte (fp32) or 16-byte (bf16) store where the
      // row segment is whole and aligned, element stores at the ragged edge
      const bool vec = (p.ldd & 7) == 0 && (reinterpret_cast<unsigned long long>(p.D) & 15) == 0;
#pragma unroll EUNR
      for (int ps = 0; ps < PASSES; ++ps) {
        const int row = ps * RPP + t_row, gm = m0 + row, gn0 = n0 + t_c0;
        if (gm >= p.M || gn0 >= p.N) continue;
        float v[8];
        lds8(row, t_c0, v);
        const long long idx = (long long)r * p.sD + (long long)gm * p.ldd + gn0;
        if (p.d_bf16) {
          if (vec && gn0 + 8 <= p.N) {
            st8<__bf16>(p.D, idx, v);
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (gn0 + q < p.N) st<__bf16>(p.D, idx + q, v[q]);
          }
        } else {
          float* out = reinterpret_cast<float*>(p.D);
          if (vec && gn0 + 8 <= p.N) {
            st8f(out + idx, v);
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (gn0 + q < p.N) out[idx + q] = v[q];
          }
        }
      }
      break;
    }
    case PK_FWD:
    case PK_DX: {
      if constexpr (!(KM & (KB(PK_FWD) | KB(PK_DX)))) break;
      const bool fwd = p.kind == PK_FWD;
      const float* __restrict__ bias = fwd && p.bias ? p.bias + (long long)r * p.sBias : nullptr;
      float* __restrict__ Z = p.Z ? p.Z + (long long)r * p.sZ : nullptr;
      const float keep_scale = p.rate > 0.f ? 1.f / (1.f - p.rate) : 1.f;
      const bool drop = p.rate > 0.f && !p.eval_mode;
      // Z rows as 32-byte pairs of 16-byte accesses where whole and aligned (element
      // accesses: Wide step 3.24 ms, 3.06 with these)
      const bool zvec = Z && (p.ldz & 3) == 0 && (reinterpret_cast<unsigned long long>(Z) & 15) == 0;
      // the bias of this thread's 8 columns, the same in every pass: loaded once
      float bia[8];
      {
        const int gn0 = n0 + t_c0;
        if (bias && gn0 + 8 <= p.N && (reinterpret_cast<unsigned long long>(bias + gn0) & 15) == 0) {
          ld8f(bias + gn0, bia);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) bia[q] = (bias && gn0 + q < p.N) ? bias[gn0 + q] : 0.f;
        }
      }
#pragma unroll EUNR
      for (int ps = 0; ps < PASSES; ++ps) {
        const int row = ps * RPP + t_row, gm = m0 + row, gn0 = n0 + t_c0;
        if (gm >= p.M || gn0 >= p.N) continue;
        const bool rv = gm < valid;
        const bool zw = zvec && gn0 + 8 <= p.N;
        float v[8], aux[8], zv[8], out[8], u[8];
        lds8(row, t_c0, v);
        if (drop) {  // t_c0 is a multiple of 8
          dropout_u8(dropout_base(ga.seed, r, p.layer, iter), gm, gn0, u);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) u[q] = 1.f;
        }
        if (fwd) {
#pragma unroll
          for (int q = 0; q < 8; ++q) aux[q] = bia[q];
        } else if (zw && rv) {
          ld8f(Z + (long long)gm * p.ldz + gn0, aux);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) aux[q] = (gn0 + q < p.N && rv) ? Z[(long long)gm * p.ldz + gn0 + q] : 0.f;
        }
        float av[8];
        if (fwd) {
#pragma unroll
          for (int q = 0; q < 8; ++q) zv[q] = v[q] + aux[q];
          act_f_v<8>(p.act, zv, av);
        } else {
          act_g_v<8>(p.act, aux, av);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const bool live = gn0 + q < p.N && rv;
          const bool keep = live && u[q] >= p.rate;
          if (!live) zv[q] = 0.f;
          out[q] = keep ? (fwd ? av[q] : v[q] * av[q]) * keep_scale : 0.f;
        }
        if (ps == 0) stamp(ga, 5);
        if (fwd && Z) {
          if (zw) {
            st8f(Z + (long long)gm * p.ldz + gn0, zv);
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (gn0 + q < p.N) Z[(long long)gm * p.ldz + gn0 + q] = zv[q];
          }
        }
        if (p.D) st8<T>(p.D, (long long)r * p.sD + (long long)gm * p.ldd + gn0, out);
        sts8(row, t_c0, out);
      }
      stamp(ga, 6);
      if (p.DT) {
        __syncthreads();
        stamp(ga, 7);
        store_transposed(p.DT, (long long)r * p.sDT, p.lddt, p.M);
      }
      break;
    }
    case PK_FWD_LOSS: {
      if constexpr ((KM & KB(PK_FWD_LOSS)) != 0u && NT == 256) {
      // whole rows live in this tile (N <= BN, tiles_n == 1)
      const float* __restrict__ bias = p.bias ? p.bias + (long long)r * p.sBias : nullptr;
      int* srow = reinterpret_cast<int*>(smem + BM * LDC);   // data row of each tile row
      float* Ys = smem + BM * LDC + BM;                       // staged targets [BM][BN]
#pragma unroll EUNR
      for (int ps = 0; ps < PASSES; ++ps) {
        const int row = ps * RPP + t_row, gn0 = t_c0;
        if (gn0 >= p.N) continue;
        float v[8], b[8];
        lds8(row, t_c0, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) b[q] = (bias && gn0 + q < p.N) ? bias[gn0 + q] : 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += b[q];
        sts8(row, t_c0, v);
      }
      stamp(ga, 5);
      const int ldy = p.Y ? (int)p.ldy : 0;
      for (int row = threadIdx.x; row < BM; row += NT) {
        const int gm = m0 + row;
        srow[row] = (gm < p.M && gm < valid) ? (int)batch_row(p, r, step, gm) : -1;
      }
      __syncthreads();
      if (p.Y) {
        const float* Yb = p.Y + (long long)r * p.sY;
        for (int e = threadIdx.x; e < BM * ldy; e += NT) {
          const int row = e / ldy, j = e % ldy;
          const int dr = srow[row];
          Ys[row * BN + j] = dr >= 0 ? Yb[(long long)dr * ldy + j] : 0.f;
        }
      }
      __syncthreads();
      stamp(ga, 6);
      const bool train = !p.eval_mode && p.D;
      const float inv_valid = valid > 0 ? 1.f / (float)valid : 0.f;
      float sums[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (softmax_cce_fast(p)) {
        if (p.N <= 16) loss_tile_cce<4, BM, LDC, BN>(p, r, m0, C, Ys, srow, train, inv_valid, sums);
        else loss_tile_cce<8, BM, LDC, BN>(p, r, m0, C, Ys, srow, train, inv_valid, sums);
      } else {
        loss_tile_lds<BM, LDC, BN>(p, r, m0, C, Ys, srow, train, inv_valid, sums);
      }
      stamp(ga, 7);
      if (p.acc && p.Y) {
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          if (q < 2 + p.nmet) {
            const float s = row_sum<64>(sums[q]);
            if ((threadIdx.x & 63) == 0 && s != 0.f)
              atomicAdd(p.acc + (long long)r * p.acc_stride + q, (double)s);
          }
        }
      }
      stamp(ga, 8);
      if (train) {
        __syncthreads();  // dz rows were produced by lane groups
#pragma unroll EUNR
        for (int ps = 0; ps < PASSES; ++ps) {
          const int row = ps * RPP + t_row, gm = m0 + row, gn0 = t_c0;
          if (gm >= p.M || gn0 >= p.N) continue;
          float v[8];
          lds8(row, t_c0, v);
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (gn0 + q >= p.N) v[q] = 0.f;
          st8<T>(p.D, (long long)r * p.sD + (long long)gm * p.ldd + gn0, v);
        }
        if (p.DT) store_transposed(p.DT, (long long)r * p.sDT, p.lddt, p.M);
      }
      }  // if constexpr
      break;
    }
    case PK_DW_UPDATE:
    case PK_DW_GRAD: {
      if constexpr (!(KM & (KB(PK_DW_UPDATE) | KB(PK_DW_GRAD)))) break;
      if (skip_update) break;
      const bool upd = p.kind == PK_DW_UPDATE;
      float* __restrict__ P = p.P + (long long)r * p.sP;
      float* __restrict__ S = p.S ? p.S + (long long)r * p.sS : nullptr;
      float* __restrict__ G = p.G ? p.G + (long long)r * p.sG : nullptr;
      const long long wpar = ((iter + 1) & 1);
      const int krows = p.ones_row >= 0 ? p.ones_row : p.M;
      const int np = S ? opt_planes(p.op) : 0;
#pragma unroll EUNR
      for (int ps = 0; ps < PASSES; ++ps) {
        const int row = ps * RPP + t_row, gm = m0 + row, gn0 = n0 + t_c0;
        if (gm >= p.M || gn0 >= p.N) continue;
        float v[8];
        lds8(row, t_c0, v);
        const long long pidx = p.p_off + (long long)gm * p.N + gn0;
        if (!upd) {
          // the raw gradient: the apply kernel (flat.hip) multiplies by grad_scale once
          // (scaling here too squared it: 1 / world^2 on the multi-rank per-step path)
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (gn0 + q < p.N) G[pidx + q] = valid > 0 ? v[q] : 0.f;
          continue;
        }
        float w[8], s0[8], s1[8];
        // whole 16-byte-aligned chunks (the common case) move as float4 pairs
        const bool vec = gn0 + 8 <= p.N && (pidx & 3) == 0 && (p.op.s_plane & 3) == 0;
        if (DW_PF && pf_vec[DW_PF ? ps : 0]) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            w[q] = pf_w[DW_PF ? ps : 0][q];
            s0[q] = pf_s0[DW_PF ? ps : 0][q];
            s1[q] = pf_s1[DW_PF ? ps : 0][q];
          }
        } else if (vec) {
          ld8f(P + pidx, w);
          if (np > 0) ld8f(S + pidx, s0); else zero8(s0);
          if (np > 1) ld8f(S + p.op.s_plane + pidx, s1); else zero8(s1);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) {  // loads first
            const bool in = gn0 + q < p.N;
            w[q] = in ? P[pidx + q] : 0.f;
            s0[q] = (in && np > 0) ? S[pidx + q] : 0.f;
            s1[q] = (in && np > 1) ? S[p.op.s_plane + pidx + q] : 0.f;
          }
        }
        {
          float gq[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) gq[q] = v[q] * p.op.grad_scale;
          opt_update_v<8>(p.op, w, gq, s0, s1, iter);  // lanes past N are discarded below
        }
        if (ps == 0) stamp(ga, 5);
        if (vec) {
          st8f(P + pidx, w);
          if (np > 0) st8f(S + pidx, s0);
          if (np > 1) st8f(S + p.op.s_plane + pidx, s1);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            if (gn0 + q < p.N) {
              P[pidx + q] = w[q];
              if (np > 0) S[pidx + q] = s0[q];
              if (np > 1) S[p.op.s_plane + pidx + q] = s1[q];
            } else {
              w[q] = 0.f;
            }
          }
        }
        if (p.Wsh && gm < krows)
          st8<T>(p.Wsh, (long long)r * p.sWsh + wpar * p.wsh_par + (long long)gm * p.ldwsh + gn0, w);
        sts8(row, t_c0, w);
      }
      stamp(ga, 6);
      if (upd && p.WTsh) {
        __syncthreads();
        stamp(ga, 7);
        store_transposed(p.WTsh, (long long)r * p.sWTsh + wpar * p.wtsh_par, p.ldwtsh, krows);
        stamp(ga, 8);
      }
      break;
    }
  }
}

// --------------------------------------------------------------- the kernel

// PF_: k-steps of fragments in flight per wave in the register-direct loop (0 = by
// tile size); the weight-gradient table launch (K = batch: one or two k-steps per
// wave) uses a shallow ring so three workgroups fit on a CU
template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT, unsigned KM = KM_ALL, int PF_ = 0,
          typename GA>
__device__ __forceinline__ void run_prob(const GA& ga, const Prob& p, const int r, const int lb, float* smem) {
  static_assert(WAVES_M * WAVES_N * KSPLIT == 4, "4 waves per block");
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  constexpr int LDC = BN + 4;  // 16-byte aligned rows for float4 LDS access
  constexpr int EPL = KT<T>::EPL, KC = KT<T>::KC;
  if ((KM & KB(PK_GATHER_T)) && p.kind == PK_GATHER_T) {
    gather_transpose_block<T>(ga, p, r, lb, smem);
  } else {
    // split-K over workgroups (PK_PARTIAL): chunk kc covers reduction elements
    // [kc * kchunk, kc * kchunk + Keff) and writes its own fp32 slab
    const bool partial = (KM & KB(PK_PARTIAL)) && p.kind == PK_PARTIAL;
    const int tk = partial ? p.tiles_k : 1;
    const int per_mn = p.tiles_m * p.tiles_n;
    const int per_r = per_mn * tk;
    // r = blockIdx.x (GroupArgs: replica-minor grid, XCD affinity); lb = this
    // replica's tile within the problem
    (void)per_r;
    const int tkm = lb;
    const int kch = partial ? tkm / per_mn : 0;
    const int t = partial ? tkm - kch * per_mn : tkm;
    const int tm = t / p.tiles_n, tn = t % p.tiles_n;
    const int koff = partial ? kch * p.kchunk : 0;
    const int Keff = partial ? min(p.kchunk, p.K - koff) : p.K;
    const int m0 = tm * BM, n0 = tn * BN;
    const long long step = ld_inv(ga.ctr) + ga.step_off;
    // (every launcher passes a valid ntrain: the plain-GEMM entry points it at zeros)
    const long long iter = iter_at(ga.ctr, p.ntrain, p.B, r, ld_inv(ga.ctr), ga.step_off);
    const int valid = (p.kind == PK_PLAIN) ? p.M : batch_valid(p, r, step);
    const bool skip_update = (p.kind == PK_DW_UPDATE) && valid == 0;
    stamp(ga, 1);

    // Epilogue thread mapping (used below): each thread owns 8 contiguous columns of
    // one row per pass.
    constexpr int CPR = BN / 8;          // 8-column chunks per row
    constexpr int RPP = 256 / CPR;       // rows per pass
    constexpr int PASSES = BM / RPP;
    const int t_row = threadIdx.x / CPR, t_c0 = (threadIdx.x % CPR) * 8;
    // Weight-update launches of one pass per thread (the LAT tile of the row-chain
    // DW table launch): the fp32 master / optimizer-state operands of the update do
    // not depend on the GEMM, so their loads are issued before the main loop and
    // their memory round trip overlaps it instead of following it.
    constexpr bool DW_PF = (KM & ~KM_DW) == 0u && PASSES <= 2;
    constexpr int PFP = DW_PF ? PASSES : 1;
    float pf_w[PFP][8], pf_s0[PFP][8], pf_s1[PFP][8];
    bool pf_vec[PFP];
#pragma unroll
    for (int ps = 0; ps < PFP; ++ps) {
      pf_vec[ps] = false;
      if constexpr (DW_PF) {
        const int gm = m0 + ps * RPP + t_row, gn0 = n0 + t_c0;
        pf_vec[ps] = p.kind == PK_DW_UPDATE && gm < p.M && gn0 + 8 <= p.N &&
                     ((p.p_off + (long long)gm * p.N + gn0) & 3) == 0 && (p.op.s_plane & 3) == 0;
        if (pf_vec[ps]) {
          const long long pidx = p.p_off + (long long)gm * p.N + gn0;
          const float* Pp = p.P + (long long)r * p.sP;
          const float* Sp = p.S ? p.S + (long long)r * p.sS : nullptr;
          const int np = Sp ? opt_planes(p.op) : 0;
          ld8f(Pp + pidx, pf_w[ps]);
          if (np > 0) ld8f(Sp + pidx, pf_s0[ps]); else zero8(pf_s0[ps]);
          if (np > 1) ld8f(Sp + p.op.s_plane + pidx, pf_s1[ps]); else zero8(pf_s1[ps]);
        }
      }
    }

    // wave index as a scalar: the k-step loop bounds below depend on it, and with a
    // VGPR wave index their branches became exec-masked and the waitcnt pass fell
    // back to vmcnt(0) at every join
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wk = wave % KSPLIT;
    const int wsp = wave / KSPLIT;
    const int wm = wsp / WAVES_N, wn = wsp % WAVES_N;
    const int g = lane >> 4, i16 = lane & 15;

    f32x4 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Weight-gradient-only launches: the operands are activation workspaces (no batch
    // gather, no weight-image parity), so no operand address depends on the step
    // counters -- the loads are issued without waiting for the counter round trip
    // (a skipped update only wastes its loads; its epilogue is skipped below).
    constexpr bool CTR_FREE = (KM & ~KM_DW) == 0u;
    const bool a_gather = CTR_FREE ? false : (bool)p.a_gather;
    if (CTR_FREE || !skip_update) {
      const T* A = reinterpret_cast<const T*>(p.A) + (long long)r * p.sA + koff;
      const T* BTp = reinterpret_cast<const T*>(p.BT) + (long long)r * p.sB +
                     ((!CTR_FREE && p.bt_shadow) ? (iter & 1) * p.bt_par : 0) + koff;
      // Every fragment load is an unconditional, in-bounds 16-byte global load
      // (invalid rows read row 0, k past the end reads k=0) followed by a value
      // select, so hipcc emits global_load_dwordx4 and never a pointer select
      // into a stack constant (which would become flat loads + scratch).
      const T* arow[WM];
      unsigned amask = 0, aones_m = 0;  // bit i: row i valid / row i is the ones row
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const int m = m0 + wm * WM * 16 + i * 16 + i16;
        arow[i] = A;
        if (m == p.ones_row) {
          aones_m |= 1u << i;
        } else if (m < p.M) {
          if (a_gather) {
            if (m < valid) {
              arow[i] = A + batch_row(p, r, step, m) * p.lda;
              amask |= 1u << i;
            }
          } else {
            arow[i] = A + (long long)m * p.lda;
            amask |= 1u << i;
          }
        }
      }
      const T* bcol[WN];
      unsigned bmask = 0;
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int n = n0 + wn * WN * 16 + j * 16 + i16;
        bcol[j] = BTp;
        if (n < p.N) {
          bcol[j] = BTp + (long long)n * p.ldb;
          bmask |= 1u << j;
        }
      }
      if constexpr (sizeof(T) == 2 && KSPLIT == 1 && BM == 128 && (BN == 128 || BN == 64) && WM == 4 &&
                    WN == BN / 32) {
        // staged rows of this lane: r = 32 t + 8 wave + lane / 8 of the A and B^T tiles
        constexpr int BR = ThrGeom<BN>::BR;
        const __bf16* arow_ld[4];
        const __bf16* bcol_ld[BR];
        unsigned aones = 0;
        const __bf16* Ab = reinterpret_cast<const __bf16*>(A);
        const __bf16* Bb = reinterpret_cast<const __bf16*>(BTp);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int rr = t * 32 + (threadIdx.x >> 3);
          const int m = m0 + rr;
          arow_ld[t] = nullptr;
          if (m == p.ones_row) {
            aones |= 1u << t;
          } else if (m < p.M) {
            if (a_gather) {
              if (m < valid) arow_ld[t] = Ab + batch_row(p, r, step, m) * p.lda;
            } else {
              arow_ld[t] = Ab + (long long)m * p.lda;
            }
          }
        }
#pragma unroll
        for (int t = 0; t < BR; ++t) {
          const int n = n0 + t * 32 + (threadIdx.x >> 3);
          bcol_ld[t] = n < p.N ? Bb + (long long)n * p.ldb : nullptr;
        }
        thr_lds_mainloop<BN>(arow_ld, bcol_ld, aones, Keff, wm, wn,
                             reinterpret_cast<f32x4(&)[4][ThrGeom<BN>::WNF]>(acc), reinterpret_cast<char*>(smem));
      } else {
      const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
      const uint4 one = ones_frag<T>();
      auto sel = [](bool c, const uint4& a, const uint4& b) {
        return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
      };
      // The ring holds RAW loaded fragments; masks are applied when a slot is consumed.
      // (Selecting on the value right after its load made the compiler wait for every
      // load as soon as it was issued -- vmcnt(0) per k-step -- so the PF-deep ring
      // never had more than one step in flight.)
      auto issue_frags = [&](int kc, uint4 (&a)[WM], uint4 (&b)[WN]) {
        const int kk = kc + g * EPL;
        const int kq = kk < Keff ? kk : 0;
#pragma unroll
        for (int i = 0; i < WM; ++i) a[i] = *reinterpret_cast<const uint4*>(arow[i] + kq);
#pragma unroll
        for (int j = 0; j < WN; ++j) b[j] = *reinterpret_cast<const uint4*>(bcol[j] + kq);
      };
      // PF-deep register ring: PF k-steps of fragments in flight per wave, so a
      // K = 784 layer waits on ~2 load round trips instead of one per step.
      constexpr int KSTEP = KSPLIT * KC;
      constexpr int PF = PF_ > 0 ? PF_ : ((WM * WN >= 16) ? 3 : 4);
      const int kbeg = wk * KC;
      const int nsteps = kbeg < Keff ? (Keff - kbeg + KSTEP - 1) / KSTEP : 0;
      uint4 ra[PF][WM], rb[PF][WN];
#pragma unroll
      for (int u = 0; u < PF; ++u) issue_frags(kbeg + u * KSTEP, ra[u], rb[u]);
      for (int s0 = 0; s0 < nsteps; s0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          const int st_ = s0 + u;
          if (st_ < nsteps) {
            const bool kin = kbeg + st_ * KSTEP + g * EPL < Keff;
            uint4 a[WM], b[WN];
#pragma unroll
            for (int i = 0; i < WM; ++i)
              a[i] = sel(kin && ((amask >> i) & 1u), ra[u][i], sel(kin && ((aones_m >> i) & 1u), one, zero));
#pragma unroll
            for (int j = 0; j < WN; ++j) b[j] = sel(kin && ((bmask >> j) & 1u), rb[u][j], zero);
            // unconditional: past the end the addresses clamp to k = 0 and the values
            // are masked at consumption (no branch around the loads)
            issue_frags(kbeg + (st_ + PF) * KSTEP, ra[u], rb[u]);
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
              for (int j = 0; j < WN; ++j) mma16<T>(acc[i][j], a[i], b[j]);
          }
        }
      }
      }  // register-direct loop
    }

    stamp(ga, 2);
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
      for (int e = threadIdx.x; e < BM * BN / 4; e += 256) {
        const int row = e / (BN / 4), c4 = (e % (BN / 4)) * 4;
        float4 s = *reinterpret_cast<const float4*>(smem + row * LDC + c4);
#pragma unroll
        for (int w = 1; w < KSPLIT; ++w) {
          const float4 o = *reinterpret_cast<const float4*>(smem + w * BM * LDC + row * LDC + c4);
          s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
        }
        *reinterpret_cast<float4*>(smem + row * LDC + c4) = s;
      }
      __syncthreads();
    }
    tile_epilogue<T, BM, BN, 256, KM, PFP, DW_PF>(ga, p, r, m0, n0, kch, valid, iter, step, skip_update, smem, pf_vec,
                                                pf_w, pf_s0, pf_s1);
  }

}

// Kernel arguments are only ever indexed with compile-time constants (the
// problem is picked by a wave-uniform branch), so hipcc keeps every Prob field
// in the kernarg segment (scalar loads) instead of copying the struct to scratch.
// KM0 / KM1: the kinds problem slot 0 / slot 1 can hold (compiled separately:
// a kernel holding both the FWD epilogue and the gather needed 68 B of scratch,
// each alone none)
template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT, unsigned KM0 = KM_ALL,
          unsigned KM1 = KM_ALL>
__global__ __launch_bounds__(256) void gemm_grouped(GroupArgs ga) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  stamp(ga, 0);
  stamp_clk(ga, 10);
  const int r = blockIdx.x, bid = blockIdx.y;
  // problem 1 owns [p[1].block_begin, ...) up to p[0]'s range when that comes after it
  // (the executor puts the problem with the deeper tiles first: longest tiles dispatched first)
  const int b0 = ga.p[0].block_begin, b1 = ga.p[1].block_begin;
  if (KM1 != KM_NONE && ga.nprob > 1 && bid >= b1 && (b1 > b0 || bid < b0))
    run_prob<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM1>(ga, ga.p[1], r, bid - ga.p[1].block_begin, smem);
  else
    run_prob<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM0>(ga, ga.p[0], r, bid - ga.p[0].block_begin, smem);

  stamp(ga, 4);
  stamp_clk(ga, 11);
}

// Two problems whose best tiles differ in ONE launch (a layer's weight gradient and input
// gradient: Otto DW 513x512x128 wants 128x64 tiles, DX 128x512x512 the 64x32 split-K
// tile): problem 0 on tile A, problem 1 on tile B, each block runs its problem's tile
// (every config is 4 waves of 64; LDS = the larger of the two). Replaces two dependent
// launches by one.
template <typename T, int WMa, int WNa, int WAMa, int WANa, int KSa, int WMb, int WNb, int WAMb, int WANb, int KSb,
          unsigned KM0, unsigned KM1>
__global__ __launch_bounds__(256) void gemm_dual(GroupArgs ga) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  stamp(ga, 0);
  stamp_clk(ga, 10);
  const int r = blockIdx.x, bid = blockIdx.y;
  const int b0 = ga.p[0].block_begin, b1 = ga.p[1].block_begin;
  if (bid >= b1 && (b1 > b0 || bid < b0))
    run_prob<T, WMb, WNb, WAMb, WANb, KSb, KM1>(ga, ga.p[1], r, bid - b1, smem);
  else
    run_prob<T, WMa, WNa, WAMa, WANa, KSa, KM0>(ga, ga.p[0], r, bid - b0, smem);
  stamp(ga, 4);
  stamp_clk(ga, 11);
}

// Wide-output loss rows run in a kernel of their own: inside gemm_grouped their
// register-resident row (16 z + 16 y values per lane) raised every GEMM tile's
// VGPR allocation (104 -> 132 on the 128x128 config, plus scratch) and slowed
// the weight-update launches of the same model by up to 50 %.
template <typename T>
__global__ __launch_bounds__(256) void loss_rows_kernel(GroupArgs ga) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  loss_rows_block<T>(ga, ga.p[0], blockIdx.x, blockIdx.y - ga.p[0].block_begin, smem);
}

// Grouped launch over a device table of problems (row-chain plan, up to
// TABLE_MAX problems of the kinds in KM): block -> problem by the kernarg
// begin[] table; the problem's fields are read through a wave-uniform pointer.
template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT, unsigned KM>
__global__ __launch_bounds__(256) void gemm_table(TableArgs ta) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  stamp(ta, 0);
  stamp_clk(ta, 10);
  const int r = blockIdx.x, bid = blockIdx.y;
  int i = 0;
#pragma unroll
  for (int j = 1; j < TABLE_MAX; ++j) i += (j < ta.nprob && bid >= ta.begin[j]) ? 1 : 0;
  i = __builtin_amdgcn_readfirstlane(i);
  // Read the problem through the constant address space (as kernel arguments are):
  // those loads are scalar and invariant, so hipcc keeps or rematerialises the
  // fields; through a plain global pointer every field read after an epilogue store
  // became a vector load with its own full memory round trip (the compiler cannot
  // tell the table from the stored-to buffers)
  const Prob p = ld_inv_struct(ta.probs + i);
  run_prob<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM, (KM == KM_DW) ? 2 : 0>(ta, p, r, bid - ta.begin[i], smem);
  stamp(ta, 4);
  stamp_clk(ta, 11);
}

// ------------------------------------------------------------- host side
template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT>
static size_t lds_bytes(bool loss = true) {
  constexpr int BM = WAVES_M * WM * 16;
  constexpr int BN = WAVES_N * WN * 16;
  const size_t tile = (size_t)BM * (BN + 4);
  size_t floats = (size_t)KSPLIT * tile;
  if (sizeof(T) == 2 && KSPLIT == 1 && BM == 128 && (BN == 128 || BN == 64))  // glds staging ring
    floats = std::max(floats, (size_t)ThrGeom<BN>::NS * ThrGeom<BN>::STAGE / sizeof(float));
  if (loss) floats = std::max(floats, tile + BM + (size_t)BM * BN);  // + row map + staged targets
  floats = std::max(floats, (size_t)64 * 65);                       // gather-transpose
  return floats * sizeof(float);
}

template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT, unsigned KM0 = KM_ALL,
          unsigned KM1 = KM_ALL>
static void set_attr() {
  (void)hipFuncSetAttribute(
      reinterpret_cast<const void*>(&gemm_grouped<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM0, KM1>),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, WM, WN, WAVES_M, WAVES_N, KSPLIT>());
}

// Kind-specialised variants (the latency-bound small-MLP path): every launch of a
// training step holds one of three kind sets, and the variant that compiles only
// those epilogues is a fraction of the all-kinds kernel's code (MNIST step
// 65.9 -> 60.6 us); launches with other kind sets take the all-kinds kernel.

template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT, unsigned KM0, unsigned KM1>
static bool launch_if(const GroupArgs& ga, size_t lds, hipStream_t s, hipError_t& err) {
  if (!(KM0 & KB(ga.p[0].kind))) return false;
  if (ga.nprob > 1 && !(KM1 & KB(ga.p[1].kind))) return false;
  hipLaunchKernelGGL((gemm_grouped<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM0, KM1>), dim3(ga.R, ga.total_blocks),
                     dim3(256), lds, s, ga);
  err = hipGetLastError();
  return true;
}

// SPEC: also launch the kind-specialised variants of this config
template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT, bool SPEC = false>
static hipError_t launch_cfg(const GroupArgs& ga, hipStream_t s) {
  if (ga.total_blocks <= 0) return hipSuccess;
  bool loss = false;
  for (int i = 0; i < ga.nprob; ++i) loss |= ga.p[i].kind == PK_FWD_LOSS;
  const size_t lds = lds_bytes<T, WM, WN, WAVES_M, WAVES_N, KSPLIT>(loss);
  if constexpr (SPEC) {
    if (ga.nprob <= 2) {
      hipError_t e = hipSuccess;
      if (launch_if<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM_FWD, KM_GATHER>(ga, lds, s, e) ||
          launch_if<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM_LOSS, KM_NONE>(ga, lds, s, e) ||
          launch_if<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM_DW, KM_DX | KM_DW>(ga, lds, s, e) ||
          launch_if<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM_PARTIAL, KM_NONE>(ga, lds, s, e))
        return e;
    }
  }
  hipLaunchKernelGGL((gemm_grouped<T, WM, WN, WAVES_M, WAVES_N, KSPLIT>), dim3(ga.R, ga.total_blocks), dim3(256), lds, s,
                     ga);
  return hipGetLastError();
}

// table launches of the row-chain plan: {layer-0 split-K partial, X^T gather} and
// {DW of every layer}
// The layer-0 table launch uses the 64x32 LAT tile (split-K 4 inside the block);
// the weight-gradient launch a 64x64 tile with 2 N-waves x split-K 2: half the
// workgroups, so every DW problem of a small MLP is resident at once (the 64x32
// tile's 536 MNIST workgroups exceed the 2 per CU its registers allow and the last
// ones ran as a second round, +7 us)
template <typename T>
static hipError_t launch_table(const TableArgs& ta, int dw, hipStream_t s) {
  if (ta.total_blocks <= 0) return hipSuccess;
  if (dw) {
    const size_t lds = lds_bytes<T, 4, 2, 1, 2, 2>(false);
    hipLaunchKernelGGL((gemm_table<T, 4, 2, 1, 2, 2, KM_DW>), dim3(ta.R, ta.total_blocks), dim3(256), lds, s, ta);
  } else {
    const size_t lds = lds_bytes<T, 4, 2, 1, 1, 4>(false);
    hipLaunchKernelGGL((gemm_table<T, 4, 2, 1, 1, 4, KM_PARTIAL | KM_GATHER>), dim3(ta.R, ta.total_blocks), dim3(256), lds,
                       s, ta);
  }
  return hipGetLastError();
}

// the supported dual pair: problem 0 (DW) on the 128x64 THR-N64 tile (cfg 2), problem 1
// (DX) on the 64x32 LAT split-K tile (cfg 0)
template <typename T>
static size_t dual20_lds() {
  return std::max(lds_bytes<T, 4, 2, 2, 2, 1>(false), lds_bytes<T, 4, 2, 1, 1, 4>(false));
}
template <typename T>
static hipError_t launch_dual(const GroupArgs& ga, int a, int b, hipStream_t s) {
  if (a != 2 || b != 0 || ga.nprob != 2) return hipErrorInvalidValue;
  if (ga.total_blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL((gemm_dual<T, 4, 2, 2, 2, 1, 4, 2, 1, 1, 4, KM_DW, KM_DX>), dim3(ga.R, ga.total_blocks), dim3(256),
                     dual20_lds<T>(), s, ga);
  return hipGetLastError();
}
template <typename T>
static void set_attr_dual() {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_dual<T, 4, 2, 2, 2, 1, 4, 2, 1, 1, 4, KM_DW, KM_DX>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)dual20_lds<T>());
}

template <typename T>
static void set_attr_table() {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_table<T, 4, 2, 1, 2, 2, KM_DW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, 4, 2, 1, 2, 2>(false));
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_table<T, 4, 2, 1, 1, 4, KM_PARTIAL | KM_GATHER>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes<T, 4, 2, 1, 1, 4>(false));
}

template <typename T, int WM, int WN, int WAVES_M, int WAVES_N, int KSPLIT>
static void set_attr_spec() {
  set_attr<T, WM, WN, WAVES_M, WAVES_N, KSPLIT>();
  set_attr<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM_FWD, KM_GATHER>();
  set_attr<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM_LOSS, KM_NONE>();
  set_attr<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM_DW, KM_DX | KM_DW>();
  set_attr<T, WM, WN, WAVES_M, WAVES_N, KSPLIT, KM_PARTIAL, KM_NONE>();
}

}  // namespace ea
