// 256x256 bf16 GEMM tile for the wide layers: 8 waves in two ping-pong groups.
//
//   C[m][n] = sum_k A[m][k] * BT[n][k]   (the NT form of gemm_impl.h, same Prob kinds)
//
// Why a second tile: the 128x128 THR tile (gemm_impl.h) runs one barrier-separated
// "wait, stage, read, MFMA" step per 64-deep k-tile with one wave per SIMD per
// workgroup, and stalls every wave on the same LDS read burst after each barrier
// (~840 TF at 4096^3 vs ~1450 for hipBLASLt, profiles/README.md). Here:
//
//   * 512 threads = 8 waves; wave w owns output rows (w >> 2) * 128 .. +128 and
//     columns (w & 3) * 64 .. +64 (8 x 4 fragments of 16x16, 128 accumulator VGPRs).
//   * Waves w and w + 4 share a SIMD; they are in different GROUPS (g = w >> 2).
//     Group 1 starts one barrier late, so on every SIMD one wave runs its 32 MFMAs
//     while its partner reads its next fragments from LDS and issues its share of
//     the global->LDS copies (a "tick" = the interval between two workgroup
//     barriers; group 0 reads sub-tile t in tick 2t and multiplies in 2t+1, group
//     1 reads in 2t+1 and multiplies in 2t+2). The matrix pipe of a SIMD is never
//     waiting for an LDS burst of its own wave.
//   * The k dimension advances in 32-deep sub-tiles (A 256x32 + B^T 256x32 bf16 =
//     32 KB) through a ring of NSLOT LDS slots (4 -> 128 KB, 5 -> 160 KB), filled
//     with 16-byte global_load_lds (no VGPR round trip). Group 0 copies the A half,
//     group 1 the B^T half (4 copies per lane per sub-tile each). Sub-tile t + NSLOT
//     - 1 is issued in the read tick of t (its slot held t - 1, whose last reader
//     retired its reads -- lgkmcnt(0) -- before the previous barrier), and each
//     group retires its copies of t + 1 with a COUNTED vmcnt before the barrier that
//     precedes the first read of t + 1, leaving the younger sub-tiles in flight.
//   * LDS image of a sub-tile row (64 bytes = 4 chunks of 8 k): chunk c of row r
//     lives in slot c ^ ((r >> 2) & 3). A fragment read (16 rows x one chunk per
//     16-lane group) then covers all 64 banks once: conflict-free. glds writes
//     lane-linear, so the swizzle is applied to each lane's SOURCE address.
//
// The epilogue stages the finished tile through LDS in two 128-row halves (one
// group's rows each, 128 x 260 fp32 = 133 KB) and runs the shared fused Dense
// epilogues (tile_epilogue, gemm_impl.h) with 512 threads.
// (reference hot loop: elephas/worker.py:41-42 -> keras fit -> Dense fwd/bwd)
#pragma once
#include "gemm_impl.h"

namespace ea {

constexpr int BIG_BM = 256, BIG_BN = 256, BIG_BK = 32, BIG_NT = 512;
constexpr int BIG_HALF = BIG_BM * BIG_BK * 2;   // bytes of one operand's sub-tile (16 KB)
constexpr int BIG_SLOT = 2 * BIG_HALF;          // A + B^T sub-tile (32 KB)
#ifndef EA_BIG_NSLOT
#define EA_BIG_NSLOT 5
#endif
constexpr int BIG_NSLOT = EA_BIG_NSLOT;
constexpr int BIG_EPI_LDS = 128 * (BIG_BN + 4) * 4;  // one 128-row half of the fp32 tile
constexpr int BIG_LDS = (BIG_NSLOT * BIG_SLOT > BIG_EPI_LDS) ? BIG_NSLOT * BIG_SLOT : BIG_EPI_LDS;
static_assert(BIG_LDS <= 160 * 1024, "LDS per workgroup");

// s_waitcnt vmcnt(4 * n): this wave's copies of the n youngest sub-tiles may stay in flight
__device__ __forceinline__ void big_wait_vm(int n) {
  if (n <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

__device__ __forceinline__ void big_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// srow[t]: source row of this lane's t-th staged row (nullptr = zero row) in the
// operand its group copies (group 0: A, group 1: B^T); ones: bit t = bias ones row.
// acc[i][j]: output rows grp*128 + i*16 + .., columns (wave & 3)*64 + j*16 + ..
__device__ __forceinline__ void big_mainloop(const __bf16* const (&srow)[4], unsigned ones, int K, f32x4 (&acc)[8][4],
                                             char* sbase) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2, wig = wave & 3;
  const int i16 = lane & 15, g = lane >> 4;
  const int ns = (K + BIG_BK - 1) / BIG_BK;
  const unsigned lds_base = (unsigned)(size_t)((__attribute__((address_space(3))) char*)sbase);
  typedef unsigned long long u64;
  const u64 zp = (u64)(const void*)g_thr_zero, op = (u64)(const void*)g_thr_ones;
  // staged chunk of this lane: LDS slot (lane & 3) of row lane >> 2 holds chunk
  // (lane & 3) ^ ((row >> 2) & 3) of that row
  const int c8 = ((lane & 3) ^ ((lane >> 4) & 3)) * 8;
  u64 base[4];
  unsigned mov = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bool o = (ones >> t) & 1u, real = srow[t] != nullptr && !o;
    base[t] = o ? op : (srow[t] ? (u64)srow[t] : zp);
    mov |= real ? 1u << t : 0u;
  }
  // copy sub-tile s into its ring slot: instruction t of wave wig covers rows
  // t*64 + wig*16 .. +16 of this group's operand (1 KB, lane-linear)
  auto stage = [&](int s) {
    const int kk = s * BIG_BK + c8;
    const bool kin = kk < K;
    const u64 koff = (u64)kk * 2u;
    char* d = sbase + (s % BIG_NSLOT) * BIG_SLOT + grp * BIG_HALF + wig * 1024;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const u64 a = base[t] + (((mov >> t) & 1u) ? koff : 0u);
      glds16((const void*)(kin ? a : zp), d + t * 4096);
    }
  };
  const unsigned swz = (unsigned)((g ^ ((i16 >> 2) & 3)) * 16);
  const unsigned a_off = (unsigned)((grp * 128 + i16) * 64) + swz;
  const unsigned b_off = (unsigned)(BIG_HALF + (wig * 64 + i16) * 64) + swz;
  uint4 fa[8], fb[4];
  auto read = [&](int s) {
    const unsigned sb = lds_base + (unsigned)((s % BIG_NSLOT) * BIG_SLOT);
#pragma unroll
    for (int j = 0; j < 4; ++j) ds_read16(fb[j], sb + b_off + (unsigned)(j * 16 * 64));
#pragma unroll
    for (int i = 0; i < 8; ++i) ds_read16(fa[i], sb + a_off + (unsigned)(i * 16 * 64));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) mma16<__bf16>(acc[i][j], fa[i], fb[j]);
    __builtin_amdgcn_s_setprio(0);
  };
  // copies of the youngest sub-tiles this wave may leave in flight once sub-tile t
  // must have landed (it has issued 0 .. min(t + NSLOT - 2, ns - 1) or, after the
  // read tick of t - 1, up to min(t + NSLOT - 2, ns - 1) as well)
  auto ahead = [&](int t) { return (t + BIG_NSLOT - 2 < ns - 1 ? t + BIG_NSLOT - 2 : ns - 1) - t; };

#pragma unroll
  for (int s = 0; s < BIG_NSLOT - 1; ++s)
    if (s < ns) stage(s);
  big_wait_vm(ahead(0));
  big_barrier();
  if (grp == 1) big_barrier();  // the ping-pong offset
  for (int t = 0; t < ns; ++t) {
    // read tick: refill the slot of t - 1, fetch this wave's fragments of t
    if (t + BIG_NSLOT - 1 < ns) stage(t + BIG_NSLOT - 1);
    read(t);
    if (grp == 1 && t + 1 < ns) big_wait_vm(ahead(t + 1));  // B^T of t + 1 landed
    big_barrier();
    // MFMA tick
    mfma();
    if (grp == 0 && t + 1 < ns) big_wait_vm(ahead(t + 1));  // A of t + 1 landed
    big_barrier();
  }
  if (grp == 0) big_barrier();  // group 1's last MFMA tick
}

// One problem tile of the big config: block setup as run_prob, the ping-pong main
// loop, then the fused epilogue over two 128-row halves.
template <unsigned KM, typename GA>
__device__ __forceinline__ void run_prob_big(const GA& ga, const Prob& p, const int r, const int lb, float* smem) {
  using T = __bf16;
  const int tm = lb / p.tiles_n, tn = lb % p.tiles_n;
  const int m0 = tm * BIG_BM, n0 = tn * BIG_BN;
  const long long step = ld_inv(ga.ctr) + ga.step_off;
  const long long iter = iter_at(ga.ctr, p.ntrain, p.B, r, ld_inv(ga.ctr), ga.step_off);
  const int valid = (p.kind == PK_PLAIN) ? p.M : batch_valid(p, r, step);
  const bool skip_update = (p.kind == PK_DW_UPDATE) && valid == 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, grp = wave >> 2, wig = wave & 3;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  stamp(ga, 1);
  if (!skip_update) {
    const __bf16* A = reinterpret_cast<const __bf16*>(p.A) + (long long)r * p.sA;
    const __bf16* BTp = reinterpret_cast<const __bf16*>(p.BT) + (long long)r * p.sB +
                        (p.bt_shadow ? (iter & 1) * p.bt_par : 0);
    const __bf16* srow[4];
    unsigned ones = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int rr = t * 64 + wig * 16 + (lane >> 2);
      srow[t] = nullptr;
      if (grp == 0) {
        const int m = m0 + rr;
        if (m == p.ones_row) {
          ones |= 1u << t;
        } else if (m < p.M) {
          if (p.a_gather) {
            if (m < valid) srow[t] = A + batch_row(p, r, step, m) * p.lda;
          } else {
            srow[t] = A + (long long)m * p.lda;
          }
        }
      } else {
        const int n = n0 + rr;
        if (n < p.N) srow[t] = BTp + (long long)n * p.ldb;
      }
    }
    big_mainloop(srow, ones, p.K, acc, reinterpret_cast<char*>(smem));
  }
  stamp(ga, 2);
  __syncthreads();  // every wave is done with the staging ring
  const int g = lane >> 4, i16 = lane & 15;
  constexpr int LDC = BIG_BN + 4;
  const bool pf_vec[1] = {false};
  const float pz[1][8] = {{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (grp == h) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) smem[(i * 16 + g * 4 + q) * LDC + wig * 64 + j * 16 + i16] = acc[i][j][q];
    }
    __syncthreads();
    tile_epilogue<T, 128, BIG_BN, BIG_NT, KM, 1, false>(ga, p, r, m0 + h * 128, n0, 0, valid, iter, step, skip_update,
                                                         smem, pf_vec, pz, pz, pz);
    __syncthreads();
  }
}

// XCD-aware tile order: blocks are dealt to the 8 XCDs round-robin, so block b
// runs on XCD b % 8; give each XCD a contiguous run of tiles, ordered in groups of
// 4 tile rows (column-major inside a group) so an XCD's concurrent tiles share A
// rows and B^T columns in its L2. Bijective for any tile count.
__device__ __forceinline__ int big_tile_of(int b, int ntiles, int tiles_m, int tiles_n) {
  const int x = b & 7, q = ntiles >> 3, rem = ntiles & 7;
  const int lin = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + (b >> 3);
  constexpr int GM = 4;
  const int per_group = GM * tiles_n;
  const int grp = lin / per_group, first = grp * GM;
  const int gsz = tiles_m - first < GM ? tiles_m - first : GM;
  const int in = lin - grp * per_group;
  return (first + in % gsz) * tiles_n + in / gsz;
}

// grid (R, total_blocks): problem by block range as gemm_grouped; the tile order
// inside a problem is XCD-aware when the launch has one replica
template <unsigned KM0, unsigned KM1>
__global__ __launch_bounds__(BIG_NT) void gemm_big(GroupArgs ga) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  stamp(ga, 0);
  const int r = blockIdx.x, bid = blockIdx.y;
  const int pi = (KM1 != KM_NONE && ga.nprob > 1 && bid >= ga.p[1].block_begin) ? 1 : 0;
  const Prob& p = pi ? ga.p[1] : ga.p[0];
  int lb = bid - p.block_begin;
  const int nt = p.tiles_m * p.tiles_n;
  if (ga.R == 1 && ga.nprob == 1) lb = big_tile_of(lb, nt, p.tiles_m, p.tiles_n);
  if (pi) run_prob_big<KM1>(ga, ga.p[1], r, lb, smem);
  else run_prob_big<KM0>(ga, ga.p[0], r, lb, smem);
  stamp(ga, 4);
}

}  // namespace ea
