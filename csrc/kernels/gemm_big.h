// 256x256 bf16 GEMM tile for the wide layers: 8 waves, 8-phase ping-pong schedule.
//
//   C[m][n] = sum_k A[m][k] * BT[n][k]   (the NT form of gemm_impl.h, same Prob kinds)
//
// Why a second tile: the 128x128 THR tile (gemm_impl.h) runs one barrier-separated
// "wait, stage, read, MFMA" step per 64-deep k-tile with one wave per SIMD per
// workgroup: every k-step drains its global->LDS copies before the barrier (~840 TF
// at 4096^3 vs ~1450 for hipBLASLt, profiles/README.md). This tile follows the
// 8-phase structure of the CDNA4 guide (cdna_hip_programming.md §5, T1-T5):
//
//   * 512 threads = 8 waves; wave w owns output rows (w >> 2) * 128 .. +128 and
//     columns (w & 3) * 64 .. +64 (8 x 4 fragments of 16x16, 128 accumulators).
//     Waves w and w + 4 share a SIMD and sit in different GROUPS (g = w >> 2);
//     group 1 runs one barrier behind group 0, so on every SIMD one wave issues its
//     16 MFMAs while its partner reads LDS fragments and issues its global->LDS
//     copies (a "tick" = the interval between two workgroup barriers).
//   * A 64-deep k-tile is 4 half-tiles of 128 rows x 128 B (A top / bottom, B^T
//     left / right); LDS holds two k-tiles (8 half-tile slots, 128 KB). A k-tile
//     is consumed in 4 phases, one output quadrant (64 rows x 32 columns x K 64 =
//     16 MFMAs) per phase in snake order (m0,n0) (m0,n1) (m1,n1) (m1,n0): fragment
//     reads 12 / 4 / 8 / 0 ds_read_b128 (the n0 B fragments stay in registers).
//   * Every phase stages ONE half-tile with 2 16-byte global_load_lds per thread:
//     phases 0 / 1 of k-tile t copy A top / bottom of t + 1 (their slots were last
//     read in phase 2 of t - 1), phases 2 / 3 copy B^T left / right of t + 2 (slots
//     last read in phase 1 of t). ONE counted wait per k-tile, in phase 3:
//     vmcnt(4) retires everything k-tile t + 1 needs and leaves the two B^T
//     half-tiles of t + 2 in flight (never vmcnt(0) in steady state); t + 1 is read
//     from the next phase on, after a barrier.
//   * LDS image rows are 128 B; chunk c of image row R holds source chunk
//     c ^ ((R >> 1) & 7) (the swizzle is applied to each lane's global SOURCE
//     address -- glds writes lane-linear): every ds_read_b128 lane group covers the
//     16 slots of a bank row once (conflict-free for the 16x16x32 fragment reads).
//
// The epilogue stages the finished tile through LDS in two 128-row halves (one
// group's rows each, 128 x 260 fp32 = 133 KB) and runs the shared fused Dense
// epilogues (tile_epilogue, gemm_impl.h) with 512 threads.
// (reference hot loop: elephas/worker.py:41-42 -> keras fit -> Dense fwd/bwd)
#pragma once
#include "gemm_impl.h"

namespace ea {

constexpr int BIG_BM = 256, BIG_BN = 256, BIG_BK = 64, BIG_NT = 512;
constexpr int BIG_HT = 128 * BIG_BK * 2;        // one half-tile: 128 rows x 128 B (16 KB)
constexpr int BIG_SET = 4 * BIG_HT;             // one k-tile: A top, A bottom, B^T left, B^T right
constexpr int BIG_EPI_LDS = 128 * (BIG_BN + 4) * 4;  // one 128-row half of the fp32 tile
constexpr int BIG_LDS = (2 * BIG_SET > BIG_EPI_LDS) ? 2 * BIG_SET : BIG_EPI_LDS;
static_assert(BIG_LDS <= 160 * 1024, "LDS per workgroup");

__device__ __forceinline__ void big_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// src[h][i]: source row of this thread's i-th staged row of half-tile h (0 A top,
// 1 A bottom, 2 B^T left, 3 B^T right; image row i * 64 + wave * 8 + lane / 8), as
// a byte address (the zero row / the bias ones row for rows without data);
// mov bit 2h + i: that row advances with k. acc[i][j]: output rows grp*128 + i*16
// + .., columns (wave & 3)*64 + j*16 + ..
// V (diagnostics / schedule variants, tools/big_variants.py): 0 the schedule above;
// 1 A half-tiles staged one phase earlier (A bottom of t + 1 in phase 0, A top of
// t + 2 in phase 3: 3 phases between the last copy k-tile t + 1 needs and its wait,
// vmcnt(6)); 5 and 6 below. (Measured with copies removed: 1042 / 1434 TF at 4096^3 /
// 8192^3; with fragment reads removed: 1129 / 1507 -- profiles/big_variants_r3.txt.)
template <int V = 0>
__device__ __forceinline__ void big_mainloop(const unsigned long long (&src)[4][2], unsigned mov, int K,
                                             f32x4 (&acc)[8][4], char* sbase) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2, wc = wave & 3;
  const int nk = (K + BIG_BK - 1) / BIG_BK;
  const unsigned lds_base = (unsigned)(size_t)((__attribute__((address_space(3))) char*)sbase);
  typedef unsigned long long u64;
  const u64 zp = (u64)(const void*)g_thr_zero;
  // staged 16-byte piece of this lane: image row i*64 + wave*8 + lane/8, image chunk
  // lane & 7 <- source chunk (lane & 7) ^ ((row >> 1) & 7) (row bits 1..3 = lane bits 4..5, wave bit 0)
  const int sc8 = ((lane & 7) ^ ((((wave & 1) << 2) | (lane >> 4)) & 7)) * 8;
  auto stage = [&](int h, int kt, int set) {
    const int kk = kt * BIG_BK + sc8;
    const bool kin = kk < K;
    const u64 koff = (u64)kk * 2u;
    char* d = sbase + set * BIG_SET + h * BIG_HT + wave * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const u64 a = src[h][i] + (((mov >> (2 * h + i)) & 1u) ? koff : 0u);
      glds16((const void*)(kin ? a : zp), d + i * 8192);
    }
  };
  // fragment reads: image row = base + (lane & 15), source chunk 4 ks + lane / 16
  const int x = (lane & 15) >> 1;
  const unsigned ck0 = (unsigned)((((lane >> 4)) ^ x) * 16), ck1 = (unsigned)(((4 + (lane >> 4)) ^ x) * 16);
  const unsigned a_row = (unsigned)(grp * BIG_HT + (lane & 15) * 128);
  const unsigned b_row = (unsigned)((2 + (wc >> 1)) * BIG_HT + ((wc & 1) * 64 + (lane & 15)) * 128);
  uint4 fa[4][2], fb0[2][2], fb1[2][2];
  auto read_a = [&](int set, int mh) {
    const unsigned b = lds_base + (unsigned)(set * BIG_SET) + a_row + (unsigned)(mh * 64 * 128);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ds_read16(fa[i][0], b + (unsigned)(i * 16 * 128) + ck0);
      ds_read16(fa[i][1], b + (unsigned)(i * 16 * 128) + ck1);
    }
  };
  auto read_b = [&](int set, int nh, uint4 (&fb)[2][2]) {
    const unsigned b = lds_base + (unsigned)(set * BIG_SET) + b_row + (unsigned)(nh * 32 * 128);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      ds_read16(fb[j][0], b + (unsigned)(j * 16 * 128) + ck0);
      ds_read16(fb[j][1], b + (unsigned)(j * 16 * 128) + ck1);
    }
  };
  auto mfma = [&](int mh, int nh, const uint4 (&fb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mma16<__bf16>(acc[mh * 4 + i][nh * 2 + j], fa[i][ks], fb[j][ks]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto lgkm0 = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };

  if constexpr (V == 0) {
  // prologue: k-tile 0 whole, B^T halves of k-tile 1; retire k-tile 0
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(h, 0, 0);
  if (nk > 1) {
    stage(2, 1, 1);
    stage(3, 1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  big_barrier();
  if (grp == 1) big_barrier();  // the ping-pong offset
  for (int t = 0; t < nk; ++t) {
    const int set = t & 1;
    // phase 0: quadrant (m0, n0); stage A top of t + 1
    read_b(set, 0, fb0);
    read_a(set, 0);
    if (t + 1 < nk) stage(0, t + 1, set ^ 1);
    lgkm0();
    big_barrier();
    mfma(0, 0, fb0);
    big_barrier();
    // phase 1: (m0, n1); stage A bottom of t + 1
    read_b(set, 1, fb1);
    if (t + 1 < nk) stage(1, t + 1, set ^ 1);
    lgkm0();
    big_barrier();
    mfma(0, 1, fb1);
    big_barrier();
    // phase 2: (m1, n1); stage B^T left of t + 2 (this set's B^T slots were last read in phase 1)
    read_a(set, 1);
    if (t + 2 < nk) stage(2, t + 2, set);
    lgkm0();
    big_barrier();
    mfma(1, 1, fb1);
    big_barrier();
    // phase 3: (m1, n0) from registers; stage B^T right of t + 2; retire k-tile t + 1
    if (t + 2 < nk) {
      stage(3, t + 2, set);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else if (t + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    big_barrier();
    mfma(1, 0, fb0);
    big_barrier();
  }
  } else {
  // V >= 1: per k-tile t, phase 0 copies A bottom of t + 1, phase 2 B^T left of t + 2,
  // phase 3 B^T right and A top of t + 2 (this set's A slots were last read in phase 2,
  // its B^T slots in phase 1); the wait in phase 3 leaves those three in flight.
  // V 6: the copies are issued in the MFMA tick (between MFMAs an LDS-DMA issue costs
  // less than beside a burst of reads); each group then retires k-tile t + 1 in its
  // read tick of phase 3 (vmcnt(2): B^T left of t + 2 in flight), before the barrier
  // that precedes the other group's first read of it. V 5: V 6 with the fragment-read
  // wait behind the barrier (the read tick ends once the reads are issued; the MFMA
  // tick absorbs what is left of their latency). Copies must stay in MFMA ticks then:
  // a read is only retired after the barrier that ends its tick, so a copy issued in
  // the next read tick of the other group could overwrite a slot still being read.
  constexpr bool LATE = V == 5, MCP = V >= 5;
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(h, 0, 0);
  if (nk > 1) {
    stage(2, 1, 1);
    stage(3, 1, 1);
    stage(0, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  big_barrier();
  if (grp == 1) big_barrier();  // the ping-pong offset
  auto tick_end = [&] {
    if (!LATE) lgkm0();
    big_barrier();
    if (LATE) lgkm0();
  };
  for (int t = 0; t < nk; ++t) {
    const int set = t & 1;
    read_b(set, 0, fb0);
    read_a(set, 0);
    if (!MCP && t + 1 < nk) stage(1, t + 1, set ^ 1);
    tick_end();
    if (MCP && t + 1 < nk) stage(1, t + 1, set ^ 1);
    mfma(0, 0, fb0);
    big_barrier();
    read_b(set, 1, fb1);
    tick_end();
    mfma(0, 1, fb1);
    big_barrier();
    read_a(set, 1);
    if (!MCP && t + 2 < nk) stage(2, t + 2, set);
    tick_end();
    if (MCP && t + 2 < nk) stage(2, t + 2, set);
    mfma(1, 1, fb1);
    big_barrier();
    if (MCP) {
      if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      big_barrier();
      if (t + 2 < nk) {
        stage(3, t + 2, set);
        stage(0, t + 2, set);
      }
    } else {
      if (t + 2 < nk) {
        stage(3, t + 2, set);
        stage(0, t + 2, set);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else if (t + 1 < nk) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      big_barrier();
    }
    mfma(1, 0, fb0);
    big_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (grp == 0) big_barrier();  // group 1's last MFMA tick
}

// One problem tile of the big config: block setup as run_prob, the ping-pong main
// loop, then the fused epilogue over two 128-row halves.
template <unsigned KM, int V = 0, typename GA>
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
    typedef unsigned long long u64;
    const u64 zp = (u64)(const void*)g_thr_zero, op = (u64)(const void*)g_thr_ones;
    u64 src[4][2];
    unsigned mov = 0;
    const int wv = threadIdx.x >> 6;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int rr = (h & 1) * 128 + i * 64 + wv * 8 + (lane >> 3);  // row of the 256-row operand tile
        u64 v = zp;
        bool real = false;
        if (h < 2) {
          const int m = m0 + rr;
          if (m == p.ones_row) {
            v = op;
          } else if (m < p.M) {
            if (p.a_gather) {
              if (m < valid) { v = (u64)(A + batch_row(p, r, step, m) * p.lda); real = true; }
            } else {
              v = (u64)(A + (long long)m * p.lda);
              real = true;
            }
          }
        } else {
          const int n = n0 + rr;
          if (n < p.N) { v = (u64)(BTp + (long long)n * p.ldb); real = true; }
        }
        src[h][i] = v;
        mov |= real ? 1u << (2 * h + i) : 0u;
      }
    }
    big_mainloop<V>(src, mov, p.K, acc, reinterpret_cast<char*>(smem));
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
__device__ __forceinline__ int big_group_of(int lin, int tiles_m, int tiles_n) {
  constexpr int GM = 4;
  const int per_group = GM * tiles_n;
  const int grp = lin / per_group, first = grp * GM;
  const int gsz = tiles_m - first < GM ? tiles_m - first : GM;
  const int in = lin - grp * per_group;
  return (first + in % gsz) * tiles_n + in / gsz;
}
__device__ __forceinline__ int big_tile_of(int b, int ntiles, int tiles_m, int tiles_n) {
  const int x = b & 7, q = ntiles >> 3, rem = ntiles & 7;
  return big_group_of((x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + (b >> 3), tiles_m, tiles_n);
}

// grid (R, total_blocks): problem by block range as gemm_grouped; the tile order
// inside a problem is XCD-aware when the launch has one replica.  With R = 8 every
// replica's tiles share one XCD (x-fastest dealing); G: take them in groups of 4 tile rows
// (column-major inside a group) so the XCD's concurrent tiles read each B^T column tile
// once per round instead of once per pair of tile rows
template <unsigned KM0, unsigned KM1, int V = 0, int G = 0>
__global__ __launch_bounds__(BIG_NT) void gemm_big(GroupArgs ga) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  stamp(ga, 0);
  const int r = blockIdx.x, bid = blockIdx.y;
  const int b0 = ga.p[0].block_begin, b1 = ga.p[1].block_begin;
  const int pi = (KM1 != KM_NONE && ga.nprob > 1 && bid >= b1 && (b1 > b0 || bid < b0)) ? 1 : 0;
  const Prob& p = pi ? ga.p[1] : ga.p[0];
  int lb = bid - p.block_begin;
  const int nt = p.tiles_m * p.tiles_n;
  if (ga.R == 1 && ga.nprob == 1) lb = big_tile_of(lb, nt, p.tiles_m, p.tiles_n);
  else if (G) lb = big_group_of(lb, p.tiles_m, p.tiles_n);
  if (pi) run_prob_big<KM1, V>(ga, ga.p[1], r, lb, smem);
  else run_prob_big<KM0, V>(ga, ga.p[0], r, lb, smem);
  stamp(ga, 4);
}

}  // namespace ea
