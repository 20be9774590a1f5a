// Persistent replica-cluster training kernel (MI355X / gfx950): a whole chunk of
// training steps of a 3-layer Dense stack in ONE launch.
//
// Why: the MNIST step is latency-bound (profiles/README.md): the row-chain plan runs
// it as three launches whose every phase is a dependent global round trip, and every
// launch re-reads the weights it updates.  Here a replica's work is spread over a
// fixed cluster of workgroups that stay resident for the whole chunk (one workgroup
// per CU; block b serves replica b % R, so with R = 8 a replica's cluster shares one
// XCD's L2 -- speed only, the protocol never depends on placement):
//
//   L0 workgroups (nk0 x nc0 per replica) each OWN a kc0 x cw tile of W0 (in LDS, for
//     the whole chunk) and its optimizer state (registers).  Per step: wait for dZ_0,
//     DW0 tile = X^T dZ_0, update the tile in place, then the NEXT step's split-K
//     partial Z_0 tile = X_next . W0_tile (+ b0 on the first k-chunk) -> workspace.
//     The next batch's X chunk streams into LDS (LDS-DMA) while they wait.
//   chain workgroups (nch = B/16 per replica, 16 batch rows each): sum the partials
//     (+ act, dropout), layer 1 and 2 forward, loss / metrics, input gradients down to
//     dZ_0 -- row-local work, W1 / W2 read from LDS -- then publish dZ_0 and the weight
//     gradient operands; in the time the L0 workgroups need for their part, each chain
//     workgroup computes DW1 / DW2 for the layer-1 columns (layer-2 rows) it owns,
//     updates them (masters and optimizer state in registers), publishes them, and
//     loads the whole new W1 / W2 for the next step.
//   (V2 roles -- plain SGD + ReLU, fit granularity: l0_role_v2 / chain_role<V2> /
//     dw_role_v2 below; layer-0 pre-activations two steps ahead plus a Gram correction
//     in the chains, W1 / W2 and the Gram slabs on weight-gradient workgroups.  bf16
//     instances run their products on v_mfma_f32_16x16x32_bf16.  docs/templates/
//     persistent-kernel.md has the roles, the modes -- per-step sync inside the launch,
//     across ranks through peer-mapped buffers, the parameter-server hook -- and safety.)
//
// Hand-offs follow the write-through form of the guide's inter-workgroup protocol
// (cdna_hip_programming.md Guideline 16, R1): every handed-off byte is stored and
// loaded with sc1 buffer instructions, each storing wave drains (s_waitcnt vmcnt(0)),
// the workgroup barriers, one lane stores the flag (agent-scope relaxed = sc1); one
// wave polls the producers' flags with sc1 loads.  Tags are the step index + 1 within
// the launch; the flag block is zero at every launch (hipMemset + hipDeviceSynchronize
// at setup, then the 1-block post kernel after each launch clears it again).  Every
// spin is bounded (timeout -> sticky error word, the workgroup returns; the host
// raises), and a launch that finds the error word set does nothing.
//
// Latency discipline (profiles/persist_*): every phase issues all of its global loads
// (or LDS fragment reads) before the first use; handed-off rows are published from LDS
// as coalesced 16-byte stores; per-lane buffer offsets stay few (the uniform parts go
// in the SGPR soffset) so that the step loop does not spill.
//
// Semantics are those of the row-chain plan (reference elephas/worker.py:41-42 ->
// one Keras fit step per batch): identical dropout masks (dropout_u1), batch windows,
// optimizer iterations and loss epilogues; master weights and state are read from P / S
// at the start of the launch and written back at its end (V1 with both weight-image
// parities; V2 the masters only -- the host rebuilds the images before their next
// reader).
#include "common.h"
#include "loss_tile.h"

// XCD-local instance (persist_local.hip compiles this file again with EA_PLOCAL = 1): a
// replica's workgroups all run on ONE XCD (the dispatch deals blocks round-robin over the 8
// XCDs, so blocks b and b + 8 share one: the host picks this instance only for R a multiple
// of 8, after probing that, and each chain verifies it at launch, below), so
// the intra-replica hand-offs need not leave that XCD's L2: their bytes and flags are stored
// PLAIN (the line stays in the L2, where the consumers' sc1 loads -- which skip only the
// CU's L1 -- find it) instead of write-through (sc1 stores drop the line, and the consumer
// re-reads it at the cross-XCD rate).  tools/micro/xchg_floor.hip: 8-workgroup exchange of
// 16 KB slabs 3.6 -> 2.6 us, flag round 1.5 -> 1.2 us (profiles/xchg_floor_r6.txt).  The
// cross-replica (sync exchange) and cross-rank hand-offs stay write-through.
//
// Exchange-local instance (persist_xlocal.hip, EA_PLOCAL = 2; per-step sync of 8 replicas on
// the V1 roles): the other way round -- workgroup q of every replica on ONE XCD (blocks
// mapped so that the 8 copies of a gradient tile share an XCD), the replica-sum exchange's
// slabs and flags stored plain, the intra-replica hand-offs (now across XCDs) write-through.
#ifndef EA_PLOCAL
#define EA_PLOCAL 0
#endif

namespace ea {

namespace {

using gu32 = __attribute__((address_space(1))) unsigned;
using rsrc_t = __amdgpu_buffer_rsrc_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

constexpr int S17 = 17;   // LDS stride of 16-wide tiles
constexpr int TU = 4;     // weight-gradient tiles per wave (<= 16 per workgroup)

// LDS row strides are width + 1 (== 1 mod 32 for widths 64 / 128 / 32 / 16): the b32
// fragment reads below -- 16 rows x k, or k x 16 columns, with k = kb + 16g + ks --
// hit 32 distinct banks per half-wave.
template <int H0, int H1>
struct ChainLds {
  static constexpr int L0S = H0 + 1, L1S = H1 + 1;
  static constexpr int STAGE = 64 * L0S + 2 * 64 * 33 + 64 * S17;    // weight-gradient operands
  static constexpr int W1 = (H0 * L1S > STAGE ? H0 * L1S : STAGE);  // W1, or the staging over it
  static constexpr int o_w2 = W1;                     // [H1][17]
  static constexpr int o_a0 = o_w2 + H1 * S17;        // [16][L0S]
  static constexpr int o_g0 = o_a0 + 16 * L0S;        // [16][L0S]
  static constexpr int o_z0 = o_g0 + 16 * L0S;        // [16][L0S] dZ_0 rows (published from here)
  static constexpr int o_a1 = o_z0 + 16 * L0S;        // [16][L1S]
  static constexpr int o_d1 = o_a1 + 16 * L1S;        // [16][L1S]
  static constexpr int o_d2 = o_d1 + 16 * L1S;        // [16][17]
  static constexpr int o_red = o_d2 + 16 * S17;       // [4][256]
  static constexpr int o_lg = o_red + 1024;           // [16][36]
  static constexpr int o_y = o_lg + 16 * 36;          // [16][32]
  static constexpr int o_b1 = o_y + 16 * 32;          // [H1]
  static constexpr int o_b2 = o_b1 + H1;              // [16]
  static constexpr int o_row = o_b2 + 16;             // [16] ints
  static constexpr int o_gs = o_row + 16;             // [16][65] V2: this chain's Gram rows (+ 1)
  static constexpr int o_wr = o_gs + 16 * 65;         // [4] V2: the W hand-off seen early (broadcast)
  static constexpr int TOTAL = o_wr + 4;
};
constexpr int L0_LDS = 2 * 64 * 129 + 128 * 33 + 64 * 33 + 128 * 33;   // + the pulled tile (PS hook)
// V2 layer-0: three X chunks (kc0 <= 112: stride 113), W0 tile (cw <= 64), dZ_0 columns, store staging
constexpr int L0V2_LDS = 3 * 64 * 113 + 128 * 65 + 64 * 65 + 64 * 65;
constexpr int DW_LDS = 64 * 129 + 2 * 64 * 33 + 64 * 17 + 32 * 17;
// + the Gram k-chunk (ng > 0): two X chunks of <= 112 columns (row stride <= 116) and
// the 64 x 64 slab staging
constexpr int DWG_LDS = DW_LDS + 2 * 64 * 116 + 64 * 65;
constexpr int DWP_LDS = DWG_LDS;
constexpr int cmax(int x, int y) { return x > y ? x : y; }
constexpr int LDS_FLOATS = (cmax(cmax(ChainLds<128, 128>::TOTAL, L0_LDS), cmax(L0V2_LDS, DWP_LDS)) + 3) & ~3;

__device__ __forceinline__ f32x4 mma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 zero4f() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// mixed_bfloat16 policy (BF instances): every MFMA operand rounded to bf16 (round to
// nearest even) at its fragment load -- a bf16 x bf16 product is exact in fp32, so the
// fp32 MFMA on rounded operands gives the numerics of a bf16 MFMA with fp32 accumulation
// (the latency-bound step gains nothing from the faster bf16 matrix rate; the data shard
// itself is bf16, half the bytes per step)
template <bool BF>
__device__ __forceinline__ float rb(float x) {
  if constexpr (BF) {
    const unsigned u = __builtin_bit_cast(unsigned, x);
    return __builtin_bit_cast(float, (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u);
  } else {
    return x;
  }
}
// two fp32 values rounded to bf16 (RNE, as rb<true>) packed in one dword, lo first
__device__ __forceinline__ unsigned bf2(float lo, float hi) {
  const unsigned a = __builtin_bit_cast(unsigned, lo), b = __builtin_bit_cast(unsigned, hi);
  return ((a + 0x7fffu + ((a >> 16) & 1u)) >> 16) | ((b + 0x7fffu + ((b >> 16) & 1u)) & 0xffff0000u);
}
__device__ __forceinline__ bf16x8 bf8(const float (&v)[8]) {
  return __builtin_bit_cast(bf16x8, u32x4{bf2(v[0], v[1]), bf2(v[2], v[3]), bf2(v[4], v[5]), bf2(v[6], v[7])});
}

// one element of a bf16 row packed two per dword in LDS (element k of a row at dword k / 2)
__device__ __forceinline__ float bf_at(const float* row, int k) {
  const unsigned d = __builtin_bit_cast(unsigned, row[k >> 1]);
  return __builtin_bit_cast(float, (k & 1) ? (d & 0xffff0000u) : (d << 16));
}
// replica r's weight image (elements of the compute dtype), as the float* img_store takes
template <bool BF>
__device__ __forceinline__ float* img_base(float* base, long long off) {
  if constexpr (BF) return reinterpret_cast<float*>(reinterpret_cast<__bf16*>(base) + off);
  else return base + off;
}
// weight-image store in the trainer's compute dtype
template <bool BF>
__device__ __forceinline__ void img_store(float* base, long long i, float v) {
  if constexpr (BF) reinterpret_cast<__bf16*>(base)[i] = (__bf16)v;
  else base[i] = v;
}

// ---- write-through (sc1) accesses of handed-off bytes through a buffer resource of
//      the replica's workspace: per-lane offset v + uniform offset s (SGPR), in floats
__device__ __forceinline__ rsrc_t ws_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ f32x4 ldw4(rsrc_t r, int v, int s) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, v * 4, s * 4, 16));
}
__device__ __forceinline__ float ldw1(rsrc_t r, int v, int s) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, v * 4, s * 4, 16));
}
// intra-replica hand-off stores: write-through (sc1 = aux 16), or plain in the XCD-local instance
constexpr int ST_AUX = EA_PLOCAL == 1 ? 0 : 16;
__device__ __forceinline__ void stw1(rsrc_t r, int v, int s, float x) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), r, v * 4, s * 4, ST_AUX);
}
__device__ __forceinline__ void stw4(rsrc_t r, int v, int s, f32x4 x) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), r, v * 4, s * 4, ST_AUX);
}
// cross-replica hand-off stores (the sync exchange slabs): write-through, or plain in the
// exchange-local instance
// a master written back to P at the end of the launch: plain -- or, when the launch ends with the
// fused averaging, write-through (4-byte agent-scope store = sc1) so its readers on other XCDs
// find it.  (Measured: the 4-byte write-through epilogue costs more than the launch the fused
// averaging saves -- 20.0 vs 19.3 us per step at the bench's 20-step shape -- so the bench
// keeps the separate replica_average kernel; ELEPHAS_AMD_FUSED_AVG=1 selects this path)
__device__ __forceinline__ void pst(const PersistArgs& a, float* p, float v) {
  if (a.avg_end) __hip_atomic_store((gu32*)(reinterpret_cast<unsigned*>(p)), __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
constexpr int SX_AUX = EA_PLOCAL == 2 ? 0 : 16;
__device__ __forceinline__ void stx4(rsrc_t r, int v, int s, f32x4 x) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), r, v * 4, s * 4, SX_AUX);
}

__device__ __forceinline__ unsigned* flag_at(const PersistArgs& a, int r, int kind) {
  return a.flags + ((long long)r * PMF_N + kind) * PM_MAXWG;
}

// R1 publish: every storing wave drains its sc1 stores, the workgroup meets, one lane
// raises the flag (agent-scope relaxed store = sc1).  XCD-local instance: the flag of an
// intra-replica hand-off is a plain store (it stays in the L2 the pollers' sc1 loads read)
__device__ __forceinline__ void publish_x(unsigned* flag, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (EA_PLOCAL == 2) __builtin_amdgcn_raw_buffer_store_b32(tag, ws_rsrc(reinterpret_cast<float*>(flag)), 0, 0, 0);
    else __hip_atomic_store((gu32*)(flag), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void publish(unsigned* flag, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (EA_PLOCAL == 1) __builtin_amdgcn_raw_buffer_store_b32(tag, ws_rsrc(reinterpret_cast<float*>(flag)), 0, 0, 0);
    else __hip_atomic_store((gu32*)(flag), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// wave 0 polls flags[0 .. n) (lane q watches producer q) until every one reaches tag;
// the whole workgroup leaves together.  false: timed out (error word set)
__device__ __forceinline__ bool wait_all(const PersistArgs& a, const unsigned* flags, int n, unsigned tag,
                                         unsigned code, long long tmo = -1) {
  int ok = 1;
  if (tmo < 0) tmo = a.timeout;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      const unsigned v = lane < n ? __hip_atomic_load((gu32*)(const_cast<unsigned*>(flags) + lane),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : tag;
      if (__all(v >= tag)) break;
      if ((long long)(wall_clock64() - t0) > tmo) {
        ok = 0;
        if (lane == 0) __hip_atomic_store((gu32*)(a.err), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no load moves above the poll
  return ok != 0;
}

// the same for two producer sets at once (lanes [0, n) watch set A, [n, n + m) set B)
__device__ __forceinline__ bool wait_two(const PersistArgs& a, const unsigned* fa, int n, unsigned ta,
                                         const unsigned* fb, int m, unsigned tb, unsigned code) {
  int ok = 1;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const bool inA = lane < n, inB = lane >= n && lane < n + m;
    const unsigned* f = inA ? fa + lane : fb + (inB ? lane - n : 0);
    const unsigned want = inA ? ta : tb;
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      const unsigned v = (inA || inB) ? __hip_atomic_load((gu32*)(const_cast<unsigned*>(f)), __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : want;
      if (__all(v >= want)) break;
      if ((long long)(wall_clock64() - t0) > a.timeout) {
        ok = 0;
        if (lane == 0) __hip_atomic_store((gu32*)(a.err), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok != 0;
}

// the same for up to four producer sets (lanes [o_s, o_s + n_s) watch set s; <= 64 in all):
// one poll, one barrier for every hand-off a phase depends on
struct WaitSet {
  const unsigned* f;
  int n;
  unsigned tag;
};
__device__ __forceinline__ bool wait_sets(const PersistArgs& a, const WaitSet (&ws)[4], unsigned code) {
  int ok = 1;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned* f = nullptr;
    unsigned want = 0;
    int o = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (lane >= o && lane < o + ws[k].n) {
        f = ws[k].f + (lane - o);
        want = ws[k].tag;
      }
      o += ws[k].n;
    }
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      const unsigned v = f ? __hip_atomic_load((gu32*)(const_cast<unsigned*>(f)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : want;
      if (__all(v >= want)) break;
      if ((long long)(wall_clock64() - t0) > a.timeout) {
        ok = 0;
        if (lane == 0) __hip_atomic_store((gu32*)(a.err), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok != 0;
}

// residency: wave 0 polls the GO flag of every workgroup of the grid (R replicas x wgs)
// until all are raised.  A workgroup that is not resident never raises
// it, so the waiting ones time out (PERR_GRID) before any of them modified state.
// XCD-local instances: a GO flag carries its workgroup's XCD + 1, and a workgroup whose L2
// partners (EA_PLOCAL 1: its replica; 2: the copies of its tile q in the other replicas) do
// not all share its XCD gives up (PERR_PLACE), state intact.
__device__ __forceinline__ unsigned xcc_id() {
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));   // HW_REG_XCC_ID[3:0]
}
__device__ __forceinline__ unsigned go_value() { return EA_PLOCAL ? xcc_id() + 1u : 1u; }
__device__ __forceinline__ bool wait_grid(const PersistArgs& a, int r, int q) {
  int ok = 1;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x, tot = a.R * a.wgs;
    const unsigned mine = go_value();
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      bool all = true, away = false;
      for (int f = lane; f < tot; f += 64) {
        const int rr = f % a.R, qq = f / a.R;
        const unsigned v = __hip_atomic_load((gu32*)(flag_at(a, rr, PMF_GO) + qq), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        all &= v != 0u;
        // the workgroups this one hands off to through the L2: its replica (1) / its tile's copies (2)
        away |= EA_PLOCAL != 0 && (EA_PLOCAL == 1 ? rr == r : qq == q) && v != 0u && v != mine;
      }
      if (__all(all)) {
        if (__any(away)) {
          ok = 0;
          if (lane == 0) __hip_atomic_store((gu32*)(a.err), (unsigned)PERR_PLACE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        break;
      }
      if ((long long)(wall_clock64() - t0) > a.timeout) {
        ok = 0;
        if (lane == 0) __hip_atomic_store((gu32*)(a.err), (unsigned)PERR_GRID, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  ok = __syncthreads_and(ok);
  return ok != 0;
}

// The rank part of the per-step exchange (replica 0's owning workgroup q): put this rank's
// tile sum v into slab [tag & 1][q] of its peer-mapped buffer, raise flag q (system scope,
// tag monotonic over the trainer's life), wait for flag q of every rank, and replace v by
// the ranks' slabs summed in rank order -- the same bits on every rank.  false: a rank did
// not arrive within xr_timeout (error word PERR_XRANK).  Shared by xchg_sum and the
// numeric self-test the host runs before it trusts the path (xrank_selftest_kernel).
template <int N>
__device__ __forceinline__ bool xrank_sum(const PersistArgs& a, int q, unsigned tag, f32x4 (&v)[N]) {
  const int tid = threadIdx.x;
  const long long soff = PEER_DATA_OFF + ((long long)(tag & 1u) * a.wgs + q) * PM_XSLOT * 4;
  int ok = 1;
  f32x4* dst = reinterpret_cast<f32x4*>(a.xr_base[a.xr_rank] + soff);
#pragma unroll
  for (int u = 0; u < N; ++u) dst[u * 256 + tid] = v[u];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    __hip_atomic_store(reinterpret_cast<unsigned*>(a.xr_base[a.xr_rank] + PEER_FLAG_OFF + (long long)q * 64), tag,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < 64) {
    // lane k watches rank k's flag q (the rank's buffer by selects: no per-lane kernarg indexing)
    char* b = a.xr_base[0];
#pragma unroll
    for (int k = 1; k < PEER_MAX_RANKS; ++k) b = (tid == k) ? a.xr_base[k] : b;
    const unsigned* fl = reinterpret_cast<const unsigned*>(b + PEER_FLAG_OFF + (long long)q * 64);
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      const unsigned f = tid < a.xr_world ? __hip_atomic_load(const_cast<unsigned*>(fl), __ATOMIC_ACQUIRE,
                                                              __HIP_MEMORY_SCOPE_SYSTEM)
                                          : tag;
      if (__all((int)(f - tag) >= 0)) break;   // wrap-safe: tags only grow
      if ((long long)(wall_clock64() - t0) > a.xr_timeout) {
        ok = 0;
        if (tid == 0) __hip_atomic_store((gu32*)(a.err), (unsigned)PERR_XRANK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (!ok) return false;
#pragma unroll
  for (int u = 0; u < N; ++u) v[u] = zero4f();
#pragma unroll 1
  for (int k = 0; k < a.xr_world; ++k) {   // rank order
    char* b = a.xr_base[0];
#pragma unroll
    for (int kk = 1; kk < PEER_MAX_RANKS; ++kk) b = (k == kk) ? a.xr_base[kk] : b;
    const f32x4* src = reinterpret_cast<const f32x4*>(b + soff);
    f32x4 x[N];
#pragma unroll
    for (int u = 0; u < N; ++u) x[u] = __builtin_nontemporal_load(src + u * 256 + tid);
#pragma unroll
    for (int u = 0; u < N; ++u) v[u] += x[u];
  }
  return true;
}

// lane 0..R-1 of wave 0 watches flag `kind` of workgroup q in replica lane's flag area
// until every one reaches tag; the whole workgroup leaves together
__device__ __forceinline__ bool wait_replicas(const PersistArgs& a, int kind, int q, unsigned tag) {
  const int tid = threadIdx.x;
  int ok = 1;
  if (tid < 64) {
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      const unsigned f = tid < a.R ? __hip_atomic_load((gu32*)(flag_at(a, tid, kind) + q), __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : tag;
      if (__all(f >= tag)) break;
      if ((long long)(wall_clock64() - t0) > a.timeout) {
        ok = 0;
        if (tid == 0) __hip_atomic_store((gu32*)(a.err), (unsigned)PERR_XCHG, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok != 0;
}

// sync: sum the weight-gradient fragments v[0 .. N) (f32x4 per lane, lane-linear slab
// layout, E = 256 N f32x4) of workgroup q over the R replicas, in replica order, as a
// reduce-scatter + all-gather inside the slabs (xchg_rs; else every replica sums all R
// slabs, 4 slabs' loads in flight): every replica stores its partial slab and
// raises PMF_X; replica r sums chunk r (f32x4 [rC, rC + C), C = ceil(E / R)) over the R
// slabs in replica order and writes the sum over its own chunk r (only r reads that
// chunk's partial), raises PMF_XS; then every replica reads chunk o's sum from replica o.
// Each workgroup moves 2 slabs instead of R (the all-gather-and-sum it replaces read R),
// and the sums are the same bits as R in-order additions everywhere.  Every storing wave
// drains its sc1 stores before a flag (publish); the slabs alternate by step parity: a
// replica writes step i + 2's partials only after seeing every replica's step i + 1
// partials, which each stored after finishing its step-i reads.
template <int N>
__device__ __forceinline__ bool xchg_sum(const PersistArgs& a, int r, int q, int i, f32x4 (&v)[N]) {
  const int tid = threadIdx.x;
  const long long slab = a.o_xg + ((long long)(i & 1) * a.wgs + q) * PM_XSLOT;
  const rsrc_t all = ws_rsrc(a.ws);   // every replica's workspace (offsets r * ws_stride)
  if (a.R > 1) {
    const unsigned tag = (unsigned)(i + 1);
#pragma unroll
    for (int u = 0; u < N; ++u) stx4(all, (u * 256 + tid) * 4, (int)((long long)r * a.ws_stride + slab), v[u]);
    publish_x(flag_at(a, r, PMF_X) + q, tag);
    if (!wait_replicas(a, PMF_X, q, tag)) return false;
    if (a.xchg_rs) {
      constexpr int E = N * 256;
      const int C = (E + a.R - 1) / a.R;
      const int lo = r * C, hi = lo + C < E ? lo + C : E;
      for (int e = lo + tid; e < hi; e += 256) {
        f32x4 s = zero4f();
        for (int rb = 0; rb < a.R; rb += 8) {   // 8 slabs' loads in flight, summed in replica order
          f32x4 x[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int rr = rb + k < a.R ? rb + k : rb;
            x[k] = ldw4(all, e * 4, (int)((long long)rr * a.ws_stride + slab));
          }
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (rb + k < a.R) s += x[k];
        }
        stx4(all, e * 4, (int)((long long)r * a.ws_stride + slab), s);
      }
      publish_x(flag_at(a, r, PMF_XS) + q, tag);
      if (!wait_replicas(a, PMF_XS, q, tag)) return false;
#pragma unroll
      for (int u = 0; u < N; ++u) {
        const int e = u * 256 + tid;
        v[u] = ldw4(all, e * 4, (int)((long long)(e / C) * a.ws_stride + slab));
      }
    } else {
#pragma unroll
      for (int u = 0; u < N; ++u) v[u] = zero4f();
      for (int rb = 0; rb < a.R; rb += 4) {   // 4 slabs' loads in flight, summed in replica order
        f32x4 x[4][N];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int rr = rb + k < a.R ? rb + k : rb;
#pragma unroll
          for (int u = 0; u < N; ++u) x[k][u] = ldw4(all, (u * 256 + tid) * 4, (int)((long long)rr * a.ws_stride + slab));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (rb + k < a.R) {
#pragma unroll
            for (int u = 0; u < N; ++u) v[u] += x[k][u];
          }
      }
    }
  }
  if (a.xr_world <= 1) return true;
  // ---- across ranks: replica 0 publishes the rank's sum, reads every rank's (over xGMI
  // on a node), sums them in rank order and leaves the total in its local total slab; the
  // other replicas read that (one remote read set per workgroup and rank, not R of them)
  const long long tslab = a.o_xt + ((long long)(i & 1) * a.wgs + q) * PM_XSLOT;   // in replica 0's workspace
  if (r == 0) {
    if (!xrank_sum<N>(a, q, a.xr_tag0 + (unsigned)i + 1u, v)) return false;
    if (a.R > 1) {   // the total for the other replicas (write-through, then the local flag)
#pragma unroll
      for (int u = 0; u < N; ++u) stx4(all, (u * 256 + tid) * 4, (int)tslab, v[u]);
      publish_x(flag_at(a, 0, PMF_XT) + q, (unsigned)(i + 1));
    }
    return true;
  }
  // replica 0 may itself wait for a late rank: the rank exchange's patience here too
  if (!wait_all(a, flag_at(a, 0, PMF_XT) + q, 1, (unsigned)(i + 1), PERR_XRANK, a.xr_timeout)) return false;
#pragma unroll
  for (int u = 0; u < N; ++u) v[u] = ldw4(all, (u * 256 + tid) * 4, (int)tslab);
  return true;
}

// ---- in-launch parameter-server hook (PersistArgs::ps_mode; layout: peer_args.h,
//      kernels: peer.hip).  theta element i lives in the buffer of the rank owning its
//      4096-parameter chunk; the memory is uncached (hipDeviceMallocUncached), so plain
//      loads and system-scope atomics see every rank's latest writes.
__device__ __forceinline__ float* ps_elem(const PsArgs& ps, long long i) {
  // the shard holding i, by selects against the (uniform) shard starts: no per-lane
  // indexing of the kernel-argument array (that would go through scratch)
  char* b = ps.base[0];
#pragma unroll
  for (int rr = 1; rr < PEER_MAX_RANKS; ++rr) b = (rr < ps.world && i >= ps.shard_begin[rr]) ? ps.base[rr] : b;
  return reinterpret_cast<float*>(b + PEER_DATA_OFF) + i;
}
__device__ __forceinline__ unsigned* ps_slice_ctr(const PsArgs& ps, int slice, int which) {
  // rank 0's flag area (unused by the parameter server's own kernels): 64-byte words
  return reinterpret_cast<unsigned*>(ps.base[0] + PEER_FLAG_OFF + (long long)which * PEER_MAX_BLOCKS * 64 +
                                     (long long)slice * 64);
}
__device__ __forceinline__ unsigned ps_ld_ctr(const unsigned* c) {
  return __hip_atomic_load(const_cast<unsigned*>(c), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// push bracket (asynchronous mode): writers of a slice never wait
__device__ __forceinline__ void ps_push_begin(const PersistArgs& a, int slice) {
  if (a.ps_mode == 2 && threadIdx.x == 0)
    __hip_atomic_fetch_add(ps_slice_ctr(a.ps, slice, 0), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
}
__device__ __forceinline__ void ps_push_end(const PersistArgs& a, int slice) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's atomics are done
  __syncthreads();
  if (a.ps_mode == 2 && threadIdx.x == 0)
    __hip_atomic_fetch_add(ps_slice_ctr(a.ps, slice, 1), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// pull: copy(); in asynchronous mode only while no writer is inside the slice (ended ==
// began before the copy, began unchanged after it), retried otherwise.  false: timed out
template <typename Copy>
__device__ __forceinline__ bool ps_pull(const PersistArgs& a, int slice, unsigned* sh, Copy copy) {
  if (a.ps_mode != 2) {
    copy();
    return true;
  }
  unsigned& snap_sh = sh[0];   // two words of the caller's LDS
  unsigned& state_sh = sh[1];
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    if (threadIdx.x == 0) {
      for (;;) {
        const unsigned e = ps_ld_ctr(ps_slice_ctr(a.ps, slice, 1));
        const unsigned b = ps_ld_ctr(ps_slice_ctr(a.ps, slice, 0));
        if (b == e) { snap_sh = b; break; }
        if ((long long)(wall_clock64() - t0) > a.timeout) { snap_sh = b; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    copy();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the copy's loads complete before the re-check
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned b2 = ps_ld_ctr(ps_slice_ctr(a.ps, slice, 0));
      const bool late = (long long)(wall_clock64() - t0) > a.timeout;
      state_sh = b2 == snap_sh ? 1 : (late ? 2 : 0);
      if (late && b2 != snap_sh)
        __hip_atomic_store((gu32*)(a.err), (unsigned)PERR_PS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (state_sh == 1) return true;
    if (state_sh == 2) return false;
  }
}

__device__ __forceinline__ float dropout_u1(uint32_t base, int row, int c) {
  // the per-column-pair hash of dropout_u8 (common.h): the row-chain / grouped masks
  const uint32_t h = fmix32(base ^ (((uint32_t)row << 16) | (uint32_t)(c >> 1)));
  return (float)((c & 1) ? (h >> 16) : (h & 0xFFFFu)) * (1.0f / 65536.0f);
}

// diagnostics (tools/persist_stamps.py): s_memrealtime of phase k of step i (i < PM_STAMP_STEPS)
__device__ __forceinline__ void pstamp(const PersistArgs& a, int i, int k) {
  if (a.stamps && threadIdx.x == 0 && i >= 0 && i < PM_STAMP_STEPS)
    a.stamps[((long long)blockIdx.x * PM_STAMP_STEPS + i) * 32 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void pcycle(const PersistArgs& a, int i, int k) {   // shader-clock stamp
  if (a.stamps && threadIdx.x == 0 && i >= 0 && i < PM_STAMP_STEPS)
    a.stamps[((long long)blockIdx.x * PM_STAMP_STEPS + i) * 32 + k] = (long long)__builtin_amdgcn_s_memtime();
}

// global (sc1) rows [0, nrows) x columns [0, ncols) of a row-major block (row stride ld,
// first element at uniform offset base) -> LDS tile (row stride lds).  ncols / 4 must
// divide 256.  Every load of the thread is issued before the first LDS write.
// Thread -> (row, float4 column) map of a 256-thread pass over rows of c4n float4s
__device__ __forceinline__ void pass_map(int c4n, int& row0, int& c4, int& rpp) {
  // row-major (a half-wave reads whole 512-byte rows): measured faster than a
  // bank-conflict-free quad-per-row map whose global reads span 4 rows per half-wave
  // (23.0 vs 20.9 us per step, profiles/persist_stamps_r3_*)
  const int t = threadIdx.x;
  row0 = t / c4n;
  c4 = t - row0 * c4n;
  rpp = 256 / c4n;
}

template <int NMAX>
__device__ __forceinline__ void stage(rsrc_t rs, int base, int ld, int nrows, int ncols, float* dst, int lds) {
  int row0, c4, rpp;
  pass_map(ncols >> 2, row0, c4, rpp);
  const int v = row0 * ld + 4 * c4;
  f32x4 x[NMAX];
  // branch-free loads (a row past nrows re-reads row 0; its value is not written): a
  // guarded load per element would split the issue into one basic block (and one
  // wait) per load
#pragma unroll
  for (int u = 0; u < NMAX; ++u) x[u] = ldw4(rs, row0 + u * rpp < nrows ? v : 4 * c4, base + u * rpp * ld);
#pragma unroll
  for (int u = 0; u < NMAX; ++u) {
    if (row0 + u * rpp < nrows) {
      float* d = dst + (row0 + u * rpp) * lds + 4 * c4;
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = x[u][q];
    }
  }
}

// stage() in two halves: issue the loads (registers), later commit them to LDS
template <int NMAX>
struct Staged {
  f32x4 x[NMAX];
  int row0, c4, rpp;
};
template <int NMAX>
__device__ __forceinline__ void stage_issue(Staged<NMAX>& st, rsrc_t rs, int base, int ld, int nrows, int ncols) {
  pass_map(ncols >> 2, st.row0, st.c4, st.rpp);
  const int v = st.row0 * ld + 4 * st.c4;
#pragma unroll
  for (int u = 0; u < NMAX; ++u) st.x[u] = ldw4(rs, st.row0 + u * st.rpp < nrows ? v : 4 * st.c4, base + u * st.rpp * ld);
}
template <int NMAX>
__device__ __forceinline__ void stage_commit(const Staged<NMAX>& st, int nrows, float* dst, int lds) {
#pragma unroll
  for (int u = 0; u < NMAX; ++u) {
    if (st.row0 + u * st.rpp < nrows) {
      float* d = dst + (st.row0 + u * st.rpp) * lds + 4 * st.c4;
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = st.x[u][q];
    }
  }
}

// 16 LDS rows (stride lds) of W floats -> global rows at uniform offset base (row
// stride W), as 16-byte write-through stores
template <int W>
__device__ __forceinline__ void publish_rows16(rsrc_t rs, int base, const float* src, int lds) {
  constexpr int C4 = W / 4, TOT = 16 * C4;
  int row0, c4, rpp;
  pass_map(C4, row0, c4, rpp);
#pragma unroll
  for (int u = 0; u < (TOT + 255) / 256; ++u) {
    if (row0 + u * rpp < 16) {
      const float* s = src + (row0 + u * rpp) * lds + 4 * c4;
      stw4(rs, row0 * W + 4 * c4, base + u * rpp * W, f32x4{s[0], s[1], s[2], s[3]});
    }
  }
}

// column sums of an LDS tile [64][ncols] (ncols <= 32) by all 256 threads: 8 row
// groups of independent loads, one barrier, then the first ncols threads add the 8
// partials (returned there).  Every thread must call it.
__device__ __forceinline__ float col_sums(const float* tile, int ld, int ncols, float* red) {
  const int tid = threadIdx.x, c = tid & 31, grp = tid >> 5;
  float s = 0.f;
  if (c < ncols) {
#pragma unroll
    for (int b = 0; b < 8; ++b) s += tile[(grp * 8 + b) * ld + c];
  }
  red[grp * 32 + c] = s;
  __syncthreads();
  float t = 0.f;
  if (tid < ncols) {
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q * 32 + tid];
  }
  return t;
}

// optimizer update of NV masters: NPT == 0 is plain SGD (no state planes, no rule
// dispatch); NPT < 0 dispatches on the rule at run time (common.h opt_update_v)
template <int NPT, int NV>
__device__ __forceinline__ void pm_update(const OptParams& op, float (&w)[NV], const float (&g)[NV], float (&s0)[NV],
                                          float (&s1)[NV], long long it) {
  if constexpr (NPT == 0) {
    const float lr = op.lr / (1.f + op.decay * (float)it);
#pragma unroll
    for (int q = 0; q < NV; ++q) w[q] -= lr * g[q];
  } else {
    opt_update_v<NV>(op, w, g, s0, s1, it);
  }
}

// hidden activation and its derivative: RELU compiles relu alone, else the run-time table
template <bool RELU, int NV>
__device__ __forceinline__ void pm_act(int act, const float (&z)[NV], float (&o)[NV], float (&g)[NV]) {
  if constexpr (RELU) {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      o[q] = fmaxf(z[q], 0.f);
      g[q] = z[q] > 0.f ? 1.f : 0.f;
    }
  } else {
    act_fg_v<NV>(act, z, o, g);
  }
}

// prologue copy of n consecutive floats of P into LDS (element e -> dst[map(e)]): 16
// loads per thread in flight per batch (a loop of dependent load -> store pairs took
// one memory latency per element group and dominated the launch's fill)
template <typename Map>
__device__ __forceinline__ void p_to_lds(const float* src, int n, float* dst, Map map) {
  for (int base = 0; base < n; base += 16 * 256) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = base + threadIdx.x + 256 * u;
      v[u] = src[e < n ? e : 0];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = base + threadIdx.x + 256 * u;
      if (e < n) dst[map(e)] = v[u];
    }
  }
}

struct Steps {
  long long s0;
  int ntr;
  __device__ __forceinline__ int valid(const PersistArgs& a, int i) const {
    const long long c = (long long)ntr - (s0 + i) * a.B;
    return (int)(c < 0 ? 0 : (c > a.B ? a.B : c));
  }
};

// ============================================================== layer-0 tiles
template <int H0, int NPT, bool PS>
__device__ __forceinline__ void l0_role(const PersistArgs& a, float* smem, int r, int kc, int cb, int q) {
  constexpr int XS = 129;                       // X chunk rows (<= 128 columns)
  const int tid = threadIdx.x, lane = tid & 63, i16 = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6) & 3;
  const int k0 = kc * a.kc0;
  const int kreal = a.K0 - k0 < a.kc0 ? a.K0 - k0 : a.kc0;
  const int KCP = (kreal + 63) & ~63;           // FWD reduction, zero padded to 64
  const int cw = a.cw, n0 = cb * cw;
  const int nct = cw >> 4, nrt = (kreal + 15) >> 4, ntiles = nrt * nct;
  const int WS = cw + 1;
  const int BR = a.nch * 16;                    // rows the chain workgroups produce
  float* sX = smem;                             // [2][64][XS] X chunks of two steps
  float* sW = sX + 2 * 64 * XS;                 // [128][WS]  the W0 tile (master, in place)
  float* sdZ = sW + 128 * WS;                   // [64][WS]   dZ_0 columns of this tile
  float* sWp = sdZ + 64 * 33;                   // [128][WS]  parameter-server hook: the tile as pulled
  __shared__ float sB0[32];
  __shared__ float sRedL[256];
  const rsrc_t rs = ws_rsrc(a.ws + (long long)r * a.ws_stride);
  float* P = a.P + (long long)r * a.sP;
  float* S = a.S ? a.S + (long long)r * a.sS : nullptr;
  const int np = NPT >= 0 ? NPT : (S ? opt_planes(a.op) : 0);
  const bool has_b = kc == 0 && a.bias0;
  Steps st{ld_inv(a.ctr), ld_inv(a.ntrain + r)};

  // ---- prologue: zero LDS (padding rows / columns stay zero), W0 tile and state
  for (int e = tid; e < L0_LDS; e += 256) smem[e] = 0.f;
  __syncthreads();
  // the W0 tile: kreal rows of cw floats (row stride H0 in P)
  for (int base = 0; base < kreal * cw; base += 16 * 256) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = base + tid + 256 * u, el = e < kreal * cw ? e : 0;
      const int k = el / cw, n = el - k * cw;
      v[u] = P[a.p_off0 + (long long)(k0 + k) * H0 + n0 + n];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = base + tid + 256 * u;
      if (e < kreal * cw) sW[(e / cw) * WS + (e % cw)] = v[u];
    }
  }
  int rt[TU], ct[TU];
  float s0[TU * 4], s1[TU * 4];
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int t = w + 4 * u;
    rt[u] = t < ntiles ? t / nct : 0;
    ct[u] = t < ntiles ? t - rt[u] * nct : 0;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int k = rt[u] * 16 + 4 * g + qq, n = ct[u] * 16 + i16;
      const bool in = t < ntiles && k < kreal;
      const long long pi = a.p_off0 + (long long)(k0 + k) * H0 + n0 + n;
      s0[4 * u + qq] = (in && np > 0) ? S[pi] : 0.f;
      s1[4 * u + qq] = (in && np > 1) ? S[a.op.s_plane + pi] : 0.f;
    }
  }
  float bw = 0.f, bs0 = 0.f, bs1 = 0.f;   // bias master / state (kc == 0, thread tid < cw)
  const bool bown = has_b && tid < cw;
  if (bown) {
    const long long pi = a.p_off0 + (long long)a.K0 * H0 + n0 + tid;
    bw = P[pi];
    bs0 = np > 0 ? S[pi] : 0.f;
    bs1 = np > 1 ? S[a.op.s_plane + pi] : 0.f;
  }
  if (tid < 32) sB0[tid] = 0.f;
  __syncthreads();
  if (bown) sB0[tid] = bw;
  float bwp = bw;   // parameter-server hook: b0 as pulled
  if constexpr (PS) {
    for (int e = tid; e < 128 * WS; e += 256) sWp[e] = sW[e];
  }
  // parameter-server hook: the tile's flat parameter indices
  auto w0_index = [&](int e) -> long long {
    const int k = e / cw, nn = e - k * cw;
    return a.p_off0 + (long long)(k0 + k) * H0 + n0 + nn;
  };

  // X chunk of step i into sX buffer (i & 1): LDS-DMA, one 64-column row segment per
  // wave instruction (rows past the valid batch repeat its first row: finite values
  // whose dZ_0 rows are zero)
  auto load_x = [&](int i) {
    const int valid = st.valid(a, i);
    const int* pr = a.perm + (long long)r * a.sPerm + (st.s0 + i) * a.B;
    const float* Xr = a.X + (long long)r * a.sX + k0;
    float* dst = sX + (i & 1) * 64 * XS;
    const int myrow = pr[lane < valid ? lane : 0];   // lane b holds batch row b's data row
    for (int v = 0; v < 16; ++v) {
      const int b = w + 4 * v;
      if (b >= BR) break;
      const int row = __builtin_amdgcn_readlane(myrow, b);
      const float* src = Xr + (long long)row * a.ldx;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (64 * h + lane < kreal) __builtin_amdgcn_global_load_lds(src + 64 * h + lane, dst + b * XS + 64 * h, 4, 0, 0);
    }
  };

  // split-K partial of step i's layer-0 pre-activations for this tile -> workspace
  const int part_base = (int)a.o_part + kc * 64 * H0 + n0;
  auto fwd = [&](int i) {
    const float* A = sX + (i & 1) * 64 * XS;
    if (w * 16 < BR) {
      f32x4 acc[2] = {zero4f(), zero4f()};
      const float* arow = A + (w * 16 + i16) * XS;
#pragma unroll 1
      for (int kb = 0; kb < KCP; kb += 64) {
        float av[16], bv0[16], bv1[16];
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
          const int k = kb + 16 * g + ks;
          av[ks] = arow[k];
          bv0[ks] = sW[k * WS + i16];
          bv1[ks] = sW[k * WS + 16 + i16];   // cw = 16: garbage, never stored
        }
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
          acc[0] = mma(av[ks], bv0[ks], acc[0]);
          acc[1] = mma(av[ks], bv1[ks], acc[1]);
        }
      }
      pstamp(a, i, 10);
      const int v = (w * 16 + 4 * g) * H0 + i16;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        if (jj < nct) {
          const float bv = has_b ? sB0[jj * 16 + i16] : 0.f;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) stw1(rs, v + qq * H0 + jj * 16, part_base, acc[jj][qq] + bv);
        }
      }
    }
    publish(flag_at(a, r, PMF_PART) + q, (unsigned)(i + 1));
    pstamp(a, i, 1);
  };

  const int n = a.nsteps;
  pstamp(a, 0, 0);
  if (st.valid(a, 0) > 0) {
    load_x(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    fwd(0);
  }
  for (int i = 0; i < n; ++i) {
    if (st.valid(a, i) == 0) break;
    const bool nxt = i + 1 < n && st.valid(a, i + 1) > 0;
    if (nxt) load_x(i + 1);
    pstamp(a, i, 2);
    if (!wait_all(a, flag_at(a, r, PMF_BWD), a.nch, (unsigned)(i + 1), 1u)) return;
    pstamp(a, i, 3);
    stage<2>(rs, (int)a.o_dz0 + n0, H0, BR, cw, sdZ, WS);   // dZ_0 columns of this tile
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // the X DMA and the dZ_0 loads
    __syncthreads();
    pstamp(a, i, 4);
    // DW0 tile = X_i^T dZ_0 (reduction over the 64 batch rows), update in place
    {
      const float* Xi = sX + (i & 1) * 64 * XS;
      f32x4 dw[TU];
#pragma unroll
      for (int u = 0; u < TU; ++u) dw[u] = zero4f();
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        float xa[TU][8], zb[2][8];
#pragma unroll
        for (int h8 = 0; h8 < 8; ++h8) {
          const int b = 16 * g + 8 * half + h8;
          zb[0][h8] = sdZ[b * WS + i16];
          zb[1][h8] = sdZ[b * WS + 16 + i16];   // cw = 16: garbage, never used
#pragma unroll
          for (int u = 0; u < TU; ++u) xa[u][h8] = Xi[b * XS + rt[u] * 16 + i16];   // rt = 0 past the tiles
        }
        // branch-free: tiles past ntiles compute garbage that is never stored
#pragma unroll
        for (int h8 = 0; h8 < 8; ++h8) {
#pragma unroll
          for (int u = 0; u < TU; ++u) dw[u] = mma(xa[u][h8], ct[u] ? zb[1][h8] : zb[0][h8], dw[u]);
        }
      }
      pstamp(a, i, 7);
      // bias gradient (first k-chunk): column sums of dZ_0 over the batch rows
      float gsum = has_b ? col_sums(sdZ, WS, cw, sRedL) : 0.f;
      if (a.sync) {   // per-step synchronous DP: the R replicas' tiles summed, same bits everywhere
        f32x4 xv[TU + 1];
#pragma unroll
        for (int u = 0; u < TU; ++u) xv[u] = dw[u];
        xv[TU] = f32x4{gsum, 0.f, 0.f, 0.f};
        if (!xchg_sum<TU + 1>(a, r, q, i, xv)) return;
#pragma unroll
        for (int u = 0; u < TU; ++u) dw[u] = xv[u];
        gsum = xv[TU][0];
      }
      pstamp(a, i, 8);
      const long long it = iter_at(a.ctr, a.ntrain, a.B, r, st.s0, i);
      float wv[TU * 4], gv[TU * 4];
#pragma unroll
      for (int u = 0; u < TU; ++u) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int k = rt[u] * 16 + 4 * g + qq;
          wv[4 * u + qq] = sW[k * WS + ct[u] * 16 + i16];
          gv[4 * u + qq] = dw[u][qq] * a.op.grad_scale;
        }
      }
      pm_update<NPT, TU * 4>(a.op, wv, gv, s0, s1, it);
      pstamp(a, i, 9);
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        if (w + 4 * u >= ntiles) continue;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int k = rt[u] * 16 + 4 * g + qq;
          if (k < kreal) sW[k * WS + ct[u] * 16 + i16] = wv[4 * u + qq];
        }
      }
      if (bown) {
        float bv[1] = {bw}, bg[1] = {gsum * a.op.grad_scale}, t0[1] = {bs0}, t1[1] = {bs1};
        pm_update<NPT, 1>(a.op, bv, bg, t0, t1, it);
        bw = bv[0];
        bs0 = t0[0];
        bs1 = t1[0];
        sB0[tid] = bw;
      }
    }
    __syncthreads();
    if constexpr (PS) {
      // reference worker.py:114-127 per batch: push theta_new - theta_pulled of this tile
      // (and b0), then pull the tile of theta for the next step
      ps_push_begin(a, q);
      for (int e = tid; e < kreal * cw; e += 256) {
        const int k = e / cw, nn = e - k * cw;
        const float dlt = sW[k * WS + nn] - sWp[k * WS + nn];
        if (dlt != 0.f) __hip_atomic_fetch_add(ps_elem(a.ps, w0_index(e)), dlt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (bown && bw != bwp)
        __hip_atomic_fetch_add(ps_elem(a.ps, a.p_off0 + (long long)a.K0 * H0 + n0 + tid), bw - bwp, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
      ps_push_end(a, q);
      if (nxt) {
        const bool ok = ps_pull(a, q, reinterpret_cast<unsigned*>(sRedL), [&]() {
          for (int base = 0; base < kreal * cw; base += 8 * 256) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int e = base + tid + 256 * u;
              v[u] = *ps_elem(a.ps, w0_index(e < kreal * cw ? e : 0));
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int e = base + tid + 256 * u;
              if (e < kreal * cw) {
                const int k = e / cw, nn = e - k * cw;
                sW[k * WS + nn] = v[u];
                sWp[k * WS + nn] = v[u];
              }
            }
          }
          if (bown) {
            bw = *ps_elem(a.ps, a.p_off0 + (long long)a.K0 * H0 + n0 + tid);
            bwp = bw;
          }
        });
        if (!ok) return;
        if (bown) sB0[tid] = bw;
        __syncthreads();
      }
    }
    pstamp(a, i, 5);
    if (nxt) fwd(i + 1);
    pstamp(a, i, 6);
  }

  // ---- epilogue: master tile, both weight-image parities, optimizer state
  __syncthreads();
  float* Wsh = a.Wsh + (long long)r * a.sWsh + a.wsh_off[0];
  float* WTsh = a.WTsh + (long long)r * a.sWTsh + a.wtsh_off[0];
  for (int e = tid; e < kreal * cw; e += 256) {
    const int k = e / cw, nn = e - k * cw;
    const float v = sW[k * WS + nn];
    pst(a, P + (a.p_off0 + (long long)(k0 + k) * H0 + n0 + nn), v);
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      Wsh[par * a.wsh_par + (long long)(k0 + k) * a.Np[0] + n0 + nn] = v;
      WTsh[par * a.wtsh_par + (long long)(n0 + nn) * a.Kp[0] + k0 + k] = v;
    }
  }
  if (np > 0) {
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      if (w + 4 * u >= ntiles) continue;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int k = rt[u] * 16 + 4 * g + qq, nn = ct[u] * 16 + i16;
        if (k >= kreal) continue;
        const long long pi = a.p_off0 + (long long)(k0 + k) * H0 + n0 + nn;
        S[pi] = s0[4 * u + qq];
        if (np > 1) S[a.op.s_plane + pi] = s1[4 * u + qq];
      }
    }
  }
  if (bown) {
    const long long pi = a.p_off0 + (long long)a.K0 * H0 + n0 + tid;
    pst(a, P + (pi), bw);
    if (np > 0) S[pi] = bs0;
    if (np > 1) S[a.op.s_plane + pi] = bs1;
  }
}

// ============================================================== V2: layer-0 tiles
// Plain SGD, fit granularity.  W0_s = W0_{s-2} - lr_{s-1} gs X_{s-1}^T dZ0_{s-1} (and
// b0 likewise with the column sums of dZ0_{s-1}), so
//   Z0_s = X_s W0_{s-2} + b0_{s-2}  -  lr_{s-1} gs (X_s X_{s-1}^T + 1) dZ0_{s-1}.
// The workgroup publishes, two steps ahead of use, Pold_s = its k-chunk's share of the
// first product (+ b0 on k-chunk 0) and its slice of the Gram block X_s X_{s-1}^T (this
// k-chunk, rows cb * 64 / nc0 ...); the chain workgroups add the correction with the
// dZ0_{s-1} rows they hand to each other.  dZ0 reaches this workgroup only for the
// update of its tile (DW0 = X^T dZ0), which is off the step's critical path.
// Step 0 is the direct product; buffers of step s live in parity s & 1.
template <int H0, int NCT, bool BF>
__device__ __forceinline__ void l0_role_v2(const PersistArgs& a, float* smem, int r, int kc, int cb, int q) {
  static_assert(NCT == 2 || NCT == 4, "column blocks of 32 or 64");
  // X rows in LDS: fp32 (stride kc0 + 1 floats), or bf16 packed two per dword (stride
  // kc0 / 2 + 1 dwords); three chunks (steps s % 3), kc0 <= 112 (host)
  constexpr int CW = NCT * 16, WS = CW + 1, TU0 = 2 * NCT;   // DW0 tiles per wave (<= 8 row tiles)
  const int XS = BF ? a.kc0 / 2 + 1 : a.kc0 + 1;
  auto xat = [](const float* row, int k) -> float { if constexpr (BF) return bf_at(row, k); else return row[k]; };
  const int tid = threadIdx.x, lane = tid & 63, i16 = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6) & 3;
  const int k0 = kc * a.kc0;
  const int kreal = a.K0 - k0 < a.kc0 ? a.K0 - k0 : a.kc0;
  const int KCP = (kreal + 63) & ~63;           // reductions over the k-chunk, zero padded to 64
  const int n0 = cb * CW;
  const int nrt = (kreal + 15) >> 4, ntiles = nrt * NCT;
  const int BR = a.nch * 16;
  float* sX = smem;                             // [3][64][XS] X chunks of steps s % 3
  float* sW = sX + 3 * 64 * XS;                 // [128][WS]   the W0 tile (master, in place)
  float* sdZ = sW + 128 * WS;                   // [64][WS]    dZ_0 columns of this tile
  float* sT = sW + 128 * 65 + 64 * 65;          // [64][65]    staging of the Pold / Gram slabs (16-byte stores)
  __shared__ float sB0[64];
  __shared__ float sBg[64];
  __shared__ float sRedL[256];
  const rsrc_t rs = ws_rsrc(a.ws + (long long)r * a.ws_stride);
  float* P = a.P + (long long)r * a.sP;
  const bool has_b = kc == 0 && a.bias0;
  Steps st{ld_inv(a.ctr), ld_inv(a.ntrain + r)};

  for (int e = tid; e < L0V2_LDS; e += 256) smem[e] = 0.f;
  __syncthreads();
  for (int base = 0; base < kreal * CW; base += 16 * 256) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = base + tid + 256 * u, el = e < kreal * CW ? e : 0;
      const int k = el / CW, nn = el - k * CW;
      v[u] = P[a.p_off0 + (long long)(k0 + k) * H0 + n0 + nn];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = base + tid + 256 * u;
      if (e < kreal * CW) sW[(e / CW) * WS + (e % CW)] = v[u];
    }
  }
  int rt[TU0], ct[TU0];
#pragma unroll
  for (int u = 0; u < TU0; ++u) {
    const int t = w + 4 * u;
    rt[u] = t < ntiles ? t / NCT : 0;
    ct[u] = t < ntiles ? t - rt[u] * NCT : 0;
  }
  float bw = 0.f;
  const bool bown = has_b && tid < CW;
  if (bown) bw = P[a.p_off0 + (long long)a.K0 * H0 + n0 + tid];
  if (tid < 64) sB0[tid] = 0.f;
  __syncthreads();
  if (bown) sB0[tid] = bw;

  auto load_x = [&](int i) {   // as l0_role: LDS-DMA of step i's X chunk into buffer i & 1
    const int valid = st.valid(a, i);
    const int* pr = a.perm + (long long)r * a.sPerm + (st.s0 + i) * a.B;
    const float* Xr = a.X + (long long)r * a.sX + k0;
    float* dst = sX + (i % 3) * 64 * XS;
    const int myrow = pr[lane < valid ? lane : 0];
    for (int v = 0; v < 16; ++v) {
      const int b = w + 4 * v;
      if (b >= BR) break;
      const int row = __builtin_amdgcn_readlane(myrow, b);
      if constexpr (BF) {   // bf16 shard: one dword (two elements) per lane, <= 128 elements per row
        const float* src = reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(a.X) +
                                                          (long long)r * a.sX + (long long)row * a.ldx + k0);
        if (lane < (kreal + 1) / 2) __builtin_amdgcn_global_load_lds(src + lane, dst + b * XS, 4, 0, 0);
      } else {
        const float* src = Xr + (long long)row * a.ldx;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (64 * h + lane < kreal) __builtin_amdgcn_global_load_lds(src + 64 * h + lane, dst + b * XS + 64 * h, 4, 0, 0);
      }
    }
  };

  // X_i . W0 tile (+ b0 on k-chunk 0) -> partial slab of step i (parity i & 1)
  auto fwd = [&](int i) {
    const float* A = sX + (i % 3) * 64 * XS;
    if (w * 16 < BR) {
      f32x4 acc[NCT];
#pragma unroll
      for (int jj = 0; jj < NCT; ++jj) acc[jj] = zero4f();
      const float* arow = A + (w * 16 + i16) * XS;
      if constexpr (BF) {
        // bf16 X rows straight into v_mfma_f32_16x16x32_bf16 (lane: elements kb + 8g + j,
        // four packed dwords, masked past the chunk), the W0 tile rounded to bf16
        const unsigned* au = reinterpret_cast<const unsigned*>(arow);
#pragma unroll 1
        for (int kb = 0; kb < KCP; kb += 32) {
          const int d0 = (kb + 8 * g) >> 1;
          u32x4 aq;
#pragma unroll
          for (int e = 0; e < 4; ++e) aq[e] = 2 * (d0 + e) < kreal ? au[d0 + e] : 0u;
          const bf16x8 a8 = __builtin_bit_cast(bf16x8, aq);
#pragma unroll
          for (int jj = 0; jj < NCT; ++jj) {
            float bv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) bv[j] = sW[(kb + 8 * g + j) * WS + jj * 16 + i16];
            acc[jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, bf8(bv), acc[jj], 0, 0, 0);
          }
        }
      } else {
#pragma unroll 1
        for (int kb = 0; kb < KCP; kb += 64) {
          float av[16], bv[NCT][16];
#pragma unroll
          for (int ks = 0; ks < 16; ++ks) {
            const int k = kb + 16 * g + ks;
            // rows are kc0 + 1 wide: k past the chunk reads the next row -- masked to zero
            av[ks] = k < kreal ? xat(arow, k) : 0.f;
#pragma unroll
            for (int jj = 0; jj < NCT; ++jj) bv[jj][ks] = sW[k * WS + jj * 16 + i16];
          }
#pragma unroll
          for (int ks = 0; ks < 16; ++ks) {
#pragma unroll
            for (int jj = 0; jj < NCT; ++jj) acc[jj] = mma(av[ks], bv[jj][ks], acc[jj]);
          }
        }
      }
#pragma unroll
      for (int jj = 0; jj < NCT; ++jj) {
        const float bv = has_b ? sB0[jj * 16 + i16] : 0.f;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) sT[(w * 16 + 4 * g + qq) * 65 + jj * 16 + i16] = acc[jj][qq] + bv;
      }
    }
    __syncthreads();
    // the slab leaves as 16-byte write-through row segments (4-byte sc1 stores cost ~6x
    // per byte: MI355X_MICROARCH.md price list)
    const int base = (int)(a.o_part + (i & 1) * a.part_par) + kc * 64 * H0 + n0;
    for (int e = tid; e < BR * (CW / 4); e += 256) {
      const int row = e / (CW / 4), c4 = e - row * (CW / 4);
      const float* src = sT + row * 65 + 4 * c4;
      stw4(rs, row * H0 + 4 * c4, base, f32x4{src[0], src[1], src[2], src[3]});
    }
    __syncthreads();
  };

  // rows [cb * 64 / nc0, (cb + 1) * 64 / nc0) of this k-chunk's X_i . X_{i-1}^T -> Gram
  // slab of step i (parity i & 1)
  auto gram = [&](int i) {
    const float* A = sX + (i % 3) * 64 * XS;
    const float* Bm = sX + ((i - 1) % 3) * 64 * XS;
    const int rows = 64 / a.nc0, r0 = cb * rows;
    const int ntg = (rows >> 4) * 4;   // 16 x 16 tiles of the slice (4 column tiles of 16)
    const int base = (int)(a.o_g + (i % 3) * a.g_par) + kc * 64 * 64;   // three Gram slabs (written a step early)
#pragma unroll 1
    for (int t = w; t < ntg; t += 4) {
      const int tr = t >> 2, tc = t & 3;
      f32x4 acc = zero4f();
      const float* arow = A + (r0 + tr * 16 + i16) * XS;
      const float* brow = Bm + (tc * 16 + i16) * XS;
#pragma unroll 1
      for (int kb = 0; kb < KCP; kb += 64) {
        float av[16], bv[16];
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
          const int k = kb + 16 * g + ks;
          av[ks] = k < kreal ? xat(arow, k) : 0.f;   // (finite X past the chunk) x 0
          bv[ks] = xat(brow, k);
        }
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) acc = mma(av[ks], bv[ks], acc);
      }
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) sT[(tr * 16 + 4 * g + qq) * 65 + tc * 16 + i16] = acc[qq];
    }
    __syncthreads();
    for (int e = tid; e < rows * 16; e += 256) {
      const int row = e >> 4, c4 = e & 15;
      const float* src = sT + row * 65 + 4 * c4;
      stw4(rs, (r0 + row) * 64 + 4 * c4, base, f32x4{src[0], src[1], src[2], src[3]});
    }
    __syncthreads();
  };

  const int n = a.nsteps;
  pstamp(a, 0, 0);
  const bool v0 = st.valid(a, 0) > 0, v1 = n > 1 && st.valid(a, 1) > 0;
  if (v0) load_x(0);
  if (v1) load_x(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (v0) {
    fwd(0);
    publish(flag_at(a, r, PMF_PART) + q, 1u);
  }
  if (v1) {
    fwd(1);
    if (a.ng == 0) gram(1);
    publish(flag_at(a, r, PMF_PART) + q, 2u);
  }
  if (n > 2 && st.valid(a, 2) > 0) load_x(2);   // in flight until iteration 0 needs it
  pstamp(a, 0, 1);
  for (int i = 0; i < n; ++i) {
    if (st.valid(a, i) == 0) break;
    // step i + 2's X chunk and its Gram slice depend on no hand-off: done while the
    // chains still run step i (the X chunk goes to buffer (i + 2) % 3, which X_{i-1} left)
    const bool ahead = i + 2 < n && st.valid(a, i + 2) > 0;
    if (ahead && a.ng == 0) {   // X_{i+2} was issued at the end of the previous iteration (or the prologue)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      pstamp(a, i, 9);
      gram(i + 2);
      pstamp(a, i, 10);
    }
    pstamp(a, i, 2);
    if (!wait_all(a, flag_at(a, r, PMF_BWD), a.nch, (unsigned)(i + 1), PERR_L0_BWD)) return;
    pstamp(a, i, 3);
    stage<NCT>(rs, (int)(a.o_dz0 + (i & 1) * a.dz0_par) + n0, H0, BR, CW, sdZ, WS);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (BF) {   // the weight gradient's dZ_0 operand (and the bias sums) in bf16
      for (int e = tid; e < 64 * WS; e += 256) sdZ[e] = rb<true>(sdZ[e]);
      __syncthreads();
    }
    pstamp(a, i, 4);
    // DW0 tile = X_i^T dZ_0 (reduction over the batch rows), SGD update in place
    {
      const float* Xi = sX + (i % 3) * 64 * XS;
      f32x4 dw[TU0];
#pragma unroll
      for (int u = 0; u < TU0; ++u) dw[u] = zero4f();
      // tile t = w + 4u: its column tile is w % NCT for every u (NCT divides 4)
      const int ctw = w % NCT;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        float xa[TU0][8], zb[8];
#pragma unroll
        for (int h8 = 0; h8 < 8; ++h8) {
          const int b = 16 * g + 8 * half + h8;
          zb[h8] = sdZ[b * WS + ctw * 16 + i16];
#pragma unroll
          for (int u = 0; u < TU0; ++u) xa[u][h8] = xat(Xi + b * XS, rt[u] * 16 + i16);
        }
        // branch-free: tiles past ntiles compute garbage that is never stored
#pragma unroll
        for (int h8 = 0; h8 < 8; ++h8) {
#pragma unroll
          for (int u = 0; u < TU0; ++u) dw[u] = mma(xa[u][h8], zb[h8], dw[u]);
        }
      }
      pstamp(a, i, 7);
      if (has_b) {   // bias gradient: column sums of dZ_0, 32 columns per pass
#pragma unroll
        for (int hc = 0; hc < (CW + 31) / 32; ++hc) {
          const float t = col_sums(sdZ + 32 * hc, WS, 32, sRedL);
          if (tid < 32) sBg[hc * 32 + tid] = t;
          __syncthreads();
        }
      }
      pstamp(a, i, 8);
      // the plain-SGD rule of pm_update<0>, in the same operation order
      const long long it = iter_at(a.ctr, a.ntrain, a.B, r, st.s0, i);
      const float lr = a.op.lr / (1.f + a.op.decay * (float)it), gs = a.op.grad_scale;
#pragma unroll
      for (int u = 0; u < TU0; ++u) {
        if (w + 4 * u >= ntiles) continue;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int k = rt[u] * 16 + 4 * g + qq;
          if (k < kreal) sW[k * WS + ct[u] * 16 + i16] -= lr * (dw[u][qq] * gs);
        }
      }
      if (bown) {
        bw -= lr * (sBg[tid] * gs);
        sB0[tid] = bw;
      }
    }
    __syncthreads();
    pstamp(a, i, 5);
    // step i + 2's Pold = X_{i+2} . W0 after step i (ng == 0: PART covers the Gram slab too)
    if (ahead) {
      fwd(i + 2);
      publish(flag_at(a, r, PMF_PART) + q, (unsigned)(i + 3));
    }
    pstamp(a, i, 6);
    // X_{i+3} into the buffer X_i just left, after the Pold MFMAs: an LDS-DMA in flight
    // makes the compiler wait for it before every later LDS access (measured: issued
    // before fwd, the Pold phase took 6.9 instead of 3.7 us)
    if (i + 3 < n && st.valid(a, i + 3) > 0) load_x(i + 3);
  }

  // ---- epilogue: master tile and both weight-image parities (plain SGD: no state)
  __syncthreads();
  float* Wsh = img_base<BF>(a.Wsh, (long long)r * a.sWsh + a.wsh_off[0]);
  float* WTsh = img_base<BF>(a.WTsh, (long long)r * a.sWTsh + a.wtsh_off[0]);
  for (int e = tid; e < kreal * CW; e += 256) {
    const int k = e / CW, nn = e - k * CW;
    const float v = sW[k * WS + nn];
    pst(a, P + (a.p_off0 + (long long)(k0 + k) * H0 + n0 + nn), v);
    if (a.imgs) {
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        img_store<BF>(Wsh, par * a.wsh_par + (long long)(k0 + k) * a.Np[0] + n0 + nn, v);
        img_store<BF>(WTsh, par * a.wtsh_par + (long long)(n0 + nn) * a.Kp[0] + k0 + k, v);
      }
    }
  }
  if (bown) pst(a, P + (a.p_off0 + (long long)a.K0 * H0 + n0 + tid), bw);
}

// ============================================================== chain (rows)
// acc[jj] (jj < 2: column tiles ct0 + 4jj) += A[16][K] . B[K][16 cols], fragments from
// LDS: A(i, k) = A[i * SAI + k], B(k, n) = B[k * SBK + n * SBN]; the 16 fragments of a
// 64-deep block are read before its MFMAs
template <int K, int SAI, int SBK, int SBN, bool BF = false>
__device__ __forceinline__ void rows_mm(const float* A, const float* B, int ct0, int nct, f32x4 (&acc)[2], int i16,
                                        int g) {
  acc[0] = zero4f();
  acc[1] = zero4f();
  if (ct0 >= nct) return;
  const bool two = ct0 + 4 < nct;
  const float* arow = A + i16 * SAI;
  const float* b0 = B + (ct0 * 16 + i16) * SBN;
  const float* b1 = two ? B + ((ct0 + 4) * 16 + i16) * SBN : b0;   // branch-free: acc[1] then unused
#pragma unroll
  for (int kb = 0; kb < K; kb += 64) {
    float av[16], bv0[16], bv1[16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int k = kb + 16 * g + ks;
      av[ks] = rb<BF>(arow[k]);
      bv0[ks] = rb<BF>(b0[k * SBK]);
      bv1[ks] = rb<BF>(b1[k * SBK]);
    }
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      acc[0] = mma(av[ks], bv0[ks], acc[0]);
      acc[1] = mma(av[ks], bv1[ks], acc[1]);
    }
  }
}

// rows_mm on the bf16 matrix cores (mixed_bfloat16 policy): the same bf16-rounded
// operands, one v_mfma_f32_16x16x32_bf16 per 32-deep block instead of eight
// 16x16x4 f32 MFMAs (lane: k = kb + 8g + j, j < 8)
template <int K, int SAI, int SBK, int SBN>
__device__ __forceinline__ void rows_mm_b(const float* A, const float* B, int ct0, int nct, f32x4 (&acc)[2], int i16,
                                          int g) {
  static_assert(K % 32 == 0, "32-deep blocks");
  acc[0] = zero4f();
  acc[1] = zero4f();
  if (ct0 >= nct) return;
  const bool two = ct0 + 4 < nct;
  const float* arow = A + i16 * SAI;
  const float* b0 = B + (ct0 * 16 + i16) * SBN;
  const float* b1 = two ? B + ((ct0 + 4) * 16 + i16) * SBN : b0;
#pragma unroll
  for (int kb = 0; kb < K; kb += 32) {
    float av[8], bv0[8], bv1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kb + 8 * g + j;
      av[j] = arow[k];
      bv0[j] = b0[k * SBK];
      bv1[j] = b1[k * SBK];
    }
    const bf16x8 a8 = bf8(av);
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, bf8(bv0), acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, bf8(bv1), acc[1], 0, 0, 0);
  }
}

// V2 (plain SGD + ReLU, fit granularity): the weight gradients leave this role (dw_role_v2
// owns W1 / W2), the layer-0 pre-activations of step i >= 1 are rebuilt from the L0
// workgroups' Pold / Gram slabs and the previous step's dZ_0 rows of every chain
// workgroup (l0_role_v2), and two more flags (A0, D2) hand the rows the DW workgroups need.
template <int H0, int H1, bool FAST, int NPT, bool RELU, bool V2, bool PS, bool BF = false>
__device__ __forceinline__ void chain_role(const PersistArgs& a, float* smem, int r, int j) {
  using Lo = ChainLds<H0, H1>;
  constexpr int L0S = Lo::L0S, L1S = Lo::L1S;
  constexpr int nt0 = H0 / 16, nt1 = H1 / 16;
  const int tid = threadIdx.x, lane = tid & 63, i16 = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6) & 3;
  const int m0 = j * 16;
  const int C = a.C;
  const int BR = a.nch * 16;
  const int nl0 = a.nk0 * a.nc0;
  float* sW1 = smem;                 // [H0][L1S] W1 (k = layer-1 input, n = unit)
  float* sW2 = smem + Lo::o_w2;      // [H1][17]
  float* sA0 = smem + Lo::o_a0;      // [16][L0S] layer-0 activations (A of FWD1)
  float* sG0 = smem + Lo::o_g0;      // [16][L0S] act'(z_0) * keep / (1 - rate)
  float* sZ0 = smem + Lo::o_z0;      // [16][L0S] dZ_0 rows
  float* sA1 = smem + Lo::o_a1;      // [16][L1S] layer-1 activations
  float* sD1 = smem + Lo::o_d1;      // [16][L1S] dZ_1 (A of DX1)
  float* sD2 = smem + Lo::o_d2;      // [16][17] dZ_2
  float* sRed = smem + Lo::o_red;    // [4][256] split-K partials / column-sum partials
  float* sLg = smem + Lo::o_lg;      // [16][36] logits -> dZ_2
  float* sY = smem + Lo::o_y;        // [16][32] targets
  float* sB1 = smem + Lo::o_b1;      // [H1]
  float* sB2 = smem + Lo::o_b2;      // [16]
  int* sRow = reinterpret_cast<int*>(smem + Lo::o_row);
  // weight-gradient staging, over the W1 region (dead between DX1 and the W1 reload)
  float* uA0 = sW1;                  // [64][L0S] layer-0 activations of every row
  float* uD1 = uA0 + 64 * L0S;       // [64][33] dZ_1 of the owned layer-1 columns
  float* uA1 = uD1 + 64 * 33;        // [64][33] layer-1 activations of the owned W2 rows
  float* uD2 = uA1 + 64 * 33;        // [64][17] dZ_2

  const rsrc_t rs = ws_rsrc(a.ws + (long long)r * a.ws_stride);
  float* P = a.P + (long long)r * a.sP;
  float* S = a.S ? a.S + (long long)r * a.sS : nullptr;
  const int np = NPT >= 0 ? NPT : (S ? opt_planes(a.op) : 0);
  Steps st{ld_inv(a.ctr), ld_inv(a.ntrain + r)};

  // owned tiles: layer-1 column tiles j + nch*c (c < nown) = layer-2 row tiles
  const int nown = (nt1 - j + a.nch - 1) / a.nch;   // <= PM_NTU (host checks)
  const int ndw1 = nt0 * nown;                      // DW1 tiles (row tile x owned col tile)
  int urt[TU], uct[TU];                             // wave w's DW1 tiles t = w + 4u (row 0 past ndw1)
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int t = w + 4 * u;
    urt[u] = t < ndw1 ? t / nown : 0;
    uct[u] = t < ndw1 ? t - (t / nown) * nown : 0;
  }

  // ---- prologue: W1, W2, biases into LDS; owned masters / state into registers
  for (int e = tid; e < Lo::TOTAL; e += 256) smem[e] = 0.f;
  __syncthreads();
  for (int e = tid; e < H0 * H1; e += 256) sW1[(e / H1) * L1S + (e % H1)] = P[a.p_off1 + e];
  for (int e = tid; e < H1 * C; e += 256) {
    const int k = e / C, nn = e - k * C;
    sW2[k * S17 + nn] = P[a.p_off2 + e];
  }
  for (int e = tid; e < H1; e += 256) sB1[e] = a.bias1 ? P[a.p_off1 + (long long)H0 * H1 + e] : 0.f;
  if (tid < C) sB2[tid] = a.bias2 ? P[a.p_off2 + (long long)H1 * C + tid] : 0.f;
  // DW1 tiles of wave w: t = w + 4u -> (row tile t / nown, owned column c = t % nown);
  // then (index 4*TU) the DW2 tile of wave w < nown: rows (j + nch*w)*16 + 4g + q, column i16
  constexpr int NM = TU * 4 + 4;
  float wm[NM], ws0[NM], ws1[NM];
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int t = w + 4 * u;
    const int rt = t / nown, c = t - rt * nown;
    if constexpr (V2) {   // the DW workgroups own the masters
      wm[4 * u] = wm[4 * u + 1] = wm[4 * u + 2] = wm[4 * u + 3] = 0.f;
      ws0[4 * u] = ws0[4 * u + 1] = ws0[4 * u + 2] = ws0[4 * u + 3] = 0.f;
      ws1[4 * u] = ws1[4 * u + 1] = ws1[4 * u + 2] = ws1[4 * u + 3] = 0.f;
      continue;
    }
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int k = rt * 16 + 4 * g + qq, nn = (j + a.nch * c) * 16 + i16;
      const bool in = t < ndw1;
      const long long pi = a.p_off1 + (long long)k * H1 + nn;
      wm[4 * u + qq] = in ? P[pi] : 0.f;
      ws0[4 * u + qq] = (in && np > 0) ? S[pi] : 0.f;
      ws1[4 * u + qq] = (in && np > 1) ? S[a.op.s_plane + pi] : 0.f;
    }
  }
  const bool w2own = !V2 && w < nown;
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    const int k = (j + a.nch * w) * 16 + 4 * g + qq;
    const bool in = w2own && i16 < C;
    const long long pi = a.p_off2 + (long long)k * C + i16;
    wm[4 * TU + qq] = in ? P[pi] : 0.f;
    ws0[4 * TU + qq] = (in && np > 0) ? S[pi] : 0.f;
    ws1[4 * TU + qq] = (in && np > 1) ? S[a.op.s_plane + pi] : 0.f;
  }
  // owned biases, where their gradients come out of the bias MFMAs (all-ones A rows):
  // b1 of the owned column tiles in wave 2 (lane -> unit (j + nch*(lane/16))*16 + lane%16),
  // b2 (chain workgroup 0) in wave 3, lanes < C -- the waves without a layer-2 tile
  const bool b1own = !V2 && a.bias1 && w == 2 && lane < 16 * nown;
  const int b1n = (j + a.nch * (lane >> 4)) * 16 + (lane & 15);
  const bool b2own = !V2 && a.bias2 && j == 0 && w == 3 && lane < C;
  float bm = 0.f, bst0 = 0.f, bst1 = 0.f;
  if (b1own || b2own) {
    const long long pi = b1own ? a.p_off1 + (long long)H0 * H1 + b1n : a.p_off2 + (long long)H1 * C + lane;
    bm = P[pi];
    bst0 = np > 0 ? S[pi] : 0.f;
    bst1 = np > 1 ? S[a.op.s_plane + pi] : 0.f;
  }
  // parameter-server hook: the owned masters as pulled, and their flat indices (-1: none)
  float wpl[PS ? NM : 1], bpl = bm;
  if constexpr (PS) {
#pragma unroll
    for (int e = 0; e < NM; ++e) wpl[e] = wm[e];
  }
  auto chain_index = [&](int u, int qq) -> long long {
    if (u < TU) {
      const int t = w + 4 * u;
      if (t >= ndw1) return -1;
      const int rt = t / nown, c = t - rt * nown;
      return a.p_off1 + (long long)(rt * 16 + 4 * g + qq) * H1 + (j + a.nch * c) * 16 + i16;
    }
    if (!(w2own && i16 < C)) return -1;
    return a.p_off2 + (long long)((j + a.nch * w) * 16 + 4 * g + qq) * C + i16;
  };
  const long long bias_index = b1own ? a.p_off1 + (long long)H0 * H1 + b1n : a.p_off2 + (long long)H1 * C + lane;
  __syncthreads();
  // every workgroup of the grid resident before any state (metric sums, hand-offs that
  // lead to weight updates) is touched: otherwise give up with PERR_GRID, state intact
  if (!wait_grid(a, r, a.nk0 * a.nc0 + j)) return;   // this chain is workgroup nl0 + j of its replica

  const int n = a.nsteps;
  // V2: this chain's rows of step s's Gram slabs (X_s . X_{s-1}^T, one per k-chunk)
  f32x4 gl[V2 ? RC_MAXSPLIT : 1];
  const int grow = tid >> 4, gc4 = (tid & 15) * 4;
  auto load_gram = [&](int s) {
    if constexpr (V2) {
      const int ngs = a.ng > 0 ? a.ng : a.nk0;
#pragma unroll
      for (int u = 0; u < RC_MAXSPLIT; ++u) {   // branch-free: slabs past ngs re-read the last one
        const int uc = u < ngs ? u : ngs - 1;
        gl[u] = ldw4(rs, grow * 64 + gc4, (int)(a.o_g + (s % 3) * a.g_par) + uc * 64 * 64 + m0 * 64);
      }
    }
  };
  // data rows of this workgroup's targets (thread: rows tid / 32 + 8h, target column
  // tid % 32), read one step ahead so the target loads have no dependent address load
  // The permutation entries load unconditionally (index clamped into the row) and the
  // row's validity is kept beside them: a select on the loaded value made the chain wait
  // for this load right after the step's hand-off poll, ahead of the partial sums' loads
  auto target_rows = [&](int s, int (&prow)[2], bool (&pok)[2]) {
    const int vs = st.valid(a, s);
    const long long first = (long long)(st.s0 + s) * a.B + m0;
    const int* pr = a.perm + (long long)r * a.sPerm;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rr = (tid >> 5) + 8 * h;
      const long long idx = first + rr < a.sPerm ? first + rr : a.sPerm - 1;
      prow[h] = pr[idx];
      pok[h] = m0 + rr < vs && (tid & 31) < a.ldy;
    }
  };
  int prow[2];
  bool pok[2];
  target_rows(0, prow, pok);
  // the loss / metric sums of this workgroup's rows over the chunk (threads < 2 + nmet):
  // one fp64 atomic per value at the end of the launch instead of one per step (an
  // atomic in flight holds up the next hand-off's drain; float partials summed in fp64
  // are exact in any order)
  double msum = 0.0;
  for (int i = 0; i < n; ++i) {
    const int valid = st.valid(a, i);
    if (valid == 0) break;
    const long long it = iter_at(a.ctr, a.ntrain, a.B, r, st.s0, i);
    // batch rows of this workgroup: targets requested before the wait
    float yv[2];
    {
      const float* Yb = a.Y + (long long)r * a.sY;
#pragma unroll
      for (int h = 0; h < 2; ++h) yv[h] = pok[h] ? Yb[(long long)prow[h] * a.ldy + (tid & 31)] : 0.f;
    }
    pstamp(a, i, 0);
    // V1: the partials and every chain workgroup's updated W1 / W2 columns of the previous
    // step.  V2: the partials, the previous step's dZ_0 rows of every chain workgroup (the
    // Z_0 correction) and (ng > 0) this step's Gram slabs -- one poll.  The DW workgroups'
    // W1 / W2 come later in the step (below)
    {
      const bool prev = i > 0;
      const WaitSet sets[4] = {
          {flag_at(a, r, PMF_PART), nl0, (unsigned)(i + 1)},
          {flag_at(a, r, V2 ? PMF_BWD : PMF_W), prev ? a.nch : 0, (unsigned)i},
          {flag_at(a, r, PMF_GR), (V2 && prev) ? a.ng : 0, (unsigned)(i + 1)},
          {nullptr, 0, 0u}};
      if (!wait_sets(a, sets, PERR_CHAIN_PART)) return;
    }
    pstamp(a, i, 1);
    if (i + 1 < n) target_rows(i + 1, prow, pok);
    Staged<H0 * H1 / 1024> w1s;
    Staged<H1 / 64> w2s;
    f32x4 bvec = zero4f();
    // V1: the weight loads go first: their latency overlaps the partial sums below
    auto issue_w = [&]() {
      stage_issue(w1s, rs, (int)a.o_w1, H1, H0, H1);
      stage_issue(w2s, rs, (int)a.o_w2, 16, H1, 16);
      if (tid < H1 / 4) bvec = ldw4(rs, 4 * tid, (int)a.o_b1);
      else if (tid >= 64 && tid < 68) bvec = ldw4(rs, 4 * (tid - 64), (int)a.o_b2);
    };
    if (!V2 && i > 0) issue_w();
    bool wready = false;   // V2: the W1 / W2 loads were issued during phase 0

    // ---- phase 0: z_0 = sum of the split-K partials (b0 is in chunk 0's) -> act, dropout
    {
      const int rr = tid & 15, c0 = (tid >> 4) * 8;
      const int m = m0 + rr;
      const bool cin = c0 < H0;
      const int v = rr * H0 + c0;
      const int pbase = (int)(a.o_part + (i & 1) * a.part_par) + m0 * H0;
      float z[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = 0.f;
      f32x4 pv[2 * RC_MAXSPLIT];
      const int vv = cin ? v : 0;
#pragma unroll
      for (int u = 0; u < RC_MAXSPLIT; ++u) {   // branch-free: chunks past nk0 re-read the last one
        const int uc = u < a.nk0 ? u : a.nk0 - 1;
        pv[2 * u] = ldw4(rs, vv, pbase + uc * 64 * H0);
        pv[2 * u + 1] = ldw4(rs, vv + 4, pbase + uc * 64 * H0);
      }
      // V2, i >= 1: this chain's rows of the Gram slabs (requested before the wait for
      // the previous step's dZ_0 rows of every chain, whose fragments follow)
      float bz[2][16];
      unsigned wflag = 0;
      if constexpr (V2) {
        if (i > 0) {
          load_gram(i);
          pstamp(a, i, 11);
          const int zs = (int)(a.o_dz0 + ((i - 1) & 1) * a.dz0_par);
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int ct = w + 4 * jj < nt0 ? w + 4 * jj : w;   // branch-free: unused past nt0
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) {   // BF: the 16x16x32 bf16 layout (two 32-deep blocks)
              const int kr = BF ? 32 * (ks >> 3) + 8 * g + (ks & 7) : 16 * g + ks;
              bz[jj][ks] = rb<BF>(ldw1(rs, kr * H0 + ct * 16 + i16, zs));
            }
          }
          // one non-blocking look at the DW workgroups' W flags, returning with the loads
          // above; read after the sums (the correction's barrier broadcasts it)
          if (tid < 64)
            wflag = tid < a.nd ? __hip_atomic_load((gu32*)(flag_at(a, r, PMF_W) + tid), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)
                               : (unsigned)i;
        }
      }
#pragma unroll
      for (int u = 0; u < RC_MAXSPLIT; ++u) {
        if (cin && u < a.nk0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            z[e] += pv[2 * u][e];
            z[4 + e] += pv[2 * u + 1][e];
          }
        }
      }
      pstamp(a, i, 13);
      pcycle(a, i, 28);
      if constexpr (V2) {
        if (i > 0) {
          // Z_0 += -lr_{i-1} gs (G + 1) dZ0_{i-1}: the G rows (+ 1 for the bias) -> LDS,
          // the product on the MFMAs, back through LDS in the row layout of z
          float* sG = smem + Lo::o_gs;
          f32x4 gsum = f32x4{1.f, 1.f, 1.f, 1.f};
          const int ngs = a.ng > 0 ? a.ng : a.nk0;
#pragma unroll
          for (int u = 0; u < RC_MAXSPLIT; ++u)
            if (u < ngs) gsum += gl[u];
#pragma unroll
          for (int e = 0; e < 4; ++e) sG[grow * 65 + gc4 + e] = gsum[e];
          int* sWr = reinterpret_cast<int*>(smem + Lo::o_wr);
          if (tid < 64) {
            const bool rdy = __all(wflag >= (unsigned)i);
            if (tid == 0) sWr[0] = rdy ? 1 : 0;
          }
          __syncthreads();
          // W1 / W2 already out: their loads overlap the correction and the act below
          wready = sWr[0] != 0;
          if (wready) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            issue_w();
          }
          const long long itp = iter_at(a.ctr, a.ntrain, a.B, r, st.s0, i - 1);
          const float coef = -(a.op.lr / (1.f + a.op.decay * (float)itp)) * a.op.grad_scale;
          float ag[16];
#pragma unroll
          for (int ks = 0; ks < 16; ++ks) ag[ks] = sG[i16 * 65 + (BF ? 32 * (ks >> 3) + 8 * g + (ks & 7) : 16 * g + ks)];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int ct = w + 4 * jj;
            f32x4 acc = zero4f();
            if constexpr (BF) {
              // dZ_0 is bf16 (rb above); G + 1 stays ~fp32 as a bf16 hi + lo pair: four
              // 16x16x32 bf16 MFMAs instead of sixteen 16x16x4 f32 ones
              float h0[8], l0[8], h1[8], l1[8], z0[8], z1[8];
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                h0[e] = rb<true>(ag[e]);
                l0[e] = ag[e] - h0[e];
                h1[e] = rb<true>(ag[8 + e]);
                l1[e] = ag[8 + e] - h1[e];
                z0[e] = bz[jj][e];
                z1[e] = bz[jj][8 + e];
              }
              const bf16x8 zb0 = bf8(z0), zb1 = bf8(z1);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf8(h0), zb0, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf8(h1), zb1, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf8(l0), zb0, acc, 0, 0, 0);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf8(l1), zb1, acc, 0, 0, 0);
            } else {
#pragma unroll
              for (int ks = 0; ks < 16; ++ks) acc = mma(ag[ks], bz[jj][ks], acc);
            }
            if (ct < nt0) {
#pragma unroll
              for (int qq = 0; qq < 4; ++qq) sZ0[(4 * g + qq) * L0S + ct * 16 + i16] = coef * acc[qq];
            }
          }
          __syncthreads();
          if (cin) {
#pragma unroll
            for (int e = 0; e < 8; ++e) z[e] += sZ0[rr * L0S + c0 + e];
          }
          pstamp(a, i, 27);
        }
      }
      if (!V2 && i > 0) {   // the previous step's weights -> LDS (read after the barrier below)
        stage_commit(w1s, H0, sW1, L1S);
        stage_commit(w2s, H1, sW2, S17);
        if (tid < H1 / 4) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) sB1[4 * tid + qq] = a.bias1 ? bvec[qq] : 0.f;
        } else if (tid >= 64 && tid < 68) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) sB2[4 * (tid - 64) + qq] = (a.bias2 && 4 * (tid - 64) + qq < C) ? bvec[qq] : 0.f;
        }
      }
      float o[8], gg[8], dv[8];
      pm_act<RELU, 8>(a.act0, z, o, gg);
      const float ks = a.rate0 > 0.f ? 1.f / (1.f - a.rate0) : 1.f;
      const uint32_t db = dropout_base(a.seed, r, 0, it);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        const bool live = cin && m < valid;
        const float u = (live && a.rate0 > 0.f) ? dropout_u1(db, m, c) : 1.f;
        const bool keep = live && u >= a.rate0;
        dv[e] = keep ? o[e] * ks : 0.f;
        if (cin) {
          sA0[rr * L0S + c] = dv[e];
          sG0[rr * L0S + c] = keep ? gg[e] * ks : 0.f;
        }
      }
      pstamp(a, i, 14);
      if (cin) {
        stw4(rs, v, (int)a.o_a0 + m0 * H0, f32x4{dv[0], dv[1], dv[2], dv[3]});
        stw4(rs, v + 4, (int)a.o_a0 + m0 * H0, f32x4{dv[4], dv[5], dv[6], dv[7]});
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) sY[(tid >> 5) * 32 + 256 * h + (tid & 31)] = yv[h];
      if (tid < 16) sRow[tid] = m0 + tid < valid ? 1 : -1;
      pstamp(a, i, 15);
    }
    if constexpr (V2) {
      if (i > 0) {   // the DW workgroups' W1 / W2 / biases of the previous step -> LDS
        if (!wready) {
          if (!wait_all(a, flag_at(a, r, PMF_W), a.nd, (unsigned)i, PERR_CHAIN_PREV)) return;
          issue_w();
        }
        pstamp(a, i, 12);
        stage_commit(w1s, H0, sW1, L1S);
        stage_commit(w2s, H1, sW2, S17);
        if (tid < H1 / 4) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) sB1[4 * tid + qq] = a.bias1 ? bvec[qq] : 0.f;
        } else if (tid >= 64 && tid < 68) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) sB2[4 * (tid - 64) + qq] = (a.bias2 && 4 * (tid - 64) + qq < C) ? bvec[qq] : 0.f;
        }
      }
    }
    __syncthreads();
    pstamp(a, i, 2);

    // ---- FWD1: column tiles w, w + 4 of the 16 x H1 output
    float G1[8];
    {
      f32x4 acc[2];
      if constexpr (BF) rows_mm_b<H0, L0S, L1S, 1>(sA0, sW1, w, nt1, acc, i16, g);
      else rows_mm<H0, L0S, L1S, 1, BF>(sA0, sW1, w, nt1, acc, i16, g);
      pstamp(a, i, 16);
      const float ks = a.rate1 > 0.f ? 1.f / (1.f - a.rate1) : 1.f;
      const uint32_t db = dropout_base(a.seed, r, 1, it);
      float z[8], o[8], gg[8];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int col = (w + 4 * jj) * 16 + i16;
        const float b = w + 4 * jj < nt1 ? sB1[col] : 0.f;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) z[4 * jj + qq] = acc[jj][qq] + b;
      }
      pm_act<RELU, 8>(a.act1, z, o, gg);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int ct = w + 4 * jj;
        if (ct >= nt1) continue;
        const int col = ct * 16 + i16;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int rr = 4 * g + qq, m = m0 + rr;
          const bool live = m < valid;
          const float u = (live && a.rate1 > 0.f) ? dropout_u1(db, m, col) : 1.f;
          const bool keep = live && u >= a.rate1;
          G1[4 * jj + qq] = keep ? gg[4 * jj + qq] * ks : 0.f;
          sA1[rr * L1S + col] = keep ? o[4 * jj + qq] * ks : 0.f;
        }
      }
      pstamp(a, i, 17);
    }
    if constexpr (V2) publish(flag_at(a, r, PMF_A0) + j, (unsigned)(i + 1));   // the A_0 rows (phase 0) are out
    else __syncthreads();
    pstamp(a, i, 3);
    publish_rows16<H1>(rs, (int)a.o_a1 + m0 * H1, sA1, L1S);   // weight-gradient operand
    // ---- FWD2: logits, the reduction split over the 4 waves (H1 / 16 k-steps each)
    {
      constexpr int PER = H1 / 16;
      f32x4 acc = zero4f();
      float av[PER], bv[PER];
#pragma unroll
      for (int s2 = 0; s2 < PER; ++s2) {
        const int sx = w * PER + s2;
        const int k = (sx >> 4) * 64 + 16 * g + (sx & 15);
        av[s2] = rb<BF>(sA1[i16 * L1S + k]);
        bv[s2] = rb<BF>(sW2[k * S17 + i16]);
      }
#pragma unroll
      for (int s2 = 0; s2 < PER; ++s2) acc = mma(av[s2], bv[s2], acc);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) sRed[w * 256 + (4 * g + qq) * 16 + i16] = acc[qq];
    }
    __syncthreads();
    pstamp(a, i, 18);
    {
      const int rr = tid >> 4, c = tid & 15;
      const float v = sRed[tid] + sRed[256 + tid] + sRed[512 + tid] + sRed[768 + tid];
      sLg[rr * 36 + c] = c < C ? v + sB2[c] : 0.f;
    }
    __syncthreads();
    pstamp(a, i, 19);
    // ---- loss / metrics -> dZ_2 = dL/dz (scaled by 1 / valid) in sLg
    {
      Prob pq;
      pq.N = C;
      pq.act = a.act2;
      pq.loss = a.loss;
      pq.nmet = a.nmet;
#pragma unroll
      for (int e = 0; e < 4; ++e) pq.met[e] = a.met[e];
      pq.Y = a.Y;
      pq.pred = nullptr;
      pq.sPred = 0;
      pq.ldp = 0;
      pq.chunk = 0;
      pq.B = a.B;
      const float inv_valid = 1.f / (float)valid;
      float sums[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (FAST) {
        if (w == 0) loss_tile_cce<4, 16, 36, 32>(pq, r, m0, sLg, sY, sRow, true, inv_valid, sums);
      } else {
        loss_tile_lds<16, 36, 32>(pq, r, m0, sLg, sY, sRow, true, inv_valid, sums);
      }
      // per-row sums sit in the row leaders (a quad per row / 16 lanes per row): through
      // LDS to 6 threads, one fp64 atomic per value (no 64-lane shuffle chains)
      float* sAcc = sRed;   // [16][8]; the FWD2 partials are consumed (barrier above)
      const bool leader = FAST ? (tid < 64 && (tid & 3) == 0) : ((tid & 15) == 0);
      const int lrow = FAST ? (tid >> 2) : (tid >> 4);
      if (leader) {
#pragma unroll
        for (int e = 0; e < 6; ++e) sAcc[lrow * 8 + e] = sums[e];
      }
      __syncthreads();
      if (a.acc && tid < 2 + a.nmet) {
        float sv = 0.f;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) sv += sAcc[rr * 8 + tid];
        msum += (double)sv;
      }
      pstamp(a, i, 20);
    }
    __syncthreads();
    {
      const int rr = tid >> 4, c = tid & 15;
      sD2[rr * S17 + c] = c < C ? sLg[rr * 36 + c] : 0.f;
    }
    __syncthreads();
    pstamp(a, i, 4);
    publish_rows16<16>(rs, (int)a.o_dz2 + m0 * 16, sD2, S17);
    // ---- DX2: dZ_1 = (dZ_2 . W2^T) * G_1 (reduction over the <= 16 logits)
    {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int ct = w + 4 * jj;
        if (ct >= nt1) continue;
        const int col = ct * 16 + i16;
        float av[4], bv[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int c = 4 * ks + g;
          av[ks] = rb<BF>(sD2[i16 * S17 + c]);
          bv[ks] = rb<BF>(sW2[col * S17 + c]);
        }
        f32x4 acc = zero4f();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc = mma(av[ks], bv[ks], acc);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) sD1[(4 * g + qq) * L1S + col] = acc[qq] * G1[4 * jj + qq];
      }
      pstamp(a, i, 21);
    }
    if constexpr (V2) {
      publish(flag_at(a, r, PMF_D2) + j, (unsigned)(i + 1));   // A_1 and dZ_2 rows are out
    } else {
      __syncthreads();
      publish_rows16<H1>(rs, (int)a.o_dz1 + m0 * H1, sD1, L1S);
    }
    pstamp(a, i, 22);
    // ---- DX1: dZ_0 = (dZ_1 . W1^T) * G_0 -> LDS, then published for the L0 tiles
    {
      f32x4 acc[2];
      if constexpr (BF) rows_mm_b<H1, L1S, 1, L1S>(sD1, sW1, w, nt0, acc, i16, g);
      else rows_mm<H1, L1S, 1, L1S, BF>(sD1, sW1, w, nt0, acc, i16, g);
      pstamp(a, i, 23);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int ct = w + 4 * jj;
        if (ct >= nt0) continue;
        const int col = ct * 16 + i16;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int rr = 4 * g + qq;
          sZ0[rr * L0S + col] = acc[jj][qq] * sG0[rr * L0S + col];
        }
      }
    }
    __syncthreads();
    publish_rows16<H0>(rs, (int)(a.o_dz0 + (i & 1) * a.dz0_par) + m0 * H0, sZ0, L0S);
    pstamp(a, i, 5);
    publish(flag_at(a, r, PMF_BWD) + j, (unsigned)(i + 1));
    pstamp(a, i, 6);
    if constexpr (V2) continue;   // weight gradients: dw_role_v2

    // ---- weight gradients of the owned layer-1 columns / layer-2 rows, update
    if (!wait_all(a, flag_at(a, r, PMF_BWD), a.nch, (unsigned)(i + 1), 3u)) return;
    pstamp(a, i, 7);
    stage<H0 / 16>(rs, (int)a.o_a0, H0, BR, H0, uA0, L0S);
#pragma unroll
    for (int c = 0; c < PM_NTU; ++c) {
      if (c < nown) {
        const int col = (j + a.nch * c) * 16;
        stage<1>(rs, (int)a.o_dz1 + col, H1, BR, 16, uD1 + c * 16, 33);
        stage<1>(rs, (int)a.o_a1 + col, H1, BR, 16, uA1 + c * 16, 33);
      }
    }
    stage<1>(rs, (int)a.o_dz2, 16, BR, 16, uD2, S17);
    // rows BR..63 of the staging must be zero for the 64-deep reductions
    for (int e = tid; e < (64 - BR) * L0S; e += 256) uA0[BR * L0S + e] = 0.f;
    for (int e = tid; e < (64 - BR) * 33; e += 256) {
      uD1[BR * 33 + e] = 0.f;
      uA1[BR * 33 + e] = 0.f;
    }
    for (int e = tid; e < (64 - BR) * S17; e += 256) uD2[BR * S17 + e] = 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    pstamp(a, i, 8);
    {
      f32x4 dw[TU + 1], db[2] = {zero4f(), zero4f()};
#pragma unroll
      for (int u = 0; u <= TU; ++u) dw[u] = zero4f();
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        float xa[TU][8], zb[2][8], a1v[8], d2v[8];
#pragma unroll
        for (int h8 = 0; h8 < 8; ++h8) {
          const int b = 16 * g + 8 * half + h8;
          zb[0][h8] = uD1[b * 33 + i16];
          zb[1][h8] = uD1[b * 33 + 16 + i16];
#pragma unroll
          for (int u = 0; u < TU; ++u) xa[u][h8] = uA0[b * L0S + urt[u] * 16 + i16];
          a1v[h8] = uA1[b * 33 + (w2own ? w : 0) * 16 + i16];
          d2v[h8] = uD2[b * S17 + i16];
        }
        // branch-free: tiles a wave does not own compute garbage that is never stored
#pragma unroll
        for (int h8 = 0; h8 < 8; ++h8) {
#pragma unroll
          for (int u = 0; u < TU; ++u)   // wave-uniform: no MFMAs for tiles past ndw1
            if (w + 4 * u < ndw1) dw[u] = mma(xa[u][h8], uct[u] ? zb[1][h8] : zb[0][h8], dw[u]);
          dw[TU] = mma(a1v[h8], d2v[h8], dw[TU]);
        }
        // bias gradients = column sums over the batch rows: an all-ones A operand (every
        // output row holds the sums), in the waves that own the biases
        if (w >= 2) {
#pragma unroll
          for (int h8 = 0; h8 < 8; ++h8) {
            db[0] = mma(1.f, w == 2 ? zb[0][h8] : d2v[h8], db[0]);
            db[1] = mma(1.f, zb[1][h8], db[1]);
          }
        }
      }
      pstamp(a, i, 24);
      if (a.sync) {   // per-step synchronous DP (see xchg_sum)
        f32x4 xv[TU + 3];
#pragma unroll
        for (int u = 0; u <= TU; ++u) xv[u] = dw[u];
        xv[TU + 1] = db[0];
        xv[TU + 2] = db[1];
        if (!xchg_sum<TU + 3>(a, r, nl0 + j, i, xv)) return;
#pragma unroll
        for (int u = 0; u <= TU; ++u) dw[u] = xv[u];
        db[0] = xv[TU + 1];
        db[1] = xv[TU + 2];
      }
      pstamp(a, i, 25);
      const float gb = (b1own && lane >= 16) ? db[1][0] : db[0][0];
      const float gs = a.op.grad_scale;
      float gv[NM];
#pragma unroll
      for (int u = 0; u <= TU; ++u)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) gv[4 * u + qq] = (u < TU || i16 < C) ? dw[u][qq] * gs : 0.f;
      pm_update<NPT, NM>(a.op, wm, gv, ws0, ws1, it);
      pstamp(a, i, 26);
      if (b1own || b2own) {
        float bv[1] = {bm}, bg[1] = {gb * gs}, t0[1] = {bst0}, t1[1] = {bst1};
        pm_update<NPT, 1>(a.op, bv, bg, t0, t1, it);
        bm = bv[0];
        bst0 = t0[0];
        bst1 = t1[0];
      }
    }
    pstamp(a, i, 9);
    const bool nxt = i + 1 < n && st.valid(a, i + 1) > 0;
    if constexpr (PS) {
      // parameter-server hook: push the owned columns' theta_new - theta_pulled, then pull
      // them for the next step (published to the other chain workgroups below)
      ps_push_begin(a, nl0 + j);
#pragma unroll
      for (int u = 0; u <= TU; ++u) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const long long idx = chain_index(u, qq);
          const float dlt = wm[4 * u + qq] - wpl[4 * u + qq];
          if (idx >= 0 && dlt != 0.f)
            __hip_atomic_fetch_add(ps_elem(a.ps, idx), dlt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      if ((b1own || b2own) && bm != bpl) __hip_atomic_fetch_add(ps_elem(a.ps, bias_index), bm - bpl, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_SYSTEM);
      ps_push_end(a, nl0 + j);
      if (nxt) {
        const bool ok = ps_pull(a, nl0 + j, reinterpret_cast<unsigned*>(sRed), [&]() {
          float v[NM];
#pragma unroll
          for (int u = 0; u <= TU; ++u) {
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
              const long long idx = chain_index(u, qq);
              v[4 * u + qq] = *ps_elem(a.ps, idx >= 0 ? idx : a.p_off1);
            }
          }
#pragma unroll
          for (int e = 0; e < NM; ++e) {
            if (chain_index(e >> 2, e & 3) >= 0) {
              wm[e] = v[e];
              wpl[e] = v[e];
            }
          }
          if (b1own || b2own) {
            bm = *ps_elem(a.ps, bias_index);
            bpl = bm;
          }
        });
        if (!ok) return;
      }
    }
    if (!nxt) break;
    // ---- publish the owned weights, gather everyone's into LDS for the next step
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int t = w + 4 * u;
      if (t >= ndw1) continue;
      const int rt = t / nown, c = t - rt * nown;
      const int v = (rt * 16 + 4 * g) * H1 + i16;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) stw1(rs, v + qq * H1, (int)a.o_w1 + (j + a.nch * c) * 16, wm[4 * u + qq]);
    }
    if (w2own && i16 < C) {
      const int v = (4 * g) * 16 + i16;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        stw1(rs, v + qq * 16, (int)a.o_w2 + (j + a.nch * w) * 256, wm[4 * TU + qq]);
    }
    if (b1own) stw1(rs, b1n, (int)a.o_b1, bm);
    if (b2own) stw1(rs, lane, (int)a.o_b2, bm);
    publish(flag_at(a, r, PMF_W) + j, (unsigned)(i + 1));
    pstamp(a, i, 10);
    pcycle(a, i, 29);
  }
  if (a.acc && tid < 2 + a.nmet && msum != 0.0) atomicAdd(a.acc + (long long)r * a.acc_stride + tid, msum);

  // ---- epilogue: owned masters, both weight-image parities, state
  if constexpr (V2) return;
  float* Wsh = a.Wsh + (long long)r * a.sWsh;
  float* WTsh = a.WTsh + (long long)r * a.sWTsh;
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int t = w + 4 * u;
    if (t >= ndw1) continue;
    const int rt = t / nown, c = t - rt * nown;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int k = rt * 16 + 4 * g + qq, nn = (j + a.nch * c) * 16 + i16;
      const long long pi = a.p_off1 + (long long)k * H1 + nn;
      pst(a, P + (pi), wm[4 * u + qq]);
      if (np > 0) S[pi] = ws0[4 * u + qq];
      if (np > 1) S[a.op.s_plane + pi] = ws1[4 * u + qq];
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        Wsh[par * a.wsh_par + a.wsh_off[1] + (long long)k * a.Np[1] + nn] = wm[4 * u + qq];
        WTsh[par * a.wtsh_par + a.wtsh_off[1] + (long long)nn * a.Kp[1] + k] = wm[4 * u + qq];
      }
    }
  }
  if (w2own && i16 < C) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int k = (j + a.nch * w) * 16 + 4 * g + qq;
      const long long pi = a.p_off2 + (long long)k * C + i16;
      pst(a, P + (pi), wm[4 * TU + qq]);
      if (np > 0) S[pi] = ws0[4 * TU + qq];
      if (np > 1) S[a.op.s_plane + pi] = ws1[4 * TU + qq];
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        Wsh[par * a.wsh_par + a.wsh_off[2] + (long long)k * a.Np[2] + i16] = wm[4 * TU + qq];
        WTsh[par * a.wtsh_par + a.wtsh_off[2] + (long long)i16 * a.Kp[2] + k] = wm[4 * TU + qq];
      }
    }
  }
  if (b1own || b2own) {
    const long long pi = b1own ? a.p_off1 + (long long)H0 * H1 + b1n : a.p_off2 + (long long)H1 * C + lane;
    pst(a, P + (pi), bm);
    if (np > 0) S[pi] = bst0;
    if (np > 1) S[a.op.s_plane + pi] = bst1;
  }
}

// ============================================================== V2: weight gradients
// nd workgroups per replica; workgroup d owns the layer-1 column tiles d + nd*c (c <
// nown) = the layer-2 row tiles of the same index, their biases, and b2 (d == 0): the
// chain's DW block of V1 on a workgroup of its own.  Per step it stages A_0 of every
// row once the chains raise A0, then (D2) the A_1 columns and dZ_2 it needs, rebuilds
// its dZ_1 columns = (dZ_2 . W2_own^T) * relu'(.) * keep / (1 - rate) -- the factor
// recovered from A_1 > 0 (ReLU, so the same MFMA as the chain's DX2 gives the same bits)
// -- computes DW1 / DW2 / the bias sums, applies plain SGD and publishes the columns.
template <int H0, int H1, bool BF>
__device__ __forceinline__ void dw_role_v2(const PersistArgs& a, float* smem, int r, int d) {
  constexpr int L0S = H0 + 1;
  constexpr int nt0 = H0 / 16, nt1 = H1 / 16;
  const int tid = threadIdx.x, lane = tid & 63, i16 = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6) & 3;
  const int C = a.C;
  const int BR = a.nch * 16;
  const int nd = a.nd;
  float* uA0 = smem;                 // [64][L0S] layer-0 activations of every row
  float* uD1 = uA0 + 64 * L0S;       // [64][33] dZ_1 of the owned layer-1 columns
  float* uA1 = uD1 + 64 * 33;        // [64][33] layer-1 activations of the owned W2 rows
  float* uD2 = uA1 + 64 * 33;        // [64][17] dZ_2
  float* sW2o = uD2 + 64 * S17;      // [32][17] the owned W2 rows (operand of the dZ_1 rebuild)
  const rsrc_t rs = ws_rsrc(a.ws + (long long)r * a.ws_stride);
  float* P = a.P + (long long)r * a.sP;
  Steps st{ld_inv(a.ctr), ld_inv(a.ntrain + r)};

  const int nown = (nt1 - d + nd - 1) / nd;   // <= PM_NTU (host checks)
  const int ndw1 = nt0 * nown;
  int urt[TU], uct[TU];
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int t = w + 4 * u;
    urt[u] = t < ndw1 ? t / nown : 0;
    uct[u] = t < ndw1 ? t - (t / nown) * nown : 0;
  }
  // Gram k-chunk of this workgroup (ng > 0): X_s . X_{s-1}^T over columns [k0g, k0g + kg)
  const bool gown = a.ng > 0 && d < a.ng;
  const int k0g = d * a.gk;
  const int kg = gown ? (a.K0 - k0g < a.gk ? a.K0 - k0g : a.gk) : 0;
  // row stride: fp32 = 4 (mod 8) floats, bf16 = 2 (mod 4) dwords -- the fragment reads
  // below (16 rows x 4 consecutive k per MFMA) hit 64 distinct banks
  const int xneed = BF ? (kg + 1) / 2 + 1 : kg + 1;
  const int XSg = BF ? xneed + ((2 - xneed) % 4 + 4) % 4 : xneed + ((4 - xneed) % 8 + 8) % 8;
  float* sXg = smem + DW_LDS;        // [2][64][XSg] X chunks of steps s & 1
  float* sTg = sXg + 2 * 64 * 116;   // [64][65] slab staging (16-byte stores)
  for (int e = tid; e < DWP_LDS; e += 256) smem[e] = 0.f;
  __syncthreads();
  constexpr int NM = TU * 4 + 4;
  float wm[NM];
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int t = w + 4 * u;
    const int rt = t / nown, c = t - rt * nown;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int k = rt * 16 + 4 * g + qq, nn = (d + nd * c) * 16 + i16;
      wm[4 * u + qq] = t < ndw1 ? P[a.p_off1 + (long long)k * H1 + nn] : 0.f;
    }
  }
  const bool w2own = w < nown;
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    const int k = (d + nd * w) * 16 + 4 * g + qq;
    const bool in = w2own && i16 < C;
    wm[4 * TU + qq] = in ? P[a.p_off2 + (long long)k * C + i16] : 0.f;
    if (w2own) sW2o[(w * 16 + 4 * g + qq) * S17 + i16] = wm[4 * TU + qq];
  }
  const bool b1own = a.bias1 && w == 2 && lane < 16 * nown;
  const int b1n = (d + nd * (lane >> 4)) * 16 + (lane & 15);
  const bool b2own = a.bias2 && d == 0 && w == 3 && lane < C;
  float bm = 0.f;
  if (b1own || b2own) bm = P[b1own ? a.p_off1 + (long long)H0 * H1 + b1n : a.p_off2 + (long long)H1 * C + lane];
  const float ks1 = a.rate1 > 0.f ? 1.f / (1.f - a.rate1) : 1.f;
  __syncthreads();

  // step s's X chunk (rows gathered through the permutation) -> buffer s & 1, LDS-DMA
  auto load_xg = [&](int s) {
    const int valid = st.valid(a, s);
    const int* pr = a.perm + (long long)r * a.sPerm + (st.s0 + s) * a.B;
    float* dst = sXg + (s & 1) * 64 * XSg;
    const int myrow = pr[lane < valid ? lane : 0];
    for (int v = 0; v < 16; ++v) {
      const int b = w + 4 * v;
      if (b >= BR) break;
      const int row = __builtin_amdgcn_readlane(myrow, b);
      if constexpr (BF) {
        const float* src = reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(a.X) +
                                                          (long long)r * a.sX + (long long)row * a.ldx + k0g);
        if (lane < (kg + 1) / 2) __builtin_amdgcn_global_load_lds(src + lane, dst + b * XSg, 4, 0, 0);
      } else {
        const float* src = a.X + (long long)r * a.sX + (long long)row * a.ldx + k0g;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (64 * h + lane < kg) __builtin_amdgcn_global_load_lds(src + 64 * h + lane, dst + b * XSg + 64 * h, 4, 0, 0);
      }
    }
  };
  // Gram slab of step s = X_s . X_{s-1}^T over this k-chunk: wave w owns column tile w
  // and all four row tiles (the B fragments read once, four independent accumulators)
  auto gram_dw = [&](int s) {
    const float* A = sXg + (s & 1) * 64 * XSg;
    const float* Bm = sXg + ((s - 1) & 1) * 64 * XSg;
    auto xat = [](const float* row, int k) -> float { if constexpr (BF) return bf_at(row, k); else return row[k]; };
    f32x4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = zero4f();
    const float* brow = Bm + (w * 16 + i16) * XSg;
    if constexpr (BF) {
      // the bf16 rows straight into v_mfma_f32_16x16x32_bf16 (lane: elements kb + 8g + j,
      // four packed dwords); both operands masked past the chunk (kg is even: whole pairs)
      const unsigned* bu = reinterpret_cast<const unsigned*>(brow);
#pragma unroll 1
      for (int kb = 0; kb < kg; kb += 32) {
        const int d0 = (kb + 8 * g) >> 1;
        u32x4 bq;
#pragma unroll
        for (int e = 0; e < 4; ++e) bq[e] = 2 * (d0 + e) < kg ? bu[d0 + e] : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned* au = reinterpret_cast<const unsigned*>(A + (u * 16 + i16) * XSg);
          u32x4 aq;
#pragma unroll
          for (int e = 0; e < 4; ++e) aq[e] = 2 * (d0 + e) < kg ? au[d0 + e] : 0u;
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, aq), __builtin_bit_cast(bf16x8, bq),
                                                           acc[u], 0, 0, 0);
        }
      }
    } else {
#pragma unroll 1
      for (int kb = 0; kb < kg; kb += 16) {
        float av[4][4], bv[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int k = kb + 4 * ks + g;
          bv[ks] = xat(brow, k);   // finite (X or zero padding) past the chunk, times a zero A
#pragma unroll
          for (int u = 0; u < 4; ++u) av[u][ks] = k < kg ? xat(A + (u * 16 + i16) * XSg, k) : 0.f;
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[u] = mma(av[u][ks], bv[ks], acc[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) sTg[(u * 16 + 4 * g + qq) * 65 + w * 16 + i16] = acc[u][qq];
    __syncthreads();
    const int base = (int)(a.o_g + (s % 3) * a.g_par) + d * 64 * 64;
    for (int e = tid; e < BR * 16; e += 256) {
      const int row = e >> 4, c4 = e & 15;
      const float* src = sTg + row * 65 + 4 * c4;
      stw4(rs, row * 64 + 4 * c4, base, f32x4{src[0], src[1], src[2], src[3]});
    }
    publish(flag_at(a, r, PMF_GR) + d, (unsigned)(s + 1));
  };

  const int n = a.nsteps;
  if (gown && n > 1 && st.valid(a, 1) > 0) {   // Gram(1); Gram(s + 2) follows iteration s
    load_xg(0);
    load_xg(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    gram_dw(1);
  }
  for (int i = 0; i < n; ++i) {
    if (st.valid(a, i) == 0) break;
    const long long it = iter_at(a.ctr, a.ntrain, a.B, r, st.s0, i);
    const bool gnext = gown && i + 2 < n && st.valid(a, i + 2) > 0;
    // X_{i+2} into the buffer X_i left (Gram(i + 1) is out): the DMA runs during the A0 wait
    if (gnext) load_xg(i + 2);
    pstamp(a, i, 0);
    if (!wait_all(a, flag_at(a, r, PMF_A0), a.nch, (unsigned)(i + 1), PERR_DW_A0)) return;
    pstamp(a, i, 1);
    stage<H0 / 16>(rs, (int)a.o_a0, H0, BR, H0, uA0, L0S);
    if (!wait_all(a, flag_at(a, r, PMF_D2), a.nch, (unsigned)(i + 1), PERR_DW_D2)) return;
    pstamp(a, i, 2);
#pragma unroll
    for (int c = 0; c < PM_NTU; ++c) {
      if (c < nown) stage<1>(rs, (int)a.o_a1 + (d + nd * c) * 16, H1, BR, 16, uA1 + c * 16, 33);
    }
    stage<1>(rs, (int)a.o_dz2, 16, BR, 16, uD2, S17);
    // rows BR..63 of the staging must be zero for the 64-deep reductions
    for (int e = tid; e < (64 - BR) * L0S; e += 256) uA0[BR * L0S + e] = 0.f;
    for (int e = tid; e < (64 - BR) * 33; e += 256) uA1[BR * 33 + e] = 0.f;
    for (int e = tid; e < (64 - BR) * S17; e += 256) uD2[BR * S17 + e] = 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    pstamp(a, i, 3);
    // dZ_1 of the owned columns, 16 rows per wave: the chain's DX2 MFMA on the same
    // operands, times relu'(z) * keep / (1 - rate) = (A_1 > 0 ? 1 / (1 - rate) : 0)
#pragma unroll
    for (int c = 0; c < PM_NTU; ++c) {
      if (c >= nown) continue;
      float av[4], bv[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int cc = 4 * kk + g;
        av[kk] = rb<BF>(uD2[(w * 16 + i16) * S17 + cc]);
        bv[kk] = rb<BF>(sW2o[(c * 16 + i16) * S17 + cc]);
      }
      f32x4 acc = zero4f();
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) acc = mma(av[kk], bv[kk], acc);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int row = w * 16 + 4 * g + qq;
        const float a1 = uA1[row * 33 + c * 16 + i16];
        uD1[row * 33 + c * 16 + i16] = acc[qq] * (a1 > 0.f ? ks1 : 0.f);
      }
    }
    __syncthreads();
    pstamp(a, i, 4);
    {
      f32x4 dw[TU + 1], db[2] = {zero4f(), zero4f()};
#pragma unroll
      for (int u = 0; u <= TU; ++u) dw[u] = zero4f();
      if constexpr (BF) {
        // v_mfma_f32_16x16x32_bf16 over two 32-row blocks of the batch (lane: rows
        // kb + 8g + j), the operands rounded to bf16 as rb<true> does
        const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u});
#pragma unroll
        for (int kb = 0; kb < 64; kb += 32) {
          float xa[TU][8], z0[8], z1[8], a1v[8], d2v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int b = kb + 8 * g + j;
            z0[j] = uD1[b * 33 + i16];
            z1[j] = uD1[b * 33 + 16 + i16];
#pragma unroll
            for (int u = 0; u < TU; ++u) xa[u][j] = uA0[b * L0S + urt[u] * 16 + i16];
            a1v[j] = uA1[b * 33 + (w2own ? w : 0) * 16 + i16];
            d2v[j] = uD2[b * S17 + i16];
          }
          const bf16x8 zb0 = bf8(z0), zb1 = bf8(z1), d28 = bf8(d2v);
#pragma unroll
          for (int u = 0; u < TU; ++u)   // wave-uniform: no MFMAs for tiles past ndw1
            if (w + 4 * u < ndw1)
              dw[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf8(xa[u]), uct[u] ? zb1 : zb0, dw[u], 0, 0, 0);
          dw[TU] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf8(a1v), d28, dw[TU], 0, 0, 0);
          if (w >= 2) {
            db[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, w == 2 ? zb0 : d28, db[0], 0, 0, 0);
            db[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, zb1, db[1], 0, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          float xa[TU][8], zb[2][8], a1v[8], d2v[8];
#pragma unroll
          for (int h8 = 0; h8 < 8; ++h8) {
            const int b = 16 * g + 8 * half + h8;
            zb[0][h8] = uD1[b * 33 + i16];
            zb[1][h8] = uD1[b * 33 + 16 + i16];
#pragma unroll
            for (int u = 0; u < TU; ++u) xa[u][h8] = uA0[b * L0S + urt[u] * 16 + i16];
            a1v[h8] = uA1[b * 33 + (w2own ? w : 0) * 16 + i16];
            d2v[h8] = uD2[b * S17 + i16];
          }
#pragma unroll
          for (int h8 = 0; h8 < 8; ++h8) {
#pragma unroll
            for (int u = 0; u < TU; ++u)   // wave-uniform: no MFMAs for tiles past ndw1
              if (w + 4 * u < ndw1) dw[u] = mma(xa[u][h8], uct[u] ? zb[1][h8] : zb[0][h8], dw[u]);
            dw[TU] = mma(a1v[h8], d2v[h8], dw[TU]);
          }
          if (w >= 2) {
#pragma unroll
            for (int h8 = 0; h8 < 8; ++h8) {
              db[0] = mma(1.f, w == 2 ? zb[0][h8] : d2v[h8], db[0]);
              db[1] = mma(1.f, zb[1][h8], db[1]);
            }
          }
        }
      }
      pstamp(a, i, 5);
      // plain SGD in the operation order of pm_update<0>
      const float lr = a.op.lr / (1.f + a.op.decay * (float)it), gs = a.op.grad_scale;
#pragma unroll
      for (int u = 0; u <= TU; ++u)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          if (u < TU || i16 < C) wm[4 * u + qq] -= lr * (dw[u][qq] * gs);
      const float gb = (b1own && lane >= 16) ? db[1][0] : db[0][0];
      if (b1own || b2own) bm -= lr * (gb * gs);
    }
    // ---- publish the owned columns (the chains read them at the next step's start)
    const bool nxt = i + 1 < n && st.valid(a, i + 1) > 0;
    if (w2own) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) sW2o[(w * 16 + 4 * g + qq) * S17 + i16] = wm[4 * TU + qq];
    }
    if (nxt) {
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int t = w + 4 * u;
        if (t >= ndw1) continue;
        const int rt = t / nown, c = t - rt * nown;
        const int v = (rt * 16 + 4 * g) * H1 + i16;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) stw1(rs, v + qq * H1, (int)a.o_w1 + (d + nd * c) * 16, wm[4 * u + qq]);
      }
      if (w2own && i16 < C) {
        const int v = (4 * g) * 16 + i16;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) stw1(rs, v + qq * 16, (int)a.o_w2 + (d + nd * w) * 256, wm[4 * TU + qq]);
      }
      if (b1own) stw1(rs, b1n, (int)a.o_b1, bm);
      if (b2own) stw1(rs, lane, (int)a.o_b2, bm);
      publish(flag_at(a, r, PMF_W) + d, (unsigned)(i + 1));
    } else {
      __syncthreads();
    }
    pstamp(a, i, 6);
    if (gnext) {   // Gram(i + 2), in the idle window before the next step's A0
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      gram_dw(i + 2);
      pstamp(a, i, 7);
    }
  }

  // ---- epilogue: owned masters and both weight-image parities (plain SGD: no state)
  float* Wsh = img_base<BF>(a.Wsh, (long long)r * a.sWsh);
  float* WTsh = img_base<BF>(a.WTsh, (long long)r * a.sWTsh);
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int t = w + 4 * u;
    if (t >= ndw1) continue;
    const int rt = t / nown, c = t - rt * nown;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int k = rt * 16 + 4 * g + qq, nn = (d + nd * c) * 16 + i16;
      pst(a, P + (a.p_off1 + (long long)k * H1 + nn), wm[4 * u + qq]);
      if (!a.imgs) continue;
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        img_store<BF>(Wsh, par * a.wsh_par + a.wsh_off[1] + (long long)k * a.Np[1] + nn, wm[4 * u + qq]);
        img_store<BF>(WTsh, par * a.wtsh_par + a.wtsh_off[1] + (long long)nn * a.Kp[1] + k, wm[4 * u + qq]);
      }
    }
  }
  if (w2own && i16 < C) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int k = (d + nd * w) * 16 + 4 * g + qq;
      pst(a, P + (a.p_off2 + (long long)k * C + i16), wm[4 * TU + qq]);
      if (!a.imgs) continue;
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        img_store<BF>(Wsh, par * a.wsh_par + a.wsh_off[2] + (long long)k * a.Np[2] + i16, wm[4 * TU + qq]);
        img_store<BF>(WTsh, par * a.wtsh_par + a.wtsh_off[2] + (long long)i16 * a.Kp[2] + k, wm[4 * TU + qq]);
      }
    }
  }
  if (b1own || b2own) pst(a, P + (b1own ? a.p_off1 + (long long)H0 * H1 + b1n : a.p_off2 + (long long)H1 * C + lane), bm);
}

}  // namespace

// ---- fused replica averaging (PersistArgs::avg_end): after every role's epilogue -- its
//      masters in P, stored write-through and drained -- each workgroup arrives at the grid
//      counter, waits for all R x wgs, then averages its slice of the parameters over the R
//      replicas: fp64 sums in replica order (the replica_average kernel's numerics), scaled,
//      into avg_out and / or every replica's P.  A launch whose error word is set skips it.
__device__ __forceinline__ void grid_average(const PersistArgs& a, int b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* ctr = flag_at(a, 0, PMF_AVG);
  const unsigned tot = (unsigned)(a.R * a.wgs);
  if (threadIdx.x == 0) __hip_atomic_fetch_add((gu32*)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!wait_all(a, ctr, 1, tot, PERR_AVG)) return;
  if (__hip_atomic_load((gu32*)(a.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
  // element-wise (P's replica stride need not keep 16-byte alignment): 8 replicas' loads in
  // flight per element; sc1 -- this XCD's L2 never held the other replicas' lines
  const long long n = a.avg_n, lo = n * b / tot, hi = n * (b + 1) / tot;
  const rsrc_t pr = ws_rsrc(a.P);
  for (long long i = lo + threadIdx.x; i < hi; i += 256) {
    double sm = 0.0;
    for (int r0 = 0; r0 < a.R; r0 += 8) {
      float x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = r0 + k < a.R ? r0 + k : r0;
        x[k] = ldw1(pr, (int)i, (int)((long long)r * a.sP));
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (r0 + k < a.R) sm += x[k];
    }
    const float m = (float)(sm * a.avg_scale);
    if (a.avg_out) a.avg_out[i] = m;
    if (a.avg_p)
      for (int r = 0; r < a.R; ++r) a.P[(long long)r * a.sP + i] = m;
  }
}

template <int H0, int H1, bool FAST, int NPT, bool RELU, bool V2, bool PS = false, bool BF = false>
__global__ __launch_bounds__(256) void mlp_persist_kernel(PersistArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[LDS_FLOATS];
  if (__hip_atomic_load((gu32*)(a.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
  const int b = blockIdx.x;
#if EA_PLOCAL == 2
  // blocks b and b + 8 share an XCD: block b -> replica (b / 8) % 8, workgroup
  // b % 8 + 8 ((b / 8) / 8) -- the 8 copies of workgroup q on one XCD (host: R = 8, wgs % 8 == 0)
  const int r = (b >> 3) & 7, q = (b & 7) + 8 * (b >> 6);
#else
  const int r = b % a.R, q = b / a.R;
#endif
  // residency: raise this workgroup's GO flag (the chain workgroups wait for the grid)
  if (threadIdx.x == 0) __hip_atomic_store((gu32*)(flag_at(a, r, PMF_GO) + q), go_value(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nl0 = a.nk0 * a.nc0;
  if constexpr (V2) {
    static_assert(NPT == 0 && RELU, "V2: plain SGD, ReLU hidden layers");
    if (q < nl0) {
      const int kc = q / a.nc0, cb = q - kc * a.nc0;
      if (a.cw == 64) l0_role_v2<H0, 4, BF>(a, smem, r, kc, cb, q);
      else l0_role_v2<H0, 2, BF>(a, smem, r, kc, cb, q);
    } else if (q < nl0 + a.nch) {
      chain_role<H0, H1, FAST, NPT, RELU, true, false, BF>(a, smem, r, q - nl0);
    } else {
      dw_role_v2<H0, H1, BF>(a, smem, r, q - nl0 - a.nch);
    }
  } else {
    if (q < nl0) l0_role<H0, NPT, PS>(a, smem, r, q / a.nc0, q - (q / a.nc0) * a.nc0, q);
    else chain_role<H0, H1, FAST, NPT, RELU, false, PS>(a, smem, r, q - nl0);
  }
  if (a.avg_end) grid_average(a, b);
}

// the instances of one hidden width: the specialised MNIST-style one (relu, softmax +
// cross-entropy, plain SGD) and the general ones
template <int H0, int H1>
hipError_t persist_launch(const PersistArgs* a, hipStream_t s) {
  bool fast = a->act2 == ACT_SOFTMAX && (a->loss == LOSS_CCE || a->loss == LOSS_SPARSE_CCE);
  for (int i = 0; i < a->nmet; ++i)
    fast = fast && (a->met[i] == MET_ACC_CAT || a->met[i] == MET_ACC_SPARSE || a->met[i] == LOSS_CCE ||
                    a->met[i] == LOSS_SPARSE_CCE);
  const bool relu = a->act0 == ACT_RELU && a->act1 == ACT_RELU;
  const bool sgd = !a->S || (a->op.opt == OPT_SGD && a->op.mom == 0.f);
  const dim3 grid(a->R * a->wgs);
#if EA_PLOCAL == 2
  // the exchange-local instance: V1 roles, per-step sync (the host picks it for nothing else)
  if (a->v2 || a->ps_mode) return hipErrorInvalidValue;
  if (fast && relu && sgd) hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, true, 0, true, false>), grid, dim3(256), 0, s, *a);
  else if (fast) hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, true, -1, false, false>), grid, dim3(256), 0, s, *a);
  else hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, false, -1, false, false>), grid, dim3(256), 0, s, *a);
  return hipGetLastError();
#endif
  if (a->v2 && a->bf16) {   // mixed_bfloat16: bf16 shard, bf16-rounded MFMA operands, fp32 masters
    if (fast) hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, true, 0, true, true, false, true>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, false, 0, true, true, false, true>), grid, dim3(256), 0, s, *a);
  } else if (a->v2) {   // the host checked plain SGD + ReLU
    if (fast) hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, true, 0, true, true>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, false, 0, true, true>), grid, dim3(256), 0, s, *a);
  } else if (a->ps_mode) {   // V1 with the in-launch parameter-server exchange
    if (fast && relu && sgd) hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, true, 0, true, false, true>), grid, dim3(256), 0, s, *a);
    else if (fast) hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, true, -1, false, false, true>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, false, -1, false, false, true>), grid, dim3(256), 0, s, *a);
  } else if (fast && relu && sgd) {
    hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, true, 0, true, false>), grid, dim3(256), 0, s, *a);
  } else if (fast) {
    hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, true, -1, false, false>), grid, dim3(256), 0, s, *a);
  } else {
    hipLaunchKernelGGL((mlp_persist_kernel<H0, H1, false, -1, false, false>), grid, dim3(256), 0, s, *a);
  }
  return hipGetLastError();
}

}  // namespace ea

using namespace ea;

#if EA_PLOCAL == 1
#define EA_PERSIST_ENTRY ea_persist_local
#elif EA_PLOCAL == 2
#define EA_PERSIST_ENTRY ea_persist_xlocal
#else
#define EA_PERSIST_ENTRY ea_persist
extern "C" int ea_persist_lds_bytes() { return (int)(LDS_FLOATS * sizeof(float)); }
#endif

// grid: R * wgs workgroups of 256 threads, every one resident (the host sizes the
// grid to at most one workgroup per CU); hidden widths (64, 64), (128, 128), (128, 64)
extern "C" hipError_t EA_PERSIST_ENTRY(const PersistArgs* a, hipStream_t s) {
  if (a->nsteps <= 0) return hipSuccess;
  if (a->H0 == 128 && a->H1 == 128) return persist_launch<128, 128>(a, s);
  if (a->H0 == 64 && a->H1 == 64) return persist_launch<64, 64>(a, s);
  if (a->H0 == 128 && a->H1 == 64) return persist_launch<128, 64>(a, s);
  return hipErrorInvalidValue;
}

#if !EA_PLOCAL
// placement probe: block b stores the XCD it runs on; the host enables the XCD-local
// instance only where blocks b and b + 8 share an XCD across the whole grid
__global__ void xcc_probe_kernel(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = ea::xcc_id();
}
extern "C" hipError_t ea_xcc_probe(int nblocks, unsigned* out, hipStream_t s) {
  hipLaunchKernelGGL(xcc_probe_kernel, dim3(nblocks), dim3(64), 0, s, out);
  return hipGetLastError();
}

namespace ea {
namespace {
// value of element e (of 4) of lane slot u of workgroup q in self-test step i on rank k:
// small integers, so every partial sum is exact in fp32 whatever the order
__device__ __forceinline__ float xr_test_value(int k, int q, int i, int u, int tid, int e) {
  return (float)((k + 1) * ((q % 5) + i + 2) + ((u * 1024 + tid * 4 + e) % 13));
}
}  // namespace

// Numeric self-test of the in-launch rank exchange (xrank_sum) before a trainer trusts it:
// nsteps exchanges of known integer tiles by every owning workgroup q (the tags continue
// the trainer's sequence); every rank checks that each exchanged element equals the exact
// rank sum.  bad[0] += 1 per workgroup and step with a wrong element, += 1 << 16 per
// workgroup that timed out.  corrupt != 0 (fault injection): this rank sends a wrong tile.
__global__ __launch_bounds__(256) void xrank_selftest_kernel(PersistArgs a, int nsteps, unsigned* bad, int corrupt) {
  constexpr int N = PM_XSLOT / 1024;
  const int q = blockIdx.x, tid = threadIdx.x;
  for (int i = 0; i < nsteps; ++i) {
    f32x4 v[N];
#pragma unroll
    for (int u = 0; u < N; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[u][e] = xr_test_value(a.xr_rank, q, i, u, tid, e) + (corrupt ? 0.5f : 0.f);
    if (!xrank_sum<N>(a, q, a.xr_tag0 + (unsigned)i + 1u, v)) {
      if (tid == 0) atomicAdd(bad, 1u << 16);
      return;
    }
    int wrong = 0;
#pragma unroll
    for (int u = 0; u < N; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float want = 0.f;
        for (int k = 0; k < a.xr_world; ++k) want += xr_test_value(k, q, i, u, tid, e);
        wrong |= v[u][e] != want;
      }
    if (__syncthreads_or(wrong) && tid == 0) atomicAdd(bad, 1u);
  }
}

}  // namespace ea

extern "C" hipError_t ea_xrank_selftest(const PersistArgs* a, int nsteps, unsigned* bad, int corrupt, hipStream_t s) {
  hipLaunchKernelGGL(xrank_selftest_kernel, dim3(a->wgs), dim3(256), 0, s, *a, nsteps, bad, corrupt);
  return hipGetLastError();
}
#endif  // !EA_PLOCAL
