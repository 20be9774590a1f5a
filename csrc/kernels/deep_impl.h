// Persistent layer-pipeline training kernel (MI355X / gfx950) -- the kernel templates;
// deep_l{2,3,4,5}.hip instantiate one layer count each (parallel builds), deep.hip dispatches.
//
// Persistent layer-pipeline training kernel (MI355X / gfx950): a whole chunk of training
// steps of a 2..DP_MAXL-layer Dense stack with wide hidden layers in ONE launch.
//
// Why: the Otto MLP (93-512-512-512-9, 8 replicas x B 128, reference examples/
// ml_pipeline_otto.py:57-68) ran as 7 latency-bound launches per step (tail-chain plan,
// 174 us, profiles/README.md); its 512-wide layers do not fit persist.hip's chain roles
// (widths <= 128, B <= 64).  Here a replica is a cluster of nw workgroups of 512 threads
// (8 waves, one workgroup per CU; block b serves replica b % R, so with R = 8 a replica's
// cluster is dispatched to one XCD -- speed only, the protocol never depends on placement).
//
// Ownership (workgroup j, column tile J = [16j, 16j + 16) of every hidden layer):
//   * W_0[:, J] (LDS, transposed [16][Kx0 + 4]) and b_0[J]: the layer-0 forward of the
//     tile and its weight gradient DW_0[:, J] = X^T dZ_0[:, J] -- dZ_0[:, J] is produced by
//     the same workgroup, so layer 0 needs no hand-off in the backward at all;
//   * the ROWS J of W_l, l >= 1 (LDS [16][N16 + 4]) and b_l[J]: the backward stripe
//     dA_{l-1}[:, J] = dZ_l W_l[J, :]^T and DW_l[J, :] = A_{l-1}[:, J]^T dZ_l, both from ONE
//     pass over dZ_l (streamed through LDS in 64-column chunks); after its update the row
//     owner rewrites its 16-column segment of the transposed image W_l^T (workspace) that
//     the forward of the next step reads (columns J of W_l for the owner of output tile J);
//   * the activation-gradient factors G_l = act'(z) keep / (1 - rate) of the forward stay
//     in the registers of the lanes that produce dA_l in the backward (same wave, same
//     lane <-> element map), the activation stripes A_l[:, J] in LDS (the DW operand).
//   The last layer (<= 32 units) is row-parallel: the tail workgroups (16 batch rows each)
//   run its forward, the loss / metrics and dZ_{L-2} rows (G_{L-2} is the one factor that
//   goes through the workspace).
//
// Phases of step s (tags = s * (2L - 2) + phase + 1; every workgroup publishes every phase):
//   FWD_0 -> | FWD_1 -> | ... FWD_{L-2} -> | tail -> | BW_{L-2} (+ DW_{L-1}) -> | ... BW_1 ->
//   then DW_0 of step s runs at the top of step s + 1 (no wait: its inputs are local).
// Hand-offs follow the write-through form of the guide's inter-workgroup protocol
// (cdna_hip_programming.md Guideline 16, R1): every handed-off byte is stored with an sc1
// buffer store and loaded with an sc1 buffer load, every storing wave drains
// (s_waitcnt vmcnt(0)) before the workgroup barrier, one lane stores the phase counter
// (agent-scope relaxed atomic store), one wave polls the replica's counters.  Every spin is
// bounded (timeout -> sticky error word; the host re-plans), the flags are zero at launch.
//
// Semantics are those of the grouped / tail-chain plans (reference elephas/worker.py:41-42 ->
// one Keras fit step per batch): the same dropout masks (dropout_u1 keyed by replica, Dense
// index, optimizer iteration, batch row, column), batch windows, optimizer iterations and
// loss epilogues (loss_tile.h).  Masters are read from P at the start of the launch and
// written back at its end; optimizer state stays in S (read-modify-write by the owner).
#pragma once
#include <mutex>

#include "common.h"
#include "loss_tile.h"

namespace ea {

namespace {

using gu32 = __attribute__((address_space(1))) unsigned;
using rsrc_t = __amdgpu_buffer_rsrc_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

constexpr int NWV = 8;          // waves per workgroup
constexpr int NTH = NWV * 64;   // threads per workgroup
constexpr int CW = DP_CW;       // dZ columns per backward chunk
constexpr int LDZ = CW + 4;     // LDS row stride of a dZ chunk

__device__ __forceinline__ f32x4 z4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// ---- accesses of handed-off bytes: per-lane offset v + uniform offset s, both in floats,
//      through a buffer resource of the replica's workspace.  Stores are write-through (sc1,
//      Guideline 16 R1); loads are PLAIN behind the one agent-scope acquire of every wait
//      (wait_phase / wait_x): a replica's workgroups re-read the same activation and
//      gradient matrices (each of the nw workgroups reads all of A_{l-1} / dZ_l).  Measured
//      on Otto (profiles/deep_stamps_otto_r5_*): sc1 loads with no acquire 107 us per step,
//      plain loads behind the acquire 115 us -- the acquire costs more than the L2 returns --
//      so the loads are sc1 (DP_LOAD_AUX 16, Guideline 16's every-load-sc1 form); 0 switches
//      to the acquire + plain-load form
#ifndef DP_LOAD_AUX
#define DP_LOAD_AUX 16
#endif
// XCD-local instance (deep_l{2..5}_local.hip compile this file again with EA_DLOCAL = 1; fit
// granularity only): block b serves replica b % R, so with R a multiple of 8 a replica's
// workgroups share one XCD (the dispatch deals blocks round-robin over the 8 XCDs; checked
// at launch, PERR_PLACE) and its hand-offs stay in that XCD's L2: stores and phase flags
// plain (the line stays in the L2, where the sc1 loads find it) instead of write-through
// (persist.hip has the measurements)
#ifndef EA_DLOCAL
#define EA_DLOCAL 0
#endif
__device__ __forceinline__ rsrc_t ws_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ f32x4 ld4(rsrc_t r, int v, long long s) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, v * 4, (int)s * 4, DP_LOAD_AUX));
}
__device__ __forceinline__ float ld1(rsrc_t r, int v, long long s) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, v * 4, (int)s * 4, DP_LOAD_AUX));
}
// after the poll: one lane's agent-scope acquire (drops this CU's stale L1 lines), its
// vmcnt drain, then the workgroup barrier -- the other waves' plain loads come after it
__device__ __forceinline__ void acquire_lane0() {
  if (DP_LOAD_AUX == 0 && threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}
constexpr int DP_ST_AUX = EA_DLOCAL ? 0 : 16;   // sc1 (write-through) / plain in the XCD-local instance
__device__ __forceinline__ void st1(rsrc_t r, int v, long long s, float x) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), r, v * 4, (int)s * 4, DP_ST_AUX);
}
__device__ __forceinline__ void st4(rsrc_t r, int v, long long s, f32x4 x) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), r, v * 4, (int)s * 4, DP_ST_AUX);
}
__device__ __forceinline__ void st2(rsrc_t r, int v, long long s, float x0, float x1) {
  const u32x2 u = {__builtin_bit_cast(unsigned, x0), __builtin_bit_cast(unsigned, x1)};
  __builtin_amdgcn_raw_buffer_store_b64(u, r, v * 4, (int)s * 4, DP_ST_AUX);
}
__device__ __forceinline__ f32x4 lds4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void lds4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// 16x16 output tile += A . B over 4 k values per lane group (fp32 MFMA, exact):
// lane group g holds k = 4g .. 4g + 3 of a 16-deep chunk, MFMA e consumes element e
__device__ __forceinline__ void mma4(f32x4& c, f32x4 a, f32x4 b) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
}

// Workgroup barrier for LDS hand-offs only (no vmcnt drain: prefetched global loads stay
// in flight across it)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// kinds: 0 GO (residency), 1 phase counter, 2 / 3 exchange (partial tile out / slice summed)
__device__ __forceinline__ unsigned* dflag(const DeepArgs& a, int r, int kind) {
  return a.flags + ((long long)r * 4 + kind) * DP_MAXWG;
}

// R1 publish of phase `tag`: every storing wave drains its sc1 stores, the workgroup
// meets, one lane raises its phase counter
__device__ __forceinline__ void publish(const DeepArgs& a, int r, int j, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (EA_DLOCAL) __builtin_amdgcn_raw_buffer_store_b32(tag, ws_rsrc(reinterpret_cast<float*>(dflag(a, r, 1) + j)), 0, 0, 0);
    else __hip_atomic_store((gu32*)(dflag(a, r, 1) + j), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// wave 0 polls the phase counters of the replica's nw workgroups (lane q watches q) until
// each reaches tag; false: timed out (error word set)
__device__ __forceinline__ bool wait_phase(const DeepArgs& a, int r, unsigned tag) {
  int ok = 1;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned* f = dflag(a, r, 1) + lane;
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      const unsigned v = lane < a.nw ? __hip_atomic_load((gu32*)(const_cast<unsigned*>(f)), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)
                                     : tag;
      if (__all(v >= tag)) break;
      if ((long long)(wall_clock64() - t0) > a.timeout) {
        ok = 0;
        if (lane == 0) __hip_atomic_store((gu32*)(a.err), (unsigned)PERR_CHAIN_PREV, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  acquire_lane0();
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no load moves above the poll
  return ok != 0;
}

// residency: every workgroup of the grid raised its GO flag (a workgroup that is not
// resident never does: the others time out before touching any state).  The GO value is the
// workgroup's XCD + 1 in the XCD-local instance, where a replica r whose workgroups do not
// all share this one's XCD gives up (PERR_PLACE), state intact
__device__ __forceinline__ unsigned dxcc_go() {
  return EA_DLOCAL ? __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) + 1u : 1u;   // HW_REG_XCC_ID
}
__device__ __forceinline__ bool wait_grid(const DeepArgs& a, int r) {
  int ok = 1;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x, tot = a.R * a.nw;
    const unsigned mine = dxcc_go();
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      bool all = true, away = false;
      for (int f = lane; f < tot; f += 64) {
        const unsigned v = __hip_atomic_load((gu32*)(dflag(a, f % a.R, 0) + f / a.R), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        all &= v != 0u;
        away |= EA_DLOCAL && f % a.R == r && v != 0u && v != mine;
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

__device__ __forceinline__ float dropout_u1(uint32_t base, int row, int c) {
  // the per-column-pair hash of dropout_u8 (common.h): the grouped / row-chain masks
  const uint32_t h = fmix32(base ^ (((uint32_t)row << 16) | (uint32_t)(c >> 1)));
  return (float)((c & 1) ? (h >> 16) : (h & 0xFFFFu)) * (1.0f / 65536.0f);
}

__device__ __forceinline__ void dstamp(const DeepArgs& a, int s, int k) {
  if (a.stamps && threadIdx.x == 0 && s >= 0 && s < DP_STAMP_STEPS)
    a.stamps[((long long)blockIdx.x * DP_STAMP_STEPS + s) * 32 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}

// per-workgroup constants
struct Ctx {
  int r, j, tid, lane, w, g, c16;
  rsrc_t rs;           // the replica's workspace
  rsrc_t xs;           // sync: the exchange buffer (partial tiles, then replica sums)
  long long xp;        // sync: this workgroup's partial tile in it
  float* P;            // the replica's masters
  float* S;            // the replica's optimizer state (null: none)
  int* prow;           // LDS: the batch rows of two steps [2][DP_ROWS] (by step parity)
};

// The lane indices, re-derived from threadIdx.x through an opaque move at the top of every
// phase: otherwise the compiler hoists every per-lane address of every phase out of the
// step loop and, with far more of them than registers, spills them to scratch (~750
// scratch stores before the loop and a scratch load in front of most workspace accesses)
__device__ __forceinline__ Ctx lanes(const Ctx& x0) {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  Ctx x = x0;
  x.tid = t;
  x.lane = t & 63;
  x.g = (t & 63) >> 4;
  x.c16 = t & 15;
  return x;
}

// The optimizer rule of one step (Keras 2.10 optimizer_v2, as common.h opt_update) with its
// per-step scalars hoisted: the decayed learning rate and the Adam / Adamax bias
// corrections are computed once per phase, not per element (the scalar rule inlined at
// every update site cost ~1 KB of scratch per lane in this kernel)
// optimizer instances of the kernel: plain SGD (no state), Adam (the Otto notebook's), every
// other rule through the run-time dispatch
constexpr int OPK_SGD0 = 0, OPK_ADAM = 1, OPK_ANY = 2;
struct OptStep {
  int kind;          // 0 plain SGD, 1 momentum, 2 Nesterov, 3 RMSprop, 4 RMSprop + momentum, 5 Adam,
                     // 6 Adagrad, 7 Adamax
  float lr, lrt;     // decayed lr; Adam / Adamax bias-corrected lr
};
__device__ __forceinline__ OptStep opt_step(const OptParams& p, long long it) {
  OptStep o;
  o.lr = p.lr / (1.f + p.decay * (float)it);
  o.lrt = o.lr;
  const float t = (float)(it + 1);
  switch (p.opt) {
    case OPT_SGD: o.kind = p.mom == 0.f ? 0 : (p.nesterov ? 2 : 1); break;
    case OPT_RMSPROP: o.kind = p.mom > 0.f ? 4 : 3; break;
    case OPT_ADAM: o.kind = 5; o.lrt = o.lr * sqrtf(1.f - powf(p.b2, t)) / (1.f - powf(p.b1, t)); break;
    case OPT_ADAGRAD: o.kind = 6; break;
    default: o.kind = 7; o.lrt = o.lr / (1.f - powf(p.b1, t)); break;
  }
  return o;
}
template <int OPK>
__device__ __forceinline__ float upd(const DeepArgs& a, const Ctx& x, const OptStep& o, long long pi, float w, float g) {
  g *= a.op.grad_scale;
  if constexpr (OPK == OPK_SGD0) {
    return w - o.lr * g;
  } else if constexpr (OPK == OPK_ADAM) {
    const OptParams& p = a.op;
    const float m = p.b1 * x.S[pi] + (1.f - p.b1) * g;
    const float v = p.b2 * x.S[pi + p.s_plane] + (1.f - p.b2) * g * g;
    x.S[pi] = m;
    x.S[pi + p.s_plane] = v;
    return w - o.lrt * m / (sqrtf(v) + p.eps);
  } else {
    const OptParams& p = a.op;
    float* S = x.S;
    const long long s1 = pi + p.s_plane;
    switch (o.kind) {
      case 0: return w - o.lr * g;
      case 1: case 2: {
        const float v = p.mom * S[pi] - o.lr * g;
        S[pi] = v;
        return o.kind == 2 ? w + p.mom * v - o.lr * g : w + v;
      }
      case 3: case 4: {
        const float ms = p.rho * S[pi] + (1.f - p.rho) * g * g;
        S[pi] = ms;
        if (o.kind == 4) {   // tf ApplyRMSProp: epsilon inside the square root
          const float m = p.mom * S[s1] + o.lr * g / sqrtf(ms + p.eps);
          S[s1] = m;
          return w - m;
        }
        return w - o.lr * g / (sqrtf(ms) + p.eps);
      }
      case 5: {
        const float m = p.b1 * S[pi] + (1.f - p.b1) * g;
        const float v = p.b2 * S[s1] + (1.f - p.b2) * g * g;
        S[pi] = m;
        S[s1] = v;
        return w - o.lrt * m / (sqrtf(v) + p.eps);
      }
      case 6: {
        const float ac = S[pi] + g * g;
        S[pi] = ac;
        return w - o.lr * g / (sqrtf(ac) + p.eps);
      }
      default: {
        const float m = p.b1 * S[pi] + (1.f - p.b1) * g;
        const float u = fmaxf(p.b2 * S[s1], fabsf(g));
        S[pi] = m;
        S[s1] = u;
        return w - o.lrt * m / (u + p.eps);
      }
    }
  }
}

// The optimizer state of N elements loaded ahead of their update (upd_p): issued before the
// phase's MFMAs, so a batch of updates waits for one global-load latency, not one per element
// (Adam on Otto: 173 us per step before, every element's state a dependent load).  The same thread updates the same elements every
// step, so its own earlier state stores are what it reads.
template <int N>
struct OptPre {
  float s0[N], s1[N];
};
template <int OPK, int N>
__device__ __forceinline__ void opt_pre(const DeepArgs& a, const Ctx& x, const OptStep& o, const long long (&pi)[N],
                                        const bool (&ok)[N], OptPre<N>& p) {
  if constexpr (OPK != OPK_SGD0) {
    if (OPK == OPK_ANY && o.kind == 0) return;
    const bool two = OPK == OPK_ADAM || o.kind == 4 || o.kind == 5 || o.kind == 7;
#pragma unroll
    for (int n = 0; n < N; ++n) p.s0[n] = ok[n] ? x.S[pi[n]] : 0.f;
    if (two) {
#pragma unroll
      for (int n = 0; n < N; ++n) p.s1[n] = ok[n] ? x.S[pi[n] + a.op.s_plane] : 0.f;
    }
  }
}
// upd with the state values s0 = S[pi], s1 = S[pi + s_plane] already loaded (opt_pre)
template <int OPK>
__device__ __forceinline__ float upd_p(const DeepArgs& a, const Ctx& x, const OptStep& o, long long pi, float w, float g,
                                       float s0, float s1) {
  g *= a.op.grad_scale;
  if constexpr (OPK == OPK_SGD0) {
    return w - o.lr * g;
  } else if constexpr (OPK == OPK_ADAM) {   // the Adam instance: no dispatch on the rule
    const OptParams& p = a.op;
    const float m = p.b1 * s0 + (1.f - p.b1) * g;
    const float v = p.b2 * s1 + (1.f - p.b2) * g * g;
    x.S[pi] = m;
    x.S[pi + p.s_plane] = v;
    return w - o.lrt * m / (sqrtf(v) + p.eps);
  } else {
    const OptParams& p = a.op;
    float* S = x.S;
    const long long i1 = pi + p.s_plane;
    switch (o.kind) {
      case 0: return w - o.lr * g;
      case 1: case 2: {
        const float v = p.mom * s0 - o.lr * g;
        S[pi] = v;
        return o.kind == 2 ? w + p.mom * v - o.lr * g : w + v;
      }
      case 3: case 4: {
        const float ms = p.rho * s0 + (1.f - p.rho) * g * g;
        S[pi] = ms;
        if (o.kind == 4) {
          const float m = p.mom * s1 + o.lr * g / sqrtf(ms + p.eps);
          S[i1] = m;
          return w - m;
        }
        return w - o.lr * g / (sqrtf(ms) + p.eps);
      }
      case 5: {
        const float m = p.b1 * s0 + (1.f - p.b1) * g;
        const float v = p.b2 * s1 + (1.f - p.b2) * g * g;
        S[pi] = m;
        S[i1] = v;
        return w - o.lrt * m / (sqrtf(v) + p.eps);
      }
      case 6: {
        const float ac = s0 + g * g;
        S[pi] = ac;
        return w - o.lr * g / (sqrtf(ac) + p.eps);
      }
      default: {
        const float m = p.b1 * s0 + (1.f - p.b1) * g;
        const float u = fmaxf(p.b2 * s1, fabsf(g));
        S[pi] = m;
        S[i1] = u;
        return w - o.lrt * m / (u + p.eps);
      }
    }
  }
}

// ---- C[16 rows x 16] of one wave: rows from global (loadA(k) -> this lane's float4
//      A[row][k .. k + 3]), B^T from LDS ([16][ldb], k contiguous), over the k-chunks
//      t = kp + KS u.  A register ring of PF chunks is issued (ring_issue) ahead of the
//      consumer; the chunk count is padded to a multiple of PF so that the loop body has
//      no load under a condition (k past Kx reads a clamped address and multiplies zeros)
template <int PF, typename LA>
__device__ __forceinline__ void ring_issue(f32x4 (&ring)[PF], LA loadA, int kp, int KS, int g) {
#pragma unroll
  for (int u = 0; u < PF; ++u) ring[u] = loadA(16 * (kp + KS * u) + 4 * g);
}
template <int PF, typename LA>
__device__ __forceinline__ f32x4 ring_run(f32x4 (&ring)[PF], LA loadA, const float* bt, int ldb, int Kx, int kp, int KS,
                                          int nmine, int lane) {
  const int g = lane >> 4, c = lane & 15;
  f32x4 acc0 = z4(), acc1 = z4();
  for (int u0 = 0; u0 < nmine; u0 += PF) {
#pragma unroll
    for (int v = 0; v < PF; ++v) {
      const int u = u0 + v;
      const int k = 16 * (kp + KS * u) + 4 * g;
      f32x4 av = ring[v];
      ring[v] = loadA(16 * (kp + KS * (u + PF)) + 4 * g);   // clamped by loadA past the end
      const bool kin = k < Kx;
      f32x4 bv = lds4(bt + c * ldb + (kin ? k : 0));
      if (!kin) { av = z4(); bv = z4(); }
      if (v & 1) mma4(acc1, av, bv);
      else mma4(acc0, av, bv);
    }
  }
  return acc0 + acc1;
}

// split-K partials of waves kp > 0 summed into the kp == 0 wave of the row tile (LDS red)
__device__ __forceinline__ f32x4 ks_reduce(const DeepArgs& a, const Ctx& x, float* red, f32x4 acc, int kp) {
  if (a.KS == 1) return acc;
  lds_barrier();   // red is the backward's bias scratch: its last readers are done
  if (kp > 0) lds4(red + ((x.w - a.RT) * 64 + x.lane) * 4, acc);
  lds_barrier();
  if (kp == 0)
    for (int p = 1; p < a.KS; ++p) acc += lds4(red + ((x.w + (p - 1) * a.RT) * 64 + x.lane) * 4);
  lds_barrier();
  return acc;
}

// ---- forward of hidden layer l (column tile j): Z = A_{l-1} W_l[:, J] + b -> act, dropout
//      -> A_l[:, J] (workspace, sc1) + A_l^T stripe (LDS) + G_l (registers) [+ G_{L-2} to
//      the workspace for the tail]
// the W^T rows J of layer l's image (16 x Kx, <= 8 float4 per thread) into registers; for
// l >= 2 issued BEFORE the phase's wait -- the image was rewritten in the previous step's
// BW_l, which every workgroup published before its FWD_0 publication this step
template <int l>
__device__ __forceinline__ void wt_load(const DeepArgs& a, const Ctx& x0, f32x4 (&stg)[8]) {
  const Ctx x = lanes(x0);
  const DeepLayer ly = a.ly[l];
  if (x.j >= ly.T) return;
  const int Kx = ly.Kx, q4n = Kx >> 2, tot = 16 * q4n, J0 = 16 * x.j;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = x.tid + NTH * u, ec = e < tot ? e : tot - 1;
    const int c = ec / q4n, q = ec - c * q4n;
    stg[u] = ld4(x.rs, (J0 + c) * Kx + 4 * q, ly.o_wt);
  }
}

// ---- forward of hidden layer l (column tile j): Z = A_{l-1} W_l[:, J] + b -> act, dropout
//      -> A_l^T stripe (LDS) + G_l (registers), then A_l[:, J] (workspace) as 16-byte rows from
//      the stripe [+ G_{L-2} to the workspace for the tail]
// STAGED (l == 1, fit granularity): the W^T rows are already in the LDS stage (LDS-DMA
// issued at the top of the step, wt_glds)
template <int L, int l, bool STAGED>
__device__ __forceinline__ void fwd_phase(const DeepArgs& a, float* smem, const Ctx& x0, int s, int valid, long long it,
                                          f32x4 (&G)[L - 1], f32x4 (&stg)[8]) {
  const Ctx x = lanes(x0);
  const DeepLayer ly = a.ly[l];
  if (x.j >= ly.T) return;
  const int J0 = 16 * x.j;
  const int rt = x.w % a.RT, kp = x.w / a.RT;
  const int Kx = ly.Kx, nkc = (Kx + 15) >> 4;
  const int m = 16 * rt + x.c16;   // this lane's A row
  f32x4 acc;
  if constexpr (l == 0) {
    constexpr int PF = 8;
    const int nmine = ((nkc - kp + a.KS - 1) / a.KS + PF - 1) / PF * PF;
    const int row = x.prow[(s & 1) * DP_ROWS + m];
    const float* xr = a.X + (long long)x.r * a.sX + (long long)row * a.ldx;
    auto loadA = [&](int k) { return *reinterpret_cast<const f32x4*>(xr + (k < Kx ? k : 0)); };
    f32x4 ring[PF];
    ring_issue<PF>(ring, loadA, kp, a.KS, x.g);
    acc = ring_run<PF>(ring, loadA, smem + ly.l_w, Kx + 4, Kx, kp, a.KS, nmine, x.lane);
  } else {
    constexpr int PF = 16;
    const int nmine = ((nkc - kp + a.KS - 1) / a.KS + PF - 1) / PF * PF;
    const DeepLayer lp = a.ly[l - 1];
    // the W^T rows J (l == 1: loaded here, after the wait), then the A ring
    float* sb = smem + a.l_stage;
    const int q4n = Kx >> 2, tot = 16 * q4n;
    if constexpr (l == 1 && !STAGED) wt_load<l>(a, x, stg);
    auto loadA = [&](int k) { return ld4(x.rs, m * Kx + (k < Kx ? k : 0), lp.o_a); };
    f32x4 ring[PF];
    ring_issue<PF>(ring, loadA, kp, a.KS, x.g);
    if constexpr (!(l == 1 && STAGED)) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = x.tid + NTH * u;
        if (e < tot) {
          const int c = e / q4n, q = e - c * q4n;
          lds4(sb + c * (Kx + 4) + 4 * q, stg[u]);
        }
      }
      lds_barrier();
    }
    if (l == 1) dstamp(a, s, 15);
    acc = ring_run<PF>(ring, loadA, sb, Kx + 4, Kx, kp, a.KS, nmine, x.lane);
    if (l == 1) dstamp(a, s, 16);
  }
  acc = ks_reduce(a, x, smem + a.l_red, acc, kp);
  if (l == 1) dstamp(a, s, 17);
  // epilogue (kp == 0 waves): lane (column c16, group g) holds rows 16 rt + 4 g + q
  float* gst = smem + a.l_red;   // G_{L-2}^T stripe [16][Bp] for the tail (l == L-2)
  if (kp == 0) {
    const int col = J0 + x.c16;
    const float bias = smem[ly.l_b + x.c16];
    float z[4], o[4], gg[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) z[q] = acc[q] + bias;
    act_fg_v<4>(ly.act, z, o, gg);
    const float scale = ly.rate > 0.f ? 1.f / (1.f - ly.rate) : 1.f;
    const uint32_t dbase = dropout_base(a.seed, x.r, l, it);
    f32x4 av, gv;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mm = 16 * rt + 4 * x.g + q;
      const bool live = mm < valid && col < ly.N;
      const float u = (live && ly.rate > 0.f) ? dropout_u1(dbase, mm, col) : 1.f;
      const bool keep = live && u >= ly.rate;
      av[q] = keep ? o[q] * scale : 0.f;
      gv[q] = keep ? gg[q] * scale : 0.f;
    }
    G[l] = gv;
    const int r0 = 16 * rt + 4 * x.g;
    lds4(smem + ly.l_at + x.c16 * (a.Bp + 4) + r0, av);
    if constexpr (l == L - 2) lds4(gst + x.c16 * a.Bp + r0, gv);
  }
  lds_barrier();
  // A_l[:, J] (and G_{L-2}[:, J]) rows out of the stripes: one 16-byte store per 4 columns
  const float* at = smem + ly.l_at;
  for (int e = x.tid; e < a.Bp * 4; e += NTH) {
    const int row = e >> 2, q = e & 3;
    f32x4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = at[(4 * q + k) * (a.Bp + 4) + row];
    st4(x.rs, row * ly.N16 + J0 + 4 * q, ly.o_a, v);
    if constexpr (l == L - 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = gst[(4 * q + k) * a.Bp + row];
      st4(x.rs, row * ly.N16 + J0 + 4 * q, a.o_g, v);
    }
  }
}

// the W^T rows J of layer l straight into the LDS stage by LDS-DMA (global_load_lds, no
// registers): one wave instruction per (row, 1 KB piece); complete once the issuing waves
// drained vmcnt and met at a barrier (publish() does both before the next phase reads it)
template <int l>
__device__ __forceinline__ void wt_glds(const DeepArgs& a, float* smem, const Ctx& x0) {
  const Ctx x = lanes(x0);
  const DeepLayer ly = a.ly[l];
  if (x.j >= ly.T) return;
  const int Kx = ly.Kx, q4n = Kx >> 2, nck = (q4n + 63) >> 6;
  float* sb = smem + a.l_stage;
  const float* src = a.ws + (long long)x.r * a.ws_stride + ly.o_wt + (long long)(16 * x.j) * Kx;
  for (int t = x.w; t < 16 * nck; t += NWV) {
    const int c = t / nck, h = t - c * nck, piece = 64 * h + x.lane;
    if (piece < q4n)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + (long long)c * Kx + 4 * piece),
                                       (__attribute__((address_space(3))) void*)(sb + c * (Kx + 4) + 256 * h), 16, 0,
                                       DP_LOAD_AUX);
  }
}

// ---- tail (row tiles j, j + nw, ...): logits = A_{L-2} W_{L-1} + b, loss / metrics,
//      dZ_{L-1} rows, dZ_{L-2} rows = (dZ_{L-1} W_{L-1}^T) * G_{L-2}
template <int L, bool FAST>
__device__ __forceinline__ void tail_phase(const DeepArgs& a, float* smem, const Ctx& x0, int s, int valid) {
  const Ctx x = lanes(x0);
  const DeepLayer la = a.ly[L - 2], lb = a.ly[L - 1];
  const int C = lb.N, C16 = lb.N16, NCT = C16 >> 4;
  const int Kx = lb.Kx, nkc = Kx >> 4;   // Kx = la.N16
  float* red = smem + a.l_stage;         // [8 waves][2 col tiles][256]
  float* sLg = red + NWV * 2 * 256;      // [16][36] logits -> dZ_{L-1}
  float* sY = sLg + 16 * 36;             // [16][32]
  int* sRow = reinterpret_cast<int*>(sY + 16 * 32);
  const float inv_valid = 1.f / (float)valid;
  for (int rt = x.j; rt < a.RT; rt += a.nw) {
    const int m0 = 16 * rt;
    const int m = m0 + x.c16;
    // ---- logits: wave w takes the k-chunks w, w + 8, ... (<= 8 of them)
    f32x4 av[8], bv0[8], bv1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = x.w + NWV * u, tc = t < nkc ? t : nkc - 1;
      const int k = 16 * tc + 4 * x.g;
      av[u] = ld4(x.rs, m * Kx + k, la.o_a);
      bv0[u] = ld4(x.rs, x.c16 * Kx + k, lb.o_wt);
      bv1[u] = ld4(x.rs, (NCT > 1 ? 16 + x.c16 : x.c16) * Kx + k, lb.o_wt);
    }
    {   // targets of the tile's rows (one element per thread)
      const int row = x.tid >> 5, c = x.tid & 31;
      const int pr = m0 + row < valid ? x.prow[(s & 1) * DP_ROWS + m0 + row] : -1;
      const float yv = (pr >= 0 && c < a.ldy) ? a.Y[(long long)x.r * a.sY + (long long)pr * a.ldy + c] : 0.f;
      sY[row * 32 + c] = yv;
      if (x.tid < 16) sRow[x.tid] = m0 + x.tid < valid ? 1 : -1;
    }
    f32x4 acc0 = z4(), acc1 = z4();
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (x.w + NWV * u < nkc) {
        mma4(acc0, av[u], bv0[u]);
        if (NCT > 1) mma4(acc1, av[u], bv1[u]);
      }
    }
    lds4(red + ((x.w * 2 + 0) * 64 + x.lane) * 4, acc0);
    lds4(red + ((x.w * 2 + 1) * 64 + x.lane) * 4, acc1);
    __syncthreads();
    if (x.tid < 2 * 256) {   // every thread: one logit (2 column tiles x 16 x 16)
      const int ct = x.tid >> 8, e = x.tid & 255, ln = e >> 2, q = e & 3;
      float sum = 0.f;
#pragma unroll
      for (int ww = 0; ww < NWV; ++ww) sum += red[((ww * 2 + ct) * 64 + ln) * 4 + q];
      const int row = 4 * (ln >> 4) + q, col = 16 * ct + (ln & 15);
      const float b = (col < C && lb.has_bias) ? ld1(x.rs, col, a.o_bl) : 0.f;
      sLg[row * 36 + col] = col < C ? sum + b : 0.f;
    }
    __syncthreads();
    if (rt == x.j) dstamp(a, s, 21);
    // ---- loss / metrics; sLg becomes dL/dz * (1 / valid)
    {
      Prob q;
      q.N = C;
      q.act = lb.act;
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
      float sums[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (FAST) {
        if (x.w == 0) {
          if (C <= 16) loss_tile_cce<4, 16, 36, 32>(q, x.r, m0, sLg, sY, sRow, true, inv_valid, sums);
          else loss_tile_cce<8, 16, 36, 32>(q, x.r, m0, sLg, sY, sRow, true, inv_valid, sums);
        }
      } else if (x.tid < 256) {
        loss_tile_lds<16, 36, 32>(q, x.r, m0, sLg, sY, sRow, true, inv_valid, sums);
      }
      if (a.acc && (FAST ? x.w == 0 : x.w < 4)) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          if (i < 2 + a.nmet) {
            const float sv = row_sum<64>(sums[i]);
            if (x.lane == 0 && sv != 0.f) atomicAdd(a.acc + (long long)x.r * a.acc_stride + i, (double)sv);
          }
        }
      }
    }
    __syncthreads();
    if (rt == x.j) dstamp(a, s, 22);
    // ---- dZ_{L-1} rows out; dZ_{L-2} rows = (dZ_{L-1} . W_{L-1}^T) * G_{L-2}: wave w takes
    //      the 16-column tiles w, w + 8, ... of layer L-2 (<= 8 of them)
    for (int e = x.tid; e < 16 * C16; e += NTH) {
      const int row = e / C16, c = e - row * C16;
      st1(x.rs, (m0 + row) * C16 + c, lb.o_dz, sLg[row * 36 + c]);
    }
    const int nit = Kx >> 4;
    f32x4 wb0[8], wb1[8], gq[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int it = x.w + NWV * u, itc = it < nit ? it : nit - 1;
      const int i = 16 * itc + x.c16;
      wb0[u] = ld4(x.rs, i * C16 + 4 * x.g, lb.o_w);
      wb1[u] = ld4(x.rs, i * C16 + (NCT > 1 ? 16 : 0) + 4 * x.g, lb.o_w);
#pragma unroll
      for (int q = 0; q < 4; ++q) gq[u][q] = ld1(x.rs, (m0 + 4 * x.g + q) * Kx + i, a.o_g);
    }
    const f32x4 d0 = lds4(sLg + x.c16 * 36 + 4 * x.g);
    const f32x4 d1 = lds4(sLg + x.c16 * 36 + 16 + 4 * x.g);
    __syncthreads();   // the stage is rewritten below: the dZ_{L-2} rows [16][Kx]
    float* sdz = red;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int it = x.w + NWV * u;
      if (it < nit) {
        f32x4 c = z4();
        mma4(c, d0, wb0[u]);
        if (NCT > 1) mma4(c, d1, wb1[u]);
        const int i = 16 * it + x.c16;
#pragma unroll
        for (int q = 0; q < 4; ++q) sdz[(4 * x.g + q) * Kx + i] = c[q] * gq[u][q];
      }
    }
    __syncthreads();
    for (int e = x.tid; e < 4 * Kx; e += NTH) {   // 16 rows x Kx / 4 float4
      const int row = e / (Kx >> 2), q4 = e - row * (Kx >> 2);
      st4(x.rs, (m0 + row) * Kx + 4 * q4, la.o_dz, lds4(sdz + row * Kx + 4 * q4));
    }
    __syncthreads();   // the LDS tiles are rewritten by the next row tile
  }
}

// ---- weight gradient of the last layer, rows J (= column tile j of layer L-2) and (on
//      workgroup 0) its bias; images of the updated rows for the next tail (SYNC: the
//      gradient goes to the exchange tile instead, the update comes after the replica sum)
template <int L, int OPK, bool SYNC>
__device__ __forceinline__ void dw_last(const DeepArgs& a, float* smem, const Ctx& x0, const OptStep& os) {
  const Ctx x = lanes(x0);
  const DeepLayer la = a.ly[L - 2], lb = a.ly[L - 1];
  const int C = lb.N, C16 = lb.N16, NCT = C16 >> 4, ldc = C16 + 4;
  const bool rows = x.j < la.T, bias = x.j == 0 && lb.has_bias;
  if (!rows && !bias) return;
  // the bias element's optimizer state, loaded before the dZ staging (the last wave: one unit per lane)
  const bool bl_ok = !SYNC && bias && x.tid >= 448 && x.tid - 448 < C;
  OptPre<1> bpre;
  {
    const long long pb[1] = {lb.p_off + (long long)lb.K * C + (x.tid >= 448 ? x.tid - 448 : 0)};
    const bool okb[1] = {bl_ok};
    opt_pre<SYNC ? OPK_SGD0 : OPK, 1>(a, x, os, pb, okb, bpre);
  }
  float* sd = smem + a.l_stage;   // dZ_{L-1} [Bp][C16 + 4]
  const int q4n = C16 >> 2, tot = a.Bp * q4n;
  for (int e = x.tid; e < tot; e += NTH) {
    const int row = e / q4n, q = e - row * q4n;
    lds4(sd + row * ldc + 4 * q, ld4(x.rs, row * C16 + 4 * q, lb.o_dz));
  }
  __syncthreads();
  if (rows && x.w < NCT) {
    const int ct = x.w, I0 = 16 * x.j, ldat = a.Bp + 4;
    const float* at = smem + la.l_at;
    const int c = 16 * ct + x.c16;
    long long pi[4];
    bool ok[4];
    OptPre<4> pre;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pi[q] = lb.p_off + (long long)(I0 + 4 * x.g + q) * C + c;
      ok[q] = !SYNC && I0 + 4 * x.g + q < lb.K && c < C;
    }
    opt_pre<SYNC ? OPK_SGD0 : OPK, 4>(a, x, os, pi, ok, pre);
    f32x4 acc = z4();
    for (int rr = 0; rr < (a.Bp >> 4); ++rr) {
      const f32x4 av = lds4(at + x.c16 * ldat + 16 * rr + 4 * x.g);
      f32x4 b;
#pragma unroll
      for (int e = 0; e < 4; ++e) b[e] = sd[(16 * rr + 4 * x.g + e) * ldc + 16 * ct + x.c16];
      mma4(acc, av, b);
    }
    float* wr = smem + lb.l_w;
    if constexpr (SYNC) {
#pragma unroll
      for (int q = 0; q < 4; ++q) st1(x.xs, (4 * x.g + q) * C16 + c, x.xp + a.x_w[L - 1], acc[q]);
    } else {
      f32x4 wv;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ip = 4 * x.g + q;
        float wt = wr[ip * ldc + c];
        if (ok[q]) {
          wt = upd_p<OPK>(a, x, os, pi[q], wt, acc[q], pre.s0[q], pre.s1[q]);
          wr[ip * ldc + c] = wt;
          st1(x.rs, (I0 + ip) * C16 + c, lb.o_w, wt);
        }
        wv[q] = wt;
      }
      st4(x.rs, c * lb.Kx + I0 + 4 * x.g, lb.o_wt, wv);
    }
  }
  if (bias && x.tid >= 448 && x.tid - 448 < C) {   // the last wave: one unit per lane
    const int c = x.tid - 448;
    float db = 0.f;
    for (int row = 0; row < a.Bp; ++row) db += sd[row * ldc + c];
    if constexpr (SYNC) {
      st1(x.xs, c, x.xp + a.x_b[L - 1], db);
    } else {
      float* bl = smem + lb.l_b;
      const float b = upd_p<OPK>(a, x, os, lb.p_off + (long long)lb.K * C + c, bl[c], db, bpre.s0[0], bpre.s1[0]);
      bl[c] = b;
      st1(x.rs, c, a.o_bl, b);
    }
  }
  __syncthreads();   // the staging is reused by the next phase
}

// ---- column sums of dZ_l[:, J] (the bias gradient of tile j of layer l) -> b_l[J]
template <int l, int OPK, bool SYNC>
__device__ __forceinline__ void bias_tile(const DeepArgs& a, float* smem, const Ctx& x0, long long o_dz, int N16,
                                          const OptStep& os) {
  const Ctx x = lanes(x0);
  const DeepLayer ly = a.ly[l];
  if (x.j >= ly.T || !ly.has_bias) return;
  const int J0 = 16 * x.j, c = x.tid & 15;
  OptPre<1> bpre;   // the bias element's optimizer state, ahead of the column sums
  {
    const long long pb[1] = {ly.p_off + (long long)ly.K * ly.N + J0 + c};
    const bool okb[1] = {!SYNC && x.tid < 16 && J0 + x.tid < ly.N};
    opt_pre<SYNC ? OPK_SGD0 : OPK, 1>(a, x, os, pb, okb, bpre);
  }
  float sm = 0.f;
#pragma unroll
  for (int k = 0; k < DP_ROWS / 32; ++k) {
    const int row = (x.tid >> 4) + 32 * k;
    const float v = ld1(x.rs, (row < a.Bp ? row : 0) * N16 + J0 + c, o_dz);
    sm += row < a.Bp ? v : 0.f;
  }
  float* red = smem + a.l_red;
  red[x.tid] = sm;
  __syncthreads();
  if (x.tid < 16 && J0 + x.tid < ly.N) {
    float db = 0.f;
    for (int k = 0; k < NTH / 16; ++k) db += red[x.tid + 16 * k];
    if constexpr (SYNC) {
      st1(x.xs, x.tid, x.xp + a.x_b[l], db);
    } else {
      float* bt = smem + ly.l_b;
      bt[x.tid] = upd_p<OPK>(a, x, os, ly.p_off + (long long)ly.K * ly.N + J0 + x.tid, bt[x.tid], db, bpre.s0[0],
                             bpre.s1[0]);
    }
  }
  __syncthreads();
}

// ---- backward of layer l >= 1 on row tile J of W_l: one pass over dZ_l in 64-column
//      chunks (LDS): dA_{l-1}[:, J] += dZ_chunk W_l[J, chunk]^T (waves = row tiles) and
//      DW_l[J, chunk] = A_{l-1}[:, J]^T dZ_chunk (waves = 4 column tiles x 2 row halves),
//      update of the chunk's masters + their W^T image segment; finally dZ_{l-1}[:, J] =
//      dA * G_{l-1} -> workspace (l >= 2) or the LDS dZ_0^T stripe (l = 1)
template <int L, int l, int OPK, bool SYNC>
__device__ __forceinline__ void bw_phase(const DeepArgs& a, float* smem, const Ctx& x0, const OptStep& os,
                                         const f32x4 (&G)[L - 1], int s) {
  const Ctx x = lanes(x0);
  const DeepLayer lp = a.ly[l - 1], ly = a.ly[l];
  if (x.j >= lp.T) {   // no row tile of W_l here; maybe its bias tile (layer l wider than l - 1)
    bias_tile<l, OPK, SYNC>(a, smem, x, ly.o_dz, ly.N16, os);
    return;
  }
  // this workgroup's bias tile j of layer l: summed from the staged chunk that holds it
  const bool btile = x.j < ly.T && ly.has_bias;
  const int hb = (16 * x.j) / CW, cb = 16 * x.j - hb * CW;

  const int I0 = 16 * x.j, Bp = a.Bp, ldat = Bp + 4, ldr = ly.N16 + 4;
  const int rt = x.w % a.RT, kp = x.w / a.RT;
  const int f = x.w & 3, hh = x.w >> 2;
  float* wr = smem + ly.l_w;
  const float* at = smem + lp.l_at;
  float* sdz = smem + a.l_stage;
  // [4][64][4] DW partials, double-buffered by chunk parity: both row halves finish a chunk's
  // update at the top of the NEXT chunk, beside the MFMAs, each for 2 of a lane's 4 rows
  // (half hh: rows 4 g + 2 hh + {0, 1}) -- slots {0, 1} hold the second half's partials of
  // the first half's rows, slots {2, 3} the first half's of the second's.  (One half doing
  // all 4 put the whole update on that half's path to every chunk barrier: Adam on Otto
  // spent +7 us per 512-wide layer there.)  The second buffer is the dZ_0^T stripe, free
  // until the phase's end.
  float* spbuf[2] = {sdz + DP_ROWS * LDZ, smem + a.l_dz0};
  const int nch = (ly.N16 + CW - 1) / CW;
  // chunk staging: Bp x 64 floats = Bp * 16 float4, <= 4 per thread, two chunks ahead
  // (register sets A / B alternate; the loop is unrolled by two so their indices stay static)
  f32x4 preA[4], preB[4];
  auto load_chunk = [&](int h, f32x4 (&pre)[4]) {
    const int c0 = h * CW;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = x.tid + NTH * u, row = e >> 4, q = e & 15;
      const int cc = c0 + 4 * q < ly.N16 ? c0 + 4 * q : c0;
      pre[u] = ld4(x.rs, (row < Bp ? row : 0) * ly.N16 + cc, ly.o_dz);
    }
  };
  load_chunk(0, preA);
  if (nch > 1) load_chunk(1, preB);
  f32x4 accB0 = z4(), accB1 = z4();
  f32x4 accWp = z4();   // this wave's DW partial of the previous chunk (first row half: pending update)
  // optimizer state of the elements finish(h) updates, loaded at the top of chunk h (stN), in
  // use one chunk later (stC)
  const int q0 = 2 * hh;   // this half's rows of a lane: 4 g + q0 + {0, 1}
  OptPre<2> stC, stN;
  auto state_pre = [&](int h, OptPre<2>& st) {
    const int c0 = h * CW, cw = ly.N16 - c0 < CW ? ly.N16 - c0 : CW;
    if (SYNC || 16 * f >= cw) return;
    const int col = c0 + 16 * f + x.c16;
    long long pi[2];
    bool ok[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      pi[q] = ly.p_off + (long long)(I0 + 4 * x.g + q0 + q) * ly.N + col;
      ok[q] = I0 + 4 * x.g + q0 + q < ly.K && col < ly.N;
    }
    opt_pre<SYNC ? OPK_SGD0 : OPK, 2>(a, x, os, pi, ok, st);
  };
  // the first-half waves complete chunk hq's rows J: partial sums, update of the masters of
  // the chunk's columns and their W^T image segment (SYNC: the gradient to the exchange tile)
  auto finish = [&](int hq, f32x4 accq) {
    const int c0 = hq * CW, cw = ly.N16 - c0 < CW ? ly.N16 - c0 : CW;
    if (16 * f >= cw) return;
    const f32x4 other = lds4(spbuf[hq & 1] + (f * 64 + x.lane) * 4);
    float gq[2];
    gq[0] = (hh ? accq[2] : accq[0]) + (hh ? other[2] : other[0]);
    gq[1] = (hh ? accq[3] : accq[1]) + (hh ? other[3] : other[1]);
    const int col = c0 + 16 * f + x.c16;
    if constexpr (SYNC) {
#pragma unroll
      for (int q = 0; q < 2; ++q) st1(x.xs, (4 * x.g + q0 + q) * ly.N16 + col, x.xp + a.x_w[l], gq[q]);
    } else {
      float wv[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ip = 4 * x.g + q0 + q;
        float wt = wr[ip * ldr + col];
        if (I0 + ip < ly.K && col < ly.N) {
          wt = upd_p<OPK>(a, x, os, ly.p_off + (long long)(I0 + ip) * ly.N + col, wt, gq[q], stC.s0[q], stC.s1[q]);
          wr[ip * ldr + col] = wt;
        }
        wv[q] = wt;
      }
      st2(x.rs, col * ly.Kx + I0 + 4 * x.g + q0, ly.o_wt, wv[0], wv[1]);
    }
  };
  auto chunk = [&](int h, f32x4 (&pre)[4]) {
    const int c0 = h * CW, cw = ly.N16 - c0 < CW ? ly.N16 - c0 : CW;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = x.tid + NTH * u, row = e >> 4, q = e & 15;
      if (row < Bp) lds4(sdz + row * LDZ + 4 * q, 4 * q < cw ? pre[u] : z4());
    }
    if (h + 2 < nch) load_chunk(h + 2, pre);   // two chunks in flight ahead of the consumer
    state_pre(h, stN);
    lds_barrier();
    if (h > 0) finish(h - 1, accWp);
    stC = stN;
    // dA_{l-1}[rows of tile rt][J] over the chunk's 16-column groups t (t % KS == kp)
#pragma unroll
    for (int t = 0; t < CW / 16; ++t) {
      if (t % a.KS == kp && 16 * t < cw) {
        const f32x4 av = lds4(sdz + (16 * rt + x.c16) * LDZ + 16 * t + 4 * x.g);
        const f32x4 bv = lds4(wr + x.c16 * ldr + c0 + 16 * t + 4 * x.g);
        if (t & 1) mma4(accB1, av, bv);
        else mma4(accB0, av, bv);
      }
    }
    // DW_l[J][chunk column tile f] over the row half hh
    f32x4 accW = z4();
    if (16 * f < cw) {
      for (int rr = hh; rr < (Bp >> 4); rr += 2) {
        const f32x4 av = lds4(at + x.c16 * ldat + 16 * rr + 4 * x.g);
        f32x4 b;
#pragma unroll
        for (int e = 0; e < 4; ++e) b[e] = sdz[(16 * rr + 4 * x.g + e) * LDZ + 16 * f + x.c16];
        mma4(accW, av, b);
      }
    }
    float* bred = smem + a.l_red;
    if (btile && h == hb && x.tid < 256) {   // bias: 16 columns x 16 row groups of Bp / 16 rows
      const int c = x.tid & 15, rg = x.tid >> 4, rows = Bp >> 4;
      float sm = 0.f;
      for (int rr = 0; rr < rows; ++rr) sm += sdz[(rg * rows + rr) * LDZ + cb + c];
      bred[x.tid] = sm;
    }
    {   // the other half's rows of this lane: half 1 -> slots 0, 1; half 0 -> slots 2, 3
      float* sp = spbuf[h & 1] + (f * 64 + x.lane) * 4 + (hh ? 0 : 2);
      sp[0] = hh ? accW[0] : accW[2];
      sp[1] = hh ? accW[1] : accW[3];
    }
    accWp = accW;
    lds_barrier();   // every read of the chunk is done, the partials are out
    if (btile && h == hb && x.tid < 16 && 16 * x.j + x.tid < ly.N) {
      float db = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) db += bred[x.tid + 16 * k];
      if constexpr (SYNC) {
        st1(x.xs, x.tid, x.xp + a.x_b[l], db);
      } else {
        float* bt = smem + ly.l_b;
        bt[x.tid] = upd<OPK>(a, x, os, ly.p_off + (long long)ly.K * ly.N + 16 * x.j + x.tid, bt[x.tid], db);
      }
    }
  };
  for (int h = 0; h < nch; h += 2) {
    chunk(h, preA);
    if (l == L - 2 && h == 0) dstamp(a, s, 18);
    if (h + 1 < nch) chunk(h + 1, preB);
  }
  finish(nch - 1, accWp);   // the last chunk's partials are out since its barrier
  if (l == L - 2) dstamp(a, s, 19);
  f32x4 acc = ks_reduce(a, x, smem + a.l_red, accB0 + accB1, kp);
  // dZ_{l-1}[:, J] = dA * G_{l-1} -> the LDS dZ^T stripe (l = 1: layer 0's DW operand; l >= 2:
  // staging of the 16-byte row stores below -- BW_1 rewrites the stripe after them); the
  // stripe held the second partial buffer until the last finish
  if (a.KS == 1) lds_barrier();
  if (kp == 0) {
    const int r0 = 16 * rt + 4 * x.g;
    f32x4 dz;
#pragma unroll
    for (int q = 0; q < 4; ++q) dz[q] = acc[q] * G[l - 1][q];
    lds4(smem + a.l_dz0 + x.c16 * ldat + r0, dz);
  }
  if constexpr (l >= 2) {
    lds_barrier();
    const float* st = smem + a.l_dz0;
    for (int e = x.tid; e < Bp * 4; e += NTH) {
      const int row = e >> 2, q = e & 3;
      f32x4 v;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = st[(4 * q + k) * ldat + row];
      st4(x.rs, row * lp.N16 + I0 + 4 * q, lp.o_dz, v);
    }
  }
}

// ---- layer-0 weight gradient of tile j for the step whose dZ_0^T stripe is in LDS:
//      DW_0[:, J] = X^T dZ_0[:, J] (waves = 64-feature groups; the X rows of that step,
//      float4 along the features: MFMA e of lane group g takes batch row 16 rr + 4 g + e,
//      output tile f the features i0 + 4 m + f), bias, in-place update of W_0^T
template <int L, int OPK, bool SYNC>
__device__ __forceinline__ void dw0_phase(const DeepArgs& a, float* smem, const Ctx& x0, int sp, const OptStep& os) {
  const Ctx x = lanes(x0);
  const DeepLayer l0 = a.ly[0];
  if (x.j >= l0.T) return;
  const int J0 = 16 * x.j, Bp = a.Bp, ldz = Bp + 4, Kx = l0.Kx, ld0 = Kx + 4;
  float* w0t = smem + l0.l_w;
  const float* dz0 = smem + a.l_dz0;
  if (x.tid < 16 && l0.has_bias && J0 + x.tid < l0.N) {
    OptPre<1> bpre;   // the state load overlaps the column sum
    const long long pb[1] = {l0.p_off + (long long)l0.K * l0.N + J0 + x.tid};
    const bool okb[1] = {!SYNC};
    opt_pre<SYNC ? OPK_SGD0 : OPK, 1>(a, x, os, pb, okb, bpre);
    float db = 0.f;
    for (int row = 0; row < Bp; ++row) db += dz0[x.tid * ldz + row];
    if constexpr (SYNC) {
      st1(x.xs, x.tid, x.xp + a.x_b0, db);
    } else {
      float* bt = smem + l0.l_b;
      bt[x.tid] = upd_p<OPK>(a, x, os, pb[0], bt[x.tid], db, bpre.s0[0], bpre.s1[0]);
    }
  }
  const int nfg = (Kx + 63) >> 6;
  const int* prow = x.prow + (sp & 1) * DP_ROWS;
  const float* Xr = a.X + (long long)x.r * a.sX;
  // A stateful rule on a narrow input layer (Otto: 93 features = 2 of the 8 waves) updates
  // through the LDS: the MFMA waves park their sums in the dead dZ_0 stripe + reduction
  // buffer and all 8 waves run the update (the state loads and the Adam math of 16 elements
  // per lane of 2 waves were 5.3 of the 22 us Adam added per Otto step)
  // (L >= 3 only: a two-layer stack keeps the one-wave-per-feature-group update -- with the
  // LDS path compiled in, its Adam kernel's results varied run to run on the GPU)
  constexpr bool STATEFUL = !SYNC && OPK != OPK_SGD0 && L >= 3;
  const int scr_n = (16 * ldz > 1024 ? 16 * ldz : 1024) + 2048;   // l_dz0 + l_red (executor.cpp)
  const bool spread = STATEFUL && nfg <= NWV && 16 * Kx <= scr_n && !(OPK == OPK_ANY && os.kind == 0);
  f32x4 keep[4] = {z4(), z4(), z4(), z4()};
  for (int fg = x.w; fg < nfg; fg += NWV) {
    const int i0 = 64 * fg, ic = i0 + 4 * x.c16;
    const bool fin = ic < Kx;
    const int col = J0 + x.c16;
    f32x4 acc[4] = {z4(), z4(), z4(), z4()};
    // two passes of 4 row groups: 16 float4 of X in flight per lane
#pragma unroll
    for (int half = 0; half < DP_ROWS / 64; ++half) {
      f32x4 xv[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = 4 * half + q;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rw = 16 * rr + 4 * x.g + e;
          const int row = prow[rw < Bp ? rw : 0];
          xv[q][e] = *reinterpret_cast<const f32x4*>(Xr + (long long)row * a.ldx + (fin ? ic : 0));
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = 4 * half + q;
        if (16 * rr < Bp) {
          const f32x4 b = lds4(dz0 + x.c16 * ldz + 16 * rr + 4 * x.g);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x4 xe = fin ? xv[q][e] : z4();
#pragma unroll
            for (int ff = 0; ff < 4; ++ff)
              acc[ff] = __builtin_amdgcn_mfma_f32_16x16x4f32(xe[ff], b[e], acc[ff], 0, 0, 0);
          }
        }
      }
    }
    if (spread) {
#pragma unroll
      for (int ff = 0; ff < 4; ++ff) keep[ff] = acc[ff];
      continue;
    }
    // lane (column c16, group g): features i0 + 16 g + 4 q + f of column J0 + c16; the
    // optimizer state of its 16 elements loaded at once (after the MFMAs: the X rows'
    // registers are free by then)
    long long pi[16];
    bool ok[16];
    OptPre<16> pre;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int ff = 0; ff < 4; ++ff) {
        const int i = i0 + 16 * x.g + 4 * q + ff;
        pi[4 * q + ff] = l0.p_off + (long long)i * l0.N + col;
        ok[4 * q + ff] = !SYNC && i < l0.K && col < l0.N;
      }
    opt_pre<SYNC ? OPK_SGD0 : OPK, 16>(a, x, os, pi, ok, pre);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ib = i0 + 16 * x.g + 4 * q;
      if (ib >= Kx) continue;
      if constexpr (SYNC) {   // W_0[:, J]^T gradient, [16][Kx0] in the exchange tile
        st4(x.xs, x.c16 * Kx + ib, x.xp, f32x4{acc[0][q], acc[1][q], acc[2][q], acc[3][q]});
        continue;
      }
      f32x4 wv = lds4(w0t + x.c16 * ld0 + ib);
#pragma unroll
      for (int ff = 0; ff < 4; ++ff) {
        if (ok[4 * q + ff])
          wv[ff] = upd_p<OPK>(a, x, os, pi[4 * q + ff], wv[ff], acc[ff][q], pre.s0[4 * q + ff], pre.s1[4 * q + ff]);
      }
      lds4(w0t + x.c16 * ld0 + ib, wv);
    }
  }
  if constexpr (STATEFUL) {
    if (!spread) return;
    float* scr = smem + a.l_dz0;   // [Kx][16]: feature-major, a column's 16 lanes contiguous
    __syncthreads();               // every dZ_0 read (the MFMAs, the bias sums) is done
    if (x.w < nfg) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int ff = 0; ff < 4; ++ff) {
          const int i = 64 * x.w + 16 * x.g + 4 * q + ff;
          if (i < Kx) scr[i * 16 + x.c16] = keep[ff][q];
        }
    }
    __syncthreads();
    constexpr int PE = 4;
    for (int e0 = 0; e0 < 16 * l0.K; e0 += PE * NTH) {
      long long pi[PE];
      bool ok[PE];
      OptPre<PE> pre;
#pragma unroll
      for (int u = 0; u < PE; ++u) {
        const int e = e0 + u * NTH + x.tid, i = e >> 4, c = e & 15;
        pi[u] = l0.p_off + (long long)i * l0.N + J0 + c;
        ok[u] = e < 16 * l0.K && J0 + c < l0.N;
      }
      opt_pre<OPK, PE>(a, x, os, pi, ok, pre);
#pragma unroll
      for (int u = 0; u < PE; ++u) {
        if (!ok[u]) continue;
        const int e = e0 + u * NTH + x.tid, i = e >> 4, c = e & 15;
        float* w = w0t + c * ld0 + i;
        *w = upd_p<OPK>(a, x, os, pi[u], *w, scr[e], pre.s0[u], pre.s1[u]);
      }
    }
  }
}

// dZ_0[:, J] of a two-layer stack comes from the tail (workspace): -> the LDS dZ_0^T stripe
__device__ __forceinline__ void load_dz0(const DeepArgs& a, float* smem, const Ctx& x0) {
  const Ctx x = lanes(x0);
  const DeepLayer l0 = a.ly[0];
  if (x.j >= l0.T) return;
  const int ldz = a.Bp + 4, J0 = 16 * x.j;
  float* dz0 = smem + a.l_dz0;
  for (int e = x.tid; e < a.Bp * 4; e += NTH) {
    const int row = e >> 2, q = e & 3;
    const f32x4 v = ld4(x.rs, row * l0.N16 + J0 + 4 * q, l0.o_dz);
#pragma unroll
    for (int k = 0; k < 4; ++k) dz0[(4 * q + k) * ldz + row] = v[k];
  }
}


// the forward phases of layers l .. L-2 (compile-time chain: every layer index is static)
template <int L, int l, bool STAGED>
__device__ __forceinline__ bool fwd_chain(const DeepArgs& a, float* smem, const Ctx& x, int s, int valid, long long it,
                                          unsigned base, f32x4 (&G)[L - 1]) {
  if constexpr (l <= L - 2) {
    f32x4 stg[8];
    if constexpr (l >= 2) wt_load<l>(a, x, stg);   // ready since this step's FWD_0 publications
    if (!wait_phase(a, x.r, base + l)) return false;
    dstamp(a, s, 2 * l + 1);
    fwd_phase<L, l, STAGED>(a, smem, x, s, valid, it, G, stg);
    publish(a, x.r, x.j, base + l + 1);
    dstamp(a, s, 2 * l + 2);
    return fwd_chain<L, l + 1, STAGED>(a, smem, x, s, valid, it, base, G);
  }
  return true;
}

// the backward phases of layers l .. 1 (BW_{L-2} also runs the last layer's update)
template <int L, int l, int OPK, bool SYNC>
__device__ __forceinline__ bool bw_chain(const DeepArgs& a, float* smem, const Ctx& x, int s, const OptStep& os,
                                         unsigned base, const f32x4 (&G)[L - 1]) {
  if constexpr (l >= 1) {
    const unsigned p = (unsigned)(L + (L - 2 - l));
    if (!wait_phase(a, x.r, base + p)) return false;
    dstamp(a, s, 11 + 2 * (L - 2 - l));
    if constexpr (l == L - 2) {
      dw_last<L, OPK, SYNC>(a, smem, x, os);
      dstamp(a, s, 23);
    }
    bw_phase<L, l, OPK, SYNC>(a, smem, x, os, G, s);
    publish(a, x.r, x.j, base + p + 1);
    dstamp(a, s, 12 + 2 * (L - 2 - l));
    return bw_chain<L, l - 1, OPK, SYNC>(a, smem, x, s, os, base, G);
  }
  return true;
}

// ---- per-step synchronous replicas: the exchange of workgroup j's weight-gradient tile
//      with workgroup j of every other replica (flag kinds 2 / 3, tag = step + 1)
__device__ __forceinline__ void publish_x(const DeepArgs& a, const Ctx& x, int kind, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store((gu32*)(dflag(a, x.r, kind) + x.j), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool wait_x(const DeepArgs& a, int j, int kind, unsigned tag) {
  int ok = 1;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      bool all = true;
      for (int rr = lane; rr < a.R; rr += 64)
        all &= __hip_atomic_load((gu32*)(dflag(a, rr, kind) + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= tag;
      if (__all(all)) break;
      if ((long long)(wall_clock64() - t0) > a.timeout) {
        ok = 0;
        if (lane == 0) __hip_atomic_store((gu32*)(a.err), (unsigned)PERR_CHAIN_PREV, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  acquire_lane0();
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok != 0;
}

// ---- rank exchange (xr_world > 1; layout args.h DeepArgs, peer_args.h): rank k's buffer by
//      selects against the uniform bases (no per-lane indexing of the kernel arguments)
__device__ __forceinline__ char* xr_base_of(const DeepArgs& a, int k) {
  char* b = a.xr_base[0];
#pragma unroll
  for (int kk = 1; kk < PEER_MAX_RANKS; ++kk) b = (k == kk) ? a.xr_base[kk] : b;
  return b;
}
// this rank's slot of flag `slot` raised to tag (every storing wave drained first, release at
// system scope), then wave 0 waits until every rank's flag `slot` reached it (lane k watches
// rank k; wrap-safe: tags only grow).  false: a rank did not arrive within xr_timeout
__device__ __forceinline__ bool deep_xrank_wait(const DeepArgs& a, int slot, unsigned tag) {
  const int tid = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    __hip_atomic_store(reinterpret_cast<unsigned*>(xr_base_of(a, a.xr_rank) + PEER_FLAG_OFF + (long long)slot * 64), tag,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  int ok = 1;
  if (tid < 64) {
    const unsigned* fl = reinterpret_cast<const unsigned*>(xr_base_of(a, tid < a.xr_world ? tid : 0) + PEER_FLAG_OFF +
                                                           (long long)slot * 64);
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      const unsigned f = tid < a.xr_world ? __hip_atomic_load(const_cast<unsigned*>(fl), __ATOMIC_ACQUIRE,
                                                              __HIP_MEMORY_SCOPE_SYSTEM)
                                          : tag;
      if (__all((int)(f - tag) >= 0)) break;
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
  return ok != 0;
}

// ---- parameter-server hook (ps_mode; server layout peer_args.h PsArgs, kernels peer.hip):
//      theta element i lives in the shard of the rank owning its chunk, in uncached memory
__device__ __forceinline__ float* dps_elem(const PsArgs& ps, long long i) {
  char* b = ps.base[0];
#pragma unroll
  for (int rr = 1; rr < PEER_MAX_RANKS; ++rr) b = (rr < ps.world && i >= ps.shard_begin[rr]) ? ps.base[rr] : b;
  return reinterpret_cast<float*>(b + PEER_DATA_OFF) + i;
}
__device__ __forceinline__ unsigned* dps_ctr(const PsArgs& ps, int slice, int which) {
  return reinterpret_cast<unsigned*>(ps.base[0] + PEER_FLAG_OFF + (long long)which * PEER_MAX_BLOCKS * 64 +
                                     (long long)slice * 64);
}
// push bracket of slice j (asynchronous mode: a puller copies a slice only while no pusher is
// inside it); hogwild: no bracket
__device__ __forceinline__ void dps_push_begin(const DeepArgs& a, int slice) {
  if (a.ps_mode == 2 && threadIdx.x == 0)
    __hip_atomic_fetch_add(dps_ctr(a.ps, slice, 0), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
}
__device__ __forceinline__ void dps_push_end(const DeepArgs& a, int slice) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (a.ps_mode == 2 && threadIdx.x == 0)
    __hip_atomic_fetch_add(dps_ctr(a.ps, slice, 1), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the masters workgroup j owns -- W_0[:, J] (transposed tile), b_0[J], rows J of W_l (l >= 1),
// b_l[J] of the hidden layers, the last layer's bias on workgroup 0 -- from src(i) (element i
// of the flat parameter vector) into LDS
template <int L, typename Src>
__device__ __forceinline__ void load_masters(const DeepArgs& a, float* smem, const Ctx& x, Src src) {
  {
    const DeepLayer l0 = a.ly[0];
    if (x.j < l0.T) {
      const int J0 = 16 * x.j, ld0 = l0.Kx + 4;
      for (int e = x.tid; e < 16 * l0.K; e += NTH) {
        const int k = e >> 4, c = e & 15;
        if (J0 + c < l0.N) smem[l0.l_w + c * ld0 + k] = src(l0.p_off + (long long)k * l0.N + J0 + c);
      }
      if (x.tid < 16 && l0.has_bias && J0 + x.tid < l0.N)
        smem[l0.l_b + x.tid] = src(l0.p_off + (long long)l0.K * l0.N + J0 + x.tid);
    }
  }
#pragma unroll
  for (int l = 1; l < L; ++l) {
    const DeepLayer ly = a.ly[l], lp = a.ly[l - 1];
    const int ldr = ly.N16 + 4;
    if (x.j < lp.T) {   // rows J of W_l
      const int I0 = 16 * x.j;
      for (int e = x.tid; e < 16 * ly.N; e += NTH) {
        const int ip = e / ly.N, c = e - ip * ly.N;
        if (I0 + ip < ly.K) smem[ly.l_w + ip * ldr + c] = src(ly.p_off + (long long)(I0 + ip) * ly.N + c);
      }
    }
    if (l < L - 1) {
      if (x.j < ly.T && x.tid < 16 && ly.has_bias && 16 * x.j + x.tid < ly.N)
        smem[ly.l_b + x.tid] = src(ly.p_off + (long long)ly.K * ly.N + 16 * x.j + x.tid);
    } else if (x.j == 0 && ly.has_bias && x.tid < ly.N) {
      smem[ly.l_b + x.tid] = src(ly.p_off + (long long)ly.K * ly.N + x.tid);
    }
  }
}

// the images the other workgroups read: W_l^T segments [c][J] (l >= 1), the last layer's
// row-major rows and (workgroup 0) its bias -- from the LDS masters
template <int L>
__device__ __forceinline__ void write_images(const DeepArgs& a, float* smem, const Ctx& x) {
#pragma unroll
  for (int l = 1; l < L; ++l) {
    const DeepLayer ly = a.ly[l], lp = a.ly[l - 1];
    if (x.j >= lp.T) continue;
    const int ldr = ly.N16 + 4, I0 = 16 * x.j;
    for (int e = x.tid; e < ly.N16 * 4; e += NTH) {
      const int c = e >> 2, q = e & 3;
      f32x4 v;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = smem[ly.l_w + (4 * q + k) * ldr + c];
      st4(x.rs, c * ly.Kx + I0 + 4 * q, ly.o_wt, v);
    }
    if (l == L - 1) {
      for (int e = x.tid; e < 16 * ly.N16; e += NTH) {
        const int ip = e / ly.N16, c = e - ip * ly.N16;
        st1(x.rs, (I0 + ip) * ly.N16 + c, ly.o_w, smem[ly.l_w + ip * ldr + c]);
      }
    }
  }
  if (x.j == 0 && x.tid < a.ly[L - 1].N16) st1(x.rs, x.tid, a.o_bl, smem[a.ly[L - 1].l_b + x.tid]);
}

// the PS pull of slice j into the LDS masters: in asynchronous mode only while no pusher is
// inside the slice (ended == began before the copy, began unchanged after it), retried
// otherwise.  false: timed out (PERR_PS)
template <int L>
__device__ __forceinline__ bool pull_masters(const DeepArgs& a, float* smem, const Ctx& x) {
  auto copy = [&]() { load_masters<L>(a, smem, x, [&](long long i) { return *dps_elem(a.ps, i); }); };
  if (a.ps_mode != 2) {
    copy();
    __syncthreads();
    return true;
  }
  unsigned* sh = reinterpret_cast<unsigned*>(smem + a.l_red);   // two words of scratch
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    if (x.tid == 0) {
      for (;;) {
        const unsigned e = __hip_atomic_load(dps_ctr(a.ps, x.j, 1), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned b = __hip_atomic_load(dps_ctr(a.ps, x.j, 0), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (b == e || (long long)(wall_clock64() - t0) > a.timeout) { sh[0] = b; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    copy();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (x.tid == 0) {
      const unsigned b2 = __hip_atomic_load(dps_ctr(a.ps, x.j, 0), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      const bool late = (long long)(wall_clock64() - t0) > a.timeout;
      sh[1] = b2 == sh[0] ? 1u : (late ? 2u : 0u);
      if (late && b2 != sh[0])
        __hip_atomic_store((gu32*)(a.err), (unsigned)PERR_PS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const unsigned st = sh[1];
    __syncthreads();
    if (st == 1u) return true;
    if (st == 2u) return false;
  }
}

// the summed gradient tile (sum0) applied to the owned masters by every replica alike --
// the same sums and the same state, so the replicas stay one model bit for bit -- with the
// images the other workgroups read (W_l^T segments, the last layer's rows and bias)
// PSM (parameter-server hook): every changed element's delta theta_new - theta_old is added to
// the server (system-scope atomics), and the images wait for the pull (pull_masters)
template <bool PSM>
__device__ __forceinline__ void ps_add(const DeepArgs& a, long long pi, float w_old, float w_new) {
  if constexpr (PSM) {
    if (w_new != w_old) __hip_atomic_fetch_add(dps_elem(a.ps, pi), w_new - w_old, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
template <int L, int OPK, bool PSM = false>
__device__ __forceinline__ void apply_sums(const DeepArgs& a, float* smem, const Ctx& x0, long long sum0,
                                           const OptStep& os) {
  const Ctx x = lanes(x0);
  const DeepLayer l0 = a.ly[0];
  if (x.j < l0.T) {
    const int J0 = 16 * x.j, Kx = l0.Kx, ld0 = Kx + 4, q4 = Kx >> 2;
    float* w0t = smem + l0.l_w;
    for (int e = x.tid; e < 16 * q4; e += NTH) {
      const int c = e / q4, k = 4 * (e - c * q4);
      long long pi[4];
      bool ok[4];
      OptPre<4> pre;
#pragma unroll
      for (int ff = 0; ff < 4; ++ff) {
        pi[ff] = l0.p_off + (long long)(k + ff) * l0.N + J0 + c;
        ok[ff] = k + ff < l0.K && J0 + c < l0.N;
      }
      opt_pre<OPK, 4>(a, x, os, pi, ok, pre);
      const f32x4 g = ld4(x.xs, c * Kx + k, sum0);
      f32x4 w = lds4(w0t + c * ld0 + k);
#pragma unroll
      for (int ff = 0; ff < 4; ++ff)
        if (ok[ff]) {
          const float wn = upd_p<OPK>(a, x, os, pi[ff], w[ff], g[ff], pre.s0[ff], pre.s1[ff]);
          ps_add<PSM>(a, pi[ff], w[ff], wn);
          w[ff] = wn;
        }
      lds4(w0t + c * ld0 + k, w);
    }
    if (x.tid < 16 && l0.has_bias && J0 + x.tid < l0.N) {
      float* bt = smem + l0.l_b;
      const long long pb = l0.p_off + (long long)l0.K * l0.N + J0 + x.tid;
      const float bn = upd<OPK>(a, x, os, pb, bt[x.tid], ld1(x.xs, a.x_b0 + x.tid, sum0));
      ps_add<PSM>(a, pb, bt[x.tid], bn);
      bt[x.tid] = bn;
    }
  }
#pragma unroll
  for (int l = 1; l < L; ++l) {
    const DeepLayer ly = a.ly[l], lp = a.ly[l - 1];
    if (x.j < lp.T) {   // rows J of W_l: 4-row groups q x columns c (consecutive threads, consecutive c)
      const int I0 = 16 * x.j, N16 = ly.N16, ldr = N16 + 4;
      float* wr = smem + ly.l_w;
      for (int e = x.tid; e < 4 * N16; e += NTH) {
        const int q = e / N16, c = e - q * N16;
        long long pi[4];
        bool ok[4];
        OptPre<4> pre;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          pi[k] = ly.p_off + (long long)(I0 + 4 * q + k) * ly.N + c;
          ok[k] = I0 + 4 * q + k < ly.K && c < ly.N;
        }
        opt_pre<OPK, 4>(a, x, os, pi, ok, pre);
        f32x4 g, w;
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] = ld1(x.xs, a.x_w[l] + (4 * q + k) * N16 + c, sum0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int ip = 4 * q + k;
          float wt = wr[ip * ldr + c];
          if (ok[k]) {
            const float wn = upd_p<OPK>(a, x, os, pi[k], wt, g[k], pre.s0[k], pre.s1[k]);
            ps_add<PSM>(a, pi[k], wt, wn);
            wt = wn;
            wr[ip * ldr + c] = wt;
          }
          w[k] = wt;
        }
        if constexpr (!PSM) {
          st4(x.rs, c * ly.Kx + I0 + 4 * q, ly.o_wt, w);
          if (l == L - 1) {
#pragma unroll
            for (int k = 0; k < 4; ++k) st1(x.rs, (I0 + 4 * q + k) * N16 + c, ly.o_w, w[k]);
          }
        }
      }
    }
    if (l < L - 1) {
      if (x.j < ly.T && ly.has_bias && x.tid < 16 && 16 * x.j + x.tid < ly.N) {
        float* bt = smem + ly.l_b;
        const long long pb = ly.p_off + (long long)ly.K * ly.N + 16 * x.j + x.tid;
        const float bn = upd<OPK>(a, x, os, pb, bt[x.tid], ld1(x.xs, a.x_b[l] + x.tid, sum0));
        ps_add<PSM>(a, pb, bt[x.tid], bn);
        bt[x.tid] = bn;
      }
    } else if (x.j == 0 && ly.has_bias && x.tid < ly.N) {
      float* bl = smem + ly.l_b;
      const long long pb = ly.p_off + (long long)ly.K * ly.N + x.tid;
      const float b = upd<OPK>(a, x, os, pb, bl[x.tid], ld1(x.xs, a.x_b[l] + x.tid, sum0));
      ps_add<PSM>(a, pb, bl[x.tid], b);
      bl[x.tid] = b;
      if constexpr (!PSM) st1(x.rs, x.tid, a.o_bl, b);
    }
  }
}

// partial tile out -> all replicas' tiles out -> slice r summed in replica order (-> with the
// rank exchange: summed over the ranks in rank order, deep_xrank) -> all slices summed -> the
// update.  Parameter-server hook (ps_mode): no replica sum -- this workgroup's own tile
// updates its masters, the deltas go to the server, the masters come back from it.
template <int L, int OPK>
__device__ __forceinline__ bool exchange(const DeepArgs& a, float* smem, const Ctx& x0, int s, const OptStep& os) {
  const Ctx x = lanes(x0);
  const unsigned tag = (unsigned)s + 1;
  if (a.ps_mode) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tile's stores are out before any wave reads it
    __syncthreads();
    dps_push_begin(a, x.j);
    apply_sums<L, OPK, true>(a, smem, x, x.xp, os);
    dps_push_end(a, x.j);
    if (!pull_masters<L>(a, smem, x)) return false;
    write_images<L>(a, smem, x);
    __syncthreads();
    return true;
  }
  publish_x(a, x, 2, tag);
  if (!wait_x(a, x.j, 2, tag)) return false;
  dstamp(a, s, 25);
  const long long sum0 = ((long long)a.R * a.nw + x.j) * a.XT;
  const int q4 = a.XT >> 2, per = (q4 + a.R - 1) / a.R;
  const int e0 = x.r * per, e1 = (x.r + 1) * per < q4 ? (x.r + 1) * per : q4;
  if (a.xr_world <= 1) {
    for (int e = e0 + x.tid; e < e1; e += NTH) {
      f32x4 v = z4();
      for (int rr = 0; rr < a.R; ++rr) v += ld4(x.xs, 4 * e, ((long long)rr * a.nw + x.j) * a.XT);
      st4(x.xs, 4 * e, sum0, v);
    }
  } else {
    // the rank's sum of slice r into this rank's peer slot, then every rank's slot summed in
    // rank order -- the same bits on every rank
    const unsigned xt = a.xr_tag0 + tag;
    const long long slot = (((long long)(xt & 1u) * a.nw + x.j) * a.XT) * 4;   // bytes past PEER_DATA_OFF
    f32x4* mine = reinterpret_cast<f32x4*>(xr_base_of(a, a.xr_rank) + PEER_DATA_OFF + slot);
    for (int e = e0 + x.tid; e < e1; e += NTH) {
      f32x4 v = z4();
      for (int rr = 0; rr < a.R; ++rr) v += ld4(x.xs, 4 * e, ((long long)rr * a.nw + x.j) * a.XT);
      mine[e] = v;
    }
    if (!deep_xrank_wait(a, x.j * a.R + x.r, xt)) return false;
    for (int e = e0 + x.tid; e < e1; e += NTH) {
      f32x4 v = z4();
      for (int k = 0; k < a.xr_world; ++k)
        v += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(xr_base_of(a, k) + PEER_DATA_OFF + slot) + e);
      st4(x.xs, 4 * e, sum0, v);
    }
  }
  publish_x(a, x, 3, tag);
  if (!wait_x(a, x.j, 3, tag)) return false;
  dstamp(a, s, 26);
  apply_sums<L, OPK>(a, smem, x, sum0, os);
  __syncthreads();
  dstamp(a, s, 27);
  return true;
}

}  // namespace

template <int L, bool FAST, int OPK, bool SYNC>
__global__ __launch_bounds__(512) void mlp_deep_kernel(DeepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (__hip_atomic_load((gu32*)(a.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
  Ctx x;
  x.r = blockIdx.x % a.R;
  x.j = blockIdx.x / a.R;
  x.tid = threadIdx.x;
  x.lane = threadIdx.x & 63;
  x.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  x.g = x.lane >> 4;
  x.c16 = x.lane & 15;
  x.rs = ws_rsrc(a.ws + (long long)x.r * a.ws_stride);
  x.xs = ws_rsrc(SYNC ? a.xg : a.ws);
  x.xp = SYNC ? ((long long)x.r * a.nw + x.j) * a.XT : 0;
  x.P = a.P + (long long)x.r * a.sP;
  x.S = a.S ? a.S + (long long)x.r * a.sS : nullptr;
  x.prow = reinterpret_cast<int*>(smem + a.lds_floats - 2 * DP_ROWS);
  if (x.tid == 0)
    __hip_atomic_store((gu32*)(dflag(a, x.r, 0) + x.j), dxcc_go(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  // ---- prologue: the owned masters from P into LDS (zero past the true widths), then the
  // images the other workgroups read
  for (int e = x.tid; e < a.lds_floats; e += NTH) smem[e] = 0.f;
  __syncthreads();
  const int Bp = a.Bp;
  load_masters<L>(a, smem, x, [&](long long i) { return x.P[i]; });
  __syncthreads();
  write_images<L>(a, smem, x);
  __syncthreads();
  if (!wait_grid(a, x.r)) return;
  // the prologue's image writes are out: tag 1 (step s then publishes s * NPH + 2 ..
  // (s + 1) * NPH + 1, so "the previous step is done" is tag base for every s)
  publish(a, x.r, x.j, 1u);

  constexpr int NPH = 2 * L - 2;
  const long long s0 = ld_inv(a.ctr);
  const int ntr = ld_inv(a.ntrain + x.r);
  f32x4 G[L - 1];
#pragma unroll
  for (int l = 0; l < L - 1; ++l) G[l] = z4();
  int last = -1;
  OptStep lastos = opt_step(a.op, 0);
  for (int s = 0; s < a.nsteps; ++s) {
    const long long cnt = (long long)ntr - (s0 + s) * a.B;
    const int valid = (int)(cnt < 0 ? 0 : (cnt > a.B ? a.B : cnt));
    if (valid == 0) break;   // uniform over the replica: no batch left in this epoch
    const long long it = iter_at(a.ctr, a.ntrain, a.B, x.r, s0, s);
    const OptStep os = opt_step(a.op, it);
    const unsigned base = (unsigned)s * NPH + 1;
    dstamp(a, s, 0);
    // ---- phase 0: the previous step's layer-0 (and, L = 2, last-layer) update, forward 0
    {
      const Ctx y = lanes(x);
      if (y.tid < Bp) {
        const int* pr = a.perm + (long long)x.r * a.sPerm + (s0 + s) * a.B;
        x.prow[(s & 1) * DP_ROWS + y.tid] = y.tid < valid ? pr[y.tid] : 0;
      }
    }
    // FWD_1's W^T rows into the LDS stage by LDS-DMA right away (fit granularity, L >= 3):
    // every workgroup's previous step -- its BW_1 image writes included -- is published at
    // tag base; the copies run beside DW_0 and FWD_0, which do not touch the stage
    constexpr bool STAGED = !SYNC && L >= 3;
    if constexpr (STAGED) {
      if (!wait_phase(a, x.r, base)) return;
      wt_glds<1>(a, smem, x);
    }
    if (!SYNC && last >= 0) {
      if constexpr (L == 2) {
        if (!wait_phase(a, x.r, base)) return;
        dw_last<L, OPK, false>(a, smem, x, lastos);
        load_dz0(a, smem, x);
      }
      __syncthreads();
      dw0_phase<L, OPK, false>(a, smem, x, last, lastos);
    }
    __syncthreads();
    dstamp(a, s, 1);
    {
      f32x4 stg0[8];
      fwd_phase<L, 0, false>(a, smem, x, s, valid, it, G, stg0);
    }
    publish(a, x.r, x.j, base + 1);
    dstamp(a, s, 2);
    if (!fwd_chain<L, 1, STAGED>(a, smem, x, s, valid, it, base, G)) return;
    if (!wait_phase(a, x.r, base + L - 1)) return;
    dstamp(a, s, 9);
    tail_phase<L, FAST>(a, smem, x, s, valid);
    publish(a, x.r, x.j, base + L);
    dstamp(a, s, 10);
    if (!bw_chain<L, L - 2, OPK, SYNC>(a, smem, x, s, os, base, G)) return;
    if constexpr (SYNC) {   // every gradient of the step into the exchange tile, then the exchange
      if constexpr (L == 2) {
        if (!wait_phase(a, x.r, base + NPH)) return;
        dw_last<L, OPK, true>(a, smem, x, os);
        load_dz0(a, smem, x);
      }
      __syncthreads();
      dw0_phase<L, OPK, true>(a, smem, x, s, os);
      dstamp(a, s, 24);
      if (!exchange<L, OPK>(a, smem, x, s, os)) return;
    }
    last = s;
    lastos = os;
  }
  // the pending layer-0 update of the last step that ran
  if (!SYNC && last >= 0) {
    if constexpr (L == 2) {
      if (!wait_phase(a, x.r, (unsigned)(last + 1) * NPH + 1)) return;
      dw_last<L, OPK, false>(a, smem, x, lastos);
      load_dz0(a, smem, x);
    }
    __syncthreads();
    dw0_phase<L, OPK, false>(a, smem, x, last, lastos);
  }
  __syncthreads();
  // ---- epilogue: the owned masters back to P
  {
    const DeepLayer l0 = a.ly[0];
    if (x.j < l0.T) {
      const int J0 = 16 * x.j, ld0 = l0.Kx + 4;
      for (int e = x.tid; e < 16 * l0.K; e += NTH) {
        const int k = e >> 4, c = e & 15;
        if (J0 + c < l0.N) x.P[l0.p_off + (long long)k * l0.N + J0 + c] = smem[l0.l_w + c * ld0 + k];
      }
      if (x.tid < 16 && l0.has_bias && J0 + x.tid < l0.N)
        x.P[l0.p_off + (long long)l0.K * l0.N + J0 + x.tid] = smem[l0.l_b + x.tid];
    }
  }
#pragma unroll
  for (int l = 1; l < L; ++l) {
    const DeepLayer ly = a.ly[l], lp = a.ly[l - 1];
    const int ldr = ly.N16 + 4;
    if (x.j < lp.T) {
      const int I0 = 16 * x.j;
      for (int e = x.tid; e < 16 * ly.N; e += NTH) {
        const int ip = e / ly.N, c = e - ip * ly.N;
        if (I0 + ip < ly.K) x.P[ly.p_off + (long long)(I0 + ip) * ly.N + c] = smem[ly.l_w + ip * ldr + c];
      }
    }
    if (l < L - 1) {
      if (x.j < ly.T && x.tid < 16 && ly.has_bias && 16 * x.j + x.tid < ly.N)
        x.P[ly.p_off + (long long)ly.K * ly.N + 16 * x.j + x.tid] = smem[ly.l_b + x.tid];
    } else if (x.j == 0 && ly.has_bias && x.tid < ly.N) {
      x.P[ly.p_off + (long long)ly.K * ly.N + x.tid] = smem[ly.l_b + x.tid];
    }
  }
}

namespace {
// dynamic LDS above the default limit: raised per instantiation and per device to the largest
// layout launched there so far (the kernel's own static LDS -- e.g. the __syncthreads_and word
// -- counts against the same 160 KB, so the device maximum itself is refused).  The check and
// the raise happen under one lock, so the attribute only ever grows and no thread launches
// a layout larger than what its device was raised to.
template <int L, bool F, int OK, bool SY>
hipError_t deep_launch_one(const DeepArgs* a, hipStream_t s) {
  static std::mutex mu;
  static int set_bytes[DP_MAX_DEVICES] = {};
  const int need = (int)(sizeof(float) * (size_t)a->lds_floats);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= DP_MAX_DEVICES) return hipErrorInvalidDevice;
  {
    std::lock_guard<std::mutex> g(mu);
    if (need > set_bytes[dev]) {
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_deep_kernel<L, F, OK, SY>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, need);
      if (e != hipSuccess) return e;
      set_bytes[dev] = need;
    }
  }
  hipLaunchKernelGGL((mlp_deep_kernel<L, F, OK, SY>), dim3(a->R * a->nw), dim3(NTH), (size_t)need, s, *a);
  return hipGetLastError();
}

template <int L, bool F, bool SY>
hipError_t deep_launch_f(const DeepArgs* a, int opk, hipStream_t s) {
  if (opk == OPK_SGD0) return deep_launch_one<L, F, OPK_SGD0, SY>(a, s);
  if (opk == OPK_ADAM) return deep_launch_one<L, F, OPK_ADAM, SY>(a, s);
  return deep_launch_one<L, F, OPK_ANY, SY>(a, s);
}

template <int L, bool SY>
hipError_t deep_launch_sy(const DeepArgs* a, bool fast, int opk, hipStream_t s) {
  return fast ? deep_launch_f<L, true, SY>(a, opk, s) : deep_launch_f<L, false, SY>(a, opk, s);
}

// opk: OPK_SGD0 / OPK_ADAM / OPK_ANY (deep.hip picks it from the optimizer)
template <int L>
hipError_t deep_launch(const DeepArgs* a, bool fast, int opk, hipStream_t s) {
  // per-step sync and the parameter-server hook both run the gradient tiles through xg (the
  // XCD-local instance has neither: fit granularity only)
#if EA_DLOCAL
  if (a->sync || a->ps_mode) return hipErrorInvalidValue;
  return deep_launch_sy<L, false>(a, fast, opk, s);
#else
  return (a->sync || a->ps_mode) ? deep_launch_sy<L, true>(a, fast, opk, s) : deep_launch_sy<L, false>(a, fast, opk, s);
#endif
}
// value of component c of f32x4 element e of replica r's slice of tile j, self-test step i on
// rank k: small integers, so every partial sum is exact in fp32 whatever the order
__device__ __forceinline__ float dxr_test_value(int k, int j, int r, int i, int e, int c) {
  return (float)((k + 1) * ((j % 7) + r + i + 2) + ((4 * e + c) % 11));
}
// Numeric self-test of the layer pipeline's rank exchange (deep_xrank_wait + the rank-order
// sum of exchange()): nsteps exchanges of known integer slices by every workgroup (j, r), with
// the tags continuing the trainer's sequence; each rank checks every summed element against
// the exact rank sum.  bad += 1 per workgroup-step with a wrong element, += 1 << 16 per
// workgroup that timed out.  corrupt != 0 (fault injection): this rank sends a wrong slice.
__global__ __launch_bounds__(NTH) void deep_xrank_selftest_kernel(DeepArgs a, int nsteps, unsigned* bad, int corrupt) {
  const int r = blockIdx.x % a.R, j = blockIdx.x / a.R, tid = threadIdx.x;
  const int q4 = a.XT >> 2, per = (q4 + a.R - 1) / a.R;
  const int e0 = r * per, e1 = (r + 1) * per < q4 ? (r + 1) * per : q4;
  for (int i = 0; i < nsteps; ++i) {
    const unsigned xt = a.xr_tag0 + (unsigned)i + 1u;
    const long long slot = (((long long)(xt & 1u) * a.nw + j) * a.XT) * 4;
    f32x4* mine = reinterpret_cast<f32x4*>(xr_base_of(a, a.xr_rank) + PEER_DATA_OFF + slot);
    for (int e = e0 + tid; e < e1; e += NTH) {
      f32x4 v;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = dxr_test_value(a.xr_rank, j, r, i, e, c) + (corrupt ? 0.5f : 0.f);
      mine[e] = v;
    }
    if (!deep_xrank_wait(a, j * a.R + r, xt)) {
      if (tid == 0) atomicAdd(bad, 1u << 16);
      return;
    }
    int wrong = 0;
    for (int e = e0 + tid; e < e1; e += NTH) {
      f32x4 v = z4();
      for (int k = 0; k < a.xr_world; ++k)
        v += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(xr_base_of(a, k) + PEER_DATA_OFF + slot) + e);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float want = 0.f;
        for (int k = 0; k < a.xr_world; ++k) want += dxr_test_value(k, j, r, i, e, c);
        wrong |= v[c] != want;
      }
    }
    if (__syncthreads_or(wrong) && tid == 0) atomicAdd(bad, 1u);
  }
}

}  // namespace

}  // namespace ea

#ifdef EA_DEEP_XRANK_ENTRY
// grid R * nw workgroups (every one resident: they wait for the other ranks' flags)
extern "C" hipError_t ea_deep_xrank_selftest(const ea::DeepArgs* a, int nsteps, unsigned* bad, int corrupt,
                                             hipStream_t s) {
  hipLaunchKernelGGL(ea::deep_xrank_selftest_kernel, dim3(a->R * a->nw), dim3(ea::NTH), 0, s, *a, nsteps, bad, corrupt);
  return hipGetLastError();
}
#endif
