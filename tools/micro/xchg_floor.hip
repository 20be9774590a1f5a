// Hardware floor of the persistent kernels' hand-off (persist.hip publish / wait_replicas /
// xchg_sum, deep_impl.h exchange) on MI355X (gfx950), timed with s_memrealtime (100 MHz).
//
// The hand-off under test, exactly as the kernels do it: write-through (sc1) 16-byte buffer
// stores of a slab, s_waitcnt vmcnt(0), workgroup barrier, one lane stores the flag
// (agent-scope relaxed atomic), the consumer's wave 0 polls the flag with agent-scope
// atomic loads, barrier, then sc1 16-byte buffer loads of the slab.
//
//   pingpong  two workgroups bounce a slab of S bytes: one-way latency of
//             store -> drain -> flag -> poll -> load, same XCD (blocks 0 / 8) or across XCDs
//             (blocks 0 / 1; block b runs on XCD b % 8 -- checked through HW_REG_XCC_ID)
//   allgather R workgroups each publish a slab, wait for all R flags, load and sum all R
//             slabs in order (xchg_sum's all-gather form): time per exchange round, with the
//             R workgroups on R different XCDs or all on one XCD
//   eager     the same, but each workgroup starts the loads of replica k's slab as soon as
//             flag k is seen (lane k of wave 0 polls flag k; the others load what arrived)
//
// Every spin is bounded (0.2 s -> error word, the workgroup leaves), every workgroup of the
// grid reaches the end.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
using rsrc_t = __amdgpu_buffer_rsrc_t;
using gu32 = __attribute__((address_space(1))) unsigned;

constexpr long long TMO = 20000000;   // 0.2 s in s_memrealtime ticks
constexpr int NTH = 256;

__device__ __forceinline__ rsrc_t mk(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ f32x4 ld4(rsrc_t r, int v) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, v * 4, 0, 16));
}
__device__ __forceinline__ void st4(rsrc_t r, int v, f32x4 x) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), r, v * 4, 0, 16);
}
__device__ __forceinline__ unsigned xcc_id() {
  // HW_REG_XCC_ID (hwreg 20), bits [3:0]
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
}
__device__ __forceinline__ void publish(unsigned* flag, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store((gu32*)flag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool SLEEP>
__device__ __forceinline__ bool wait_flags(const unsigned* flags, int n, unsigned tag, unsigned* err) {
  int ok = 1;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      const unsigned v = lane < n ? __hip_atomic_load((gu32*)(const_cast<unsigned*>(flags) + lane), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT)
                                  : tag;
      if (__all(v >= tag)) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > TMO) {
        ok = 0;
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      if (SLEEP) __builtin_amdgcn_s_sleep(1);
    }
  }
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok != 0;
}

// out[0] = ticks for iters round trips (block 0), out[2 + b] = XCC id of block b
template <int NF4, bool SLEEP>
__global__ __launch_bounds__(NTH) void pingpong(float* buf, unsigned* flags, int peer, int iters, long long* out,
                                                unsigned* err) {
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) out[2 + b] = xcc_id();
  if (b != 0 && b != peer) return;
  const int me = b == 0 ? 0 : 1;
  const rsrc_t mine = mk(buf + (long long)me * NF4 * NTH * 4), other = mk(buf + (long long)(1 - me) * NF4 * NTH * 4);
  f32x4 v[NF4 > 0 ? NF4 : 1];
#pragma unroll
  for (int u = 0; u < (NF4 > 0 ? NF4 : 1); ++u) v[u] = f32x4{1.f, 2.f, 3.f, (float)tid};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    const unsigned tag = (unsigned)(i + 1);
    {
      if (me == 0) {   // A: send, then wait for the reply
#pragma unroll
        for (int u = 0; u < NF4; ++u) st4(mine, (u * NTH + tid) * 4, v[u]);
        publish(flags + 0, tag);
        if (!wait_flags<SLEEP>(flags + 64, 1, tag, err)) break;
#pragma unroll
        for (int u = 0; u < NF4; ++u) v[u] = ld4(other, (u * NTH + tid) * 4) + 1.f;
      } else {         // B: wait, read, reply
        if (!wait_flags<SLEEP>(flags + 0, 1, tag, err)) break;
#pragma unroll
        for (int u = 0; u < NF4; ++u) v[u] = ld4(other, (u * NTH + tid) * 4) + 1.f;
#pragma unroll
        for (int u = 0; u < NF4; ++u) st4(mine, (u * NTH + tid) * 4, v[u]);
        publish(flags + 64, tag);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < NF4; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
  if (me == 0 && tid == 0) { out[0] = t1 - t0; out[1] = (long long)s; }
}

// R participants: blocks 0, st, 2 st, ... (st = 1: R XCDs; st = 8: one XCD).  Slabs alternate by
// iteration parity (a writer of round i + 2 has seen every round-(i + 1) flag, which each reader
// raised after its round-i loads).  EAGER: lane k polls flag k, and the loads of slab k are
// issued in the first poll round that sees it (all threads follow the wave-0 bitmask via LDS).
template <int NF4, bool SLEEP, bool EAGER>
__global__ __launch_bounds__(NTH) void allgather(float* buf, unsigned* flags, int R, int st, int iters, long long* out,
                                                 unsigned* err) {
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) out[2 + b] = xcc_id();
  if (b % st != 0 || b / st >= R) return;
  const int r = b / st;
  const long long slab_f = (long long)NF4 * NTH * 4;
  __shared__ unsigned seen;
  f32x4 v[NF4];
#pragma unroll
  for (int u = 0; u < NF4; ++u) v[u] = f32x4{1.f, (float)r, 3.f, (float)tid};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    const unsigned tag = (unsigned)(i + 1);
    float* par = buf + (long long)(i & 1) * 8 * slab_f;
#pragma unroll
    for (int u = 0; u < NF4; ++u) st4(mk(par + r * slab_f), (u * NTH + tid) * 4, v[u]);
    publish(flags + r, tag);
    f32x4 acc[NF4];
#pragma unroll
    for (int u = 0; u < NF4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (!EAGER) {
      if (!wait_flags<SLEEP>(flags, R, tag, err)) break;
      for (int k = 0; k < R; ++k) {
        f32x4 x[NF4];
#pragma unroll
        for (int u = 0; u < NF4; ++u) x[u] = ld4(mk(par + k * slab_f), (u * NTH + tid) * 4);
#pragma unroll
        for (int u = 0; u < NF4; ++u) acc[u] += x[u];
      }
    } else {
      // partial sums per replica kept in arrival order would change the bits; a real exchange
      // would keep R slabs in registers and add in replica order -- here: loads issued at
      // arrival, summed in replica order at the end (R <= 8 slabs of NF4 f32x4 in registers)
      f32x4 x[8][NF4];
      unsigned done = 0;
      const unsigned all = (1u << R) - 1;
      const long long tw = __builtin_amdgcn_s_memrealtime();
      bool bad = false;
      while (done != all) {
        if (tid < 64) {
          const unsigned f = tid < R ? __hip_atomic_load((gu32*)(flags + tid), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
          const unsigned long long m = __ballot(tid < R && f >= tag);
          if (tid == 0) seen = (unsigned)m;
        }
        __syncthreads();
        const unsigned now = seen & ~done;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (now & (1u << k)) {
#pragma unroll
            for (int u = 0; u < NF4; ++u) x[k][u] = ld4(mk(par + k * slab_f), (u * NTH + tid) * 4);
          }
        done |= now;
        __syncthreads();
        if (done != all) {
          if (__builtin_amdgcn_s_memrealtime() - tw > TMO) { bad = true; break; }
          if (SLEEP) __builtin_amdgcn_s_sleep(1);
        }
      }
      if (bad) { if (tid == 0) atomicOr(err, 2u); break; }
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < R) {
#pragma unroll
          for (int u = 0; u < NF4; ++u) acc[u] += x[k][u];
        }
    }
#pragma unroll
    for (int u = 0; u < NF4; ++u) v[u] = acc[u] * 0.125f;
    // the round's reads are done before anyone may overwrite this parity's slabs (round i + 2):
    // a second flag round, as the kernels' next step provides
    publish(flags + 64 + r, tag);
    if (!wait_flags<SLEEP>(flags + 64, R, tag, err)) break;
  }
  const long long t1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < NF4; ++u) s += v[u].x + v[u].w;
  if (r == 0 && tid == 0) { out[0] = t1 - t0; out[1] = (long long)s; }
}

// a flag-only barrier round among R workgroups (the second flag round of allgather alone)
template <bool SLEEP>
__global__ __launch_bounds__(NTH) void flagbar(unsigned* flags, int R, int st, int iters, long long* out, unsigned* err) {
  const int b = blockIdx.x;
  if (b % st != 0 || b / st >= R) return;
  const int r = b / st;
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    publish(flags + r, (unsigned)(i + 1));
    if (!wait_flags<SLEEP>(flags, R, (unsigned)(i + 1), err)) break;
  }
  const long long t1 = __builtin_amdgcn_s_memrealtime();
  if (r == 0 && threadIdx.x == 0) out[0] = t1 - t0;
}


// ---- chip-wide: G groups of R = 8 workgroups exchanging at once (the persistent kernels run
//      32 such groups, one per gradient tile), with the hand-off at device scope (sc1 stores and
//      loads, agent-scope atomic flags: what the kernels do) or XCD-local (plain stores, which
//      keep the line in the XCD's L2, read by the same sc1 loads -- L1 skipped, L2-served --
//      and a plain flag store polled by the same agent-scope loads) --
//      valid only when every member of a group runs on one XCD, which the kernel checks
//      through HW_REG_XCC_ID (err bit 4 otherwise).
//   LOCAL: members of group g on one XCD: b = (g % 8) + 8 * ((g / 8) * 8 + r); else b = 8 g + r
template <bool XCDL>
__device__ __forceinline__ void st4s(rsrc_t r, int v, f32x4 x) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), r, v * 4, 0, XCDL ? 0 : 16);
}
template <bool XCDL>
__device__ __forceinline__ f32x4 ld4s(rsrc_t r, int v) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, v * 4, 0, 16));   // sc1: skips L1, L2-served
}
template <bool XCDL>
__device__ __forceinline__ void flag_st(unsigned* f, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (XCDL) __builtin_amdgcn_raw_buffer_store_b32(tag, mk((float*)f), 0, 0, 0);
    else __hip_atomic_store((gu32*)f, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
template <bool XCDL>
__device__ __forceinline__ bool flag_wait(const unsigned* flags, int n, unsigned tag, unsigned* err) {
  int ok = 1;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      const unsigned v = lane < n ? __hip_atomic_load((gu32*)(const_cast<unsigned*>(flags) + lane), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT)
                                  : tag;
      if (__all(v >= tag)) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > TMO) {
        ok = 0;
        if (lane == 0) atomicOr(err, 1u);
        if (lane < n && blockIdx.x < 64 && blockIdx.x % 8 == 0)
          printf("block %d lane %d flag[%d] %u want %u xcc %u\n", blockIdx.x, lane, (int)(flags - (const unsigned*)0) & 255, v, tag, xcc_id());
        break;
      }
    }
  }
  ok = __syncthreads_and(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok != 0;
}

template <int NF4, bool XCDL, bool LOCAL>
__global__ __launch_bounds__(NTH) void groups(float* buf, unsigned* flags, unsigned* xcc, int G, int iters, long long* out,
                                              unsigned* err) {
  const int b = blockIdx.x, tid = threadIdx.x;
  constexpr int R = 8;
  int g, r;
  if (LOCAL) { const int k = b / 8; g = (b % 8) + 8 * (k / 8); r = k % 8; }
  else { g = b / 8; r = b % 8; }
  if (g >= G) return;
  const long long slab_f = (long long)NF4 * NTH * 4;
  float* gb = buf + (long long)g * 2 * R * slab_f;
  unsigned* gf = flags + g * 256;
  // membership check: every member of the group on one XCD (XCDL only)
  if (tid == 0) __hip_atomic_store((gu32*)(xcc + g * R + r), xcc_id() + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (XCDL) {
    __shared__ int same;
    if (tid < 64) {
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned v = 0;
      for (;;) {
        v = tid < R ? __hip_atomic_load((gu32*)(xcc + g * R + tid), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1u;
        if (__all(v != 0u) || __builtin_amdgcn_s_memrealtime() - t0 > TMO) break;
      }
      const unsigned v0 = __shfl(v, 0);
      const bool eq = __all(tid >= R || v == v0);
      if (tid == 0) same = eq ? 1 : 0;
    }
    __syncthreads();
    if (!same) { if (tid == 0) { atomicOr(err, 16u); if (g == 0) printf("group 0 member %d: not one XCD\n", r); } return; }
  }
  constexpr int NV = NF4 > 0 ? NF4 : 1;
  f32x4 v[NV];
#pragma unroll
  for (int u = 0; u < NV; ++u) v[u] = f32x4{1.f, (float)r, 3.f, (float)tid};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    const unsigned tag = (unsigned)(i + 1);
    float* par = gb + (long long)(i & 1) * R * slab_f;
#pragma unroll
    for (int u = 0; u < NF4; ++u) st4s<XCDL>(mk(par + r * slab_f), (u * NTH + tid) * 4, v[u]);
    flag_st<XCDL>(gf + r, tag);
    if (!flag_wait<XCDL>(gf, R, tag, err)) break;
    f32x4 x[R][NV];
#pragma unroll
    for (int k = 0; k < R; ++k)
#pragma unroll
      for (int u = 0; u < NF4; ++u) x[k][u] = ld4s<XCDL>(mk(par + k * slab_f), (u * NTH + tid) * 4);
#pragma unroll
    for (int u = 0; u < NF4; ++u) {
      f32x4 acc = x[0][u];
#pragma unroll
      for (int k = 1; k < R; ++k) acc += x[k][u];
      v[u] = acc * 0.125f;
    }
    flag_st<XCDL>(gf + 64 + r, tag);
    if (!flag_wait<XCDL>(gf + 64, R, tag, err)) break;
  }
  const long long t1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < NF4; ++u) s += v[u].x + v[u].w;
  if (g == 0 && r == 0 && tid == 0) { out[0] = t1 - t0; out[1] = (long long)s; }
}

struct Dev {
  float* buf;
  float* gbuf;
  unsigned* gflags;
  unsigned* xcc;
  unsigned* flags;
  long long* out;
  unsigned* err;
};

template <int NF4, bool SLEEP>
static void pp(Dev& d, int peer) {
  std::vector<double> v;
  const int iters = 2000;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemset(d.flags, 0, 4096));
    CK(hipMemset(d.err, 0, 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL((pingpong<NF4, SLEEP>), dim3(16), dim3(NTH), 0, 0, d.buf, d.flags, peer, iters, d.out, d.err);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    long long h[2 + 16];
    unsigned e = 0;
    CK(hipMemcpy(h, d.out, sizeof(h), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&e, d.err, 4, hipMemcpyDeviceToHost));
    if (e) { printf("pingpong timed out\n"); return; }
    v.push_back(h[0] * 10.0 / (2.0 * iters));
    if (rep == 0 && NF4 == 0 && !SLEEP)
      printf("  XCC of blocks 0..15:"), [&] { for (int b = 0; b < 16; ++b) printf(" %lld", h[2 + b]); printf("\n"); }();
  }
  std::sort(v.begin(), v.end());
  printf("pingpong  %-10s slab %6d B  poll %-8s one-way %7.0f ns (median of 5, %d round trips)\n",
         peer == 8 ? "same XCD" : "cross XCD", NF4 * NTH * 16, SLEEP ? "s_sleep1" : "spin", v[2], iters);
}

template <int NF4, bool SLEEP, bool EAGER>
static void ag(Dev& d, int R, int st) {
  std::vector<double> v;
  const int iters = 1000;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemset(d.flags, 0, 4096));
    CK(hipMemset(d.err, 0, 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL((allgather<NF4, SLEEP, EAGER>), dim3(64), dim3(NTH), 0, 0, d.buf, d.flags, R, st, iters, d.out, d.err);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    long long h[2];
    unsigned e = 0;
    CK(hipMemcpy(h, d.out, sizeof(h), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&e, d.err, 4, hipMemcpyDeviceToHost));
    if (e) { printf("allgather timed out (err %u)\n", e); return; }
    v.push_back(h[0] * 10.0 / iters);
  }
  std::sort(v.begin(), v.end());
  // subtract the flag-only round measured separately by the caller
  printf("allgather%s R %d %-9s slab %6d B poll %-8s round %7.0f ns (incl. one flag-only barrier round)\n",
         EAGER ? "-eager" : "      ", R, st == 8 ? "one XCD" : "R XCDs", NF4 * NTH * 16, SLEEP ? "s_sleep1" : "spin", v[2]);
}

template <bool SLEEP>
static void fb(Dev& d, int R, int st) {
  std::vector<double> v;
  const int iters = 2000;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemset(d.flags, 0, 4096));
    CK(hipMemset(d.err, 0, 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL((flagbar<SLEEP>), dim3(64), dim3(NTH), 0, 0, d.flags, R, st, iters, d.out, d.err);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    long long h[1];
    unsigned e = 0;
    CK(hipMemcpy(h, d.out, sizeof(h), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&e, d.err, 4, hipMemcpyDeviceToHost));
    if (e) { printf("flagbar timed out\n"); return; }
    v.push_back(h[0] * 10.0 / iters);
  }
  std::sort(v.begin(), v.end());
  printf("flag-only barrier  R %d %-9s poll %-8s round %7.0f ns\n", R, st == 8 ? "one XCD" : "R XCDs",
         SLEEP ? "s_sleep1" : "spin", v[2]);
}

template <int NF4, bool XCDL, bool LOCAL>
static void gr(Dev& d, int G) {
  std::vector<double> v;
  const int iters = 1000;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemset(d.gflags, 0, 32 * 256 * 4));
    CK(hipMemset(d.xcc, 0, 32 * 8 * 4));
    CK(hipMemset(d.err, 0, 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL((groups<NF4, XCDL, LOCAL>), dim3(256), dim3(NTH), 0, 0, d.gbuf, d.gflags, d.xcc, G, iters, d.out, d.err);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    long long h[2];
    unsigned e = 0;
    CK(hipMemcpy(h, d.out, sizeof(h), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&e, d.err, 4, hipMemcpyDeviceToHost));
    if (e) { printf("groups G %d %s %s: error %u (16 = members not on one XCD)\n", G, XCDL ? "xcd-local" : "device", LOCAL ? "one-XCD" : "spread", e); return; }
    if (h[0] >= TMO) { printf("groups G %d %s %s: timed out without an error word\n", G, XCDL ? "xcd-local" : "device", LOCAL ? "one-XCD" : "spread"); return; }
    v.push_back(h[0] * 10.0 / iters);
  }
  std::sort(v.begin(), v.end());
  printf("groups G %2d x R 8 %-16s members %-8s slab %6d B  round %7.0f ns (exchange + one flag-only round)\n", G,
         XCDL ? "xcd-local (L2)" : "device (sc1)", LOCAL ? "one XCD" : "8 XCDs", NF4 * NTH * 16, v[2]);
}

int main() {
  Dev d;
  CK(hipMalloc(&d.buf, 2 * 8 * 8 * 256 * 16));
  CK(hipMemset(d.buf, 0, 2 * 8 * 8 * 256 * 16));
  CK(hipMalloc(&d.flags, 4096));
  CK(hipMalloc(&d.out, 8 * 80));
  CK(hipMalloc(&d.err, 4));
  CK(hipMalloc(&d.gbuf, 32LL * 2 * 8 * 8 * 256 * 16));
  CK(hipMemset(d.gbuf, 0, 32LL * 2 * 8 * 8 * 256 * 16));
  CK(hipMalloc(&d.gflags, 32 * 256 * 4));
  CK(hipMalloc(&d.xcc, 32 * 8 * 4));
  if (getenv("XF_DEBUG")) {
    gr<0, true, true>(d, 1);
    gr<4, true, false>(d, 32);
    return 0;
  }
  for (int G : {1, 32}) {
    gr<0, false, false>(d, G);
    gr<0, false, true>(d, G);
    gr<0, true, true>(d, G);
    gr<4, false, false>(d, G);
    gr<4, false, true>(d, G);
    gr<4, true, true>(d, G);
    gr<8, false, false>(d, G);
    gr<8, true, true>(d, G);
  }
  gr<4, true, false>(d, 32);   // must report the membership error
  for (int peer : {8, 1}) {
    pp<0, false>(d, peer);
    pp<0, true>(d, peer);
    pp<1, false>(d, peer);
    pp<4, false>(d, peer);
    pp<4, true>(d, peer);
    pp<8, false>(d, peer);
  }
  for (int st : {8, 1}) {
    fb<false>(d, 8, st);
    fb<true>(d, 8, st);
    ag<1, false, false>(d, 8, st);
    ag<4, false, false>(d, 8, st);
    ag<4, true, false>(d, 8, st);
    ag<4, false, true>(d, 8, st);
    ag<8, false, false>(d, 8, st);
    ag<8, false, true>(d, 8, st);
  }
  return 0;
}
