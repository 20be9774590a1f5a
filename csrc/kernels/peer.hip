// Peer-memory collectives and the sharded device parameter server.
//
// Every rank owns one uncached device buffer (hipDeviceMallocUncached, so no
// rank ever reads a stale L2 line of memory another GPU wrote over xGMI) that all
// other ranks map through HIP IPC.  Kernels here read and write those peer
// buffers directly: no host round trip, no RCCL, no host-side synchronisation.
//
// 1. All-reduce (sum) for small / medium messages -- the per-step gradient path
//    (reference elephas/spark_model.py:220-227 collects and averages every
//    worker's delta; the batch-granularity path does it every step):
//      one-shot : every rank stages its input into its own buffer, flags each
//                 chunk, waits for the same chunk's flag on every peer, then sums
//                 the chunk over all ranks (in rank order: bit-identical results on
//                 every rank).  One barrier, (W-1)*n bytes read per rank.
//      two-shot : reduce-scatter (rank p sums slice p) + all-gather (everyone copies
//                 slice p from rank p).  Two barriers, 2*(W-1)/W*n bytes per rank:
//                 the choice for larger messages on point-to-point xGMI links.
//    Synchronisation is per WORKGROUP (one flag per chunk and phase, value = call
//    epoch), not grid-wide; staging buffers alternate by epoch parity so no
//    closing barrier is needed (a rank can only overwrite a parity after every
//    peer has entered the following call, i.e. finished reading this one).
// 2. Parameter server (reference elephas/parameter/server.py:107-132,201-218):
//    theta is sharded in chunks over the ranks' buffers; a pull gathers the chunks
//    from their owners, a push adds a delta into them with fp32 atomics.  Both are
//    single stream-ordered kernels (capturable in a hipGraph) instead of a host
//    lock + hipStreamSynchronize; see the parameter-server section for the
//    'asynchronous' (chunk-consistent pulls) and 'hogwild' semantics.
//
// Every wait spins with a wall-clock limit: on expiry the workgroup records an
// error word in its own buffer and exits, so every wave reaches its end even if
// a peer never arrives (the host raises when it reads the error word).
#include <hip/hip_runtime.h>

#include "peer_args.h"

namespace ea {

__device__ __forceinline__ unsigned* flag_ptr(char* base, int phase, int b) {
  return reinterpret_cast<unsigned*>(base + PEER_FLAG_OFF + (long long)phase * PEER_MAX_BLOCKS * 64 + (long long)b * 64);
}
__device__ __forceinline__ unsigned* err_ptr(char* base) { return reinterpret_cast<unsigned*>(base + PEER_ERR_OFF); }
__device__ __forceinline__ float* stage_ptr(char* base, long long cap, int parity) {
  return reinterpret_cast<float*>(base + PEER_DATA_OFF) + (long long)parity * cap;
}
__device__ __forceinline__ float* red_ptr(char* base, long long cap, int parity) {
  return reinterpret_cast<float*>(base + PEER_DATA_OFF) + (2 + (long long)parity) * cap;
}

__device__ __forceinline__ void store_flag(unsigned* f, unsigned v) {
  __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned load_flag(const unsigned* f) {
  return __hip_atomic_load(const_cast<unsigned*>(f), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait until every peer's flag (phase, b) has reached `epoch`; lanes 0..W-1 of
// wave 0 each watch one peer. Returns false (and records the error) on timeout.
__device__ bool wait_peers(const PeerArgs& a, int phase, int b, unsigned epoch) {
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world && t != a.rank) {
    const unsigned* f = flag_ptr(a.base[t], phase, b);
    const unsigned long long t0 = wall_clock64();
    while ((int)(load_flag(f) - epoch) < 0) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        __hip_atomic_store(err_ptr(a.base[a.rank]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system-scope acquire for every wave's reads
  return ok != 0;
}

// Publish this workgroup's writes, then raise its flag.
__device__ __forceinline__ void signal(const PeerArgs& a, int phase, int b, unsigned epoch) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // each wave's own stores complete at system scope
  __syncthreads();
  if (threadIdx.x == 0) store_flag(flag_ptr(a.base[a.rank], phase, b), epoch);
}

__device__ __forceinline__ float4 f4add(float4 x, float4 y) {
  return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
}

// Copy [lo, hi) of src to dst (float4 body; lo is a multiple of 4, the tail is scalar).
__device__ __forceinline__ void copy_span(const float* __restrict__ src, float* __restrict__ dst, long long lo,
                                          long long hi) {
  const long long v0 = lo / 4, v1 = hi / 4;
  for (long long i = v0 + threadIdx.x; i < v1; i += blockDim.x)
    reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
  for (long long i = v1 * 4 + threadIdx.x; i < hi; i += blockDim.x) dst[i] = src[i];
}

// A wait that timed out poisons the outputs it would have written with NaN (besides the
// error word the host checks): a late peer never leaves a rank's local value looking
// like a reduced one.
__device__ __forceinline__ void poison_span(float* __restrict__ dst, long long lo, long long hi) {
  for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) dst[i] = __builtin_nanf("");
}

// dst[i] = sum_{r < W} srcs[r][i] over [lo, hi), summed in rank order.
__device__ __forceinline__ void sum_span(const PeerArgs& a, int parity, long long lo, long long hi, float* out,
                                         float* out2) {
  const long long v0 = lo / 4, v1 = hi / 4;
  for (long long i = v0 + threadIdx.x; i < v1; i += blockDim.x) {
    float4 v[PEER_MAX_RANKS];
#pragma unroll
    for (int r = 0; r < PEER_MAX_RANKS; ++r)  // issue every peer's load before the adds
      if (r < a.world) v[r] = reinterpret_cast<const float4*>(stage_ptr(a.base[r], a.cap, parity))[i];
    float4 s = v[0];
#pragma unroll
    for (int r = 1; r < PEER_MAX_RANKS; ++r)
      if (r < a.world) s = f4add(s, v[r]);
    reinterpret_cast<float4*>(out)[i] = s;
    if (out2) reinterpret_cast<float4*>(out2)[i] = s;
  }
  for (long long i = v1 * 4 + threadIdx.x; i < hi; i += blockDim.x) {
    float s = stage_ptr(a.base[0], a.cap, parity)[i];
    for (int r = 1; r < a.world; ++r) s += stage_ptr(a.base[r], a.cap, parity)[i];
    out[i] = s;
    if (out2) out2[i] = s;
  }
}

// Epoch of this call for workgroup b: the host's counter, or (graph mode: the same
// kernel replayed from a hipGraph with frozen arguments) one past the epoch this
// rank's workgroup b flagged last -- identical on every rank because every rank
// makes the same calls with the same sizes.
__device__ __forceinline__ unsigned call_epoch(const PeerArgs& a, int b) {
  if (!a.dev_epoch) return a.epoch;
  __shared__ unsigned e;
  if (threadIdx.x == 0) e = __hip_atomic_load(flag_ptr(a.base[a.rank], 0, b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  return e;
}

__global__ __launch_bounds__(256) void allreduce_oneshot_kernel(PeerArgs a) {
  const int b = blockIdx.x;
  a.epoch = call_epoch(a, b);
  const int parity = a.epoch & 1;
  const long long lo = (long long)b * a.chunk;
  const long long hi = lo + a.chunk < a.n ? lo + a.chunk : a.n;
  char* mine = a.base[a.rank];
  if (lo < hi) copy_span(a.in, stage_ptr(mine, a.cap, parity), lo, hi);
  signal(a, 0, b, a.epoch);
  if (!wait_peers(a, 0, b, a.epoch)) {
    if (lo < hi) poison_span(a.out, lo, hi);
    return;
  }
  if (lo < hi) sum_span(a, parity, lo, hi, a.out, nullptr);
}

// slice p = [p*slice, min(n, (p+1)*slice)); block b owns sub-chunk b of every slice.
__global__ __launch_bounds__(256) void allreduce_twoshot_kernel(PeerArgs a) {
  const int b = blockIdx.x;
  a.epoch = call_epoch(a, b);
  const int parity = a.epoch & 1;
  char* mine = a.base[a.rank];
  auto span = [&](int p, long long& lo, long long& hi) {
    const long long s0 = (long long)p * a.slice;
    const long long s1 = s0 + a.slice < a.n ? s0 + a.slice : a.n;
    lo = s0 + (long long)b * a.chunk;
    hi = lo + a.chunk < s1 ? lo + a.chunk : s1;
  };
  long long lo, hi;
  for (int p = 0; p < a.world; ++p) {
    span(p, lo, hi);
    if (lo < hi) copy_span(a.in, stage_ptr(mine, a.cap, parity), lo, hi);
  }
  signal(a, 0, b, a.epoch);
  // a timed-out wait raises no later flag (a peer must never read a slice this rank did
  // not reduce): the peers' own waits time out and poison their outputs the same way
  bool ok = wait_peers(a, 0, b, a.epoch);
  if (ok) {
    span(a.rank, lo, hi);
    if (lo < hi) sum_span(a, parity, lo, hi, red_ptr(mine, a.cap, parity), a.out);
    signal(a, 1, b, a.epoch);
    ok = wait_peers(a, 1, b, a.epoch);
  }
  if (!ok) {
    for (int p = 0; p < a.world; ++p) {
      span(p, lo, hi);
      if (lo < hi) poison_span(a.out, lo, hi);
    }
    return;
  }
  for (int p = 0; p < a.world; ++p) {
    if (p == a.rank) continue;
    span(p, lo, hi);
    if (lo < hi) copy_span(red_ptr(a.base[p], a.cap, parity), a.out, lo, hi);
  }
}

// ------------------------------------------------------------------ parameter server
// theta is cut into chunks; chunk c lives in the buffer of rank c * W / nchunks,
// with (at ctr_off) two counters per chunk: writer workgroups that
// BEGAN and that ENDED an update of the chunk.  Writers never wait: a push adds its
// delta with fp32 atomics (no update is ever lost, whatever the interleaving) between
// bumping `began` and `ended`.  An 'asynchronous' reader copies a chunk only while
// no writer workgroup is inside it (ended == began before the copy, began unchanged
// after it), so a pulled chunk never holds a half-applied push; it waits only for
// writer workgroups that are already running, so no interleaving of streams or
// processes can deadlock.  'hogwild' readers copy without looking at the counters.
__device__ __forceinline__ float* ps_theta(const PsArgs& a, int owner) {
  return reinterpret_cast<float*>(a.base[owner] + PEER_DATA_OFF);
}
__device__ __forceinline__ unsigned* ps_ctr(const PsArgs& a, int owner, long long c, int which) {
  return reinterpret_cast<unsigned*>(a.base[owner] + a.ctr_off) + c * 32 + which * 16;
}
__device__ __forceinline__ int ps_owner(const PsArgs& a, long long c) { return (int)(c * a.world / a.nchunks); }

__device__ __forceinline__ bool ps_timed_out(const PsArgs& a, unsigned long long t0) {
  if (wall_clock64() - t0 <= a.timeout_ticks) return false;
  __hip_atomic_store(err_ptr(a.base[a.rank]), 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return true;
}

// dst = theta, one chunk per workgroup
// dst = theta; with P != null also every replica row P[r] (stride sP) = theta: a pull
// straight into the masters of a trainer whose step kernel reads only those
__global__ __launch_bounds__(256) void ps_gather_kernel(PsArgs a, float* __restrict__ dst, int consistent,
                                                        float* __restrict__ P, long long sP, int R) {
  const long long c = blockIdx.x;
  const long long lo = c * a.chunk, hi = lo + a.chunk < a.n ? lo + a.chunk : a.n;
  const int owner = ps_owner(a, c);
  const float* th = ps_theta(a, owner);
  auto copy_all = [&]() {
    copy_span(th, dst, lo, hi);
    for (int r = 0; P && r < R; ++r) {
      float* row = P + (long long)r * sP;
      if ((reinterpret_cast<uintptr_t>(row) & 15) == 0) {
        copy_span(th, row, lo, hi);
      } else {  // replica rows of an odd-sized vector are only 8-byte aligned
        for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) row[i] = th[i];
      }
    }
  };
  if (!consistent) {
    copy_all();
    return;
  }
  unsigned* began = ps_ctr(a, owner, c, 0);
  unsigned* ended = ps_ctr(a, owner, c, 1);
  // pushes made INSIDE a persistent launch (persist.hip ps_push_begin / ps_push_end) bracket
  // their slice with per-slice began / ended words in rank 0's flag area instead of these
  // chunk counters: the consistent pull also waits until no such writer is inside any
  // slice, and retries if one began during the copy (thread t watches slice t)
  const unsigned* sb = reinterpret_cast<const unsigned*>(a.base[0] + PEER_FLAG_OFF) + threadIdx.x * 16;
  const unsigned* se = sb + PEER_MAX_BLOCKS * 16;
  __shared__ unsigned snap, ssum;
  __shared__ int state;  // 0 retry, 1 done, 2 give up
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    if (threadIdx.x == 0) {
      for (;;) {
        const unsigned e = load_flag(ended);
        const unsigned b = load_flag(began);
        if (b == e) { snap = b; break; }
        if (ps_timed_out(a, t0)) { snap = b; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      ssum = 0u;
    }
    unsigned mb = 0u;
    for (;;) {   // every slice quiet (one wait for the whole workgroup)
      const unsigned e = load_flag(se);
      mb = load_flag(sb);
      if (__syncthreads_and(mb == e)) break;
      if (__syncthreads_or(ps_timed_out(a, t0))) break;   // one decision for the workgroup
      __builtin_amdgcn_s_sleep(1);
    }
    atomicAdd(&ssum, mb);
    __syncthreads();
    const unsigned s0 = ssum;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    copy_all();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the copy's loads complete before the re-check
    __syncthreads();
    if (threadIdx.x == 0) ssum = 0u;
    __syncthreads();
    atomicAdd(&ssum, load_flag(sb));
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned b2 = load_flag(began);
      state = (b2 == snap && ssum == s0) ? 1 : (ps_timed_out(a, t0) ? 2 : 0);
    }
    __syncthreads();
    if (state != 0) return;
  }
}

// theta += sum_r (P[r] - before) with fp32 atomics, one chunk per workgroup
__global__ __launch_bounds__(256) void ps_push_kernel(PsArgs a, const float* __restrict__ P, long long sP, int R,
                                                      const float* __restrict__ before) {
  const long long c = blockIdx.x;
  const long long lo = c * a.chunk, hi = lo + a.chunk < a.n ? lo + a.chunk : a.n;
  const int owner = ps_owner(a, c);
  float* th = ps_theta(a, owner);
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(ps_ctr(a, owner, c, 0), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const float b = before[i];
    float d = 0.f;
    for (int r = 0; r < R; ++r) d += P[(long long)r * sP + i] - b;  // Sterbenz-exact differences
    if (d != 0.f) __hip_atomic_fetch_add(th + i, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(ps_ctr(a, owner, c, 1), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// theta = src (initialisation, no concurrent writers)
__global__ __launch_bounds__(256) void ps_set_kernel(PsArgs a, const float* __restrict__ src) {
  const long long c = blockIdx.x;
  const long long lo = c * a.chunk, hi = lo + a.chunk < a.n ? lo + a.chunk : a.n;
  copy_span(src, ps_theta(a, ps_owner(a, c)), lo, hi);
}

}  // namespace ea

using namespace ea;

extern "C" hipError_t ea_allreduce_peer(const PeerArgs* a, int twoshot, int nblocks, hipStream_t s) {
  if (twoshot) hipLaunchKernelGGL(allreduce_twoshot_kernel, dim3(nblocks), dim3(256), 0, s, *a);
  else hipLaunchKernelGGL(allreduce_oneshot_kernel, dim3(nblocks), dim3(256), 0, s, *a);
  return hipGetLastError();
}

extern "C" hipError_t ea_ps_gather(const PsArgs* a, float* dst, int consistent, float* P, long long sP, int R,
                                   hipStream_t s) {
  hipLaunchKernelGGL(ps_gather_kernel, dim3((unsigned)a->nchunks), dim3(256), 0, s, *a, dst, consistent, P, sP, R);
  return hipGetLastError();
}

extern "C" hipError_t ea_ps_push(const PsArgs* a, const float* P, long long sP, int R, const float* before,
                                 hipStream_t s) {
  hipLaunchKernelGGL(ps_push_kernel, dim3((unsigned)a->nchunks), dim3(256), 0, s, *a, P, sP, R, before);
  return hipGetLastError();
}

extern "C" hipError_t ea_ps_set(const PsArgs* a, const float* src, hipStream_t s) {
  hipLaunchKernelGGL(ps_set_kernel, dim3((unsigned)a->nchunks), dim3(256), 0, s, *a, src);
  return hipGetLastError();
}
