#include "peer.h"

#include <cstdlib>
#include <cstring>
#include <stdexcept>

extern "C" hipError_t ea_allreduce_peer(const ea::PeerArgs* a, int twoshot, int nblocks, hipStream_t s);
extern "C" hipError_t ea_ps_gather(const ea::PsArgs* a, float* dst, int consistent, float* P, long long sP, int R,
                                   hipStream_t s);
extern "C" hipError_t ea_ps_push(const ea::PsArgs* a, const float* P, long long sP, int R, const float* before,
                                 hipStream_t s);
extern "C" hipError_t ea_ps_set(const ea::PsArgs* a, const float* src, hipStream_t s);

namespace ea {

static void chk(hipError_t e, const char* w) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + w + ": " + hipGetErrorString(e));
}

static unsigned long long ticks_for(double seconds, int device) {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) khz = 100000;
  return (unsigned long long)(seconds * (double)khz * 1000.0);
}

// ---------------------------------------------------------------- PeerBuffer
PeerBuffer::PeerBuffer(int rank, int world, long long data_bytes, int device)
    : rank_(rank), world_(world), device_(device), data_bytes_(data_bytes), bases_(world, nullptr) {
  if (world < 1 || world > PEER_MAX_RANKS || rank < 0 || rank >= world)
    throw std::invalid_argument("PeerBuffer: need 0 <= rank < world <= 8");
  chk(hipSetDevice(device), "hipSetDevice");
  const size_t bytes = (size_t)(PEER_DATA_OFF + data_bytes);
  void* p = nullptr;
  // uncached: stores reach HBM and loads bypass L2, so memory written by another
  // GPU over xGMI is never read stale; ELEPHAS_AMD_PEER_CACHED=1 selects plain
  // coarse-grained memory (diagnostics)
  const char* env = std::getenv("ELEPHAS_AMD_PEER_CACHED");
  if (env && env[0] == '1') chk(hipMalloc(&p, bytes), "hipMalloc(peer)");
  else chk(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(peer, uncached)");
  chk(hipMemset(p, 0, bytes), "hipMemset(peer)");
  chk(hipDeviceSynchronize(), "hipDeviceSynchronize(peer)");
  bases_[rank] = static_cast<char*>(p);
  if (world == 1) opened_ = true;
}

// A buffer other ranks have mapped is freed only after release(): a peer's kernel may
// still be reading it (the last collective's reads trail its flag wait), and freeing
// mapped memory under a running kernel faults the reader.  Without release() the
// process exit reclaims it.
PeerBuffer::~PeerBuffer() {
  for (int r = 0; r < world_; ++r) {
    if (!bases_[r] || r == rank_) continue;
    (void)hipIpcCloseMemHandle(bases_[r]);
  }
  if (bases_[rank_] && (world_ == 1 || released_)) (void)hipFree(bases_[rank_]);
}

std::string PeerBuffer::handle() const {
  hipIpcMemHandle_t h;
  chk(hipIpcGetMemHandle(&h, bases_[rank_]), "hipIpcGetMemHandle(peer)");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void PeerBuffer::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::invalid_argument("PeerBuffer::open: one handle per rank");
  if (opened_ && world_ > 1) throw std::runtime_error("PeerBuffer::open: already open");
  chk(hipSetDevice(device_), "hipSetDevice");
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) continue;
    if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("bad IPC handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    chk(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(peer)");
    bases_[r] = static_cast<char*>(p);
  }
  opened_ = true;
}

unsigned PeerBuffer::error() const {
  unsigned v = 0;
  chk(hipMemcpy(&v, bases_[rank_] + PEER_ERR_OFF, sizeof(v), hipMemcpyDeviceToHost), "peer error read");
  return v;
}

void PeerBuffer::clear_error() {
  chk(hipMemset(bases_[rank_] + PEER_ERR_OFF, 0, sizeof(unsigned)), "peer error clear");
}

// ------------------------------------------------------------- PeerAllReduce
PeerAllReduce::PeerAllReduce(int rank, int world, long long cap_elems, int device, double timeout_s)
    : buf_(rank, world, 4 * ((cap_elems + 3) / 4 * 4) * (long long)sizeof(float), device),
      cap_((cap_elems + 3) / 4 * 4),
      timeout_ticks_(ticks_for(timeout_s, device)) {}

void PeerAllReduce::all_reduce(const float* in, float* out, long long n, hipStream_t s, int algo) {
  if (graph_n_ >= 0) throw std::runtime_error("PeerAllReduce: object is in graph mode");
  launch(in, out, n, s, algo, false);
}

void PeerAllReduce::all_reduce_graph(const float* in, float* out, long long n, hipStream_t s, int algo) {
  if (n > cap_) throw std::invalid_argument("PeerAllReduce::all_reduce_graph: n exceeds the staging capacity");
  if (epoch_ != 0) throw std::runtime_error("PeerAllReduce: host-epoch calls were made on this object");
  if (graph_n_ >= 0 && (graph_n_ != n || graph_algo_ != algo))
    throw std::invalid_argument("PeerAllReduce::all_reduce_graph: every call needs the same n and algo");
  graph_n_ = n;
  graph_algo_ = algo;
  launch(in, out, n, s, algo, true);
}

void PeerAllReduce::launch(const float* in, float* out, long long n, hipStream_t s, int algo, bool dev_epoch) {
  if (!buf_.opened()) throw std::runtime_error("PeerAllReduce: peers not opened");
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15)
    throw std::invalid_argument("PeerAllReduce: buffers must be 16-byte aligned");
  const int W = buf_.world();
  if (W == 1) {
    if (in != out && n > 0) chk(hipMemcpyAsync(out, in, n * sizeof(float), hipMemcpyDeviceToDevice, s), "copy");
    return;
  }
  for (long long off = 0; off < n; off += cap_) {
    const long long m = n - off < cap_ ? n - off : cap_;
    const bool two = algo == 1 || (algo < 0 && m * (long long)sizeof(float) >= twoshot_min_bytes_);
    PeerArgs a;
    std::memset(&a, 0, sizeof(a));
    for (int r = 0; r < W; ++r) a.base[r] = buf_.base(r);
    a.in = in + off;
    a.out = out + off;
    a.n = m;
    a.cap = cap_;
    a.world = W;
    a.rank = buf_.rank();
    a.timeout_ticks = timeout_ticks_;
    a.dev_epoch = dev_epoch ? 1 : 0;
    a.epoch = dev_epoch ? 0u : ++epoch_;
    // work per workgroup: >= 1024 elements, <= PEER_MAX_BLOCKS workgroups
    const long long span = two ? (m + W - 1) / W : m;
    long long chunk = (span + PEER_MAX_BLOCKS - 1) / PEER_MAX_BLOCKS;
    if (chunk < 1024) chunk = 1024;
    chunk = (chunk + 3) / 4 * 4;
    a.chunk = chunk;
    a.slice = two ? ((span + 3) / 4 * 4) : m;
    const int nb = (int)((span + chunk - 1) / chunk);
    chk(ea_allreduce_peer(&a, two ? 1 : 0, nb < 1 ? 1 : nb, s), "allreduce_peer");
  }
}

// ---------------------------------------------------- ShardedParameterServer
// Buffer of every rank: [theta | zero vector] (padded(n) floats each), then two
// 64-byte counter lines per chunk.  Every rank allocates the full layout and
// uses the chunks it owns (the rest is a few MB of slack on a 288 GB device).
ShardedParameterServer::ShardedParameterServer(int rank, int world, long long n, int consistent, int device,
                                               long long chunk, double timeout_s)
    : n_(n),
      chunk_((chunk + 3) / 4 * 4),
      nchunks_((n + (chunk + 3) / 4 * 4 - 1) / ((chunk + 3) / 4 * 4)),
      consistent_(consistent),
      timeout_ticks_(ticks_for(timeout_s, device)),
      buf_(rank, world, 2 * padded(n) * (long long)sizeof(float) + 256 + nchunks_ * 128, device) {
  if (n <= 0) throw std::invalid_argument("ShardedParameterServer: n must be positive");
}

PsArgs ShardedParameterServer::args() const {
  if (!buf_.opened()) throw std::runtime_error("ShardedParameterServer: peers not opened");
  PsArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int r = 0; r < buf_.world(); ++r) a.base[r] = buf_.base(r);
  a.n = n_;
  a.chunk = chunk_;
  a.nchunks = nchunks_;
  a.ctr_off = (PEER_DATA_OFF + 2 * padded(n_) * (long long)sizeof(float) + 255) / 256 * 256;
  a.timeout_ticks = timeout_ticks_;
  a.world = buf_.world();
  a.rank = buf_.rank();
  for (int r = 0; r < PEER_MAX_RANKS; ++r) a.shard_begin[r] = r < a.world ? shard_begin(r) : n_;
  return a;
}

long long ShardedParameterServer::shard_begin(int r) const {
  // first chunk c with c * world / nchunks >= r
  const long long W = buf_.world();
  const long long c = (r * nchunks_ + W - 1) / W;
  const long long b = c * chunk_;
  return b < n_ ? b : n_;
}

void ShardedParameterServer::set(const float* src, hipStream_t s) {
  const PsArgs a = args();
  chk(ea_ps_set(&a, src, s), "ps_set");
}

void ShardedParameterServer::pull(float* dst, hipStream_t s) {
  if (reinterpret_cast<uintptr_t>(dst) & 15) throw std::invalid_argument("ps pull: destination must be 16-byte aligned");
  const PsArgs a = args();
  chk(ea_ps_gather(&a, dst, consistent_, nullptr, 0, 0, s), "ps_gather");
}

void ShardedParameterServer::pull_replicas(float* dst, float* P, long long sP, int R, hipStream_t s) {
  if (reinterpret_cast<uintptr_t>(dst) & 15) throw std::invalid_argument("ps pull: destination must be 16-byte aligned");
  if (reinterpret_cast<uintptr_t>(P) & 15) throw std::invalid_argument("ps pull: replica rows must start 16-byte aligned");
  const PsArgs a = args();
  chk(ea_ps_gather(&a, dst, consistent_, P, sP, R, s), "ps_gather");
}

void ShardedParameterServer::push_replicas(const float* P, long long sP, int R, const float* before, hipStream_t s) {
  const PsArgs a = args();
  chk(ea_ps_push(&a, P, sP, R, before, s), "ps_push");
}

void ShardedParameterServer::push_delta(const float* delta, hipStream_t s) {
  // theta += (0 - delta): P = the zero vector that follows theta in this rank's buffer
  const PsArgs a = args();
  const float* zero = reinterpret_cast<const float*>(buf_.local() + PEER_DATA_OFF) + padded(n_);
  chk(ea_ps_push(&a, zero, 0, 1, delta, s), "ps_push");
}

}  // namespace ea
