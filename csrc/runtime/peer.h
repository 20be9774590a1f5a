// Host side of the peer-memory collectives and the sharded device parameter
// server (kernels: csrc/kernels/peer.hip).
//
// PeerBuffer  one uncached device allocation per rank, exported with a HIP IPC
//             handle and mapped by every other rank of the node (the handles are
//             exchanged by the caller, e.g. torch.distributed all_gather_object).
// PeerAllReduce  in-place / out-of-place sum all-reduce over the mapped buffers
//             (one-shot below `twoshot_min_bytes`, two-shot above); messages larger
//             than the staging capacity run as consecutive capacity-sized calls.
// ShardedParameterServer  theta sharded in chunks over the ranks' buffers; pulls
//             and pushes are single kernels reading / atomically updating the
//             owners' memory (replaces the reference's Flask / socket servers,
//             reference elephas/parameter/server.py).
// All operations are enqueued on the caller's stream and never synchronise it;
// collective calls must be issued in the same order on every rank, each rank on
// one stream.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "kernels/peer_args.h"

namespace ea {

class PeerBuffer {
 public:
  PeerBuffer(int rank, int world, long long data_bytes, int device);
  ~PeerBuffer();
  PeerBuffer(const PeerBuffer&) = delete;
  PeerBuffer& operator=(const PeerBuffer&) = delete;
  std::string handle() const;
  // handles[r] for every rank (own entry ignored)
  void open(const std::vector<std::string>& handles);
  bool opened() const { return opened_; }
  char* base(int r) const { return bases_[r]; }
  char* local() const { return bases_[rank_]; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  long long data_bytes() const { return data_bytes_; }
  // error word written by kernels whose wait timed out (0 = none); synchronous read
  unsigned error() const;
  void clear_error();
  // the caller guarantees no rank will touch this buffer again (every rank has
  // synchronised its device and passed a process-group barrier): free it on destruction
  void release() { released_ = true; }

 private:
  int rank_, world_, device_;
  long long data_bytes_;
  bool opened_ = false;
  bool released_ = false;
  std::vector<char*> bases_;
};

class PeerAllReduce {
 public:
  // cap_elems: staging elements per parity (the buffer holds 4 x cap_elems floats)
  PeerAllReduce(int rank, int world, long long cap_elems, int device, double timeout_s = 20.0);
  std::string handle() const { return buf_.handle(); }
  void open(const std::vector<std::string>& handles) { buf_.open(handles); }
  // out = sum over ranks of in (may alias); algo: -1 auto, 0 one-shot, 1 two-shot
  void all_reduce(const float* in, float* out, long long n, hipStream_t s, int algo = -1);
  // Graph-capturable form: the epoch is derived on the device, so one captured call
  // can be replayed any number of times.  Every call on this object must then use
  // graph mode with the same n and algo (n <= capacity), on every rank.
  void all_reduce_graph(const float* in, float* out, long long n, hipStream_t s, int algo = -1);
  unsigned error() const { return buf_.error(); }
  void clear_error() { buf_.clear_error(); }
  void release() { buf_.release(); }
  long long capacity() const { return cap_; }
  long long calls() const { return epoch_; }
  void set_twoshot_min_bytes(long long b) { twoshot_min_bytes_ = b; }
  long long twoshot_min_bytes() const { return twoshot_min_bytes_; }

 private:
  void launch(const float* in, float* out, long long n, hipStream_t s, int algo, bool dev_epoch);
  PeerBuffer buf_;
  long long cap_;
  unsigned epoch_ = 0;
  long long graph_n_ = -1;
  int graph_algo_ = -2;
  unsigned long long timeout_ticks_;
  long long twoshot_min_bytes_ = 1LL << 20;
};

class ShardedParameterServer {
 public:
  // consistent: 1 = 'asynchronous' (a pulled chunk never holds a half-applied push),
  // 0 = 'hogwild' (pulls copy whatever is there); pushes never lose an update
  ShardedParameterServer(int rank, int world, long long n, int consistent, int device, long long chunk = 4096,
                         double timeout_s = 30.0);
  std::string handle() const { return buf_.handle(); }
  void open(const std::vector<std::string>& handles) { buf_.open(handles); }
  void set(const float* src, hipStream_t s);          // theta = src (no concurrent pushes)
  void pull(float* dst, hipStream_t s);               // dst = theta
  void pull_replicas(float* dst, float* P, long long sP, int R, hipStream_t s);  // dst = P[r] = theta
  // theta += sum_r (P[r] - before), P rows of stride sP
  void push_replicas(const float* P, long long sP, int R, const float* before, hipStream_t s);
  void push_delta(const float* delta, hipStream_t s);  // theta -= delta (reference update semantics)
  unsigned error() const { return buf_.error(); }
  void clear_error() { buf_.clear_error(); }
  void release() { buf_.release(); }
  long long size() const { return n_; }
  int consistent() const { return consistent_; }
  long long nchunks() const { return nchunks_; }
  long long shard_begin(int r) const;                 // first parameter owned by rank r
  // the kernel view of the server (a persistent step kernel's in-launch hook, persist.hip)
  PsArgs kernel_args() const { return args(); }

 private:
  static long long padded(long long n) { return (n + 3) / 4 * 4 + 4; }
  PsArgs args() const;
  long long n_, chunk_, nchunks_;
  int consistent_;
  unsigned long long timeout_ticks_;
  PeerBuffer buf_;
};

}  // namespace ea
