// Kernel arguments and buffer layout of the peer-memory collectives and the
// sharded parameter server (csrc/kernels/peer.hip, csrc/runtime/peer.cpp).
#pragma once

namespace ea {

constexpr int PEER_MAX_RANKS = 8;          // one node: 8 MI355X on xGMI
constexpr int PEER_MAX_BLOCKS = 256;       // flags per phase (one per workgroup)
// byte offsets inside every rank's buffer (identical on all ranks)
constexpr long long PEER_FLAG_OFF = 0;                                   // [2 phases][256 blocks] x 64 B
constexpr long long PEER_ERR_OFF = 2LL * PEER_MAX_BLOCKS * 64;           // error word (timeouts)
constexpr long long PEER_DATA_OFF = 64 * 1024;                           // data (16-byte aligned)

struct PeerArgs {
  char* base[PEER_MAX_RANKS];   // every rank's buffer, mapped into this process
  const float* in;
  float* out;
  long long n;                  // elements in this call
  long long cap;                // elements per staging parity
  long long chunk;              // elements per workgroup (multiple of 4)
  long long slice;              // two-shot: elements per rank slice (multiple of 4)
  unsigned long long timeout_ticks;  // 100 MHz wall-clock ticks
  unsigned epoch;
  int dev_epoch;                // 1: each workgroup derives the epoch from its own last flag
  int world, rank;
};

struct PsArgs {
  char* base[PEER_MAX_RANKS];
  long long n;                  // parameters
  long long chunk;              // parameters per chunk (multiple of 4)
  long long nchunks;            // chunk c lives on rank c * world / nchunks
  long long ctr_off;            // byte offset of the per-chunk began/ended counters
  unsigned long long timeout_ticks;
  int world, rank;
  long long shard_begin[PEER_MAX_RANKS];   // first parameter of every rank's shard (n past the last)
};

}  // namespace ea
