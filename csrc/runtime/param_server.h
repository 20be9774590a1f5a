// Device-resident parameter server for the asynchronous / hogwild modes.
//
// Replaces the reference's Flask/socket parameter servers
// (reference elephas/parameter/server.py:42-233, client.py:41-91): the master
// parameters live in HBM of the owning GPU as one flat fp32 vector.
//   pull  = device-to-device copy (peer copy over xGMI for a remote owner)
//   push  = remote-subtract kernel  theta <- theta - delta  run by the pusher
//           directly on the owner's memory (peer RMW over xGMI)
// 'asynchronous' mode serialises pushes and pulls with a writer-priority
// reader/writer lock (reference utils/rwlock.py:10-67 semantics), in-process or
// shared between processes through POSIX shared memory; 'hogwild' takes no lock
// and lets concurrent updates race (reference server.py:109-131 guards).
#pragma once
#include <hip/hip_runtime.h>
#include "rwlock.h"

#include <atomic>
#include <memory>
#include <shared_mutex>
#include <stdexcept>
#include <string>

namespace ea {

// Run `enqueue(theta)` (device work reading the server's vector on stream s) under
// the read lock; with `sync` the stream is drained before the lock is released.
template <class Lock, class F>
inline void locked_read(Lock* lock, bool locked, bool sync, float* theta, hipStream_t s, F&& enqueue) {
  if (locked) lock->lock_shared();
  try {
    enqueue(theta);
    if (sync) {
      const hipError_t e = hipStreamSynchronize(s);
      if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ps read sync: ") + hipGetErrorString(e));
    }
  } catch (...) {
    if (locked) lock->unlock_shared();
    throw;
  }
  if (locked) lock->unlock_shared();
}

class DeviceParameterServer {
 public:
  DeviceParameterServer(long long n, int locked, int device, const std::string& lock_name = "");
  ~DeviceParameterServer();
  void pull(float* dst, hipStream_t s);
  void push(const float* delta, hipStream_t s);
  // R lockstep replicas (rows of P, stride sP): pull into all of them + `before`;
  // push theta += sum_r P[r] - R * before
  void pull_replicas(float* P, long long sP, int R, float* before, hipStream_t s);
  void push_replicas(const float* P, long long sP, int R, const float* before, hipStream_t s);
  void set(const float* src, hipStream_t s);
  // pull fused into a caller's kernel (e.g. Executor::refresh_from)
  template <class F> void pull_with(hipStream_t s, F&& enqueue) {
    locked_read(lock_.get(), locked_ != 0, locked_ != 0, p_, s, enqueue);
    pulls_++;
  }
  std::string ipc_handle() const;
  float* data() const { return p_; }
  long long size() const { return n_; }
  long long pushes() const { return pushes_.load(); }
  long long pulls() const { return pulls_.load(); }

 private:
  long long n_;
  int locked_;
  int device_;
  float* p_ = nullptr;
  std::unique_ptr<RWLockBase> lock_;
  std::atomic<long long> pushes_{0}, pulls_{0};
};

class RemoteParameterServer {
 public:
  RemoteParameterServer(const std::string& handle, long long n, int locked, const std::string& lock_name);
  ~RemoteParameterServer();
  void pull(float* dst, hipStream_t s);
  void push(const float* delta, hipStream_t s);
  void pull_replicas(float* P, long long sP, int R, float* before, hipStream_t s);
  void push_replicas(const float* P, long long sP, int R, const float* before, hipStream_t s);
  template <class F> void pull_with(hipStream_t s, F&& enqueue) {
    locked_read(lock_.get(), locked_ != 0, true, p_, s, enqueue);
  }
  long long size() const { return n_; }

 private:
  long long n_;
  int locked_;
  float* p_ = nullptr;
  std::unique_ptr<RWLockBase> lock_;
};

}  // namespace ea
