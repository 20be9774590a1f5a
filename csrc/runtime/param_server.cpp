#include "param_server.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

extern "C" hipError_t ea_ps_sub(float* p, const float* d, long long n, float scale, int atomic, hipStream_t s);
extern "C" hipError_t ea_ps_pull_replicas(const float* src, float* P, long long sP, int R, float* before, long long n,
                                          hipStream_t s);
extern "C" hipError_t ea_ps_push_replicas(float* p, const float* P, long long sP, int R, const float* before,
                                          long long n, int atomic, hipStream_t s);

namespace ea {

static void chk(hipError_t e, const char* w) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + w + ": " + hipGetErrorString(e));
}

// ------------------------------------------------------------ local owner
DeviceParameterServer::DeviceParameterServer(long long n, int locked, int device, const std::string& lock_name)
    : n_(n), locked_(locked), device_(device), lock_(make_lock(lock_name)) {
  chk(hipSetDevice(device), "hipSetDevice");
  chk(hipMalloc(&p_, (size_t)n * sizeof(float)), "hipMalloc(ps)");
  chk(hipMemset(p_, 0, (size_t)n * sizeof(float)), "hipMemset(ps)");
}

DeviceParameterServer::~DeviceParameterServer() {
  if (p_) (void)hipFree(p_);
}

void DeviceParameterServer::pull(float* dst, hipStream_t s) {
  if (locked_) lock_->lock_shared();
  try {
    chk(hipMemcpyAsync(dst, p_, (size_t)n_ * sizeof(float), hipMemcpyDeviceToDevice, s), "ps.pull");
    if (locked_) chk(hipStreamSynchronize(s), "ps.pull sync");
  } catch (...) {
    if (locked_) lock_->unlock_shared();
    throw;
  }
  if (locked_) lock_->unlock_shared();
  pulls_++;
}

void DeviceParameterServer::push(const float* delta, hipStream_t s) {
  if (locked_) lock_->lock();
  try {
    chk(ea_ps_sub(p_, delta, n_, 1.f, 0, s), "ps.push");
    if (locked_) chk(hipStreamSynchronize(s), "ps.push sync");
  } catch (...) {
    if (locked_) lock_->unlock();
    throw;
  }
  if (locked_) lock_->unlock();
  pushes_++;
}

void DeviceParameterServer::pull_replicas(float* P, long long sP, int R, float* before, hipStream_t s) {
  if (locked_) lock_->lock_shared();
  try {
    chk(ea_ps_pull_replicas(p_, P, sP, R, before, n_, s), "ps.pull_replicas");
    if (locked_) chk(hipStreamSynchronize(s), "ps.pull_replicas sync");
  } catch (...) {
    if (locked_) lock_->unlock_shared();
    throw;
  }
  if (locked_) lock_->unlock_shared();
  pulls_++;
}

void DeviceParameterServer::push_replicas(const float* P, long long sP, int R, const float* before, hipStream_t s) {
  if (locked_) lock_->lock();
  try {
    chk(ea_ps_push_replicas(p_, P, sP, R, before, n_, 0, s), "ps.push_replicas");
    if (locked_) chk(hipStreamSynchronize(s), "ps.push_replicas sync");
  } catch (...) {
    if (locked_) lock_->unlock();
    throw;
  }
  if (locked_) lock_->unlock();
  pushes_++;
}

void DeviceParameterServer::set(const float* src, hipStream_t s) {
  lock_->lock();
  try {
    chk(hipMemcpyAsync(p_, src, (size_t)n_ * sizeof(float), hipMemcpyDeviceToDevice, s), "ps.set");
    chk(hipStreamSynchronize(s), "ps.set sync");
  } catch (...) {
    lock_->unlock();
    throw;
  }
  lock_->unlock();
}

std::string DeviceParameterServer::ipc_handle() const {
  hipIpcMemHandle_t h;
  chk(hipIpcGetMemHandle(&h, p_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

// ----------------------------------------------------------- remote (xGMI)
RemoteParameterServer::RemoteParameterServer(const std::string& handle, long long n, int locked,
                                             const std::string& lock_name)
    : n_(n), locked_(locked), lock_(make_lock(lock_name)) {
  if (handle.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("bad IPC handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  void* p = nullptr;
  chk(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  p_ = reinterpret_cast<float*>(p);
}

RemoteParameterServer::~RemoteParameterServer() {
  if (p_) (void)hipIpcCloseMemHandle(p_);
}

void RemoteParameterServer::pull(float* dst, hipStream_t s) {
  if (locked_) lock_->lock_shared();
  try {
    chk(hipMemcpyAsync(dst, p_, (size_t)n_ * sizeof(float), hipMemcpyDeviceToDevice, s), "remote.pull");
    chk(hipStreamSynchronize(s), "remote.pull sync");
  } catch (...) {
    if (locked_) lock_->unlock_shared();
    throw;
  }
  if (locked_) lock_->unlock_shared();
}

void RemoteParameterServer::push(const float* delta, hipStream_t s) {
  if (locked_) lock_->lock();
  try {
    chk(ea_ps_sub(p_, delta, n_, 1.f, 0, s), "remote.push");
    chk(hipStreamSynchronize(s), "remote.push sync");
  } catch (...) {
    if (locked_) lock_->unlock();
    throw;
  }
  if (locked_) lock_->unlock();
}

void RemoteParameterServer::pull_replicas(float* P, long long sP, int R, float* before, hipStream_t s) {
  if (locked_) lock_->lock_shared();
  try {
    chk(ea_ps_pull_replicas(p_, P, sP, R, before, n_, s), "remote.pull_replicas");
    chk(hipStreamSynchronize(s), "remote.pull_replicas sync");
  } catch (...) {
    if (locked_) lock_->unlock_shared();
    throw;
  }
  if (locked_) lock_->unlock_shared();
}

void RemoteParameterServer::push_replicas(const float* P, long long sP, int R, const float* before, hipStream_t s) {
  if (locked_) lock_->lock();
  try {
    chk(ea_ps_push_replicas(p_, P, sP, R, before, n_, 0, s), "remote.push_replicas");
    chk(hipStreamSynchronize(s), "remote.push_replicas sync");
  } catch (...) {
    if (locked_) lock_->unlock();
    throw;
  }
  if (locked_) lock_->unlock();
}

}  // namespace ea
