// Reader/writer locks of the parameter server (host code only: no HIP), split
// out of param_server.cpp so it can be built and stress-tested under
// AddressSanitizer / ThreadSanitizer on the CPU (tests/test_host_sanitizers.py).
//   LocalLock -- in-process std::shared_mutex
//   ShmLock   -- process-shared pthread rwlock in POSIX shared memory with writer
//                priority (the reference RWLock, utils/rwlock.py:10-67)
#pragma once
#include <memory>
#include <string>

namespace ea {

class RWLockBase {
 public:
  virtual ~RWLockBase() = default;
  virtual void lock_shared() = 0;
  virtual void unlock_shared() = 0;
  virtual void lock() = 0;
  virtual void unlock() = 0;
};

std::unique_ptr<RWLockBase> make_lock(const std::string& shm_name);  // "" -> in-process
void shm_rwlock_create(const std::string& name);
void shm_rwlock_destroy(const std::string& name);

}  // namespace ea
