#include "rwlock.h"

#include <fcntl.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <shared_mutex>
#include <stdexcept>

namespace ea {

// ------------------------------------------------------------------ locks
class LocalLock : public RWLockBase {
 public:
  void lock_shared() override { m_.lock_shared(); }
  void unlock_shared() override { m_.unlock_shared(); }
  void lock() override { m_.lock(); }
  void unlock() override { m_.unlock(); }

 private:
  std::shared_mutex m_;
};

static std::string shm_path(const std::string& name) { return name[0] == '/' ? name : "/" + name; }

class ShmLock : public RWLockBase {
 public:
  explicit ShmLock(const std::string& name) {
    int fd = shm_open(shm_path(name).c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open failed for lock " + name);
    void* p = mmap(nullptr, sizeof(pthread_rwlock_t), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("mmap failed for lock " + name);
    l_ = reinterpret_cast<pthread_rwlock_t*>(p);
  }
  ~ShmLock() override { munmap(l_, sizeof(pthread_rwlock_t)); }
  void lock_shared() override { pthread_rwlock_rdlock(l_); }
  void unlock_shared() override { pthread_rwlock_unlock(l_); }
  void lock() override { pthread_rwlock_wrlock(l_); }
  void unlock() override { pthread_rwlock_unlock(l_); }

 private:
  pthread_rwlock_t* l_;
};

void shm_rwlock_create(const std::string& name) {
  int fd = shm_open(shm_path(name).c_str(), O_CREAT | O_RDWR | O_TRUNC, 0600);
  if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name);
  if (ftruncate(fd, sizeof(pthread_rwlock_t)) != 0) {
    close(fd);
    throw std::runtime_error("ftruncate failed for " + name);
  }
  void* p = mmap(nullptr, sizeof(pthread_rwlock_t), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("mmap failed for " + name);
  pthread_rwlockattr_t a;
  pthread_rwlockattr_init(&a);
  pthread_rwlockattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  // writer priority, as the reference RWLock (utils/rwlock.py:24-46)
  pthread_rwlockattr_setkind_np(&a, PTHREAD_RWLOCK_PREFER_WRITER_NONRECURSIVE_NP);
  pthread_rwlock_init(reinterpret_cast<pthread_rwlock_t*>(p), &a);
  pthread_rwlockattr_destroy(&a);
  munmap(p, sizeof(pthread_rwlock_t));
}

void shm_rwlock_destroy(const std::string& name) { shm_unlink(shm_path(name).c_str()); }

std::unique_ptr<RWLockBase> make_lock(const std::string& shm_name) {
  if (shm_name.empty()) return std::make_unique<LocalLock>();
  return std::make_unique<ShmLock>(shm_name);
}

}  // namespace ea
