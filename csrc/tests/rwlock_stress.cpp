// Host-side stress test of the parameter-server locks (csrc/runtime/rwlock.cpp),
// built with -fsanitize=address or -fsanitize=thread by tests/test_host_sanitizers.py.
//
// Invariants checked (the reference's lock tests are TODO stubs,
// tests/utils/test_rwlock.py:1):
//   * a writer is alone: no reader and no other writer inside while it holds the lock
//   * readers do overlap (the lock is not a plain mutex)
//   * a "parameter vector" updated as theta -= delta under the write lock loses no
//     update (the reference SocketServer loses them: server.py:204-208)
//   * the process-shared variant gives the same guarantees across fork()ed processes
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "runtime/rwlock.h"

using namespace ea;

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

static int in_process() {
  auto lock = make_lock("");
  std::atomic<int> readers{0}, writers{0}, max_readers{0};
  std::atomic<bool> bad{false};
  std::vector<double> theta(256, 0.0);
  const int kWriters = 4, kReaders = 6, kIters = 4000;
  std::vector<std::thread> ts;
  for (int w = 0; w < kWriters; ++w)
    ts.emplace_back([&] {
      for (int i = 0; i < kIters; ++i) {
        lock->lock();
        if (writers.fetch_add(1) != 0 || readers.load() != 0) bad = true;
        for (auto& v : theta) v -= 1.0;  // theta <- theta - delta
        writers.fetch_sub(1);
        lock->unlock();
      }
    });
  for (int r = 0; r < kReaders; ++r)
    ts.emplace_back([&] {
      for (int i = 0; i < kIters; ++i) {
        lock->lock_shared();
        const int now = readers.fetch_add(1) + 1;
        int m = max_readers.load();
        while (now > m && !max_readers.compare_exchange_weak(m, now)) {}
        if (writers.load() != 0) bad = true;
        const double first = theta[0];
        for (auto v : theta)
          if (v != first) bad = true;  // a torn (half-applied) update is visible
        readers.fetch_sub(1);
        lock->unlock_shared();
      }
    });
  for (auto& t : ts) t.join();
  if (bad) return fail("in-process exclusion / torn read");
  for (auto v : theta)
    if (v != -1.0 * kWriters * kIters) return fail("in-process lost update");
  if (max_readers.load() < 2) std::fprintf(stderr, "note: readers never overlapped (scheduler)\n");
  return 0;
}

static int cross_process() {
  const std::string name = "/elephas_amd_stress_" + std::to_string(getpid());
  shm_rwlock_create(name);
  // shared counters + parameter vector
  struct Shared {
    std::atomic<int> writers, readers, bad;
    double theta[64];
  };
  auto* sh = static_cast<Shared*>(
      mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0));
  new (sh) Shared();
  for (double& v : sh->theta) v = 0.0;
  const int kProcs = 3, kIters = 2000;
  std::vector<pid_t> kids;
  for (int p = 0; p < kProcs; ++p) {
    pid_t pid = fork();
    if (pid == 0) {
      auto lock = make_lock(name);
      for (int i = 0; i < kIters; ++i) {
        if (i % 3 == 0) {
          lock->lock_shared();
          if (sh->writers.load() != 0) sh->bad = 1;
          const double f = sh->theta[0];
          for (double v : sh->theta)
            if (v != f) sh->bad = 1;
          lock->unlock_shared();
        } else {
          lock->lock();
          if (sh->writers.fetch_add(1) != 0) sh->bad = 1;
          for (double& v : sh->theta) v += 1.0;
          sh->writers.fetch_sub(1);
          lock->unlock();
        }
      }
      _exit(0);
    }
    kids.push_back(pid);
  }
  int rc = 0;
  for (pid_t k : kids) {
    int st = 0;
    waitpid(k, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = fail("child crashed");
  }
  int writes = 0;
  for (int i = 0; i < kIters; ++i) writes += (i % 3 != 0);
  if (sh->bad.load()) rc = fail("cross-process exclusion / torn read");
  for (double v : sh->theta)
    if (v != (double)writes * kProcs) { rc = fail("cross-process lost update"); break; }
  shm_rwlock_destroy(name);
  munmap(sh, sizeof(Shared));
  return rc;
}

int main(int argc, char** argv) {
  const std::string which = argc > 1 ? argv[1] : "all";
  int rc = 0;
  if (which == "all" || which == "threads") rc |= in_process();
  if (which == "all" || which == "procs") rc |= cross_process();
  if (rc == 0) std::printf("rwlock stress OK\n");
  return rc;
}
