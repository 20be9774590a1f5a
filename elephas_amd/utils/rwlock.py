"""Reader/writer lock with writer priority (reference elephas/utils/rwlock.py:10-67).

Several readers may hold the lock, or exactly one writer; a waiting writer
blocks new readers.  Used by the host-side (http/socket) parameter servers;
the device parameter server uses the native std::shared_mutex / POSIX shm
rwlock equivalent (csrc/runtime/param_server.cpp)."""
import threading


class RWLock:
    def __init__(self):
        self.rwlock = 0          # >0: readers holding, -1: writer holding
        self.writers_waiting = 0
        self.monitor = threading.Lock()
        self.readers_ok = threading.Condition(self.monitor)
        self.writers_ok = threading.Condition(self.monitor)

    def acquire_read(self):
        with self.monitor:
            while self.rwlock < 0 or self.writers_waiting:
                self.readers_ok.wait()
            self.rwlock += 1

    def acquire_write(self):
        with self.monitor:
            while self.rwlock != 0:
                self.writers_waiting += 1
                self.writers_ok.wait()
                self.writers_waiting -= 1
            self.rwlock = -1

    def release(self):
        with self.monitor:
            if self.rwlock < 0:
                self.rwlock = 0
            elif self.rwlock > 0:
                self.rwlock -= 1
            else:
                raise RuntimeError("release of an unlocked RWLock")
            wake_writers = self.writers_waiting and self.rwlock == 0
            wake_readers = self.writers_waiting == 0
            if wake_writers:
                self.writers_ok.notify()
            elif wake_readers:
                self.readers_ok.notify_all()

    # context-manager helpers
    class _Ctx:
        def __init__(self, acq, rel):
            self.acq, self.rel = acq, rel

        def __enter__(self):
            self.acq()

        def __exit__(self, *a):
            self.rel()

    def read_locked(self):
        return RWLock._Ctx(self.acquire_read, self.release)

    def write_locked(self):
        return RWLock._Ctx(self.acquire_write, self.release)
