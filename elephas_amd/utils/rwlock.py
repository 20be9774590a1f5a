"""Writer-preferring shared/exclusive lock for the host-side (http / socket)
parameter servers -- the role of reference elephas/utils/rwlock.py:10-67.

Design: one condition variable guards a small state record (number of shared
holders, whether an exclusive holder exists, how many exclusive requests are
queued).  Shared requests back off while any exclusive request is queued, so a
stream of pulls cannot starve a push; every state change wakes all waiters and
each re-checks its own admission predicate (simpler to reason about than
targeted wake-ups, and the waiter count here is the number of worker threads).
The device parameter server does not use it: its pulls and pushes are
lock-free kernels with per-chunk counters (csrc/kernels/peer.hip).
"""
import threading
from contextlib import contextmanager


class RWLock:
    def __init__(self):
        self._cv = threading.Condition(threading.Lock())
        self._shared = 0          # threads holding the lock shared
        self._exclusive = False   # a thread holds it exclusively
        self._queued = 0          # exclusive requests waiting for admission

    # ----------------------------------------------------------- admission
    def acquire_read(self) -> None:
        with self._cv:
            self._cv.wait_for(lambda: not self._exclusive and self._queued == 0)
            self._shared += 1

    def acquire_write(self) -> None:
        with self._cv:
            self._queued += 1
            try:
                self._cv.wait_for(lambda: not self._exclusive and self._shared == 0)
            finally:
                self._queued -= 1
            self._exclusive = True

    def release(self) -> None:
        """Release one hold, shared or exclusive (whichever this lock is in)."""
        with self._cv:
            if self._exclusive:
                self._exclusive = False
            elif self._shared:
                self._shared -= 1
            else:
                raise RuntimeError("release of an unlocked RWLock")
            self._cv.notify_all()

    # ------------------------------------------------------------ helpers
    @contextmanager
    def read_locked(self):
        self.acquire_read()
        try:
            yield self
        finally:
            self.release()

    @contextmanager
    def write_locked(self):
        self.acquire_write()
        try:
            yield self
        finally:
            self.release()
