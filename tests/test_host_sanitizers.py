"""Race detection / sanitizers on the native HOST code.

The parameter-server reader/writer locks (csrc/runtime/rwlock.cpp) are built
with AddressSanitizer and with ThreadSanitizer into a standalone stress program
(csrc/tests/rwlock_stress.cpp) and run on the CPU: writer exclusion, reader
concurrency, no lost theta <- theta - delta updates, in-process and across
fork()ed processes through the POSIX shared-memory lock. (GPU sanitizers are not
available on this pool; device code is covered by the numerics / determinism
tests in test_native_gpu.py.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
CXX = shutil.which("g++") or shutil.which("clang++")


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
@pytest.mark.parametrize("san,mode", [("address", "all"), ("thread", "threads")])
def test_rwlock_under_sanitizer(tmp_path, san, mode):
    exe = str(tmp_path / f"rwlock_{san}")
    cmd = [CXX, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-I", CSRC,
           os.path.join(CSRC, "runtime", "rwlock.cpp"), os.path.join(CSRC, "tests", "rwlock_stress.cpp"),
           "-o", exe, "-lpthread", "-lrt"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, mode], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rwlock stress OK" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
