"""In-tree build of the native runtime ``elephas_amd._C`` for gfx950.

Every source is compiled directly with ``hipcc --offload-arch=gfx950`` (no
hipify, no torch headers) and linked into one pybind11 extension that lives
next to this file, so it travels with the repository snapshot to the GPU box.
Object files are cached under ``build/`` and rebuilt only when a source or a
header is newer.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("ELEPHAS_AMD_ARCH", "gfx950")

SOURCES = [
    "kernels/gemm.hip",
    "kernels/gemm_cfg0_bf16.hip",
    "kernels/gemm_cfg1_bf16.hip",
    "kernels/gemm_cfg2_bf16.hip",
    "kernels/gemm_big_bf16.hip",
    "kernels/gemm_f32.hip",
    "kernels/flat.hip",
    "kernels/rowchain.hip",
    "kernels/persist.hip",
    "kernels/persist_local.hip",
    "kernels/persist_xlocal.hip",
    "kernels/deep.hip",
    "kernels/deep_l2.hip",
    "kernels/deep_l3.hip",
    "kernels/deep_l4.hip",
    "kernels/deep_l5.hip",
    "kernels/deep_l2_local.hip",
    "kernels/deep_l3_local.hip",
    "kernels/deep_l4_local.hip",
    "kernels/deep_l5_local.hip",
    "kernels/peer.hip",
    "kernels/shuffle.hip",
    "runtime/executor.cpp",
    "runtime/peer.cpp",
    "runtime/rwlock.cpp",
    "runtime/host_loader.cpp",
    "runtime/bindings.cpp",
]


def source_digest() -> str:
    """sha256 (first 16 hex digits) over every native source under csrc/ (path + bytes, in
    path order): compiled into _C as ``source_digest`` so a run can show that the loaded
    binary was built from the sources it ships with (ops/native.py provenance())."""
    import hashlib
    h = hashlib.sha256()
    for dirpath, _, files in sorted(os.walk(CSRC)):
        for fn in sorted(files):
            if fn.endswith((".hip", ".h", ".cpp")) and "tests" not in os.path.relpath(dirpath, CSRC).split(os.sep):
                path = os.path.join(dirpath, fn)
                h.update(os.path.relpath(path, CSRC).encode())
                with open(path, "rb") as f:
                    h.update(f.read())
    return h.hexdigest()[:16]


def ext_path() -> str:
    return os.path.join(ROOT, "elephas_amd", "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    return os.path.join(rocm, "bin", "hipcc")


_INCLUDE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(path, seen=None):
    """path plus every local header it includes, transitively (quoted includes
    resolved against the including file's directory, then csrc/)."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path) as f:
        text = f.read()
    for inc in _INCLUDE.findall(text):
        for base in (os.path.dirname(path), CSRC):
            cand = os.path.normpath(os.path.join(base, inc))
            if os.path.exists(cand):
                _deps(cand, seen)
                break
    return seen


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths)


def build(verbose: bool = False, force: bool = False, jobs: int = 6) -> str:
    import pybind11

    os.makedirs(BUILD, exist_ok=True)
    inc = ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"], "-I" + CSRC]
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
             "-Wno-unused-result"]
    objs, cmds = [], []
    digest = source_digest()
    stamp = os.path.join(BUILD, "source_digest.txt")
    old_digest = open(stamp).read().strip() if os.path.exists(stamp) else ""
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, src.replace("/", "_") + ".o")
        objs.append(o)
        extra = []
        stale = force or not os.path.exists(o) or os.path.getmtime(o) < _newest(_deps(s))
        if src == "runtime/bindings.cpp":
            extra = [f'-DEA_SRC_DIGEST="{digest}"']
            stale = stale or old_digest != digest   # the digest covers every source
        if stale:
            lang = [] if src.endswith(".hip") else ["-x", "hip"]
            cmds.append([_hipcc()] + flags + extra + inc + lang + ["-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r

    # a build that fails part-way may already have compiled bindings.cpp with this digest:
    # drop the stamp first, so the next build recompiles it for whatever tree it sees
    if cmds and os.path.exists(stamp):
        os.remove(stamp)
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(run, cmds))
    with open(stamp, "w") as f:
        f.write(digest)
    out = ext_path()
    if force or cmds or not os.path.exists(out) or os.path.getmtime(out) < _newest(objs):
        run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + ["-o", out, "-lrt", "-lpthread"])
    return out


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, force="-f" in sys.argv))
