"""Loader for the in-tree native runtime ``elephas_amd._C`` (HIP/gfx950).

On a machine with a visible AMD GPU the extension is mandatory: ``require()``
raises instead of silently falling back to the torch path, so GPU tests and the
benchmark always exercise the hand-written kernels.  On a CPU-only machine the
import is optional (the torch engine is the reference implementation there).
"""
from __future__ import annotations

import importlib.util
import os
import sys
import threading

import torch  # noqa: F401  -- must be imported first: _C binds torch's libamdhip64.so.7

_lock = threading.Lock()
_mod = None
_err = None

# enums mirrored from csrc/kernels/args.h
PK = dict(PLAIN=0, FWD=1, FWD_LOSS=2, DX=3, DW_UPDATE=4, DW_GRAD=5, GATHER_T=6, LOSS_ROWS=7)


def _path() -> str:
    import sysconfig
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def load(build_if_missing: bool = True):
    global _mod, _err
    with _lock:
        if _mod is not None:
            return _mod
        path = _path()
        if not os.path.exists(path) and build_if_missing and os.environ.get("ELEPHAS_AMD_NO_BUILD") != "1":
            try:
                from .. import _build
                _build.build()
            except Exception as e:  # pragma: no cover - reported through require()
                _err = e
        if not os.path.exists(path):
            _err = _err or FileNotFoundError(path)
            return None
        try:
            spec = importlib.util.spec_from_file_location("elephas_amd._C", path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["elephas_amd._C"] = mod
            _mod = mod
        except Exception as e:  # pragma: no cover
            _err = e
            return None
        return _mod


def available() -> bool:
    return load() is not None


def gpu_present() -> bool:
    return torch.cuda.is_available()


def require():
    m = load()
    if m is None:
        raise RuntimeError(f"elephas_amd native runtime (_C) is not available: {_err!r}. "
                           f"Build it with `python -m elephas_amd._build`.")
    return m


def provenance() -> dict:
    """Which sources the loaded binary was built from: the digest compiled into _C vs the
    digest of the csrc/ tree next to it (equal = the binary matches these sources)."""
    from .._build import source_digest
    m = load(build_if_missing=False)
    built = getattr(m, "source_digest", None) if m is not None else None
    tree = source_digest()
    return dict(built=built, tree=tree, match=built == tree, path=_path() if m is not None else None)


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)
