"""Self-contained HDF5 writer/reader, cross-checked against the system libhdf5
(/opt/conda/lib/libhdf5.so, read-only use through ctypes) when it exists."""
import ctypes
import json
import os

import numpy as np
import pytest

from elephas_amd.io import h5lite

LIBHDF5 = "/opt/conda/lib/libhdf5.so"


def test_lookup3_known_values():
    # values from Bob Jenkins' lookup3.c driver5(): hashlittle("", 0) == 0xdeadbeef,
    # hashlittle("Four score and seven years ago", 30, 0) == 0x17770551
    assert h5lite.lookup3(b"") == 0xDEADBEEF
    assert h5lite.lookup3(b"Four score and seven years ago") == 0x17770551


def test_roundtrip(tmp_path):
    p = str(tmp_path / "a.h5")
    f = h5lite.File(p, "w")
    f.attrs["s"] = "héllo"
    f.attrs["b"] = b"bytes"
    f.attrs["names"] = ["dense", "dense_1"]
    f.attrs["x"] = np.float64(2.5)
    f.attrs["v"] = np.arange(3, dtype=np.int64)
    f.attrs["big"] = "z" * 200000          # > one object-header message
    g = f.create_group("a/b")
    g.create_dataset("w:0", data=np.arange(12, dtype=np.float32).reshape(3, 4))
    g.create_dataset("empty", data=np.zeros((0,), np.float32))
    f.close()
    r = h5lite.File(p, "r")
    assert r.attrs["s"].decode() == "héllo" and r.attrs["b"] == b"bytes"
    assert list(r.attrs["names"]) == [b"dense", b"dense_1"]
    assert r.attrs["x"] == 2.5 and list(r.attrs["v"]) == [0, 1, 2]
    assert len(r.attrs["big"]) == 200000
    assert np.array_equal(r["a/b/w:0"][()], np.arange(12, dtype=np.float32).reshape(3, 4))
    assert r["a/b/empty"].shape == (0,)
    # append mode keeps content
    a = h5lite.File(p, "a")
    a.attrs["distributed_config"] = json.dumps({"class_name": "SparkModel"}).encode()
    a.close()
    assert json.loads(h5lite.File(p, "r").attrs["distributed_config"])["class_name"] == "SparkModel"


@pytest.mark.skipif(not os.path.exists(LIBHDF5), reason="no system libhdf5 to cross-check against")
def test_libhdf5_reads_our_files(tmp_path, classification_model):
    p = str(tmp_path / "m.h5")
    classification_model.compile("sgd", "categorical_crossentropy", ["acc"])
    classification_model.save(p)
    L = ctypes.CDLL(LIBHDF5)
    L.H5open()
    L.H5Fopen.restype = ctypes.c_int64
    L.H5Fopen.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_int64]
    fid = L.H5Fopen(p.encode(), 0, 0)
    assert fid >= 0
    L.H5Dopen2.restype = ctypes.c_int64
    L.H5Dopen2.argtypes = [ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64]
    did = L.H5Dopen2(fid, b"/model_weights/dense/dense/kernel:0", 0)
    assert did >= 0
    buf = np.zeros((784, 128), np.float32)
    native_float = ctypes.c_int64.in_dll(L, "H5T_NATIVE_FLOAT_g").value
    L.H5Dread.argtypes = [ctypes.c_int64] * 5 + [ctypes.c_void_p]
    assert L.H5Dread(did, native_float, 0, 0, 0, buf.ctypes.data) >= 0
    assert np.array_equal(buf, classification_model.get_weights()[0])
    L.H5Aopen.restype = ctypes.c_int64
    L.H5Aopen.argtypes = [ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64]
    L.H5Aget_type.restype = ctypes.c_int64
    L.H5Aget_type.argtypes = [ctypes.c_int64]
    L.H5Tget_size.restype = ctypes.c_size_t
    L.H5Tget_size.argtypes = [ctypes.c_int64]
    L.H5Aread.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
    aid = L.H5Aopen(fid, b"model_config", 0)
    tid = L.H5Aget_type(aid)
    n = L.H5Tget_size(tid)
    s = ctypes.create_string_buffer(n)
    assert L.H5Aread(aid, tid, s) >= 0
    assert json.loads(s.raw.rstrip(b"\x00").decode()) == json.loads(classification_model.to_json())
