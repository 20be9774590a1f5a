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


class _H5:
    """The handful of libhdf5 C calls needed to write files the way h5py does with
    the library defaults (superblock v0, symbol-table groups): used only to produce
    reference-format inputs for h5lite's reader."""

    def __init__(self):
        L = ctypes.CDLL(LIBHDF5)
        L.H5open()
        hid, c = ctypes.c_int64, ctypes
        for name, res, args in [
                ("H5Fcreate", hid, [c.c_char_p, c.c_uint, hid, hid]),
                ("H5Gcreate2", hid, [hid, c.c_char_p, hid, hid, hid]),
                ("H5Screate_simple", hid, [c.c_int, c.POINTER(c.c_uint64), c.c_void_p]),
                ("H5Screate", hid, [c.c_int]),
                ("H5Dcreate2", hid, [hid, c.c_char_p, hid, hid, hid, hid, hid]),
                ("H5Dwrite", c.c_int, [hid, hid, hid, hid, hid, c.c_void_p]),
                ("H5Acreate2", hid, [hid, c.c_char_p, hid, hid, hid, hid]),
                ("H5Awrite", c.c_int, [hid, hid, c.c_void_p]),
                ("H5Tcopy", hid, [hid]),
                ("H5Tset_size", c.c_int, [hid, c.c_size_t]),
                ("H5Pcreate", hid, [hid]),
                ("H5Pset_chunk", c.c_int, [hid, c.c_int, c.POINTER(c.c_uint64)]),
                ("H5Pset_deflate", c.c_int, [hid, c.c_uint]),
                ("H5Pset_shuffle", c.c_int, [hid]),
                ("H5Pset_fletcher32", c.c_int, [hid]),
                ("H5Dclose", c.c_int, [hid]), ("H5Aclose", c.c_int, [hid]), ("H5Sclose", c.c_int, [hid]),
                ("H5Gclose", c.c_int, [hid]), ("H5Fclose", c.c_int, [hid]), ("H5Tclose", c.c_int, [hid]),
                ("H5Pclose", c.c_int, [hid])]:
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        self.L = L
        g = lambda n: ctypes.c_int64.in_dll(L, n).value
        self.FLOAT, self.INT64, self.C_S1 = g("H5T_NATIVE_FLOAT_g"), g("H5T_NATIVE_LLONG_g"), g("H5T_C_S1_g")
        self.DCREATE = g("H5P_CLS_DATASET_CREATE_ID_g")

    def space(self, shape):
        if shape == ():
            return self.L.H5Screate(0)  # H5S_SCALAR
        dims = (ctypes.c_uint64 * len(shape))(*shape)
        return self.L.H5Screate_simple(len(shape), dims, None)

    def str_attr(self, obj, name, value, vlen=False):
        L = self.L
        t = L.H5Tcopy(self.C_S1)
        if isinstance(value, list):
            n = max([len(v) for v in value] + [1])
            L.H5Tset_size(t, n)
            sp = self.space((len(value),))
            buf = b"".join(v.ljust(n, b"\x00") for v in value)
        elif vlen:
            L.H5Tset_size(t, ctypes.c_size_t(-1).value)  # H5T_VARIABLE
            sp = self.space(())
            cs = ctypes.c_char_p(value)
            a = L.H5Acreate2(obj, name, t, sp, 0, 0)
            assert L.H5Awrite(a, t, ctypes.byref(cs)) >= 0
            L.H5Aclose(a), L.H5Sclose(sp), L.H5Tclose(t)
            return
        else:
            L.H5Tset_size(t, len(value))
            sp = self.space(())
            buf = value
        a = L.H5Acreate2(obj, name, t, sp, 0, 0)
        assert L.H5Awrite(a, t, buf) >= 0
        L.H5Aclose(a), L.H5Sclose(sp), L.H5Tclose(t)

    def dataset(self, parent, name, arr, chunks=None, gzip=False, shuffle=False, fletcher=False):
        L = self.L
        arr = np.ascontiguousarray(arr)
        sp = self.space(arr.shape)
        dcpl = 0
        if chunks:
            dcpl = L.H5Pcreate(self.DCREATE)
            L.H5Pset_chunk(dcpl, len(chunks), (ctypes.c_uint64 * len(chunks))(*chunks))
            if fletcher:
                L.H5Pset_fletcher32(dcpl)
            if shuffle:
                L.H5Pset_shuffle(dcpl)
            if gzip:
                L.H5Pset_deflate(dcpl, 4)
        t = self.FLOAT if arr.dtype == np.float32 else self.INT64
        d = L.H5Dcreate2(parent, name, t, sp, 0, dcpl, 0)
        assert d >= 0
        assert L.H5Dwrite(d, t, 0, 0, 0, arr.ctypes.data) >= 0
        L.H5Dclose(d), L.H5Sclose(sp)
        if dcpl:
            L.H5Pclose(dcpl)


@pytest.mark.skipif(not os.path.exists(LIBHDF5), reason="no system libhdf5 to write reference-format files")
def test_reads_libhdf5_default_format(tmp_path):
    """Files written through libhdf5's default (earliest) format, as h5py / TF-Keras
    model.save produce them: superblock v0, symbol-table groups, chunked datasets with
    gzip / shuffle / fletcher32, fixed and variable-length string attributes."""
    h = _H5()
    L = h.L
    p = str(tmp_path / "ref.h5")
    f = L.H5Fcreate(p.encode(), 2, 0, 0)   # H5F_ACC_TRUNC, default fcpl / fapl
    h.str_attr(f, b"fixed", b"abc")
    h.str_attr(f, b"vlen", "variable-length é".encode(), vlen=True)
    h.str_attr(f, b"names", [b"dense", b"dense_1", b"dense_2"])
    g = L.H5Gcreate2(f, b"grp", 0, 0, 0)
    sub = L.H5Gcreate2(g, b"sub", 0, 0, 0)
    rng = np.random.default_rng(0)
    a = rng.normal(size=(37, 21)).astype(np.float32)
    b = rng.normal(size=(100,)).astype(np.float32)
    c = np.arange(60, dtype=np.int64).reshape(3, 4, 5)
    h.dataset(g, b"contig", a)
    h.dataset(sub, b"chunked_gzip", a, chunks=(8, 5), gzip=True, shuffle=True, fletcher=True)
    h.dataset(sub, b"chunked_plain", b, chunks=(7,))
    h.dataset(g, b"ints", c, chunks=(2, 2, 2), gzip=True)
    for i in range(40):   # enough links to split the group's B-tree into several nodes
        h.dataset(g, f"w{i}".encode(), np.full((3,), i, np.float32))
    L.H5Gclose(sub), L.H5Gclose(g), L.H5Fclose(f)
    with open(p, "rb") as fh:
        assert fh.read(9)[8] == 0   # superblock version 0
    r = h5lite.File(p, "r")
    assert r.attrs["fixed"] == b"abc"
    assert r.attrs["vlen"].tobytes().rstrip(b"\x00").decode() == "variable-length é"
    assert list(r.attrs["names"]) == [b"dense", b"dense_1", b"dense_2"]
    np.testing.assert_array_equal(r["grp/contig"][()], a)
    np.testing.assert_array_equal(r["grp/sub/chunked_gzip"][()], a)
    np.testing.assert_array_equal(r["grp/sub/chunked_plain"][()], b)
    np.testing.assert_array_equal(r["grp/ints"][()], c)
    for i in range(40):
        np.testing.assert_array_equal(r[f"grp/w{i}"][()], np.full((3,), i, np.float32))


@pytest.mark.skipif(not os.path.exists(LIBHDF5), reason="no system libhdf5 to write reference-format files")
def test_load_keras_h5_written_by_libhdf5(tmp_path, classification_model):
    """A Keras-layout .h5 produced through libhdf5 defaults (as tf.keras model.save +
    Elephas' h5py distributed_config append write it) loads with load_spark_model:
    weights, compile config and the distributed config all round-trip."""
    from elephas_amd.spark_model import load_spark_model
    from elephas_amd.models.optimizers import SGD
    classification_model.compile(SGD(0.05), "categorical_crossentropy", ["acc"])
    h = _H5()
    L = h.L
    p = str(tmp_path / "keras.h5")
    f = L.H5Fcreate(p.encode(), 2, 0, 0)
    h.str_attr(f, b"keras_version", b"2.10.0")
    h.str_attr(f, b"backend", b"tensorflow")
    h.str_attr(f, b"model_config", classification_model.to_json().encode())
    tc = {"loss": "categorical_crossentropy", "metrics": ["acc"], "weighted_metrics": None,
          "loss_weights": None, "optimizer_config": {"class_name": "SGD", "config": {
              "name": "SGD", "learning_rate": 0.05, "decay": 0.0, "momentum": 0.0, "nesterov": False}}}
    h.str_attr(f, b"training_config", json.dumps(tc).encode())
    mw = L.H5Gcreate2(f, b"model_weights", 0, 0, 0)
    layers = [l for l in classification_model._layers]
    h.str_attr(mw, b"layer_names", [l.name.encode() for l in layers])
    h.str_attr(mw, b"backend", b"tensorflow")
    h.str_attr(mw, b"keras_version", b"2.10.0")
    rng = np.random.default_rng(3)
    want = []
    for l in layers:
        lg = L.H5Gcreate2(mw, l.name.encode(), 0, 0, 0)
        ws = l.get_weights()
        names = [f"{l.name}/kernel:0", f"{l.name}/bias:0"][:len(ws)]
        h.str_attr(lg, b"weight_names", [n.encode() for n in names])   # empty for Activation/Dropout
        inner = L.H5Gcreate2(lg, l.name.encode(), 0, 0, 0) if ws else None
        for n, w in zip(names, ws):
            v = rng.normal(size=w.shape).astype(np.float32)
            want.append(v)
            h.dataset(inner, n.split("/")[1].encode(), v)
        if inner is not None:
            L.H5Gclose(inner)
        L.H5Gclose(lg)
    L.H5Gclose(mw)
    dc = {"class_name": "SparkModel", "config": {"parameter_server_mode": "http", "mode": "synchronous",
                                                  "frequency": "epoch", "num_workers": 2, "batch_size": 32}}
    h.str_attr(f, b"distributed_config", json.dumps(dc).encode())
    L.H5Fclose(f)
    sm = load_spark_model(p)
    got = sm.master_network.get_weights()
    assert len(got) == len(want)
    for g_, w_ in zip(got, want):
        np.testing.assert_array_equal(g_, w_)
    assert sm.get_config()["num_workers"] == 2 and sm.get_config()["mode"] == "synchronous"
    assert float(sm.master_network.optimizer.learning_rate) == pytest.approx(0.05)


def test_optimizer_weights_round_trip(tmp_path):
    """A trained model's optimizer state (Keras optimizer_weights group: iter + slot
    variables named '<opt>/<layer>/<kernel|bias>/<slot>:0') is saved and restored:
    continuing training after load matches continuing the original model."""
    from elephas_amd.models import Sequential, Dense
    from elephas_amd.models.optimizers import Adam
    from elephas_amd.models import load_model
    from elephas_amd import config
    config.set_engine("torch")
    rng = np.random.default_rng(1)
    x = rng.normal(size=(64, 6)).astype(np.float32)
    y = np.eye(3, dtype=np.float32)[rng.integers(0, 3, 64)]
    m = Sequential()
    m.add(Dense(5, activation="relu", input_dim=6))
    m.add(Dense(3, activation="softmax"))
    m.compile(Adam(0.01), "categorical_crossentropy", ["acc"])
    m.fit(x, y, epochs=2, batch_size=16, verbose=0, shuffle=False)
    p = str(tmp_path / "opt.h5")
    m.save(p)
    f = h5lite.File(p, "r")
    names = [n.decode() for n in f["optimizer_weights"].attrs["weight_names"]]
    assert names[0] == "Adam/iter:0" and int(f["optimizer_weights/Adam/iter:0"][()]) == 8
    assert "Adam/dense/kernel/m:0" in names and "Adam/dense_1/bias/v:0" in names
    m2 = load_model(p)
    m.fit(x, y, epochs=1, batch_size=16, verbose=0, shuffle=False)
    m2.fit(x, y, epochs=1, batch_size=16, verbose=0, shuffle=False)
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    config.set_engine("auto")
