"""Minimal self-contained HDF5 reader/writer (no h5py / libhdf5 dependency).

Writes HDF5 files that libhdf5 >= 1.8 (and therefore h5py/Keras) can open:
  * superblock version 2, object headers version 2 (Jenkins lookup3 checksums)
  * groups with compact link storage (Link Info + Group Info + Link messages)
  * attributes in compact storage (fixed-length strings, numeric scalars/arrays)
  * datasets with contiguous layout (little-endian ints/floats, fixed strings)
Attributes larger than one object-header message (64 KiB) are stored as a
uint8 dataset ``__attr__<name>`` next to the object, and read back
transparently (libhdf5 would need dense attribute storage for them).

Reads, in addition, what h5py writes with libhdf5's default (earliest) file
format -- i.e. files produced by TF/Keras ``model.save('x.h5')`` and Elephas:
  * superblock versions 0/1, object header version 1
  * old-style groups: symbol-table message -> v1 B-tree (group nodes) -> symbol
    table nodes, link names in the group's local heap
  * chunked datasets (v1 B-tree of raw-data chunks) with the deflate (gzip),
    shuffle and fletcher32 filters
  * variable-length strings (h5py ``str`` attributes) through the global heap
Not read: dense (fractal-heap) link/attribute storage, which only the
``libver='latest'`` format writes for groups or objects with many entries.

The API is the h5py subset that Keras' HDF5 format and the reference use
(reference elephas/spark_model.py:117-125, 377-381; ml_model.py:61-70,130-132,
178-185, 265-266): ``File(path, mode)``, ``.attrs[...]``, ``create_group``,
``create_dataset``, item access and ``[()]``.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Optional, Union

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF
BIG_ATTR = "__attr__"
MAX_MSG = 65000

# ----------------------------------------------------------------- lookup3


def _rot(x, k):
    return ((x << k) | (x >> (32 - k))) & 0xFFFFFFFF


def lookup3(data: bytes, initval: int = 0) -> int:
    """Bob Jenkins' hashlittle (lookup3.c) as used by H5_checksum_lookup3."""
    M = 0xFFFFFFFF
    length = len(data)
    a = b = c = (0xDEADBEEF + length + initval) & M
    i = 0
    while length > 12:
        a = (a + int.from_bytes(data[i:i + 4], "little")) & M
        b = (b + int.from_bytes(data[i + 4:i + 8], "little")) & M
        c = (c + int.from_bytes(data[i + 8:i + 12], "little")) & M
        a = (a - c) & M; a ^= _rot(c, 4); c = (c + b) & M
        b = (b - a) & M; b ^= _rot(a, 6); a = (a + c) & M
        c = (c - b) & M; c ^= _rot(b, 8); b = (b + a) & M
        a = (a - c) & M; a ^= _rot(c, 16); c = (c + b) & M
        b = (b - a) & M; b ^= _rot(a, 19); a = (a + c) & M
        c = (c - b) & M; c ^= _rot(b, 4); b = (b + a) & M
        i += 12
        length -= 12
    if length == 0:
        return c
    tail = data[i:i + length] + b"\x00" * (12 - length)
    a = (a + int.from_bytes(tail[0:4], "little")) & M
    b = (b + int.from_bytes(tail[4:8], "little")) & M
    c = (c + int.from_bytes(tail[8:12], "little")) & M
    c ^= b; c = (c - _rot(b, 14)) & M
    a ^= c; a = (a - _rot(c, 11)) & M
    b ^= a; b = (b - _rot(a, 25)) & M
    c ^= b; c = (c - _rot(b, 16)) & M
    a ^= c; a = (a - _rot(c, 4)) & M
    b ^= a; b = (b - _rot(a, 14)) & M
    c ^= b; c = (c - _rot(b, 24)) & M
    return c


# ----------------------------------------------------------------- datatypes


def _dtype_msg(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    if dt.kind == "f":
        if dt.itemsize == 4:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            bits = bytes([0x20, 31, 0])
        elif dt.itemsize == 8:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            bits = bytes([0x20, 63, 0])
        elif dt.itemsize == 2:
            props = struct.pack("<HHBBBBI", 0, 16, 10, 5, 0, 10, 15)
            bits = bytes([0x20, 15, 0])
        else:
            raise TypeError(dt)
        return bytes([0x11]) + bits + struct.pack("<I", dt.itemsize) + props
    if dt.kind in "iub":
        signed = 0x08 if dt.kind == "i" else 0
        return bytes([0x10, signed, 0, 0]) + struct.pack("<I", dt.itemsize) + struct.pack("<HH", 0, dt.itemsize * 8)
    if dt.kind == "S":
        # fixed-length, null padded, ASCII
        return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", max(dt.itemsize, 1))
    raise TypeError(f"unsupported dtype {dt}")


def _parse_dtype(buf: bytes, off: int):
    cv = buf[off]
    cls, ver = cv & 0x0F, cv >> 4
    bits = buf[off + 1:off + 4]
    size = struct.unpack_from("<I", buf, off + 4)[0]
    if cls == 1:
        dt = np.dtype({2: "<f2", 4: "<f4", 8: "<f8"}[size])
        if bits[0] & 1:
            dt = dt.newbyteorder(">")
        return dt, 8 + 12
    if cls == 0:
        signed = bool(bits[0] & 0x08)
        dt = np.dtype(("<i" if signed else "<u") + str(size))
        if bits[0] & 1:
            dt = dt.newbyteorder(">")
        return dt, 8 + 4
    if cls == 3:
        return np.dtype(f"S{size}"), 8
    if cls == 9 and (bits[0] & 0x0F) == 1:  # variable-length string: {u32 len, u64 heap addr, u32 index}
        return VLEN_STR, 8 + 12
    raise NotImplementedError(f"HDF5 datatype class {cls} (version {ver}) is not supported by h5lite")


# marker for variable-length strings: elements are 16-byte global-heap references
VLEN_STR = np.dtype([("len", "<u4"), ("addr", "<u8"), ("idx", "<u4")])


def _space_msg(shape) -> bytes:
    if shape == ():
        return bytes([2, 0, 0, 0])
    return bytes([2, len(shape), 0, 1]) + b"".join(struct.pack("<Q", int(d)) for d in shape)


def _parse_space(buf, off):
    ver = buf[off]
    rank = buf[off + 1]
    flags = buf[off + 2]
    if ver == 1:
        p = off + 8
        dims = struct.unpack_from("<" + "Q" * rank, buf, p)
        return tuple(dims)
    typ = buf[off + 3]
    if typ == 0:
        return ()
    if typ == 2:
        return None
    dims = struct.unpack_from("<" + "Q" * rank, buf, off + 4)
    return tuple(dims)


def _to_array(value) -> np.ndarray:
    if isinstance(value, str):
        b = value.encode("utf-8")
        return np.array(b, dtype=f"S{max(len(b), 1)}")
    if isinstance(value, bytes):
        return np.array(value, dtype=f"S{max(len(value), 1)}")
    if isinstance(value, (list, tuple)) and (len(value) == 0 or isinstance(value[0], (str, bytes))):
        items = [v.encode("utf-8") if isinstance(v, str) else bytes(v) for v in value]
        n = max([len(v) for v in items] + [1])
        return np.array(items, dtype=f"S{n}")
    a = np.asarray(value)
    if a.dtype.kind == "U":
        a = np.char.encode(a, "utf-8")
    if a.dtype.kind == "O":
        raise TypeError("object arrays are not supported")
    if a.dtype.kind == "b":
        a = a.astype(np.uint8)
    return np.array(a, order="C", copy=True)  # (ascontiguousarray would turn 0-d into 1-d)


def _ascii_name(name: str) -> bytes:
    return name.encode("utf-8")


# ------------------------------------------------------------------ objects


class Attributes:
    def __init__(self):
        self._d: Dict[str, np.ndarray] = {}

    def __setitem__(self, k, v):
        self._d[str(k)] = _to_array(v)

    def __getitem__(self, k):
        a = self._d[k]
        return a[()] if a.shape == () else a

    def get(self, k, default=None):
        return self[k] if k in self._d else default

    def __contains__(self, k):
        return k in self._d

    def __delitem__(self, k):
        del self._d[k]

    def keys(self):
        return self._d.keys()

    def items(self):
        return [(k, self[k]) for k in self._d]

    def __iter__(self):
        return iter(self._d)

    def __len__(self):
        return len(self._d)


class Dataset:
    def __init__(self, name, data: np.ndarray):
        self.name = name
        self.attrs = Attributes()
        self._data = data

    @property
    def shape(self):
        return self._data.shape

    @property
    def dtype(self):
        return self._data.dtype

    def __getitem__(self, item):
        if item == () or item is Ellipsis:
            return self._data.copy() if self._data.shape != () else self._data[()]
        return self._data[item]

    def __array__(self, dtype=None):
        return np.asarray(self._data, dtype=dtype)


class Group:
    def __init__(self, name: str = "/"):
        self.name = name
        self.attrs = Attributes()
        self._children: Dict[str, Union["Group", Dataset]] = {}

    def _walk(self, path: str, create: bool = False):
        node = self
        parts = [p for p in path.split("/") if p]
        for i, p in enumerate(parts):
            if p not in node._children:
                if not create:
                    raise KeyError(path)
                node._children[p] = Group(node.name.rstrip("/") + "/" + p)
            node = node._children[p]
        return node

    def create_group(self, name: str) -> "Group":
        parent_path, _, leaf = name.rstrip("/").rpartition("/")
        parent = self._walk(parent_path, create=True) if parent_path else self
        if leaf in parent._children:
            raise ValueError(f"Unable to create group (name already exists): {name}")
        g = Group(parent.name.rstrip("/") + "/" + leaf)
        parent._children[leaf] = g
        return g

    def require_group(self, name):
        try:
            return self._walk(name)
        except KeyError:
            return self.create_group(name)

    def create_dataset(self, name: str, shape=None, dtype=None, data=None, **kwargs) -> Dataset:
        if data is None:
            data = np.zeros(shape, dtype=dtype or np.float32)
        arr = _to_array(data) if not isinstance(data, np.ndarray) else np.array(data, order="C", copy=True)
        if dtype is not None and arr.dtype.kind != "S":
            arr = arr.astype(dtype)
        parent_path, _, leaf = name.rstrip("/").rpartition("/")
        parent = self._walk(parent_path, create=True) if parent_path else self
        if leaf in parent._children:
            raise ValueError(f"Unable to create dataset (name already exists): {name}")
        d = Dataset(parent.name.rstrip("/") + "/" + leaf, arr)
        parent._children[leaf] = d
        return d

    def __getitem__(self, path):
        return self._walk(path)

    def __contains__(self, path):
        try:
            self._walk(path)
            return True
        except KeyError:
            return False

    def __delitem__(self, name):
        del self._children[name]

    def keys(self):
        return self._children.keys()

    def items(self):
        return self._children.items()

    def __iter__(self):
        return iter(self._children)

    def __len__(self):
        return len(self._children)

    def visit(self, fn, prefix=""):
        for k, v in self._children.items():
            p = prefix + k
            r = fn(p)
            if r is not None:
                return r
            if isinstance(v, Group):
                r = v.visit(fn, p + "/")
                if r is not None:
                    return r
        return None


# ------------------------------------------------------------------ writer


class _Writer:
    def __init__(self):
        self.buf = bytearray()

    def alloc(self, n: int) -> int:
        off = len(self.buf)
        self.buf += b"\x00" * n
        # keep 8-byte alignment for the next object
        pad = (-len(self.buf)) % 8
        self.buf += b"\x00" * pad
        return off

    def put(self, off: int, data: bytes):
        self.buf[off:off + len(data)] = data


def _msg(mtype: int, data: bytes, flags: int = 0) -> bytes:
    if len(data) > 0xFFFF:
        raise ValueError("object header message too large")
    return struct.pack("<BHB", mtype, len(data), flags) + data


def _attr_msg(name: str, arr: np.ndarray) -> bytes:
    nm = _ascii_name(name) + b"\x00"
    dt = _dtype_msg(arr.dtype)
    sp = _space_msg(arr.shape)
    raw = arr.astype(arr.dtype.newbyteorder("<") if arr.dtype.kind in "iuf" else arr.dtype).tobytes()
    body = struct.pack("<BBHHHB", 3, 0, len(nm), len(dt), len(sp), 1) + nm + dt + sp + raw
    return _msg(0x0C, body)


def _ohdr(messages: bytes) -> bytes:
    size = len(messages)
    if size < 256:
        flags, sz = 0x00, struct.pack("<B", size)
    elif size < 65536:
        flags, sz = 0x01, struct.pack("<H", size)
    else:
        flags, sz = 0x02, struct.pack("<I", size)
    head = b"OHDR" + bytes([2, flags]) + sz + messages
    return head + struct.pack("<I", lookup3(head))


def _split_attrs(obj) -> Dict[str, np.ndarray]:
    return dict(obj.attrs._d)


def _write_obj(w: _Writer, obj) -> int:
    if isinstance(obj, Dataset):
        arr = obj._data
        raw = arr.astype(arr.dtype.newbyteorder("<") if arr.dtype.kind in "iuf" else arr.dtype).tobytes()
        data_off = w.alloc(len(raw)) if raw else UNDEF
        if raw:
            w.put(data_off, raw)
        msgs = _msg(0x01, _space_msg(arr.shape)) + _msg(0x03, _dtype_msg(arr.dtype), 0x01)
        msgs += _msg(0x05, bytes([3, 0x0A]))
        msgs += _msg(0x08, bytes([3, 1]) + struct.pack("<QQ", data_off, len(raw)))
        for k, v in _split_attrs(obj).items():
            msgs += _attr_msg(k, v)
        hdr = _ohdr(msgs)
        off = w.alloc(len(hdr))
        w.put(off, hdr)
        return off
    # group: write children first (their addresses go into link messages)
    links = []
    attrs = _split_attrs(obj)
    big = {k: v for k, v in attrs.items() if len(v.tobytes()) > MAX_MSG}
    for k, v in big.items():
        del attrs[k]
    children = list(obj._children.items())
    for k, v in big.items():
        ds = Dataset(BIG_ATTR + k, np.frombuffer(v.tobytes(), dtype=np.uint8).copy())
        ds.attrs["__dtype__"] = v.dtype.str
        ds.attrs["__shape__"] = np.asarray(v.shape, dtype=np.int64)
        children.append((BIG_ATTR + k, ds))
    for name, child in children:
        links.append((name, _write_obj(w, child)))
    msgs = _msg(0x02, bytes([0, 0]) + struct.pack("<QQ", UNDEF, UNDEF))  # link info: compact
    msgs += _msg(0x0A, bytes([0, 0]))  # group info
    for name, addr in links:
        nb = _ascii_name(name)
        if len(nb) < 256:
            body = bytes([1, 0x10, 1, len(nb)]) + nb + struct.pack("<Q", addr)  # charset field: UTF-8
        else:
            body = bytes([1, 0x11, 1]) + struct.pack("<H", len(nb)) + nb + struct.pack("<Q", addr)
        msgs += _msg(0x06, body)
    for k, v in attrs.items():
        msgs += _attr_msg(k, v)
    hdr = _ohdr(msgs)
    off = w.alloc(len(hdr))
    w.put(off, hdr)
    return off


def write_file(path: str, root: Group) -> None:
    w = _Writer()
    w.alloc(48)  # superblock
    root_addr = _write_obj(w, root)
    eof = len(w.buf)
    sb = SIGNATURE + bytes([2, 8, 8, 0]) + struct.pack("<QQQQ", 0, UNDEF, eof, root_addr)
    sb += struct.pack("<I", lookup3(sb))
    w.put(0, sb)
    tmp = path + ".tmp-h5lite"
    with open(tmp, "wb") as f:
        f.write(bytes(w.buf))
    os.replace(tmp, path)


# ------------------------------------------------------------------ reader


class _Reader:
    def __init__(self, data: bytes):
        self.b = data

    def superblock(self) -> int:
        b = self.b
        if b[:8] != SIGNATURE:
            raise OSError("not an HDF5 file (bad signature)")
        ver = b[8]
        if ver in (2, 3):
            so, sl = b[9], b[10]
            if so != 8 or sl != 8:
                raise NotImplementedError("only 8-byte offsets/lengths")
            base, ext, eof, root = struct.unpack_from("<QQQQ", b, 12)
            return root
        if ver in (0, 1):
            return self._sb_v0(ver)
        raise NotImplementedError(f"superblock version {ver}")

    def _sb_v0(self, ver):
        b = self.b
        so, sl = b[13], b[14]
        p = 24 if ver == 0 else 28
        base, fsi, eof, drv = struct.unpack_from("<QQQQ", b, p)
        p += 32
        # root group symbol table entry: link name offset, object header address
        _, ohdr = struct.unpack_from("<QQ", b, p)
        return ohdr

    def messages(self, addr: int):
        b = self.b
        out = []
        if b[addr:addr + 4] == b"OHDR":
            flags = b[addr + 5]
            p = addr + 6
            if flags & 0x20:
                p += 16
            if flags & 0x10:
                p += 4
            szlen = 1 << (flags & 0x03)
            size = int.from_bytes(b[p:p + szlen], "little")
            p += szlen
            self._v2_chunk(p, p + size, flags, out)
        else:
            ver = b[addr]
            if ver != 1:
                raise NotImplementedError(f"object header version {ver}")
            nmsg = struct.unpack_from("<H", b, addr + 2)[0]
            size = struct.unpack_from("<I", b, addr + 8)[0]
            self._v1_chunk(addr + 16, addr + 16 + size, out)
        return out

    def _v2_chunk(self, p, end, flags, out):
        b = self.b
        while p + 4 <= end - 4:
            mtype = b[p]
            msize = struct.unpack_from("<H", b, p + 1)[0]
            mflags = b[p + 3]
            p += 4
            if flags & 0x04:
                p += 2
            if mtype == 0x10:  # continuation
                off, ln = struct.unpack_from("<QQ", b, p)
                if b[off:off + 4] == b"OCHK":
                    self._v2_chunk(off + 4, off + ln, flags, out)
            elif mtype != 0:
                out.append((mtype, p, msize))
            p += msize

    def _v1_chunk(self, p, end, out):
        b = self.b
        while p + 8 <= end:
            mtype, msize, mflags = struct.unpack_from("<HHB", b, p)
            p += 8
            if mtype == 0x10:
                off, ln = struct.unpack_from("<QQ", b, p)
                self._v1_chunk(off, off + ln, out)
            elif mtype != 0:
                out.append((mtype, p, msize))
            p += msize

    def read_obj(self, addr: int, name: str):
        b = self.b
        msgs = self.messages(addr)
        types = {m[0] for m in msgs}
        attrs = Attributes()
        for mtype, p, size in msgs:
            if mtype == 0x0C:
                k, v = self._attr(p)
                attrs._d[k] = v
        if 0x08 in types:  # dataset
            shape, dt, raw, chunked, filters = None, None, None, None, []
            for mtype, p, size in msgs:
                if mtype == 0x01:
                    shape = _parse_space(b, p)
                elif mtype == 0x03:
                    dt, _ = _parse_dtype(b, p)
                elif mtype == 0x0B:
                    filters = self._filters(p)
                elif mtype == 0x08:
                    ver, cls = b[p], b[p + 1]
                    if ver != 3:
                        raise NotImplementedError(f"layout message version {ver}")
                    if cls == 1:
                        off, ln = struct.unpack_from("<QQ", b, p + 2)
                        raw = b"" if off == UNDEF else b[off:off + ln]
                    elif cls == 0:
                        ln = struct.unpack_from("<H", b, p + 2)[0]
                        raw = b[p + 4:p + 4 + ln]
                    elif cls == 2:
                        nd = b[p + 2]
                        bt = struct.unpack_from("<Q", b, p + 3)[0]
                        cdims = struct.unpack_from("<" + "I" * nd, b, p + 11)
                        chunked = (bt, cdims)
                    else:
                        raise NotImplementedError(f"layout class {cls}")
            shape = shape or ()
            n = int(np.prod(shape)) if shape else 1
            if chunked is not None:
                arr = self._read_chunked(chunked[0], chunked[1], shape, dt, filters)
            else:
                arr = np.frombuffer(raw, dtype=dt, count=n if raw else 0)
                arr = arr.reshape(shape) if raw else np.zeros(shape, dtype=dt)
            if dt == VLEN_STR:
                arr = self._vlen_strings(arr)
                dt = arr.dtype
            ds = Dataset(name, arr.astype(dt.newbyteorder("=")) if dt.kind in "iuf" else arr.copy())
            ds.attrs = attrs
            return ds
        g = Group(name)
        g.attrs = attrs
        for mtype, p, size in msgs:
            if mtype == 0x06:
                lname, laddr = self._link(p)
                if laddr is None:
                    continue
                child = self.read_obj(laddr, name.rstrip("/") + "/" + lname)
                if lname.startswith(BIG_ATTR) and isinstance(child, Dataset):
                    dt = np.dtype(child.attrs["__dtype__"].decode() if isinstance(child.attrs["__dtype__"], bytes)
                                  else str(child.attrs["__dtype__"]))
                    shp = tuple(int(x) for x in np.atleast_1d(child.attrs["__shape__"])) \
                        if child.attrs["__shape__"].size else ()
                    g.attrs._d[lname[len(BIG_ATTR):]] = np.frombuffer(child._data.tobytes(), dtype=dt).reshape(shp)
                else:
                    g._children[lname] = child
            elif mtype == 0x11:  # old-style symbol table
                self._symbol_table(p, g, name)
        return g

    def _attr(self, p):
        b = self.b
        ver = b[p]
        if ver == 3:
            _, _, nlen, dlen, slen, _ = struct.unpack_from("<BBHHHB", b, p)
            q = p + 9
            name = b[q:q + nlen].rstrip(b"\x00").decode("utf-8")
            q += nlen
            dt, _ = _parse_dtype(b, q)
            q += dlen
            shape = _parse_space(b, q)
            q += slen
        elif ver in (1, 2):
            _, _, nlen, dlen, slen = struct.unpack_from("<BBHHH", b, p)
            q = p + 8
            pad = (lambda x: (x + 7) // 8 * 8) if ver == 1 else (lambda x: x)
            name = b[q:q + nlen].rstrip(b"\x00").decode("utf-8")
            q += pad(nlen)
            dt, _ = _parse_dtype(b, q)
            q += pad(dlen)
            shape = _parse_space(b, q)
            q += pad(slen)
        else:
            raise NotImplementedError(f"attribute message version {ver}")
        shape = shape if shape is not None else (0,)
        n = int(np.prod(shape)) if shape else 1
        arr = np.frombuffer(b, dtype=dt, count=n, offset=q).reshape(shape).copy()
        if dt == VLEN_STR:
            return name, self._vlen_strings(arr)
        if dt.kind in "iuf":
            arr = arr.astype(dt.newbyteorder("="))
        return name, arr

    def _link(self, p):
        b = self.b
        ver, flags = b[p], b[p + 1]
        q = p + 2
        ltype = 0
        if flags & 0x08:
            ltype = b[q]
            q += 1
        if flags & 0x04:
            q += 8
        if flags & 0x10:
            q += 1
        ls = 1 << (flags & 0x03)
        nlen = int.from_bytes(b[q:q + ls], "little")
        q += ls
        name = b[q:q + nlen].decode("utf-8")
        q += nlen
        if ltype != 0:
            return name, None
        return name, struct.unpack_from("<Q", b, q)[0]

    # -------------------------------------------------- old-style (v1) structures
    def _symbol_table(self, p, g, name):
        """Symbol-table message: v1 B-tree of the group's symbol table nodes + the
        local heap holding the link names."""
        b = self.b
        btree, heap = struct.unpack_from("<QQ", b, p)
        if b[heap:heap + 4] != b"HEAP":
            raise OSError("bad local heap signature")
        data_addr = struct.unpack_from("<Q", b, heap + 24)[0]
        for snod in self._btree_children(btree, 0):
            if b[snod:snod + 4] != b"SNOD":
                raise OSError("bad symbol table node signature")
            nsym = struct.unpack_from("<H", b, snod + 6)[0]
            q = snod + 8
            for _ in range(nsym):
                noff, ohdr = struct.unpack_from("<QQ", b, q)
                q += 40  # name offset, header address, cache type, reserved, scratch pad
                end = b.index(b"\x00", data_addr + noff)
                lname = b[data_addr + noff:end].decode("utf-8")
                g._children[lname] = self.read_obj(ohdr, name.rstrip("/") + "/" + lname)

    def _btree_nodes(self, addr, node_type, ndims=0):
        """Leaf entries (key, child address) of a v1 B-tree (type 0: group nodes,
        type 1: raw-data chunks with ndims-dimensional keys)."""
        b = self.b
        if b[addr:addr + 4] != b"TREE":
            raise OSError("bad v1 B-tree signature")
        ntype, level = b[addr + 4], b[addr + 5]
        if ntype != node_type:
            raise OSError(f"unexpected B-tree node type {ntype}")
        used = struct.unpack_from("<H", b, addr + 6)[0]
        q = addr + 24
        ksize = 8 if node_type == 0 else 8 + 8 * ndims
        out = []
        for _ in range(used):
            key = b[q:q + ksize]
            child = struct.unpack_from("<Q", b, q + ksize)[0]
            q += ksize + 8
            if level == 0:
                out.append((key, child))
            else:
                out.extend(self._btree_nodes(child, node_type, ndims))
        return out

    def _btree_children(self, addr, node_type):
        return [c for _, c in self._btree_nodes(addr, node_type)]

    def _filters(self, p):
        """Filter pipeline message (versions 1 and 2) -> [(filter id, client values)]."""
        b = self.b
        ver, nf = b[p], b[p + 1]
        q = p + (8 if ver == 1 else 2)
        out = []
        for _ in range(nf):
            fid = struct.unpack_from("<H", b, q)[0]
            q += 2
            nlen = 0
            if ver == 1 or fid >= 256:
                nlen = struct.unpack_from("<H", b, q)[0]
                q += 2
            flags, nval = struct.unpack_from("<HH", b, q)
            q += 4
            if ver == 1:
                nlen = (nlen + 7) // 8 * 8
            q += nlen
            vals = struct.unpack_from("<" + "I" * nval, b, q)
            q += 4 * nval
            if ver == 1 and nval % 2:
                q += 4
            out.append((fid, vals))
        return out

    def _read_chunked(self, btree, cdims, shape, dt, filters):
        """Assemble a chunked dataset from the raw-data chunk B-tree (the last chunk
        dimension is the element size), undoing the filter pipeline per chunk."""
        import zlib
        nd = len(cdims) - 1
        csh = tuple(int(c) for c in cdims[:nd])
        if not shape:
            shape = ()
        full = tuple(-(-int(s) // c) * c for s, c in zip(shape, csh)) if nd else ()
        out = np.zeros(full, dtype=dt)
        if btree == UNDEF:
            return out[tuple(slice(0, s) for s in shape)] if nd else out
        esz = dt.itemsize
        for key, addr in self._btree_nodes(btree, 1, len(cdims)):
            csize, fmask = struct.unpack_from("<II", key, 0)
            offs = struct.unpack_from("<" + "Q" * len(cdims), key, 8)[:nd]
            raw = self.b[addr:addr + csize]
            for i, (fid, vals) in reversed(list(enumerate(filters))):
                if fmask & (1 << i):
                    continue  # filter skipped for this chunk
                if fid == 1:
                    raw = zlib.decompress(raw)
                elif fid == 2:  # shuffle: byte planes -> elements
                    n = len(raw) // esz
                    raw = np.frombuffer(raw, np.uint8)[:n * esz].reshape(esz, n).T.tobytes()
                elif fid == 3:  # fletcher32: trailing checksum
                    raw = raw[:-4]
                else:
                    raise NotImplementedError(f"HDF5 filter {fid} is not supported by h5lite")
            blk = np.frombuffer(raw, dtype=dt, count=int(np.prod(csh))).reshape(csh)
            out[tuple(slice(o, o + c) for o, c in zip(offs, csh))] = blk
        return out[tuple(slice(0, s) for s in shape)]

    def _vlen_strings(self, refs):
        """Global-heap references of variable-length strings -> fixed-length bytes array."""
        b = self.b
        vals = []
        for ref in refs.reshape(-1):
            ln, addr, idx = int(ref["len"]), int(ref["addr"]), int(ref["idx"])
            if addr == 0 or ln == 0:
                vals.append(b"")
                continue
            if b[addr:addr + 4] != b"GCOL":
                raise OSError("bad global heap signature")
            csize = struct.unpack_from("<Q", b, addr + 8)[0]
            q, end, found = addr + 16, addr + csize, b""
            while q + 16 <= end:
                oid, _, _, osz = struct.unpack_from("<HHIQ", b, q)
                if oid == 0:  # free space: end of the collection's objects
                    break
                if oid == idx:
                    found = b[q + 16:q + 16 + min(ln, osz)]
                    break
                q += 16 + (osz + 7) // 8 * 8
            vals.append(found)
        n = max([len(v) for v in vals] + [1])
        return np.array(vals, dtype=f"S{n}").reshape(refs.shape)


def read_file(path: str) -> Group:
    with open(path, "rb") as f:
        data = f.read()
    r = _Reader(data)
    root = r.superblock()
    return r.read_obj(root, "/")


class File(Group):
    """h5py-like file object; the whole tree is held in memory and written on close."""

    def __init__(self, path, mode: str = "r"):
        super().__init__("/")
        self.filename = str(path)
        self.mode = mode
        if mode in ("r", "r+", "a") and os.path.exists(self.filename):
            src = read_file(self.filename)
            self.attrs = src.attrs
            self._children = src._children
        elif mode in ("r", "r+"):
            raise FileNotFoundError(self.filename)
        elif mode in ("w-", "x") and os.path.exists(self.filename):
            raise FileExistsError(self.filename)
        self._open = True

    def flush(self):
        if self.mode != "r":
            write_file(self.filename, self)

    def close(self):
        if self._open:
            self.flush()
            self._open = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
