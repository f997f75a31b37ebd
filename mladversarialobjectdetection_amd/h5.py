"""A minimal HDF5 codec for Keras weight files (`Model.save_weights('….h5')` / `load_weights`), so the
defender's `antipatch.h5` (attack_detection.py:54-55 load, :300-318 save) is interchangeable with the
reference's.  h5py is not installed in this image, so the file format is written and parsed here,
with numpy and struct only.

What it writes (HDF5 file format specification, version 0 superblock):
  * superblock v0 (8-byte offsets and lengths, group leaf K 4, internal K 16), root group cached;
  * "old-style" groups: a v1 object header holding a Symbol Table message, a v1 B-tree (group
    nodes) over symbol-table nodes (SNOD, <= 8 entries each, names in sorted order) and a local heap
    of the member names;
  * datasets: v1 object header with Dataspace (v1), Datatype (IEEE float32/64 little-endian or
    fixed-length string), Fill Value (v2, undefined) and Layout (v3, contiguous) messages;
  * attributes: Attribute messages (v1) with fixed-length, null-padded ASCII strings — the form
    h5py gives Keras's `layer_names` / `weight_names` arrays and the `backend` / `keras_version`
    strings.
The Keras weight layout (keras/saving/hdf5_format.py save_weights_to_hdf5_group):
  root attrs layer_names [n], backend, keras_version; per layer a group named after the layer with
  attr weight_names [k]; each weight a dataset at <layer>/<weight name> (a name with '/' makes
  nested groups).

The reader understands what this writer produces plus the variants an h5py-written Keras file may
hold: superblock v0 / v1, v1 object headers with continuation messages, multi-level group B-trees,
contiguous or compact layouts (layout message v1-v3), float16/32/64 and integer datasets of either
byte order, attribute messages v1-v3 with fixed-length strings.  It does not read v2 object headers
("OHDR", h5py's libver='latest'), chunked / filtered datasets or variable-length strings, and says so.

Parity: pinned only by its own writer (no HDF5 library and no reference-written .h5 file exist in
this environment).
"""
from __future__ import annotations

import struct

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
_SIG = b"\x89HDF\r\n\x1a\n"
_LEAF_K, _NODE_K = 4, 16


def _pad8(b: bytes) -> bytes:
    return b + b"\0" * (-len(b) % 8)


# ---- writer ------------------------------------------------------------------------------------

class _Group:
    def __init__(self):
        self.members: dict[str, object] = {}
        self.attrs: dict[str, object] = {}


class _Dataset:
    def __init__(self, arr):
        self.arr = np.ascontiguousarray(arr)
        self.attrs: dict[str, object] = {}


def _datatype(arr) -> bytes:
    """Datatype message body (version 1) for a numpy array's dtype."""
    dt = arr.dtype
    if dt.kind == "f":
        if dt.itemsize == 4:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
        elif dt.itemsize == 8:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
        else:
            raise ValueError(f"h5: float{dt.itemsize * 8} not written")
        order = 1 if dt.byteorder == ">" else 0
        bits = bytes([0x20 | order, dt.itemsize * 8 - 1, 0])  # implied-msb mantissa, sign bit position
        return bytes([0x11]) + bits + struct.pack("<I", dt.itemsize) + props
    if dt.kind == "S":
        # fixed-length ASCII, null padded
        return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", max(1, dt.itemsize))
    raise ValueError(f"h5: dtype {dt} not written")


def _dataspace(shape) -> bytes:
    return struct.pack("<BBBB4x", 1, len(shape), 0, 0) + b"".join(struct.pack("<Q", d) for d in shape)


def _attr_value(v) -> np.ndarray:
    a = np.asarray(v)
    if a.dtype.kind == "U":
        a = np.char.encode(a, "ascii")
    if a.dtype.kind == "O":
        a = np.array([x if isinstance(x, bytes) else str(x).encode("ascii") for x in a.ravel()]).reshape(a.shape)
    if a.dtype.kind == "S" and a.dtype.itemsize == 0:
        a = a.astype("S1")
    return a


def _attr_message(name: str, value) -> bytes:
    a = _attr_value(value)
    nb = name.encode("ascii") + b"\0"
    dtb, dsb = _datatype(a), _dataspace(a.shape)
    data = a.astype(a.dtype.newbyteorder("<") if a.dtype.kind == "f" else a.dtype).tobytes()
    return struct.pack("<BBHHH", 1, 0, len(nb), len(dtb), len(dsb)) + _pad8(nb) + _pad8(dtb) + _pad8(dsb) + data


class _Writer:
    def __init__(self):
        self.buf = bytearray(96)  # the superblock, filled in last

    def alloc(self, data: bytes) -> int:
        # every object starts on an 8-byte boundary
        self.buf += b"\0" * (-len(self.buf) % 8)
        at = len(self.buf)
        self.buf += data
        return at

    def header(self, msgs) -> int:
        body = b""
        for typ, data, flags in msgs:
            d = _pad8(data)
            body += struct.pack("<HHB3x", typ, len(d), flags) + d
        return self.alloc(struct.pack("<BBHII4x", 1, 0, len(msgs), 1, len(body)) + body)

    def dataset(self, ds: _Dataset) -> int:
        a = ds.arr
        if a.dtype.kind == "f" and a.dtype.byteorder == ">":
            a = a.astype(a.dtype.newbyteorder("<"))
        raw = a.tobytes()
        at = self.alloc(raw) if raw else UNDEF
        msgs = [(0x0001, _dataspace(a.shape), 0),
                (0x0003, _datatype(a), 1),
                (0x0005, struct.pack("<BBBB", 2, 2, 2, 0), 1),  # v2: late allocation, fill undefined
                (0x0008, struct.pack("<BBQQ", 3, 1, at, len(raw)), 0)]
        msgs += [(0x000C, _attr_message(k, v), 0) for k, v in ds.attrs.items()]
        return self.header(msgs)

    def group(self, g: _Group):
        """Returns (object header address, B-tree address, local heap address)."""
        names = sorted(g.members, key=lambda s: s.encode("ascii"))
        addrs = {}
        for n in names:
            m = g.members[n]
            addrs[n] = self.dataset(m) if isinstance(m, _Dataset) else self.group(m)[0]
        # local heap: offset 0 is the empty string, then each name null-terminated, 8-aligned
        heap = bytearray(8)
        off = {}
        for n in names:
            off[n] = len(heap)
            heap += _pad8(n.encode("ascii") + b"\0")
        heap += b"\0" * 16  # a free block, as the library leaves one
        free_at = len(heap) - 16
        heap[free_at:free_at + 16] = struct.pack("<QQ", 1, 16)  # (next free = 1: last, size)
        data_at = self.alloc(bytes(heap))
        heap_at = self.alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), free_at, data_at))
        # symbol-table nodes, 2 * leaf K entries each (full size on disk)
        per = 2 * _LEAF_K
        snods, last_names = [], []
        for i in range(0, max(1, len(names)), per):
            chunk = names[i:i + per]
            ent = b"".join(struct.pack("<QQII16x", off[n], addrs[n], 0, 0) for n in chunk)
            ent += b"\0" * (40 * (per - len(chunk)))
            snods.append(self.alloc(b"SNOD" + struct.pack("<BBH", 1, 0, len(chunk)) + ent))
            last_names.append(chunk[-1] if chunk else None)
        if len(snods) > 2 * _NODE_K:
            raise ValueError(f"h5: a group of {len(names)} members needs a multi-level B-tree (not written)")
        # v1 B-tree, group nodes, level 0: key0, child0, key1, ..., key_n (key = heap offset of the
        # largest name in the child to its left; key0 = the empty string)
        n_used = len(snods) if names else 0
        keys = [0] + [off[n] for n in last_names[:n_used]]
        body = b""
        for i in range(n_used):
            body += struct.pack("<QQ", keys[i], snods[i])
        body += struct.pack("<Q", keys[n_used] if n_used else 0)
        body += b"\0" * ((2 * _NODE_K + 1) * 8 + 2 * _NODE_K * 8 - len(body))
        bt_at = self.alloc(b"TREE" + struct.pack("<BBHQQ", 0, 0, n_used, UNDEF, UNDEF) + body)
        msgs = [(0x0011, struct.pack("<QQ", bt_at, heap_at), 0)]
        msgs += [(0x000C, _attr_message(k, v), 0) for k, v in g.attrs.items()]
        return self.header(msgs), bt_at, heap_at

    def finish(self, root: _Group) -> bytes:
        oh, bt, hp = self.group(root)
        eof = len(self.buf)
        sb = _SIG + struct.pack("<BBBBBBBB", 0, 0, 0, 0, 0, 8, 8, 0) + struct.pack("<HHI", _LEAF_K, _NODE_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, oh, 1, 0) + struct.pack("<QQ", bt, hp)
        assert len(sb) == 96
        self.buf[:96] = sb
        return bytes(self.buf)


def _member(root: _Group, path: str, create_group=True):
    g = root
    parts = [p for p in path.split("/") if p]
    for p in parts[:-1]:
        g = g.members.setdefault(p, _Group())
        if not isinstance(g, _Group):
            raise ValueError(f"h5: {path}: {p} is a dataset")
    return g, parts[-1]


def write_keras_weights(path, layers, *, backend="tensorflow", keras_version="2.9.0"):
    """layers: [(layer name, [(weight name, array), ...]), ...] in the model's layer order (Keras
    `save_weights` h5 layout; weight names as Keras prints them, e.g. 'conv0/cnv1/kernel:0')."""
    root = _Group()
    root.attrs["layer_names"] = np.array([n.encode("ascii") for n, _ in layers])
    root.attrs["backend"] = np.array(backend.encode("ascii"))
    root.attrs["keras_version"] = np.array(keras_version.encode("ascii"))
    for lname, weights in layers:
        parent, leaf = _member(root, lname)
        lg = parent.members.setdefault(leaf, _Group())
        lg.attrs["weight_names"] = np.array([w.encode("ascii") for w, _ in weights]) if weights else \
            np.zeros((0,), "S1")
        for wname, arr in weights:
            g, leafw = _member(lg, wname)
            g.members[leafw] = _Dataset(np.asarray(arr))
    with open(path, "wb") as f:
        f.write(_Writer().finish(root))


# ---- reader ------------------------------------------------------------------------------------

class H5Error(ValueError):
    pass


class H5File:
    """Read-only access to groups, datasets and attributes of a file in the subset described above."""

    def __init__(self, path):
        with open(path, "rb") as f:
            self.b = f.read()
        b = self.b
        base = b.find(_SIG)
        if base != 0:
            raise H5Error("h5: no HDF5 signature at offset 0")
        ver = b[8]
        if ver not in (0, 1):
            raise H5Error(f"h5: superblock version {ver} not read")
        so, sl = b[13], b[14]
        if so != 8 or sl != 8:
            raise H5Error("h5: only 8-byte offsets / lengths are read")
        p = 16 + 4 + 4 + (4 if ver == 1 else 0)  # K values, flags, (v1: indexed-storage K + reserved)
        p += 32  # base, free-space, EOF, driver addresses
        self.root = struct.unpack_from("<Q", b, p + 8)[0]

    # object headers
    def _messages(self, addr):
        b = self.b
        if b[addr:addr + 4] == b"OHDR":
            raise H5Error("h5: version 2 object headers (libver='latest') are not read")
        ver, _, nmsg, _, size = struct.unpack_from("<BBHII", b, addr)
        if ver != 1:
            raise H5Error(f"h5: object header version {ver}")
        blocks = [(addr + 16, size)]
        out = []
        while blocks and len(out) < nmsg:
            start, size = blocks.pop(0)
            p = start
            while p + 8 <= start + size and len(out) < nmsg:
                typ, msz, flags = struct.unpack_from("<HHB", b, p)
                data = b[p + 8:p + 8 + msz]
                p += 8 + msz
                if typ == 0x0010:  # continuation
                    blocks.append(struct.unpack_from("<QQ", data))
                out.append((typ, data, flags))
        return out

    def _children(self, oh):
        for typ, data, _ in self._messages(oh):
            if typ == 0x0011:
                bt, heap = struct.unpack_from("<QQ", data)
                return self._btree_entries(bt, self._heap_data(heap))
        raise H5Error("h5: not a (symbol-table) group")

    def _heap_data(self, heap):
        b = self.b
        if b[heap:heap + 4] != b"HEAP":
            raise H5Error("h5: bad local heap")
        size, _, data_at = struct.unpack_from("<QQQ", b, heap + 8)
        return b[data_at:data_at + size]

    def _btree_entries(self, bt, heap):
        b = self.b
        if b[bt:bt + 4] != b"TREE" or b[bt + 4] != 0:
            raise H5Error("h5: bad group B-tree")
        level, used = b[bt + 5], struct.unpack_from("<H", b, bt + 6)[0]
        p = bt + 24
        out = {}
        for i in range(used):
            child = struct.unpack_from("<Q", b, p + 8 + 16 * i)[0]
            if level > 0:
                out.update(self._btree_entries(child, heap))
                continue
            if b[child:child + 4] != b"SNOD":
                raise H5Error("h5: bad symbol-table node")
            n = struct.unpack_from("<H", b, child + 6)[0]
            for k in range(n):
                name_off, oh = struct.unpack_from("<QQ", b, child + 8 + 40 * k)
                name = heap[name_off:heap.index(b"\0", name_off)].decode("ascii")
                out[name] = oh
        return out

    def _resolve(self, path):
        oh = self.root
        for part in [p for p in path.split("/") if p]:
            kids = self._children(oh)
            if part not in kids:
                raise KeyError(path)
            oh = kids[part]
        return oh

    def members(self, path="/"):
        return sorted(self._children(self._resolve(path)))

    def is_group(self, path):
        return any(t == 0x0011 for t, _, _ in self._messages(self._resolve(path)))

    # datatypes / dataspaces
    @staticmethod
    def _dtype(d):
        cls, ver = d[0] & 0x0F, d[0] >> 4
        bits = d[1] | d[2] << 8 | d[3] << 16
        size = struct.unpack_from("<I", d, 4)[0]
        if cls == 1:  # float
            if size not in (2, 4, 8):
                raise H5Error(f"h5: float of {size} bytes")
            return np.dtype(("<" if not bits & 1 else ">") + {2: "f2", 4: "f4", 8: "f8"}[size]), 8 + 12
        if cls == 0:  # fixed-point integer
            return np.dtype(("<" if not bits & 1 else ">") + ("i" if bits & 8 else "u") + str(size)), 8 + 4
        if cls == 3:  # fixed-length string
            return np.dtype(f"S{size}"), 8
        raise H5Error(f"h5: datatype class {cls} (version {ver}) not read")

    @staticmethod
    def _shape(d):
        ver, rank, flags = d[0], d[1], d[2]
        if ver == 1:
            p = 8
        elif ver == 2:
            if d[3] == 2:  # null dataspace
                return None, 4
            p = 4
        else:
            raise H5Error(f"h5: dataspace version {ver}")
        shape = tuple(struct.unpack_from("<Q", d, p + 8 * i)[0] for i in range(rank))
        p += 8 * rank * (2 if flags & 1 else 1)
        return shape, p

    def _attrs_of(self, oh):
        out = {}
        for typ, data, _ in self._messages(oh):
            if typ != 0x000C:
                continue
            ver = data[0]
            if ver == 1:
                nsz, tsz, ssz = struct.unpack_from("<HHH", data, 2)
                p = 8
                name = data[p:p + nsz - 1].decode("ascii")
                p += nsz + (-nsz % 8)
                dt, _ = self._dtype(data[p:p + tsz])
                p += tsz + (-tsz % 8)
                shape, _ = self._shape(data[p:p + ssz])
                p += ssz + (-ssz % 8)
            elif ver in (2, 3):
                nsz, tsz, ssz = struct.unpack_from("<HHH", data, 2)
                p = 8 + (1 if ver == 3 else 0)
                name = data[p:p + nsz - 1].decode("ascii")
                p += nsz
                dt, _ = self._dtype(data[p:p + tsz])
                p += tsz
                shape, _ = self._shape(data[p:p + ssz])
                p += ssz
            else:
                raise H5Error(f"h5: attribute message version {ver}")
            n = int(np.prod(shape)) if shape else 1
            if shape is None:
                out[name] = None
                continue
            arr = np.frombuffer(data, dt, count=n, offset=p).copy()
            out[name] = arr.reshape(shape) if shape else arr[0]
        return out

    def attrs(self, path="/"):
        return self._attrs_of(self._resolve(path))

    def dataset(self, path):
        shape = dt = None
        raw = None
        for typ, data, _ in self._messages(self._resolve(path)):
            if typ == 0x0001:
                shape, _ = self._shape(data)
            elif typ == 0x0003:
                dt, _ = self._dtype(data)
            elif typ == 0x000B:
                raise H5Error(f"h5: {path}: filtered (compressed) datasets are not read")
            elif typ == 0x0008:
                ver = data[0]
                if ver == 3:
                    cls = data[1]
                    if cls == 1:
                        at, size = struct.unpack_from("<QQ", data, 2)
                        raw = b"" if at == UNDEF else self.b[at:at + size]
                    elif cls == 0:
                        size = struct.unpack_from("<H", data, 2)[0]
                        raw = data[4:4 + size]
                    else:
                        raise H5Error(f"h5: {path}: chunked datasets are not read")
                elif ver in (1, 2):
                    rank, cls = data[1], data[2]
                    p = 8
                    if cls == 1:
                        at = struct.unpack_from("<Q", data, p)[0]
                        raw = None if at == UNDEF else at
                    elif cls == 0:
                        p += 4 * rank
                        size = struct.unpack_from("<I", data, p)[0]
                        raw = data[p + 4:p + 4 + size]
                    else:
                        raise H5Error(f"h5: {path}: chunked datasets are not read")
                else:
                    raise H5Error(f"h5: layout message version {ver}")
        if shape is None or dt is None:
            raise H5Error(f"h5: {path} is not a dataset")
        n = int(np.prod(shape)) if shape else 1
        if isinstance(raw, int):
            raw = self.b[raw:raw + n * dt.itemsize]
        if raw is None or len(raw) < n * dt.itemsize:
            if n == 0:
                raw = b""
            else:
                raise H5Error(f"h5: {path}: no stored data")
        return np.frombuffer(raw, dt, count=n).reshape(shape).astype(dt.newbyteorder("=")) \
            if dt.kind != "S" else np.frombuffer(raw, dt, count=n).reshape(shape)


def read_keras_weights(path):
    """[(layer name, [(weight name, array), ...]), ...] in the file's layer order (Keras
    load_weights reads it in this order)."""
    f = H5File(path)
    ra = f.attrs("/")
    if "layer_names" not in ra:
        raise H5Error("h5: no layer_names attribute (not a Keras weights file)")
    out = []
    for ln in np.atleast_1d(ra["layer_names"]):
        lname = ln.decode("ascii")
        wn = f.attrs(lname).get("weight_names")
        names = [] if wn is None else [w.decode("ascii") for w in np.atleast_1d(wn)]
        out.append((lname, [(w, f.dataset(lname + "/" + w)) for w in names]))
    return out
