"""Victim checkpoint converter: a TensorFlow V2 checkpoint (tensor bundle) ->
the libphx weight blob, without TensorFlow.

The reference loads the released automl checkpoints with `util_keras.restore_ckpt`
(automl/efficientdet/tf2/util_keras.py:108-203, called by infer_lib.KerasDriver,
tf2/infer_lib.py:385-403, with ema_decay = config.moving_average_decay = 0.9998 and
skip_mismatch=False).  For a name-keyed (TF1 graph) checkpoint its rule is, per model variable v:

  * every trainable variable and every BN moving mean / variance is an "EMA variable"
    (get_ema_vars, util_keras.py:69-80); the checkpoint key of v is its name, and with
    ema_decay > 0 the key `<name>/ExponentialMovingAverage` (ExponentialMovingAverage.average_name)
    also maps to v — the EMA entry is inserted after the raw one, so it is the value v ends with;
  * every key of that map must be present with v's shape (skip_mismatch=False: KeyError /
    ValueError otherwise).

The libphx manifest (`phx_weight_manifest`) uses the reference's Keras variable names and TF
layouts (HWIO kernels, [k, k, C, 1] depthwise kernels), so conversion is a copy of each tensor into
its manifest offset.

Object-graph checkpoints (`tf.train.Checkpoint` / Keras `save_weights` in the TF2 format), the
reference's other branch (util_keras.py:131-152), restore by object path: tf.train.Checkpoint matches
the saved TrackableObjectGraph against the model's attributes and assigns every matched variable; the
EMA rule does not apply, unmatched variables keep their initial values, and a restore that matches
nothing fails (assert_nontrivial_match).  The object graph (the DT_STRING tensor
`_CHECKPOINTABLE_OBJECT_GRAPH`, a serialized TrackableObjectGraph) records for every variable its
`full_name` — the Keras variable name the manifest uses — next to its `checkpoint_key`, so the same
architecture's variables are found by full_name here (object_graph_keys).

Format (TensorFlow core/util/tensor_bundle, LevelDB table format): `<prefix>.index` is an SSTable
whose keys are tensor names (the empty key holds the BundleHeaderProto) and whose values are
BundleEntryProto {dtype, shape, shard_id, offset, size, crc32c (masked CRC-32C of the bytes)};
`<prefix>.data-SSSSS-of-NNNNN` hold the raw little-endian tensor bytes.  Only what the bundle
writer emits is read: uncompressed blocks, float32 / float16 / bfloat16 / float64 tensors.
"""
from __future__ import annotations

import os
import re
import struct

import numpy as np

# ---------------------------------------------------------------------------------------------
# CRC-32C (Castagnoli) and LevelDB's mask
# ---------------------------------------------------------------------------------------------
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes, crc: int = 0) -> int:
    crc ^= 0xFFFFFFFF
    tab = _CRC_TABLE
    for b in data:
        crc = tab[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def crc32c_mask(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def crc32c_unmask(masked: int) -> int:
    rot = (masked - 0xA282EAD8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------------------------------------------
# protobuf wire format (the few messages the bundle uses)
# ---------------------------------------------------------------------------------------------
def _varint(buf: bytes, pos: int):
    v = shift = 0
    while True:
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if b < 0x80:
            return v, pos
        shift += 7


def _fields(buf: bytes):
    """(field number, wire type, value) of a serialized message; length-delimited values are bytes."""
    pos = 0
    while pos < len(buf):
        tag, pos = _varint(buf, pos)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"checkpoint: unsupported protobuf wire type {wt}")
        yield f, wt, v


def _enc_varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _enc_field(f: int, wt: int, v) -> bytes:
    key = _enc_varint((f << 3) | wt)
    if wt == 0:
        return key + _enc_varint(v)
    if wt == 2:
        return key + _enc_varint(len(v)) + v
    if wt == 5:
        return key + struct.pack("<I", v)
    raise ValueError(wt)


# tensorflow/core/framework/types.proto
DT_FLOAT, DT_DOUBLE, DT_STRING, DT_BFLOAT16, DT_HALF = 1, 2, 7, 14, 19
_NP_OF = {DT_FLOAT: np.dtype("<f4"), DT_DOUBLE: np.dtype("<f8"), DT_HALF: np.dtype("<f2")}


class BundleEntry:
    """BundleEntryProto: dtype (1), shape (2: TensorShapeProto, dim (2) {size (1)}), shard_id (3),
    offset (4), size (5), crc32c (6), slices (7)."""

    def __init__(self, raw: bytes):
        self.dtype, self.shape, self.shard, self.offset, self.size, self.crc = 0, (), 0, 0, 0, None
        self.sliced = False
        for f, _, v in _fields(raw):
            if f == 1:
                self.dtype = v
            elif f == 2:
                dims = []
                for g, _, d in _fields(v):
                    if g == 2:
                        size = 0
                        for h, _, s in _fields(d):
                            if h == 1:
                                size = s - (1 << 64) if s >= 1 << 63 else s
                        dims.append(size)
                self.shape = tuple(dims)
            elif f == 3:
                self.shard = v
            elif f == 4:
                self.offset = v
            elif f == 5:
                self.size = v
            elif f == 6:
                self.crc = v
            elif f == 7:
                self.sliced = True


# ---------------------------------------------------------------------------------------------
# LevelDB table (SSTable) reader
# ---------------------------------------------------------------------------------------------
_TABLE_MAGIC = 0xDB4775248B80FB57
_FOOTER = 48


def _block_entries(block: bytes):
    """Key/value pairs of one table block (prefix-compressed keys, restart array at the end)."""
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrest
    pos, key = 0, b""
    while pos < end:
        shared, pos = _varint(block, pos)
        nonshared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        key = key[:shared] + block[pos:pos + nonshared]
        pos += nonshared
        yield key, block[pos:pos + vlen]
        pos += vlen


def _read_block(data: bytes, off: int, size: int, verify: bool) -> bytes:
    block = data[off:off + size]
    ctype = data[off + size]
    if ctype != 0:
        raise NotImplementedError("checkpoint index: compressed table blocks are not supported "
                                  "(the tensor-bundle writer stores them uncompressed)")
    if verify:
        want = struct.unpack_from("<I", data, off + size + 1)[0]
        got = crc32c_mask(crc32c(data[off:off + size + 1]))
        if want != got:
            raise ValueError("checkpoint index: block checksum mismatch")
    return block


def read_index(path: str, verify: bool = True) -> dict:
    """All (key -> value bytes) of a tensor-bundle index file."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < _FOOTER or struct.unpack_from("<Q", data, len(data) - 8)[0] != _TABLE_MAGIC:
        raise ValueError(f"{path}: not a TensorFlow checkpoint index (table magic missing)")
    foot = data[len(data) - _FOOTER:]
    pos = 0
    _, pos = _varint(foot, pos)        # metaindex handle (unused: no filter block)
    _, pos = _varint(foot, pos)
    ioff, pos = _varint(foot, pos)
    isize, pos = _varint(foot, pos)
    out = {}
    for _, handle in _block_entries(_read_block(data, ioff, isize, verify)):
        boff, p = _varint(handle, 0)
        bsize, _ = _varint(handle, p)
        for k, v in _block_entries(_read_block(data, boff, bsize, verify)):
            out[k] = v
    return out


class CheckpointReader:
    """tf.train.load_checkpoint for a name-keyed tensor bundle: list_variables / get_tensor."""

    def __init__(self, prefix: str, verify: bool = True):
        if os.path.isdir(prefix):
            prefix = latest_checkpoint(prefix)
        self.prefix = prefix
        self.verify = verify
        raw = read_index(prefix + ".index", verify)
        self.num_shards = 1
        if b"" in raw:
            for f, _, v in _fields(raw.pop(b"")):
                if f == 1:
                    self.num_shards = v
                elif f == 2 and v != 0:
                    raise NotImplementedError("checkpoint: big-endian bundles are not supported")
        self.entries = {k.decode(): BundleEntry(v) for k, v in raw.items()}
        self._shards = {}

    def list_variables(self):
        return sorted((k, list(e.shape)) for k, e in self.entries.items())

    def shape_map(self):
        return {k: e.shape for k, e in self.entries.items()}

    def _shard(self, i):
        if i not in self._shards:
            p = f"{self.prefix}.data-{i:05d}-of-{self.num_shards:05d}"
            self._shards[i] = np.memmap(p, dtype=np.uint8, mode="r")
        return self._shards[i]

    def get_strings(self, name: str) -> list:
        """A DT_STRING tensor as a flat list of bytes.  tensor_bundle's string layout: every element's
        length as a varint64, a masked CRC-32C of the lengths (taken over their uint64 little-endian
        bytes), then the element bytes; the entry's crc32c extends the same running CRC over the
        lengths' uint64 bytes, the 4 checksum bytes and the element bytes."""
        e = self.entries[name]
        if e.dtype != DT_STRING:
            raise ValueError(f"checkpoint: {name} is not a string tensor")
        raw = bytes(self._shard(e.shard)[e.offset:e.offset + e.size])
        n = int(np.prod(e.shape)) if e.shape else 1
        lens, pos = [], 0
        for _ in range(n):
            v, pos = _varint(raw, pos)
            lens.append(v)
        lraw = b"".join(struct.pack("<Q", v) for v in lens)
        lck = struct.unpack_from("<I", raw, pos)[0]
        if self.verify and crc32c_mask(crc32c(lraw)) != lck:
            raise ValueError(f"checkpoint: length checksum mismatch for {name}")
        body = raw[pos + 4:]
        if self.verify and e.crc is not None and \
                crc32c_mask(crc32c(lraw + raw[pos:pos + 4] + body)) != e.crc:
            raise ValueError(f"checkpoint: checksum mismatch for {name}")
        out, q = [], 0
        for v in lens:
            out.append(body[q:q + v])
            q += v
        return out

    def get_tensor(self, name: str) -> np.ndarray:
        e = self.entries[name]
        if e.sliced:
            raise NotImplementedError(f"checkpoint: partitioned variable {name}")
        raw = bytes(self._shard(e.shard)[e.offset:e.offset + e.size])
        if self.verify and e.crc is not None and crc32c_mask(crc32c(raw)) != e.crc:
            raise ValueError(f"checkpoint: checksum mismatch for {name}")
        if e.dtype == DT_BFLOAT16:
            u = np.frombuffer(raw, dtype="<u2").astype(np.uint32) << 16
            arr = u.view(np.float32)
        elif e.dtype in _NP_OF:
            arr = np.frombuffer(raw, dtype=_NP_OF[e.dtype])
        else:
            raise NotImplementedError(f"checkpoint: dtype {e.dtype} of {name}")
        return arr.reshape(e.shape).astype(np.float32)


def latest_checkpoint(directory: str) -> str:
    """tf.train.latest_checkpoint: the `model_checkpoint_path` of the directory's `checkpoint` file."""
    cp = os.path.join(directory, "checkpoint")
    if os.path.exists(cp):
        with open(cp) as f:
            for line in f:
                if line.startswith("model_checkpoint_path:"):
                    p = line.split(":", 1)[1].strip().strip('"')
                    return p if os.path.isabs(p) else os.path.join(directory, p)
    idx = [n[:-6] for n in os.listdir(directory) if n.endswith(".index")]
    if not idx:
        raise FileNotFoundError(f"no checkpoint in {directory}")
    if len(idx) == 1:
        return os.path.join(directory, idx[0])
    # no `checkpoint` file and several prefixes: the newest is the one with the largest trailing
    # step number (`model.ckpt-10` after `model.ckpt-9`); refuse to guess when they have none
    steps = {}
    for n in idx:
        m = re.search(r"-(\d+)$", n)
        if m is None:
            raise FileNotFoundError(f"{directory}: several checkpoints {sorted(idx)} and no `checkpoint` file")
        steps[n] = int(m.group(1))
    return os.path.join(directory, max(idx, key=lambda n: steps[n]))


# ---------------------------------------------------------------------------------------------
# writer (the same format; used to export blobs and by the tests)
# ---------------------------------------------------------------------------------------------
def _block(entries) -> bytes:
    out = bytearray()
    restarts = []
    prev = b""
    for i, (k, v) in enumerate(entries):
        if i % 16 == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                shared += 1
        out += _enc_varint(shared) + _enc_varint(len(k) - shared) + _enc_varint(len(v)) + k[shared:] + v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def _put_block(f, content: bytes) -> bytes:
    off = f.tell()
    f.write(content)
    f.write(b"\x00" + struct.pack("<I", crc32c_mask(crc32c(content + b"\x00"))))
    return _enc_varint(off) + _enc_varint(len(content))


def write_checkpoint(prefix: str, tensors: dict, block_entries: int = 64, update_latest: bool | None = None,
                     strings: dict | None = None):
    """Write float32 tensors as a single-shard tensor bundle (<prefix>.index + .data-00000-of-00001).

    update_latest: rewrite the directory's `checkpoint` file to point at this prefix.  None (the
    default) writes it only when the directory has none, so exporting into an existing checkpoint
    directory never silently redirects its latest pointer."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    strings = strings or {}
    names = sorted(list(tensors) + list(strings))
    entries = []
    with open(prefix + ".data-00000-of-00001", "wb") as d:
        for n in names:
            if n in strings:  # DT_STRING, shape [] for one element (tensor_bundle's string layout)
                elems = [bytes(x) for x in strings[n]]
                lraw = b"".join(struct.pack("<Q", len(x)) for x in elems)
                lck = struct.pack("<I", crc32c_mask(crc32c(lraw)))
                raw = b"".join(_enc_varint(len(x)) for x in elems) + lck + b"".join(elems)
                body_crc = crc32c_mask(crc32c(lraw + lck + b"".join(elems)))
                shape = b"" if len(elems) == 1 else _enc_field(2, 2, _enc_field(1, 0, len(elems)))
                msg = (_enc_field(1, 0, DT_STRING) + _enc_field(2, 2, shape) + _enc_field(4, 0, d.tell())
                       + _enc_field(5, 0, len(raw)) + _enc_field(6, 5, body_crc))
                entries.append((n.encode(), msg))
                d.write(raw)
                continue
            a = np.ascontiguousarray(np.asarray(tensors[n], dtype="<f4"))
            raw = a.tobytes()
            shape = b"".join(_enc_field(2, 2, _enc_field(1, 0, int(s))) for s in a.shape)
            msg = (_enc_field(1, 0, DT_FLOAT) + _enc_field(2, 2, shape) + _enc_field(4, 0, d.tell())
                   + _enc_field(5, 0, len(raw)) + _enc_field(6, 5, crc32c_mask(crc32c(raw))))
            entries.append((n.encode(), msg))
            d.write(raw)
    header = _enc_field(1, 0, 1) + _enc_field(3, 2, _enc_field(1, 0, 1))
    entries.insert(0, (b"", header))
    with open(prefix + ".index", "wb") as f:
        index = []
        for i in range(0, len(entries), block_entries):
            chunk = entries[i:i + block_entries]
            index.append((chunk[-1][0], _put_block(f, _block(chunk))))
        meta = _put_block(f, _block([]))
        ih = _put_block(f, _block(index))
        footer = meta + ih
        footer += b"\x00" * (_FOOTER - 8 - len(footer)) + struct.pack("<Q", _TABLE_MAGIC)
        f.write(footer)
    cp = os.path.join(os.path.dirname(os.path.abspath(prefix)), "checkpoint")
    if update_latest is None:
        update_latest = not os.path.exists(cp)
    if update_latest:
        with open(cp, "w") as f:
            f.write(f'model_checkpoint_path: "{os.path.basename(prefix)}"\n')


def _enc_varint_field(f: int, v: int) -> bytes:
    return _enc_field(f, 0, v)


def write_object_graph_checkpoint(prefix: str, tensors: dict, paths: dict | None = None):
    """A TF2 object-based checkpoint of float32 variables, as tf.train.Checkpoint(model=...).save
    lays it out: each variable under `<object path>/.ATTRIBUTES/VARIABLE_VALUE`, and the
    TrackableObjectGraph (nodes = root, one node per path component, one per variable with its
    SerializedTensor {name "VARIABLE_VALUE", full_name, checkpoint_key}) as the DT_STRING scalar
    `_CHECKPOINTABLE_OBJECT_GRAPH`.  paths: full_name -> object path (default "model/<full_name>")."""
    paths = paths or {k: "model/" + k for k in tensors}
    nodes = [dict(children={}, attr=None)]  # node 0: the root
    for full, path in paths.items():
        cur = 0
        for comp in path.split("/"):
            nxt = nodes[cur]["children"].get(comp)
            if nxt is None:
                nodes.append(dict(children={}, attr=None))
                nxt = len(nodes) - 1
                nodes[cur]["children"][comp] = nxt
            cur = nxt
        nodes[cur]["attr"] = (full, path + "/.ATTRIBUTES/VARIABLE_VALUE")
    graph = b""
    for nd in nodes:
        body = b"".join(_enc_field(1, 2, _enc_varint_field(1, i) + _enc_field(2, 2, c.encode()))
                        for c, i in nd["children"].items())
        if nd["attr"]:
            full, key = nd["attr"]
            body += _enc_field(2, 2, _enc_field(1, 2, b"VARIABLE_VALUE") + _enc_field(2, 2, full.encode())
                               + _enc_field(3, 2, key.encode()))
        graph += _enc_field(1, 2, body)
    t = {paths[k] + "/.ATTRIBUTES/VARIABLE_VALUE": v for k, v in tensors.items()}
    write_checkpoint(prefix, t, strings={"_CHECKPOINTABLE_OBJECT_GRAPH": [graph]})


def object_graph_keys(reader) -> dict:
    """full_name -> checkpoint_key of every variable attribute in the checkpoint's object graph
    (TrackableObjectGraph: nodes (1) {children (1), attributes (2) {name (1), full_name (2),
    checkpoint_key (3)}})."""
    graph = reader.get_strings("_CHECKPOINTABLE_OBJECT_GRAPH")[0]
    out = {}
    for f, _, node in _fields(graph):
        if f != 1:
            continue
        for g, _, att in _fields(node):
            if g != 2:
                continue
            a = {h: v for h, _, v in _fields(att)}
            if a.get(1) == b"VARIABLE_VALUE" and 2 in a and 3 in a:
                out[a[2].decode()] = a[3].decode()
    return out


# ---------------------------------------------------------------------------------------------
# restore_ckpt for the libphx manifest
# ---------------------------------------------------------------------------------------------
EMA_SUFFIX = "/ExponentialMovingAverage"


def _is_ema_var(p) -> bool:
    """get_ema_vars (util_keras.py:69-80): every trainable variable plus the BN moving statistics —
    which is every entry of the manifest (it holds no other variables)."""
    return True


def checkpoint_to_blob(ckpt, manifest, ema_decay: float = 0.9998, skip_mismatch: bool = False,
                       verify: bool = True) -> np.ndarray:
    """util_keras.restore_ckpt (name-keyed branch, util_keras.py:153-203) onto the manifest: returns the
    weight blob.  With skip_mismatch, missing / mis-shaped entries keep 0 (the reference leaves the
    variable's initial value) and are reported through the returned blob's `.missing` list."""
    reader = ckpt if isinstance(ckpt, CheckpointReader) else CheckpointReader(ckpt, verify)
    keys = [k for k, _ in reader.list_variables()]
    if keys and keys[0] == "_CHECKPOINTABLE_OBJECT_GRAPH":
        return _object_graph_to_blob(reader, manifest)
    shapes = reader.shape_map()
    n = max(p["offset"] + int(np.prod(p["shape"])) for p in manifest)
    blob = np.zeros(n, np.float32)
    missing = []
    for p in manifest:
        name, shape = p["name"], tuple(p["shape"])
        cands = [name]
        if ema_decay and ema_decay > 0 and _is_ema_var(p):
            cands.append(name + EMA_SUFFIX)  # inserted after the raw key: the value the variable ends with
        val = None
        for key in cands:
            if key not in shapes:
                msg = f"Not found {key} in {reader.prefix}"
                if not skip_mismatch:
                    raise KeyError(msg)
                missing.append(key)
                continue
            if tuple(shapes[key]) != shape:
                msg = f"Shape mismatch: {key}, expected {shape}, but got {tuple(shapes[key])}"
                if not skip_mismatch:
                    raise ValueError(msg)
                missing.append(key)
                continue
            val = reader.get_tensor(key)
        if val is not None:
            off = p["offset"]
            blob[off:off + val.size] = val.reshape(-1)
    out = blob.view(_Blob)
    out.missing = missing
    return out


def _object_graph_to_blob(reader, manifest) -> np.ndarray:
    """The object-graph branch of restore_ckpt (util_keras.py:131-152): every manifest variable whose
    full_name the object graph records gets its saved value (no EMA rule); the others keep 0 and
    are listed in `.missing`; a restore that matches nothing (assert_nontrivial_match) falls back to
    the hub-checkpoint loader, which fails on any missing key."""
    by_name = object_graph_keys(reader)
    shapes = reader.shape_map()
    n = max(p["offset"] + int(np.prod(p["shape"])) for p in manifest)
    blob = np.zeros(n, np.float32)
    missing, matched = [], 0
    for p in manifest:
        key = by_name.get(p["name"])
        if key is None or key not in shapes:
            missing.append(p["name"])
            continue
        if tuple(shapes[key]) != tuple(p["shape"]):
            raise ValueError(f"Shape mismatch: {key}, expected {tuple(p['shape'])}, but got {tuple(shapes[key])}")
        val = reader.get_tensor(key)
        blob[p["offset"]:p["offset"] + val.size] = val.reshape(-1)
        matched += 1
    if not matched:
        # assert_nontrivial_match failed: restore_ckpt falls back to load_from_hub_checkpoint
        # (util_keras.py:141-147)
        return hub_checkpoint_to_blob(reader, manifest)
    out = blob.view(_Blob)
    out.missing = missing
    return out


# util_keras.HUB_CPT_NAME (util_keras.py:24-26): variable-name prefix -> EfficientDetNetTrainHub
# object, tried in this order ('' matches everything else)
HUB_CPT_NAME = (("class_net/class-predict/", "classes"), ("box_net/box-predict/", "boxes"), ("", "base_model"))


def hub_checkpoint_key(var_name: str) -> str:
    """load_from_hub_checkpoint's _get_cpt_var_name (util_keras.py:86-96) for a Keras variable name
    (with its ':0'): the prefix is replaced by the hub object's name, '/' becomes '.S' (the object
    graph's escaping of a slash inside one path component), and ':0' is dropped except under
    base_model, whose keys keep it."""
    for prefix, hub in HUB_CPT_NAME:
        if var_name.startswith(prefix):
            key = hub + "/" + var_name[len(prefix):].replace("/", ".S")
            if prefix:
                key = key.replace(":0", "")
            return key + "/.ATTRIBUTES/VARIABLE_VALUE"
    raise AssertionError("unreachable: the '' prefix matches every name")


def hub_checkpoint_to_blob(ckpt, manifest, verify: bool = True) -> np.ndarray:
    """load_from_hub_checkpoint (util_keras.py:83-105): every variable of the model (model.weights:
    the manifest, named '<name>:0') is assigned tf.train.load_variable(ckpt, hub key) — a missing key
    or a mis-shaped value fails, as the reference's assign does."""
    reader = ckpt if isinstance(ckpt, CheckpointReader) else CheckpointReader(ckpt, verify)
    shapes = reader.shape_map()
    n = max(p["offset"] + int(np.prod(p["shape"])) for p in manifest)
    blob = np.zeros(n, np.float32)
    for p in manifest:
        key = hub_checkpoint_key(p["name"] + ":0")
        if key not in shapes:
            raise KeyError(f"Key {key} not found in checkpoint {reader.prefix} (load_from_hub_checkpoint)")
        if tuple(shapes[key]) != tuple(p["shape"]):
            raise ValueError(f"Shape mismatch: {key}, expected {tuple(p['shape'])}, but got {tuple(shapes[key])}")
        val = reader.get_tensor(key)
        blob[p["offset"]:p["offset"] + val.size] = val.reshape(-1)
    out = blob.view(_Blob)
    out.missing = []
    return out


def write_hub_checkpoint(prefix: str, manifest, blob: np.ndarray):
    """An EfficientDetNetTrainHub-style object checkpoint of a weight blob: every variable under its
    hub key (hub_checkpoint_key), with an object graph whose full names are the hub objects' own
    (so it matches no EfficientDetNet variable, and restore_ckpt takes the hub fallback)."""
    tensors, paths = {}, {}
    for p in manifest:
        v = np.asarray(blob[p["offset"]:p["offset"] + int(np.prod(p["shape"]))], np.float32).reshape(p["shape"])
        path = hub_checkpoint_key(p["name"] + ":0")[: -len("/.ATTRIBUTES/VARIABLE_VALUE")]
        tensors["hub/" + path] = v
        paths["hub/" + path] = path
    write_object_graph_checkpoint(prefix, tensors, paths)


class _Blob(np.ndarray):
    missing: list = []


def blob_to_checkpoint(prefix: str, manifest, blob: np.ndarray, ema: bool = True):
    """Export a weight blob under the manifest's names (and, with ema, the same values as the
    ExponentialMovingAverage shadows the reference's loader prefers)."""
    t = {}
    for p in manifest:
        v = np.asarray(blob[p["offset"]:p["offset"] + int(np.prod(p["shape"]))], np.float32).reshape(p["shape"])
        t[p["name"]] = v
        if ema and _is_ema_var(p):
            t[p["name"] + EMA_SUFFIX] = v
    write_checkpoint(prefix, t)
