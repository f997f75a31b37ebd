"""Victim checkpoint converter (mladversarialobjectdetection_amd/ckpt.py) on CPU.

No TensorFlow checkpoint ships with the reference or exists in this image, so the bundle reader is
checked against the format's published constants (CRC-32C check value, LevelDB's checksum mask and
table magic) and against bundles written by this module's writer (parity unpinned beyond those);
the restore rule is the reference's (util_keras.restore_ckpt, util_keras.py:153-203): EMA shadows win,
missing keys raise KeyError and shape mismatches ValueError unless skip_mismatch.
"""
import os
import struct

import numpy as np
import pytest

from mladversarialobjectdetection_amd import ckpt as C
from mladversarialobjectdetection_amd import weights as W


def test_crc32c_known_answers():
    assert C.crc32c(b"123456789") == 0xE3069283          # the CRC-32C check value
    assert C.crc32c(b"") == 0
    assert C.crc32c(bytes(32)) == 0x8A9136AA             # RFC 3720 B.4: 32 bytes of zeros
    assert C.crc32c(bytes([0xFF] * 32)) == 0x62A8AB43     # RFC 3720 B.4: 32 bytes of ones
    assert C.crc32c(bytes(range(32))) == 0x46DD794E       # RFC 3720 B.4: incrementing
    for v in (0, 1, 0xE3069283, 0xFFFFFFFF):
        assert C.crc32c_unmask(C.crc32c_mask(v)) == v
    assert C.crc32c_mask(0) == 0xA282EAD8


def _manifest():
    from mladversarialobjectdetection_amd import _lib
    return _lib.Context("efficientdet-d0", 128, 1).manifest()


@pytest.fixture(scope="module")
def d0():
    man = _manifest()
    return man, W.synthetic_blob(man, seed=3)


def test_round_trip_is_bit_exact(tmp_path, d0):
    man, blob = d0
    prefix = str(tmp_path / "ckpt" / "model")
    C.blob_to_checkpoint(prefix, man, blob)
    with open(prefix + ".index", "rb") as f:
        raw = f.read()
    assert struct.unpack_from("<Q", raw, len(raw) - 8)[0] == 0xDB4775248B80FB57
    r = C.CheckpointReader(os.path.dirname(prefix))       # directory: `checkpoint` file -> prefix
    assert len(r.list_variables()) == 2 * len(man)
    out = C.checkpoint_to_blob(r, man)
    assert out.dtype == np.float32 and out.shape == blob.shape
    assert np.array_equal(out.view(np.uint32), blob.view(np.uint32))


def test_ema_shadow_wins_unless_disabled(tmp_path, d0):
    man, blob = d0
    t = {}
    for p in man[:40]:
        v = blob[p["offset"]:p["offset"] + int(np.prod(p["shape"]))].reshape(p["shape"])
        t[p["name"]] = v
        t[p["name"] + C.EMA_SUFFIX] = v * 2 + 1
    prefix = str(tmp_path / "m")
    C.write_checkpoint(prefix, t)
    part = man[:40]
    n = part[-1]["offset"] + int(np.prod(part[-1]["shape"]))
    ema = C.checkpoint_to_blob(prefix, part, ema_decay=0.9998)
    raw = C.checkpoint_to_blob(prefix, part, ema_decay=0)
    np.testing.assert_array_equal(raw[:n], blob[:n])
    np.testing.assert_array_equal(ema[:n], blob[:n] * 2 + 1)


def test_missing_and_mismatched_keys(tmp_path, d0):
    man, blob = d0
    part = man[:10]
    t = {p["name"]: blob[p["offset"]:p["offset"] + int(np.prod(p["shape"]))].reshape(p["shape"]) for p in part}
    prefix = str(tmp_path / "m")
    C.write_checkpoint(prefix, t)
    with pytest.raises(KeyError):                        # no EMA shadows, ema_decay > 0
        C.checkpoint_to_blob(prefix, part)
    ok = C.checkpoint_to_blob(prefix, part, ema_decay=0)
    n = part[-1]["offset"] + int(np.prod(part[-1]["shape"]))
    np.testing.assert_array_equal(ok[:n], blob[:n])
    bad = dict(t)
    bad[part[0]["name"]] = np.zeros((2, 2), np.float32)
    C.write_checkpoint(prefix, bad)
    with pytest.raises(ValueError):
        C.checkpoint_to_blob(prefix, part, ema_decay=0)
    skipped = C.checkpoint_to_blob(prefix, part, ema_decay=0, skip_mismatch=True)
    assert skipped.missing == [part[0]["name"]]
    assert not skipped[:int(np.prod(part[0]["shape"]))].any()


def test_corruption_and_object_graph_are_rejected(tmp_path):
    prefix = str(tmp_path / "m")
    C.write_checkpoint(prefix, {"a/kernel": np.arange(6, dtype=np.float32).reshape(2, 3)})
    assert np.array_equal(C.CheckpointReader(prefix).get_tensor("a/kernel"), np.arange(6).reshape(2, 3))
    data = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    data[0] ^= 1
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(ValueError):
        C.CheckpointReader(prefix).get_tensor("a/kernel")
    # an object-graph key that is not a serialized TrackableObjectGraph string
    C.write_checkpoint(prefix, {"_CHECKPOINTABLE_OBJECT_GRAPH": np.zeros(1, np.float32)})
    with pytest.raises(ValueError):
        C.checkpoint_to_blob(prefix, [{"name": "x", "shape": [1], "offset": 0}])


def test_many_blocks_and_shared_prefixes(tmp_path):
    # more than one data block and restart interval, long shared key prefixes
    rng = np.random.default_rng(0)
    t = {f"efficientnet-b0/blocks_{i}/conv2d/kernel": rng.standard_normal((i % 5 + 1, 3)).astype(np.float32)
         for i in range(300)}
    prefix = str(tmp_path / "m")
    C.write_checkpoint(prefix, t, block_entries=7)
    r = C.CheckpointReader(prefix)
    assert sorted(r.entries) == sorted(t)
    for k in list(t)[::37]:
        np.testing.assert_array_equal(r.get_tensor(k), t[k])


def test_latest_checkpoint_without_pointer_file(tmp_path):
    """No `checkpoint` file: the largest trailing step wins (model.ckpt-10 after -9), and several
    prefixes without step numbers are refused rather than guessed."""
    a = {"a/kernel": np.ones((1,), np.float32)}
    for step in (9, 10, 2):
        C.write_checkpoint(str(tmp_path / f"model.ckpt-{step}"), a, update_latest=False)
    assert not (tmp_path / "checkpoint").exists()
    assert C.latest_checkpoint(str(tmp_path)) == str(tmp_path / "model.ckpt-10")
    other = tmp_path / "other"
    C.write_checkpoint(str(other / "x"), a, update_latest=False)
    assert C.latest_checkpoint(str(other)) == str(other / "x")      # a single prefix is unambiguous
    C.write_checkpoint(str(other / "y"), a, update_latest=False)
    with pytest.raises(FileNotFoundError):
        C.latest_checkpoint(str(other))


def test_export_keeps_an_existing_latest_pointer(tmp_path):
    a = {"a/kernel": np.ones((1,), np.float32)}
    C.write_checkpoint(str(tmp_path / "model.ckpt-5"), a)           # no pointer yet: written
    C.write_checkpoint(str(tmp_path / "export"), a)                 # pointer exists: kept
    assert C.latest_checkpoint(str(tmp_path)) == str(tmp_path / "model.ckpt-5")
    C.write_checkpoint(str(tmp_path / "export"), a, update_latest=True)
    assert C.latest_checkpoint(str(tmp_path)) == str(tmp_path / "export")


def test_object_graph_checkpoint_restores_by_full_name(tmp_path, d0):
    """The reference's object-graph branch (util_keras.py:131-152): variables are found through the
    TrackableObjectGraph's full_name -> checkpoint_key records (Keras-style object paths), no EMA
    rule applies, unmatched variables are reported, and a graph matching nothing is refused."""
    man, blob = d0
    t = {p["name"]: blob[p["offset"]:p["offset"] + int(np.prod(p["shape"]))].reshape(p["shape"]) for p in man}
    # Keras-like object paths (attribute names, layer lists), unrelated to the variable names
    paths = {name: f"model/net/_layers/{i}/{name.rsplit('/', 1)[-1]}" for i, name in enumerate(t)}
    prefix = str(tmp_path / "og" / "ckpt-1")
    C.write_object_graph_checkpoint(prefix, t, paths)
    r = C.CheckpointReader(prefix)
    assert r.list_variables()[0][0] == "_CHECKPOINTABLE_OBJECT_GRAPH"
    keys = C.object_graph_keys(r)
    assert len(keys) == len(man) and keys[man[0]["name"]] == paths[man[0]["name"]] + "/.ATTRIBUTES/VARIABLE_VALUE"
    out = C.checkpoint_to_blob(prefix, man, ema_decay=0.9998)
    assert np.array_equal(out.view(np.uint32), blob.view(np.uint32)) and out.missing == []
    # a partial graph: the others keep 0 and are listed
    half = dict(list(t.items())[: len(t) // 2])
    C.write_object_graph_checkpoint(str(tmp_path / "og2" / "ckpt-1"), half, {k: paths[k] for k in half})
    part = C.checkpoint_to_blob(str(tmp_path / "og2"), man)
    assert len(part.missing) == len(man) - len(half)
    p0 = man[0]
    n0 = int(np.prod(p0["shape"]))
    np.testing.assert_array_equal(part[p0["offset"]:p0["offset"] + n0], blob[p0["offset"]:p0["offset"] + n0])
    # nothing matches: assert_nontrivial_match fails and the hub fallback finds no hub key either
    C.write_object_graph_checkpoint(str(tmp_path / "og3" / "ckpt-1"), {"other/kernel": np.ones(2, np.float32)})
    with pytest.raises(KeyError):
        C.checkpoint_to_blob(str(tmp_path / "og3"), man)
    # the string tensor's checksums are verified
    data = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    e = r.entries["_CHECKPOINTABLE_OBJECT_GRAPH"]
    data[e.offset + e.size - 1] ^= 1
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(ValueError):
        C.object_graph_keys(C.CheckpointReader(prefix))


def test_hub_checkpoint_key_follows_util_keras():
    """_get_cpt_var_name (util_keras.py:86-96): prefix -> hub object, '/' -> '.S', ':0' dropped except
    under base_model."""
    assert C.hub_checkpoint_key("class_net/class-predict/depthwise_kernel:0") == \
        "classes/depthwise_kernel/.ATTRIBUTES/VARIABLE_VALUE"
    assert C.hub_checkpoint_key("box_net/box-predict/bias:0") == "boxes/bias/.ATTRIBUTES/VARIABLE_VALUE"
    assert C.hub_checkpoint_key("efficientnet-b0/stem/conv2d/kernel:0") == \
        "base_model/efficientnet-b0.Sstem.Sconv2d.Skernel:0/.ATTRIBUTES/VARIABLE_VALUE"
    assert C.hub_checkpoint_key("class_net/class-0/bias:0") == \
        "base_model/class_net.Sclass-0.Sbias:0/.ATTRIBUTES/VARIABLE_VALUE"


def test_hub_checkpoint_fallback_restores_every_variable(tmp_path, d0):
    """restore_ckpt's AssertionError branch (util_keras.py:141-147): an EfficientDetNetTrainHub
    checkpoint (object graph of the hub objects, matching no EfficientDetNet variable) is loaded by
    load_from_hub_checkpoint bit for bit; a missing or mis-shaped hub key fails."""
    man, blob = d0
    prefix = str(tmp_path / "hub" / "ckpt-1")
    C.write_hub_checkpoint(prefix, man, blob)
    out = C.checkpoint_to_blob(str(tmp_path / "hub"), man)
    assert np.array_equal(out.view(np.uint32), blob.view(np.uint32)) and out.missing == []
    short = [p for p in man if p is not man[3]]
    C.write_hub_checkpoint(str(tmp_path / "hub2" / "ckpt-1"), short, blob)
    with pytest.raises(KeyError):
        C.checkpoint_to_blob(str(tmp_path / "hub2"), man)
