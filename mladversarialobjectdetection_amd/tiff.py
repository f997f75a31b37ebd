"""Minimal baseline-TIFF I/O for the reference's patch checkpoint format.

PatchAttacker.save_weights writes the raw normalised patch with ``tifffile.imwrite(
'patch.tiff', patch)`` (attacker.py:341) and ``initial_patch=dir`` / the defender's evaluation
patch read it back with ``tifffile.imread`` (attacker.py:46-48, attack_detection.py:57-59).
tifffile is not installed here, so this module writes and reads the same kind of file directly:
one image, float32 samples (SampleFormat 3), samples-per-pixel 1..4 interleaved
(PlanarConfiguration 1), uncompressed strips.  Either byte order is accepted on read.
"""
from __future__ import annotations

import struct

import numpy as np

# tag ids (TIFF 6.0)
_W, _H, _BPS, _COMP, _PHOTO, _OFFS, _SPP, _RPS, _COUNTS, _PLANAR, _FMT = (
    256, 257, 258, 259, 262, 273, 277, 278, 279, 284, 339)
_SHORT, _LONG = 3, 4


def write_float_tiff(path: str, img: np.ndarray) -> None:
    """img [H,W] or [H,W,C] (C <= 4) -> little-endian float32 TIFF, one strip."""
    a = np.ascontiguousarray(np.asarray(img, dtype="<f4"))
    if a.ndim == 2:
        a = a[..., None]
    if a.ndim != 3 or not 1 <= a.shape[2] <= 4:
        raise ValueError(f"expected [H,W] or [H,W,C<=4], got {a.shape}")
    h, w, c = a.shape
    data = a.tobytes()
    ntags = 11
    ifd_off = 8
    ifd_size = 2 + 12 * ntags + 4
    extra_off = ifd_off + ifd_size          # BitsPerSample / SampleFormat arrays when c > 2
    extra = b""

    def shorts(vals):
        nonlocal extra
        if len(vals) <= 2:
            return struct.pack("<2H", *(list(vals) + [0] * (2 - len(vals))))
        off = extra_off + len(extra)
        extra += struct.pack(f"<{len(vals)}H", *vals)
        if len(extra) % 2:
            extra += b"\0"
        return struct.pack("<I", off)

    entries = [
        (_W, _LONG, 1, struct.pack("<I", w)),
        (_H, _LONG, 1, struct.pack("<I", h)),
        (_BPS, _SHORT, c, shorts([32] * c)),
        (_COMP, _SHORT, 1, struct.pack("<2H", 1, 0)),
        (_PHOTO, _SHORT, 1, struct.pack("<2H", 2 if c >= 3 else 1, 0)),
        (_OFFS, _LONG, 1, None),  # patched below
        (_SPP, _SHORT, 1, struct.pack("<2H", c, 0)),
        (_RPS, _LONG, 1, struct.pack("<I", h)),
        (_COUNTS, _LONG, 1, struct.pack("<I", len(data))),
        (_PLANAR, _SHORT, 1, struct.pack("<2H", 1, 0)),
        (_FMT, _SHORT, c, shorts([3] * c)),
    ]
    data_off = extra_off + len(extra)
    ifd = struct.pack("<H", ntags)
    for tag, typ, cnt, val in entries:
        if val is None:
            val = struct.pack("<I", data_off)
        ifd += struct.pack("<HHI", tag, typ, cnt) + val
    ifd += struct.pack("<I", 0)
    with open(path, "wb") as f:
        f.write(b"II*\0" + struct.pack("<I", ifd_off) + ifd + extra + data)


def read_float_tiff(path: str) -> np.ndarray:
    """First image of an uncompressed, interleaved float32 TIFF -> [H,W,C] (C == 1 squeezed)."""
    with open(path, "rb") as f:
        buf = f.read()
    bo = {b"II": "<", b"MM": ">"}.get(buf[:2])
    if bo is None or struct.unpack(bo + "H", buf[2:4])[0] != 42:
        raise ValueError(f"{path}: not a classic TIFF")
    off = struct.unpack(bo + "I", buf[4:8])[0]
    n = struct.unpack(bo + "H", buf[off:off + 2])[0]
    sizes = {1: 1, 3: 2, 4: 4}
    tags = {}
    for i in range(n):
        e = off + 2 + 12 * i
        tag, typ, cnt = struct.unpack(bo + "HHI", buf[e:e + 8])
        sz = sizes.get(typ)
        if sz is None:
            continue
        raw = buf[e + 8:e + 12] if sz * cnt <= 4 else buf[struct.unpack(bo + "I", buf[e + 8:e + 12])[0]:][:sz * cnt]
        code = {1: "B", 3: "H", 4: "I"}[typ]
        tags[tag] = list(struct.unpack(bo + code * cnt, raw[:sz * cnt]))
    w, h = tags[_W][0], tags[_H][0]
    c = tags.get(_SPP, [1])[0]
    if tags.get(_COMP, [1])[0] != 1:
        raise ValueError(f"{path}: compressed TIFF not supported")
    if tags.get(_PLANAR, [1])[0] != 1 and c > 1:
        raise ValueError(f"{path}: planar (separate) TIFF not supported")
    if set(tags.get(_BPS, [32])) != {32} or set(tags.get(_FMT, [1])) != {3}:
        raise ValueError(f"{path}: not float32 samples")
    data = b"".join(buf[o:o + k] for o, k in zip(tags[_OFFS], tags[_COUNTS]))
    a = np.frombuffer(data, dtype=bo + "f4", count=h * w * c).astype(np.float32).reshape(h, w, c)
    return a[..., 0] if c == 1 else a
