"""CPU: host-side pieces of the mirror that need no GPU — the reference's patch checkpoint format
(patch.tiff, attacker.py:341 / :46-48) and config_override validation (hparams_config.py:91-109)."""
import struct

import numpy as np
import pytest

from mladversarialobjectdetection_amd import _lib
from mladversarialobjectdetection_amd import tiff
from mladversarialobjectdetection_amd.attacker import NmsConfig, VictimConfig


def test_float_tiff_round_trip(tmp_path):
    p = np.random.default_rng(0).uniform(-1, 1, (640, 640, 3)).astype(np.float32)
    f = str(tmp_path / "patch.tiff")
    tiff.write_float_tiff(f, p)
    q = tiff.read_float_tiff(f)
    assert q.dtype == np.float32 and q.shape == (640, 640, 3)
    np.testing.assert_array_equal(q, p)
    g = np.arange(12, dtype=np.float32).reshape(3, 4)
    tiff.write_float_tiff(f, g)
    np.testing.assert_array_equal(tiff.read_float_tiff(f), g)


def test_big_endian_multi_strip_tiff(tmp_path):
    """A tifffile-style big-endian file with two strips and the tags at the end of the file."""
    img = np.arange(2 * 3 * 3, dtype=np.float32).reshape(2, 3, 3) / 7
    data = img.astype(">f4").tobytes()
    half = len(data) // 2
    ents = []
    def tag(t, typ, cnt, val):
        ents.append(struct.pack(">HHI", t, typ, cnt) + val)
    bps_off = 8 + len(data)
    fmt_off = bps_off + 6
    ifd_off = fmt_off + 6
    tag(256, 3, 1, struct.pack(">HH", 3, 0))
    tag(257, 3, 1, struct.pack(">HH", 2, 0))
    tag(258, 3, 3, struct.pack(">I", bps_off))
    tag(259, 3, 1, struct.pack(">HH", 1, 0))
    tag(262, 3, 1, struct.pack(">HH", 2, 0))
    tag(273, 4, 2, struct.pack(">I", ifd_off + 2 + 12 * 11 + 4))
    tag(277, 3, 1, struct.pack(">HH", 3, 0))
    tag(278, 3, 1, struct.pack(">HH", 1, 0))
    tag(279, 4, 2, struct.pack(">I", ifd_off + 2 + 12 * 11 + 4 + 8))
    tag(284, 3, 1, struct.pack(">HH", 1, 0))
    tag(339, 3, 3, struct.pack(">I", fmt_off))
    buf = (b"MM\0*" + struct.pack(">I", ifd_off) + data + struct.pack(">3H", 32, 32, 32)
           + struct.pack(">3H", 3, 3, 3) + struct.pack(">H", 11) + b"".join(ents) + struct.pack(">I", 0)
           + struct.pack(">2I", 8, 8 + half) + struct.pack(">2I", half, len(data) - half))
    f = tmp_path / "be.tiff"
    f.write_bytes(buf)
    np.testing.assert_array_equal(tiff.read_float_tiff(str(f)), img)


def test_config_override_validation():
    ctx = _lib.Context("efficientdet-d0", image_size=128, max_batch=1)
    c = VictimConfig("efficientdet-d0", 128, [0] * 3, [1] * 3, NmsConfig(score_thresh=0.5))
    c.override({"nms_configs": {"iou_thresh": .5, "score_thresh": .25}}, ctx)  # attacker_train.py:31 shape
    assert c.nms_configs.score_thresh == .25 and ctx.model_info()["nms_score_thresh"] == pytest.approx(.25)
    for bad in ({"nms_configs": {"method": "hard"}}, {"nms_configs": {"max_output_size": 50}},
                {"nms_configs": {"sigma": 0.3}}, {"image_size": 256}, {"nms_configs": {"foo": 1}}):
        with pytest.raises(ValueError):
            c.override(bad, ctx)


def test_config_override_reaches_the_owning_context():
    """victim.config.override({...}) as the reference writes it (no ctx argument) must reach the
    library threshold; a config owned by no context refuses a computation-changing override."""
    ctx = _lib.Context("efficientdet-d0", image_size=128, max_batch=1)
    c = VictimConfig("efficientdet-d0", 128, [0] * 3, [1] * 3, NmsConfig(score_thresh=0.5), ctx=ctx)
    c.override({"nms_configs": {"score_thresh": .3}})
    assert ctx.model_info()["nms_score_thresh"] == pytest.approx(.3)
    loose = VictimConfig("efficientdet-d0", 128, [0] * 3, [1] * 3, NmsConfig(score_thresh=0.5))
    with pytest.raises(ValueError):
        loose.override({"nms_configs": {"score_thresh": .3}})
    loose.override({"nms_configs": {"iou_thresh": .5}})   # changes nothing the library computes


def test_derive_asr_counts_coordinates_like_calc_asr():
    """calc_asr (attacker.py:253-255) divides tf.size of the flattened [n,4] box tensors:
    1 - 4n / (4d + 1e-7).  With d = 0 and n > 0 that is 1 - 4e7 n, not 1 - 1e7 n."""
    from mladversarialobjectdetection_amd.attacker import PatchAttacker
    import oracle.step as ostep
    row = np.zeros(_lib.NMETRIC + 1)
    row[_lib.M_NIMG], row[_lib.NMETRIC] = 2, 0.4
    row[_lib.M_ASR_NUM], row[_lib.M_ASR_DEN] = 3, 0
    d = PatchAttacker._derive(row)
    assert d["asr"] == ostep.calc_asr(3, 0)
    assert d["asr"] == pytest.approx(1 - 4 * 3 / np.float32(1e-7), rel=1e-6)
    row[_lib.M_ASR_NUM], row[_lib.M_ASR_DEN] = 1, 5
    assert PatchAttacker._derive(row)["asr"] == pytest.approx(1 - 4 / (20 + 1e-7), rel=1e-6)
    row[_lib.M_ASR_NUM], row[_lib.M_ASR_DEN] = 0, 0
    assert PatchAttacker._derive(row)["asr"] == 1.0
