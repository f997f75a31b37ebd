"""CPU checks of the inference compositor's oracle (oracle/adv_patch.py, the restatement of
adv_patch.py + the OpenCV operations it calls; cv2 is absent, so these hand-checkable cases are what
pins it — parity unpinned beyond them) and of the Python mirror's host side."""
import numpy as np
import pytest

from oracle import adv_patch as A


def test_yuv_round_trip_of_greys_and_extremes():
    g = np.stack([np.arange(256, dtype=np.uint8)] * 3, -1)[None]
    yuv = A.rgb2yuv(g)
    assert (yuv[..., 0] == np.arange(256)).all() and (yuv[..., 1:] == 128).all()  # greys: Y = level, U = V = 128
    assert (A.yuv2rgb(yuv) == g).all()
    # coefficients sum to 2^14: white and black are exact
    assert A.rgb2yuv(np.array([[[255, 255, 255]]], np.uint8)).tolist() == [[[255, 128, 128]]]
    # pure red: Y = (255 * 4899 + 2^13) >> 14 = 76, V saturates, U = ((0 - 76) * 8061 + 128 * 2^14 + 2^13) >> 14
    assert A.rgb2yuv(np.array([[[255, 0, 0]]], np.uint8)).tolist() == [[[76, 91, 255]]]


def test_resizes_of_constant_images_are_constant():
    c = np.full((640, 640, 3), 77, np.uint8)
    for dw in (97, 160, 320, 333):
        assert (A.resize_area_u8(c, dw, dw) == 77).all(), dw
    for dw in (641, 700, 1023):
        assert (A.resize_cubic_u8(c, dw, dw) == 77).all(), dw
    for dw, dh in ((300, 200), (1280, 960)):
        assert (A.resize_linear_u8(c, dw, dh) == 77).all()


def test_resize_hand_cases():
    rng = np.random.default_rng(0)
    im = rng.integers(0, 256, (8, 8, 3), dtype=np.uint8)
    # identity, exact 2x decimation (INTER_LINEAR -> INTER_AREA: (sum + 2) >> 2)
    assert (A.resize_linear_u8(im, 8, 8) == im).all()
    cells = im.astype(np.int64).reshape(4, 2, 4, 2, 3).sum(axis=(1, 3))
    assert (A.resize_linear_u8(im, 4, 4) == ((cells + 2) >> 2)).all()
    assert (A.resize_area_u8(im, 4, 4) == ((cells + 2) >> 2)).all()
    # 4x integer area: cvRound(sum * (1/16)) — half to even
    big = np.zeros((4, 4, 3), np.uint8)
    big[0, 0] = 8  # sum 8 -> 0.5 -> 0
    big[0, 1, 1] = 24  # sum 24 -> 1.5 -> 2
    r = A.resize_area_u8(big, 1, 1)
    assert r[0, 0].tolist() == [0, 2, 0]
    # exact 2x upscale with INTER_LINEAR: every destination pixel between two sources takes (3, 1) / 4
    row = np.zeros((1, 2, 3), np.uint8)
    row[0, 1] = 100
    up = A.resize_linear_u8(np.repeat(row, 2, 0), 4, 2)
    assert up[0, :, 0].tolist() == [0, 25, 75, 100]


def test_print_patch_and_placement():
    p = np.arange(256, dtype=np.uint8).reshape(16, 16, 1).repeat(3, -1)
    assert (A.print_patch(p) == (p.astype(np.int64) + 127) // 2).all()
    # _create: centred, clamped at the far edges (adv_patch.py:60-91)
    assert A.create((480, 640, 3), (100, 100, 300, 200), 0.4) == (160, 110, 80, 80)
    assert A.create((480, 640, 3), (0, 600, 470, 640), 0.5) == (117, 405, 235, 235)
    assert A.create((480, 640, 3), (10, 10, 30, 20), 0.4) == (16, 11, 8, 8)


def test_noise_is_bounded_and_keyed():
    a = A.noise(3, 1, 0, 0, (40, 40, 3))
    b = A.noise(3, 1, 0, 1, (40, 40, 3))
    assert a.dtype == np.float64 and np.abs(a).max() < 0.01 and not np.array_equal(a, b)
    assert np.array_equal(a, A.noise(3, 1, 0, 0, (40, 40, 3)))


def test_compositor_pastes_only_inside_boxes():
    rng = np.random.default_rng(1)
    im = rng.integers(0, 256, (240, 320, 3), dtype=np.uint8)
    patch = rng.integers(0, 256, (640, 640, 3), dtype=np.uint8)
    out = A.add_adv_to_img(im, [[20, 30, 120, 90]], A.print_patch(patch), 0.5, seed=0, step=0)
    y, x, ph, pw = A.create(im.shape, (20, 30, 120, 90), 0.5)
    mask = np.zeros(im.shape[:2], bool)
    mask[y:y + ph, x:x + pw] = True
    assert (out[~mask] == im[~mask]).all()
    assert (out[mask] != im[mask]).mean() > 0.9
