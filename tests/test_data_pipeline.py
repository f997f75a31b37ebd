"""Input pipeline: DataSequence._map_fn letterbox and the train-set
augmentation chain (train_data_generator.py:55-77, 201-204, 222-225).

CPU tests pin the oracle's cv2 INTER_LINEAR restatement on hand-checkable cases (cv2 is absent
here, so beyond these cases the resize semantics are parity unpinned) and the augmentation draws.
GPU tests compare the HIP kernels (through the C ABI) with the oracle on the same inputs:
  letterbox   |d| <= 2e-6 absolute (fp32 normalisation + float32 cv2 weights vs float64 oracle)
  augment     |d| <= 2e-6 absolute (fp64 channel sums vs numpy mean; fused multiply-add)
"""
import os

import numpy as np
import pytest

from oracle import data as OD

MEAN = [0.485 * 255, 0.456 * 255, 0.406 * 255]  # hparams_config.py:224-225
STD = [0.229 * 255, 0.224 * 255, 0.225 * 255]


# ---- oracle pins (CPU) -------------------------------------------------------------------------
def test_resize_identity_is_copy():
    x = np.random.default_rng(0).normal(size=(7, 9, 3))
    np.testing.assert_array_equal(OD.cv2_resize_linear(x, 9, 7), x)


def test_resize_exact_half_is_box_mean():
    # cv2 takes its INTER_AREA path for an exact 2x INTER_LINEAR downscale: a 2x2 box mean
    x = np.random.default_rng(1).normal(size=(8, 6, 3))
    box = 0.25 * (x[0::2, 0::2] + x[1::2, 0::2] + x[0::2, 1::2] + x[1::2, 1::2])
    np.testing.assert_allclose(OD.cv2_resize_linear(x, 3, 4), box, rtol=0, atol=1e-12)


def test_resize_upscale_hand_values():
    # cv2.resize([[0, 1]], (4, 1)) = [[0, .25, .75, 1]] (half-pixel centres, clamped borders)
    x = np.array([[[0.0], [1.0]]])
    np.testing.assert_allclose(OD.cv2_resize_linear(x, 4, 1)[0, :, 0], [0, 0.25, 0.75, 1.0], atol=1e-7)
    # rows: [[0],[1]] -> 4 rows, same weights (rows clamp, weights unchanged)
    y = np.array([[[0.0]], [[1.0]]])
    np.testing.assert_allclose(OD.cv2_resize_linear(y, 1, 4)[:, 0, 0], [0, 0.25, 0.75, 1.0], atol=1e-7)


def test_map_fn_geometry():
    im = np.full((100, 200, 3), 255, np.uint8)
    out = OD.map_fn(im, (512, 512), MEAN, STD)
    assert out.shape == (512, 512, 3) and out.dtype == np.float32
    # scale = min(512/200, 512/100) = 2.56 -> 256 x 512, zero canvas below
    assert np.all(out[256:] == 0) and np.all(out[:256] > 0)
    np.testing.assert_allclose(out[0, 0], (255 - np.array(MEAN)) / np.array(STD), rtol=1e-6)


def test_map_fn_burj_photo():
    """The reference's own test photo (brightness_matcher.py:169-179 inputs) through _map_fn."""
    p = os.path.join(os.path.dirname(__file__), "golden", "burj_khalifa_96.npz")
    if not os.path.exists(p):
        pytest.skip("burj fixture absent")
    d = np.load(p)
    im = d["burj_khalifa_day"]  # 96x96 uint8
    out = OD.map_fn(im, (128, 192), MEAN, STD)  # upscale 4/3 into a non-square canvas
    assert np.isfinite(out).all() and out.shape == (128, 192, 3)
    assert np.all(out[:, 128:] == 0)
    np.testing.assert_allclose(out[0, 0], (im[0, 0] - np.array(MEAN)) / np.array(STD), rtol=1e-6)


def test_augment_draws_and_range():
    m, f, d = OD.aug_draws(123, 7, 0, 256)
    assert 0.35 < m.mean() < 0.65
    assert 0.8 <= f < 1.2 and -0.2 <= d < 0.2
    # per-image draws depend on the global image index only; batch draws on the step only
    m2, f2, d2 = OD.aug_draws(123, 7, 100, 8)
    np.testing.assert_array_equal(m2, m[100:108])
    assert f2 == f and d2 == d
    x = np.random.default_rng(2).uniform(-1, 1, (3, 16, 8, 3)).astype(np.float32)
    y = OD.augment(x, 123, 7)
    assert y.shape == x.shape and y.min() >= -1 and y.max() <= 1


# ---- GPU parity ----------------------------------------------------------------------------
def _victim():
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim
    return EfficientDetVictim("efficientdet-d0", "synthetic", seed=0, image_size=128, max_batch=2, rng_seed=11)


@pytest.mark.gpu
def test_letterbox_matches_oracle():
    import torch
    from mladversarialobjectdetection_amd import data as D
    v = _victim()
    rng = np.random.default_rng(3)
    shapes = [(480, 640), (640, 480), (256, 256), (1024, 1024), (100, 37), (512, 512), (1, 300), (333, 1)]
    ims = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in shapes]
    src, off, dims = D.pack_images(ims, torch.device("cuda", 0))
    for out_size in [(512, 512), (384, 640), (100, 102)]:  # the last: ow % 4 != 0 (per-element kernel)
        got = D.letterbox(v, src, off, dims, out_size, MEAN, STD).cpu().numpy()
        for i, im in enumerate(ims):
            h, w = shapes[i]
            sc = min(out_size[1] / w, out_size[0] / h)
            if int(h * sc) == 0 or int(w * sc) == 0:
                # the reference's cv2.resize raises on an empty destination; the kernel leaves
                # the zero canvas
                assert np.all(got[i] == 0)
                continue
            ref = OD.map_fn(im, out_size, MEAN, STD)
            err = np.abs(got[i] - ref).max()
            assert err <= 2e-6, (shapes[i], out_size, err)


@pytest.mark.gpu
def test_augment_matches_oracle():
    import torch
    from mladversarialobjectdetection_amd import data as D
    v = _victim()
    # W = 52: pixel-quad kernels; W = 50: per-element kernels (W % 4 != 0)
    for W in (50, 52):
        xw = np.random.default_rng(W).uniform(-1, 1, (6, 40, W, 3)).astype(np.float32)
        xwt = torch.as_tensor(xw, device="cuda")
        for step in (0, 1, 5):
            got = D.augment(v, xwt, step).cpu().numpy()
            ref = OD.augment(xw, 11, step)
            assert np.abs(got - ref).max() <= 2e-6, (W, step)
    x = np.random.default_rng(4).uniform(-1, 1, (6, 40, 52, 3)).astype(np.float32)
    xt = torch.as_tensor(x, device="cuda")
    # data-parallel shard: images 2..5 as rank 1 with global offset 2 equal the global batch's
    full = D.augment(v, xt, 9).cpu().numpy()
    part = D.augment(v, xt[2:], 9, global_image_offset=2).cpu().numpy()
    np.testing.assert_array_equal(part, full[2:])
    # in-place call is refused (the mirror reads other pixels of the same image)
    from mladversarialobjectdetection_amd._lib import PhxError
    with pytest.raises(PhxError):
        v.ctx.call("phx_augment", xt.data_ptr(), 6, 40, 52, 0, 0, xt.data_ptr(), None)
