"""CPU oracle of the training input pipeline (TEST INFRASTRUCTURE ONLY — imported by tests/ and
never by the product path).

Restates, in numpy:
  * DataSequence._map_fn (train_data_generator.py:55-77): normalise in float64, scale =
    min(S_h/h, S_w/w), cv2.resize(image, [int(w*scale), int(h*scale)]) with the default
    INTER_LINEAR, pasted top-left into a zero [S_h, S_w, 3] canvas, yielded as float32 (:111);
  * the train-set map chain of partition() (train_data_generator.py:201-204, 222-225):
    tf.image.random_flip_left_right -> tf.keras.layers.RandomFlip('horizontal') ->
    tf.keras.layers.RandomContrast(.2) -> tf.image.random_brightness(.2) -> clip [-1, 1].

cv2 and TensorFlow are third-party and absent here (opencv-python is unpinned in the reference's
requirements.txt; tensorflow==2.8.1 requirements.txt:4), so their arithmetic is restated from
their published behaviour [recall, parity unpinned beyond the hand-checkable cases in
tests/test_data_pipeline.py]:
  cv2.resize INTER_LINEAR, CV_64F source: inv_scale = dsize/ssize, scale = 1/inv_scale;
    fx = float32((dx + .5) * scale - .5), sx = floor(fx), fx -= sx; if sx < 0: sx, fx = 0, 0;
    if sx >= w - 1: sx, fx = w - 1, 0; horizontal weights (1 - fx, fx) in float32 on taps
    (sx, min(sx+1, w-1)); vertical: fy likewise but rows clamp(sy), clamp(sy+1) to [0, h-1]
    with unchanged weights; sums in float64.  (An exact 2x downscale takes cv2's INTER_AREA
    path, a 2x2 box mean — the same value as these weights up to rounding.)
  tf.image.adjust_contrast: per image, per channel mean over (H, W) (fp32 reduce_mean);
    (x - mean) * factor + mean.  RandomContrast(.2) in TF 2.8 draws ONE factor U(0.8, 1.2) per
    call (tf.image.random_contrast) and does not clip.  random_brightness draws ONE delta
    U(-.2, .2) per call.  random_flip_left_right / RandomFlip flip image b when U[b] < 0.5.
Random draws are the product's Philox streams (oracle/philox.py, stream RNG_AUG): per image
(c0=0, c2=global image) words x, y for the two flips; per batch (c0=1, c2=0xFFFFFFFF) words x, y for
the contrast factor and brightness delta.
"""
from __future__ import annotations

import numpy as np

from . import philox as PX


def cv2_resize_linear(img: np.ndarray, dw: int, dh: int) -> np.ndarray:
    """cv2.resize(img, (dw, dh)) INTER_LINEAR for a float64 HWC image (see module docstring)."""
    h, w = img.shape[:2]
    scx = 1.0 / (dw / w)
    scy = 1.0 / (dh / h)
    dx = np.arange(dw, dtype=np.float64)
    fx = ((dx + 0.5) * scx - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    lo = sx < 0
    sx[lo], fx[lo] = 0, 0.0
    hi = sx >= w - 1
    sx[hi], fx[hi] = w - 1, 0.0
    sx1 = np.minimum(sx + 1, w - 1)
    ax0 = (np.float32(1.0) - fx).astype(np.float64)[None, :, None]
    ax1 = fx.astype(np.float64)[None, :, None]
    rows = img[:, sx] * ax0 + img[:, sx1] * ax1  # [h, dw, c]
    dy = np.arange(dh, dtype=np.float64)
    fy = ((dy + 0.5) * scy - 0.5).astype(np.float32)
    sy = np.floor(fy).astype(np.int64)
    fy = (fy - sy.astype(np.float32)).astype(np.float32)
    y0 = np.clip(sy, 0, h - 1)
    y1 = np.clip(sy + 1, 0, h - 1)
    by0 = (np.float32(1.0) - fy).astype(np.float64)[:, None, None]
    by1 = fy.astype(np.float64)[:, None, None]
    return rows[y0] * by0 + rows[y1] * by1


def map_fn(image_u8: np.ndarray, output_size, mean_rgb, stddev_rgb) -> np.ndarray:
    """DataSequence._map_fn (train_data_generator.py:55-77) + the float32 cast of __call__ (:111)."""
    h, w, c = image_u8.shape
    image = image_u8.astype(float)
    image -= np.asarray(mean_rgb, dtype=np.float64)
    image /= np.asarray(stddev_rgb, dtype=np.float64)
    image_scale = min(output_size[1] / w, output_size[0] / h)
    sh, sw = int(h * image_scale), int(w * image_scale)
    scaled = cv2_resize_linear(image, sw, sh)
    out = np.zeros((*output_size, c))
    out[:sh, :sw, :] = scaled
    return out.astype(np.float32)


def aug_draws(seed: int, step: int, gimg0: int, B: int):
    """(mirror[B] bool, contrast factor, brightness delta) of one call."""
    idx = np.arange(gimg0, gimg0 + B, dtype=np.uint32)
    x, y, _, _ = PX.draw(seed, 0, 0, idx, step, PX.RNG_AUG)
    mirror = (PX.u01(x) < np.float32(0.5)) != (PX.u01(y) < np.float32(0.5))
    bx, by, _, _ = PX.draw(seed, 1, 0, 0xFFFFFFFF, step, PX.RNG_AUG)
    f = PX.runif(bx, 0.8, 1.2)
    delta = PX.runif(by, -0.2, 0.2)
    return mirror, np.float32(f), np.float32(delta)


def augment(images: np.ndarray, seed: int, step: int, gimg0: int = 0) -> np.ndarray:
    """train_data_generator.py:222-225 map chain on a float32 batch [B,H,W,3]."""
    B = images.shape[0]
    mirror, f, delta = aug_draws(seed, step, gimg0, B)
    x = np.where(mirror[:, None, None, None], images[:, :, ::-1, :], images).astype(np.float32)
    mean = x.astype(np.float64).mean(axis=(1, 2), keepdims=True).astype(np.float32)
    t = ((x - mean) * f + mean).astype(np.float32)
    t = (t + delta).astype(np.float32)
    return np.clip(t, -1.0, 1.0).astype(np.float32)
