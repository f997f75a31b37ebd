"""CPU restatement of the reference's inference-time patch compositor (adv_patch.py:16-201) —
TEST INFRASTRUCTURE ONLY: tests/ use it as the checker of the HIP compositor (phx_adv_patch); the
product never imports it.

The reference runs numpy + OpenCV 4.5.5 (requirements.txt:11) on uint8 RGB images.  cv2 is not
installed here, so the three OpenCV operations the compositor calls are restated from OpenCV's
published integer / float arithmetic (parity unpinned beyond the hand-checkable cases in
tests/test_adv_patch.py):
  * cv2.resize INTER_LINEAR, 8-bit (AdversarialPatch.rescale, adv_patch.py:99-104): 11-bit
    fixed-point weights, the horizontal pass into int rows, the vertical pass as
    ((b0*(S0>>4))>>16 + (b1*(S1>>4))>>16 + 2) >> 2; an exact 2x downscale runs INTER_AREA instead;
  * cv2.resize INTER_AREA (adv_patch.py:158-160, downscale): an integer factor averages its cell
    (2x2: (sum + 2) >> 2; otherwise cvRound(sum * (1.f / area))), a fractional factor takes OpenCV's
    fractional-cell weights (float) applied row by row in float32 and rounds half to even;
  * cv2.resize INTER_CUBIC (adv_patch.py:161-163, upscale): Keys' kernel with A = -0.75, 11-bit
    fixed-point weights per tap, replicated borders, (sum + 2^21) >> 22 clamped to [0, 255];
  * cv2.cvtColor RGB2YUV / YUV2RGB, 8-bit (adv_patch.py:122-131): 14-bit fixed point, Y = (4899 R +
    9617 G + 1868 B + 2^13) >> 14, U = ((B - Y) 8061 + 128 * 2^14 + 2^13) >> 14, V likewise with R and
    14369; back: R = Y + ((V - 128) 18678 + 2^13) >> 14, G = Y + ((U - 128) (-6472) + (V - 128)
    (-9519) + 2^13) >> 14, B = Y + ((U - 128) 33292 + 2^13) >> 14, saturated.
numpy's uniform noise (adv_patch.py:147) is the one random draw: here U(-0.01, 0.01) in float64 from
Philox4x32-10 keyed by (seed; element / 2, box slot, image, step << 8 | RNG_APNOISE), the draw the
product makes (oracle/philox.py).  The reference's random patch (np.random.rand, adv_patch.py:31) is
likewise a seeded draw here.
"""
import math

import numpy as np

from oracle import philox as ph

PATCH = 640
MEAN_RGB, STDDEV_RGB = 127.0, 128.0
RNG_APNOISE = 10  # common.hpp RngStream

# ---- OpenCV fixed-point constants (imgproc: resize.cpp, color_yuv.simd.hpp) ---------------------
COEF_BITS, COEF_SCALE = 11, 2048
R2Y, G2Y, B2Y, R2VI, B2UI = 4899, 9617, 1868, 14369, 8061
V2RI, V2GI, U2GI, U2BI = 18678, -9519, -6472, 33292
YUV_SHIFT = 14


def _descale(x, n=YUV_SHIFT):
    """CV_DESCALE: (x + 2^(n-1)) >> n (arithmetic shift)"""
    return (x + (1 << (n - 1))) >> n


def _sat_u8(x):
    return np.clip(x, 0, 255).astype(np.uint8)


def rgb2yuv(img):
    """cv2.cvtColor(img, cv2.COLOR_RGB2YUV), uint8 [..., 3] (RGB2YCrCb_i<uchar> with the YUV
    coefficients: Y, then U = Cb-like from B, V = Cr-like from R)"""
    r, g, b = (img[..., i].astype(np.int64) for i in range(3))
    y = _descale(r * R2Y + g * G2Y + b * B2Y)
    delta = 128 << YUV_SHIFT
    v = _descale((r - y) * R2VI + delta)
    u = _descale((b - y) * B2UI + delta)
    return np.stack([_sat_u8(y), _sat_u8(u), _sat_u8(v)], -1)


def yuv2rgb(img):
    """cv2.cvtColor(img, cv2.COLOR_YUV2RGB), uint8 (YUV2RGB_i<uchar>)"""
    y, u, v = (img[..., i].astype(np.int64) for i in range(3))
    b = y + _descale((u - 128) * U2BI)
    g = y + _descale((u - 128) * U2GI + (v - 128) * V2GI)
    r = y + _descale((v - 128) * V2RI)
    return np.stack([_sat_u8(r), _sat_u8(g), _sat_u8(b)], -1)


def y_of_rgb(img):
    """the Y channel of rgb2yuv"""
    r, g, b = (img[..., i].astype(np.int64) for i in range(3))
    return _descale(r * R2Y + g * G2Y + b * B2Y)


# ---- cv2.resize ----------------------------------------------------------------------------------
def _cv_round_short(x):
    """saturate_cast<short>(float): round half to even, saturate"""
    return np.clip(np.rint(np.float32(x)), -32768, 32767).astype(np.int64)


def _linear_tabs(ssize, dsize):
    """per destination index: (source index, weight 0, weight 1) as resize() computes them for
    INTER_LINEAR in fixed point (fx in float32 from a double expression; the horizontal pass clamps
    (sx, fx) at both ends)"""
    scale = 1.0 / (dsize / ssize)
    ofs = np.zeros(dsize, np.int64)
    w = np.zeros((dsize, 2), np.int64)
    for d in range(dsize):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0.0), 0
        if s >= ssize - 1:
            f, s = np.float32(0.0), ssize - 1
        ofs[d] = s
        w[d] = [_cv_round_short((np.float32(1.0) - f) * COEF_SCALE), _cv_round_short(f * COEF_SCALE)]
    return ofs, w


def _linear_vtabs(ssize, dsize):
    """vertical INTER_LINEAR: (sy, beta0, beta1); rows sy, sy + 1 clamped to the image, weights not"""
    scale = 1.0 / (dsize / ssize)
    ofs = np.zeros(dsize, np.int64)
    w = np.zeros((dsize, 2), np.int64)
    for d in range(dsize):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = np.float32(f - np.float32(s))
        ofs[d] = s
        w[d] = [_cv_round_short((np.float32(1.0) - f) * COEF_SCALE), _cv_round_short(f * COEF_SCALE)]
    return ofs, w


def resize_linear_u8(img, dw, dh):
    """cv2.resize(img, (dw, dh)) with the default INTER_LINEAR, uint8 [H,W,C]"""
    H, W, C = img.shape
    if (dh, dw) == (H, W):
        return img.copy()
    if W == 2 * dw and H == 2 * dh:  # resize(): INTER_LINEAR at an exact 2x decimation runs INTER_AREA
        return resize_area_u8(img, dw, dh)
    xo, xw = _linear_tabs(W, dw)
    yo, yw = _linear_vtabs(H, dh)
    src = img.astype(np.int64)
    xo1 = np.minimum(xo + 1, W - 1)
    # horizontal pass: int rows (S[sx] * a0 + S[sx+1] * a1)
    rows = src[:, xo, :] * xw[None, :, 0, None] + src[:, xo1, :] * xw[None, :, 1, None]
    r0 = np.clip(yo, 0, H - 1)
    r1 = np.clip(yo + 1, 0, H - 1)
    s0, s1 = rows[r0], rows[r1]
    b0, b1 = yw[:, 0, None, None], yw[:, 1, None, None]
    out = (((b0 * (s0 >> 4)) >> 16) + ((b1 * (s1 >> 4)) >> 16) + 2) >> 2
    return out.astype(np.uint8)


def _area_tab(ssize, dsize):
    """computeResizeAreaTab (double geometry, float weights): list of (d, s, alpha)"""
    scale = 1.0 / (dsize / ssize)
    tab = []
    for d in range(dsize):
        fs1 = d * scale
        fs2 = fs1 + scale
        cell = min(scale, ssize - fs1)
        s1 = math.ceil(fs1)
        s2 = math.floor(fs2)
        s2 = min(s2, ssize - 1)
        s1 = min(s1, s2)
        if s1 - fs1 > 1e-3:
            tab.append((d, s1 - 1, np.float32((s1 - fs1) / cell)))
        for s in range(s1, s2):
            tab.append((d, s, np.float32(1.0 / cell)))
        if fs2 - s2 > 1e-3:
            tab.append((d, s2, np.float32(min(min(fs2 - s2, 1.0), cell) / cell)))
    return tab


def resize_area_u8(img, dw, dh):
    """cv2.resize(..., interpolation=INTER_AREA) for a downscale, uint8 [H,W,C]"""
    H, W, C = img.shape
    sx, sy = W / dw, H / dh
    ix, iy = int(round(sx)), int(round(sy))
    if abs(sx - ix) < np.finfo(np.float64).eps and abs(sy - iy) < np.finfo(np.float64).eps:
        src = img.astype(np.int64)
        cells = src[:dh * iy, :dw * ix].reshape(dh, iy, dw, ix, C).sum(axis=(1, 3))
        if ix == 2 and iy == 2:
            return ((cells + 2) >> 2).astype(np.uint8)
        scale = np.float32(1.0) / np.float32(ix * iy)
        return _sat_u8(np.rint(cells.astype(np.float32) * scale))
    xtab, ytab = _area_tab(W, dw), _area_tab(H, dh)
    # the x entries of each destination column in order, padded with zero weights (x + 0 == x in
    # float32, so the padding leaves every per-column sum — taken in OpenCV's order — unchanged)
    per = [[] for _ in range(dw)]
    for d, s, a in xtab:
        per[d].append((s, a))
    J = max(len(e) for e in per)
    XS = np.zeros((dw, J), np.int64)
    XA = np.zeros((dw, J), np.float32)
    for d, e in enumerate(per):
        for j, (s, a) in enumerate(e):
            XS[d, j], XA[d, j] = s, a
    src = img.astype(np.float32)
    out = np.zeros((dh, dw, C), np.uint8)
    acc = None
    prev = ytab[0][0]
    for d, s, beta in ytab:
        row = src[s]
        buf = np.zeros((dw, C), np.float32)
        for j in range(J):
            buf = buf + row[XS[:, j]] * XA[:, j, None]  # float32, one rounding per operation
        if acc is None:
            acc = beta * buf
        elif d != prev:
            out[prev] = _sat_u8(np.rint(acc))
            acc = beta * buf
            prev = d
        else:
            acc = acc + beta * buf
    out[prev] = _sat_u8(np.rint(acc))
    return out


def _cubic_coeffs(x):
    """interpolateCubic (A = -0.75), float32 arithmetic"""
    A = np.float32(-0.75)
    x = np.float32(x)
    one = np.float32(1.0)
    c0 = ((A * (x + one) - np.float32(5) * A) * (x + one) + np.float32(8) * A) * (x + one) - np.float32(4) * A
    c1 = ((A + np.float32(2)) * x - (A + np.float32(3))) * x * x + one
    c2 = ((A + np.float32(2)) * (one - x) - (A + np.float32(3))) * (one - x) * (one - x) + one
    c3 = one - c0 - c1 - c2
    return [np.float32(c0), np.float32(c1), np.float32(c2), np.float32(c3)]


def _cubic_tabs(ssize, dsize):
    scale = 1.0 / (dsize / ssize)
    ofs = np.zeros(dsize, np.int64)
    w = np.zeros((dsize, 4), np.int64)
    for d in range(dsize):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = np.float32(f - np.float32(s))
        ofs[d] = s
        w[d] = [_cv_round_short(c * COEF_SCALE) for c in _cubic_coeffs(f)]
    return ofs, w


def resize_cubic_u8(img, dw, dh):
    """cv2.resize(..., interpolation=INTER_CUBIC), uint8 [H,W,C]"""
    H, W, C = img.shape
    xo, xw = _cubic_tabs(W, dw)
    yo, yw = _cubic_tabs(H, dh)
    src = img.astype(np.int64)
    rows = np.zeros((H, dw, C), np.int64)
    for k in range(4):
        xi = np.clip(xo - 1 + k, 0, W - 1)
        rows += src[:, xi, :] * xw[None, :, k, None]
    acc = np.zeros((dh, dw, C), np.int64)
    for k in range(4):
        yi = np.clip(yo - 1 + k, 0, H - 1)
        acc += rows[yi] * yw[:, k, None, None]
    return _sat_u8((acc + (1 << (2 * COEF_BITS - 1))) >> (2 * COEF_BITS))


# ---- the compositor (adv_patch.py) ---------------------------------------------------------------
def print_patch(patch_u8):
    """AdversarialPatch.print_patch (adv_patch.py:40-58): ((p - 127) / 128 * .5) * 128 + 127, clipped,
    truncated — every step exact in float64, = (p + 127) // 2"""
    p = patch_u8.astype(np.float64) - MEAN_RGB
    p /= STDDEV_RGB
    p *= 0.5
    p *= STDDEV_RGB
    p += MEAN_RGB
    return np.clip(p, 0.0, 255.0).astype(np.uint8)


def create(img_shape, bbox, scale):
    """AdversarialPatch._create (adv_patch.py:60-91): (ymin, xmin, patch_h, patch_w).  The reference's
    numpy 1.22 promotion: float32 boxes (the detector's dtype) take h, w in float32 (array-scalar
    subtraction), every product / sum with a Python float is float64 (numpy >= 2 would keep float32
    there, so the float64 steps are written out)."""
    ymin, xmin, ymax, xmax = bbox
    h, w = ymax - ymin, xmax - xmin
    ymin, xmin, h, w = float(ymin), float(xmin), float(h), float(w)
    long_side = max(h, w)
    pw = int(long_side * scale)
    ph = pw
    oy = ymin + h / 2.0
    ox = xmin + w / 2.0
    ymp = max(oy - ph / 2.0, 0.0)
    xmp = max(ox - pw / 2.0, 0.0)
    ih, iw = img_shape[0], img_shape[1]
    if ymp + ph > ih:
        ymp = ih - ph
    if xmp + pw > iw:
        xmp = iw - pw
    return int(ymp), int(xmp), ph, pw


def rescale(image, out_h=PATCH, out_w=PATCH):
    """AdversarialPatch.rescale (adv_patch.py:93-108)"""
    h, w, c = image.shape
    s = min(out_w / w, out_h / h)
    sh, sw = int(h * s), int(w * s)
    out = np.full((out_h, out_w, c), 127, np.uint8)
    out[:sh, :sw] = resize_linear_u8(image, sw, sh)
    return out


def target_y_sum(image, out_h=PATCH, out_w=PATCH):
    """sum of the Y channel of rgb2yuv(rescale(image)) (exact integer)"""
    return int(y_of_rgb(rescale(image, out_h, out_w)).sum())


def brightness_match(printed, image, out_h=PATCH, out_w=PATCH):
    """AdversarialPatch.brightness_match (adv_patch.py:110-131): np.mean of uint8 = exact sum / n in
    float64; Y' = trunc(clip(Y - mean_src + mean_tgt, 0, 255))"""
    tm = target_y_sum(image, out_h, out_w) / float(out_h * out_w)
    src = rgb2yuv(printed)
    sm = int(src[..., 0].astype(np.int64).sum()) / float(src.shape[0] * src.shape[1])
    res = np.clip(src[..., 0].astype(np.float64) - sm + tm, 0.0, 255.0)
    src = src.copy()
    src[..., 0] = res.astype(np.uint8)
    return yuv2rgb(src)


def resize_patch(patch, ph, pw):
    """AdversarialPatch.resize (adv_patch.py:151-164)"""
    h = patch.shape[0]
    if h > ph:
        return resize_area_u8(patch, pw, ph)
    if h < ph:
        return resize_cubic_u8(patch, pw, ph)
    return patch


def noise(seed, step, image, slot, shape):
    """U(-0.01, 0.01) float64 per element: Philox block (image, slot, element pair) — two doubles
    per draw (53-bit mantissas from words (x, y) and (z, w))"""
    n = int(np.prod(shape))
    npair = (n + 1) // 2
    r = ph.draw(seed, np.arange(npair), np.full(npair, slot), np.full(npair, image), step, RNG_APNOISE)
    hi = lambda a, b: ((a.astype(np.uint64) << np.uint64(32)) | b.astype(np.uint64)) >> np.uint64(11)  # noqa: E731
    u = np.empty(2 * npair, np.float64)
    u[0::2] = hi(r[0], r[1]).astype(np.float64) * (1.0 / 9007199254740992.0)
    u[1::2] = hi(r[2], r[3]).astype(np.float64) * (1.0 / 9007199254740992.0)
    return (-0.01 + u[:n] * 0.02).reshape(shape)


def transformed_patch(printed, image, ph, pw, nz):
    """AdversarialPatch.get_transformed_patch (adv_patch.py:166-187)"""
    p = brightness_match(printed, image)
    p = resize_patch(p, ph, pw)
    p = p - MEAN_RGB
    p /= STDDEV_RGB
    p = np.clip(p + nz, -1.0, 1.0)
    p *= STDDEV_RGB
    p += MEAN_RGB
    return np.clip(p, 0.0, 255.0).astype(np.uint8)


def add_adv_to_img(img, bboxes, printed, scale, seed=0, step=0, image_index=0):
    """AdversarialPatch.add_adv_to_img (adv_patch.py:189-201): boxes in order, each brightness match
    against the image as patched so far"""
    img = img.copy()
    for k, bbox in enumerate(bboxes):
        y, x, ph, pw = create(img.shape, bbox, scale)
        nz = noise(seed, step, image_index, k, (ph, pw, 3))
        img[y:y + ph, x:x + pw] = transformed_patch(printed, img, ph, pw, nz)
    return img
