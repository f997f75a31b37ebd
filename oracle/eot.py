"""EOT patch pipeline restated for the oracle (torch fp64 values, numpy fp32 geometry).

  Patcher.random_print_adjust    attacker.py:365-372
  Patcher.add_patches_to_image   attacker.py:374-403
  Patcher.add_patch_to_image     attacker.py:405-446
  Patcher.create                 attacker.py:448-488
  BrightnessMatcher.call         brightness_matcher.py:25-73 (TF rgb_to_yuv / yuv_to_rgb kernels)
  tf.image.resize(antialias)     TF ScaleAndTranslate: triangle kernel, half-pixel centres, span
                                 weights normalised, exact adjoint gradient [TF-recall]
  tfa.image.rotate               angles_to_projective_transforms + ImageProjectiveTransformV3
                                 (bilinear, constant fill); gradient = TF's registered rule, an
                                 inverse-transform warp of the upstream gradient with fill 0
                                 [TF-recall]
Random draws come from the product's counter-based Philox streams (oracle/philox.py) so the
oracle and the GPU see identical EOT parameters.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import philox as ph

f32 = np.float32
P = 640


# ------------------------------------------------------------------------------------------
# random parameters
# ------------------------------------------------------------------------------------------
def print_params(seed, step, gimg):
    """w ~ N(0.5, 0.1)[3], b ~ N(0, 0.01)[3] (attacker.py:370-371)"""
    r = ph.draw(seed, 0, 0, gimg, step, ph.RNG_PRINT)
    r2 = ph.draw(seed, 1, 0, gimg, step, ph.RNG_PRINT)
    r3 = ph.draw(seed, 2, 0, gimg, step, ph.RNG_PRINT)
    w = [ph.rnorm(r[0], r[1], 0.5, 0.1), ph.rnorm(r[2], r[3], 0.5, 0.1), ph.rnorm(r2[0], r2[1], 0.5, 0.1)]
    b = [ph.rnorm(r2[2], r2[3], 0.0, 0.01), ph.rnorm(r3[0], r3[1], 0.0, 0.01), ph.rnorm(r3[2], r3[3], 0.0, 0.01)]
    return np.array(w, np.float32).reshape(3), np.array(b, np.float32).reshape(3)


def placement(box, scale, H, W, seed, step, gimg, k, tol=0.2):
    """Patcher.create (attacker.py:448-488) in TF's fp32 op order; returns dict or None.
    tol: the centre tolerance (0.2 the attacker's; 0 the defender Masker's evaluation branch,
    attack_detection.py:454-456, whose create has the same arithmetic)."""
    ymin, xmin, ymax, xmax = (f32(v) for v in box)
    scale = f32(scale)
    h = f32(ymax - ymin)
    w = f32(xmax - xmin)
    longer = max(h, w)
    psf = f32(np.floor(f32(longer * scale)))
    diag = min(f32(f32(1.41421354) * psf), f32(W))
    r = ph.draw(seed, 0, k, gimg, step, ph.RNG_PLACE)
    tol = f32(tol)
    ry = ph.runif(r[0], f32(f32(-tol * h) / f32(2.0)), f32(f32(tol * h) / f32(2.0)))
    rx = ph.runif(r[1], f32(f32(-tol * w) / f32(2.0)), f32(f32(tol * w) / f32(2.0)))
    oy = f32(f32(ymin + f32(h / f32(2.0))) + ry)
    ox = f32(f32(xmin + f32(w / f32(2.0))) + rx)
    yp = max(f32(oy - f32(diag / f32(2.0))), f32(0.0))
    xp = max(f32(ox - f32(diag / f32(2.0))), f32(0.0))
    if f32(yp + diag) > f32(H):
        yp = f32(f32(H) - diag)
    if f32(xp + diag) > f32(W):
        xp = f32(f32(W) - diag)
    q = ph.draw(seed, 1, k, gimg, step, ph.RNG_BOX)
    delta = ph.runif(q[0], -0.3, 0.3)
    amax = f32(20.0 * np.pi / 180.0)
    angle = ph.runif(q[1], -amax, amax)
    valid = bool(f32(psf * psf) > f32(4.0))
    ps_i, diag_i = int(psf), int(diag)
    return dict(valid=valid, ymin=int(yp), xmin=int(xp), ps=ps_i, diag=diag_i,
                pad=int(math.floor((diag_i - ps_i) / 2)), angle=f32(angle), delta=f32(delta))


def noise(seed, step, gimg, k, ps):
    """U(-.01,.01) [ps,ps,3] (attacker.py:426), counter c0 = pixel index."""
    px = np.arange(ps * ps, dtype=np.uint32)
    r = ph.draw(seed, px, k, gimg, step, ph.RNG_NOISE)
    return np.stack([ph.runif(r[0], -0.01, 0.01), ph.runif(r[1], -0.01, 0.01), ph.runif(r[2], -0.01, 0.01)],
                    -1).reshape(ps, ps, 3)


# ------------------------------------------------------------------------------------------
# brightness matcher
# ------------------------------------------------------------------------------------------
RGB2YUV = torch.tensor([[0.299, -0.14714119, 0.61497538],
                        [0.587, -0.28886916, -0.51496512],
                        [0.114, 0.43601035, -0.10001026]], dtype=torch.float64)
YUV2RGB = torch.tensor([[1, 1, 1],
                        [0, -0.394642334, 2.03206185],
                        [1.13988303, -0.58062185, 0]], dtype=torch.float64)


def brightness_match(src, tgt):
    """BrightnessMatcher.call((src, tgt)) — brightness_matcher.py:43-73."""
    k01 = float(f32(127.0 / 255.0))
    kb = float(f32(255.0 / 127.0))
    s = (src + 1.0) * k01
    t = (tgt + 1.0) * k01
    s = s @ RGB2YUV.to(src.dtype)
    t = t @ RGB2YUV.to(tgt.dtype)
    source, target = s[..., 0], t[..., 0]
    pxmap = torch.clamp(source - source.mean() + target.mean(), 0.0, 1.0)
    res = torch.stack([pxmap, s[..., 1], s[..., 2]], -1) @ YUV2RGB.to(src.dtype)
    res = torch.clamp(res, 0.0, 1.0)
    return res * kb - 1.0


# ------------------------------------------------------------------------------------------
# antialiased resize = ScaleAndTranslate(triangle, antialias) as a weight matrix
# ------------------------------------------------------------------------------------------
def resize_matrix(ps, in_size=P):
    """[ps, in_size] weights of tf.image.resize(..., antialias=True) along one axis (fp32)."""
    scale = f32(f32(ps) / f32(in_size))
    inv_scale = f32(1.0 / float(scale))
    kscale = max(inv_scale, f32(1.0))
    one_over_k = f32(f32(1.0) / kscale)
    Wm = np.zeros((ps, in_size), np.float32)
    for i in range(ps):
        sample_f = f32(f32(f32(i) + f32(0.5)) * inv_scale)
        start = int(math.ceil(f32(f32(sample_f - kscale) - f32(0.5))))
        end = int(math.floor(f32(f32(sample_f + kscale) - f32(0.5))))
        start = min(max(start, 0), in_size - 1)
        end = min(max(end, 0), in_size - 1) + 1
        ws = []
        tot = f32(0.0)
        for src in range(start, end):
            pos = f32(f32(f32(src) + f32(0.5)) - sample_f)
            x = abs(f32(pos * one_over_k))
            wv = f32(1.0) - x if x < 1.0 else f32(0.0)
            ws.append(f32(wv))
            tot = f32(tot + f32(wv))
        if abs(tot) >= 1000.0 * np.finfo(np.float32).tiny:
            inv = f32(f32(1.0) / tot)
            for j, src in enumerate(range(start, end)):
                Wm[i, src] = f32(ws[j] * inv)
    return Wm


# ------------------------------------------------------------------------------------------
# rotation (ImageProjectiveTransformV3, bilinear, constant fill) with TF's gradient rule
# ------------------------------------------------------------------------------------------
def rotate_transform(angle, side):
    """tfa.image.angles_to_projective_transforms (fp32)."""
    a = f32(angle)
    s1 = f32(side - 1)
    c, s = f32(np.cos(a)), f32(np.sin(a))
    xo = f32(f32(s1 - f32(f32(c * s1) - f32(s * s1))) / f32(2.0))
    yo = f32(f32(s1 - f32(f32(s * s1) + f32(c * s1))) / f32(2.0))
    return np.array([c, -s, xo, s, c, yo], np.float32)


def inverse_transform(t):
    a, b, tx, d, e, ty = (float(v) for v in t)
    det = a * e - b * d
    return np.array([e / det, -b / det, (b * ty - e * tx) / det, -d / det, a / det, (d * tx - a * ty) / det],
                    np.float32)


def _sample_coords(t, side):
    oy, ox = np.meshgrid(np.arange(side, dtype=np.float32), np.arange(side, dtype=np.float32), indexing="ij")
    inx = f32(t[0]) * ox + f32(t[1]) * oy
    inx = (inx + f32(t[2])).astype(np.float32)
    iny = f32(t[3]) * ox + f32(t[4]) * oy
    iny = (iny + f32(t[5])).astype(np.float32)
    return inx, iny


def projective_bilinear(img, t, fill):
    """img [S,S,C] torch -> [S,S,C]: TF ProjectiveGenerator bilinear (constant fill)."""
    S = img.shape[0]
    inx, iny = _sample_coords(t, S)
    xf, yf = np.floor(inx), np.floor(iny)
    xc, yc = xf + 1, yf + 1
    wx1 = torch.as_tensor((inx - xf).astype(np.float64), dtype=img.dtype)[..., None]
    wx0 = torch.as_tensor((xc - inx).astype(np.float64), dtype=img.dtype)[..., None]
    wy1 = torch.as_tensor((iny - yf).astype(np.float64), dtype=img.dtype)[..., None]
    wy0 = torch.as_tensor((yc - iny).astype(np.float64), dtype=img.dtype)[..., None]

    def read(yy, xx):
        yy = yy.astype(np.int64)
        xx = xx.astype(np.int64)
        ok = (yy >= 0) & (yy < S) & (xx >= 0) & (xx < S)
        v = img[np.clip(yy, 0, S - 1), np.clip(xx, 0, S - 1)]
        okt = torch.as_tensor(ok)[..., None]
        return torch.where(okt, v, torch.full_like(v, fill))

    v_yf = wx0 * read(yf, xf) + wx1 * read(yf, xc)
    v_yc = wx0 * read(yc, xf) + wx1 * read(yc, xc)
    return wy0 * v_yf + wy1 * v_yc


class Rotate(torch.autograd.Function):
    """forward: tfa.image.rotate(bilinear, fill -2); backward: TF's registered gradient."""

    @staticmethod
    def forward(ctx, img, angle):
        S = img.shape[0]
        t = rotate_transform(angle, S)
        ctx.tinv = inverse_transform(t)
        return projective_bilinear(img, t, -2.0)

    @staticmethod
    def backward(ctx, g):
        return projective_bilinear(g, ctx.tinv, 0.0), None


# ------------------------------------------------------------------------------------------
# Patcher
# ------------------------------------------------------------------------------------------
def patch_image(image, patch, boxes, scale, seed, step, gimg, return_places=False):
    """add_patches_to_image (attacker.py:374-403) for one image [H,W,3]; patch [640,640,3]."""
    H, W = image.shape[0], image.shape[1]
    w, b = print_params(seed, step, gimg)
    p = torch.clamp(torch.as_tensor(w.astype(np.float64), dtype=patch.dtype) * patch
                    + torch.as_tensor(b.astype(np.float64), dtype=patch.dtype), -1.0, 1.0)
    p = brightness_match(p, image.detach() if image.requires_grad else image)
    img = image
    places = []
    for k, box in enumerate(boxes):
        pl = placement(box, scale, H, W, seed, step, gimg, k)
        places.append(pl)
        if not pl["valid"]:
            continue
        ps, diag, pad = pl["ps"], pl["diag"], pl["pad"]
        Wm = torch.as_tensor(resize_matrix(ps).astype(np.float64), dtype=patch.dtype)
        im = torch.einsum("iy,yxc,jx->ijc", Wm, p, Wm)
        im = im + torch.as_tensor(noise(seed, step, gimg, k, ps).astype(np.float64), dtype=patch.dtype)
        im = im + float(pl["delta"])
        im = torch.clamp(im, -1.0, 1.0)
        padded = torch.full((diag, diag, 3), -2.0, dtype=patch.dtype)
        padded = padded.index_put((torch.arange(pad, pad + ps)[:, None], torch.arange(pad, pad + ps)[None, :]), im)
        im = Rotate.apply(padded, pl["angle"])
        y0, x0 = pl["ymin"], pl["xmin"]
        bg = img[y0:y0 + diag, x0:x0 + diag]
        im = torch.where(im < -1.0, bg, im)
        im = torch.clamp(im, -1.0, 1.0)
        img = img.clone()
        img[y0:y0 + diag, x0:x0 + diag] = im
    if return_places:
        return img, places
    return img
