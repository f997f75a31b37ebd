"""The defender step restated for the oracle (test infrastructure only: only tests/, smoke() and
bench.py's cpu_baseline import it).

  PatchAttackDefender.call        attack_detection.py:168-206 (training=True): first pass ->
                                  Masker -> 2 * PatchNeutralizer(images) -> Σ_b mean((t - u)^2)
  odet_model / _postprocessing    attack_detection.py:96-166: frozen victim (its layers are not
                                  trainable, :46-47 -> inference BN), pre_nms, person filter,
                                  gaussian soft-NMS (score_thresh 0.5, defender_train.py:30),
                                  clip, then filter_valid_boxes (:79-94: area > 100, score >= 0.5)
  Masker (training)               attack_detection.py:321-498: patches = shuffled 240x240 crops of
                                  the batch, random left-right / up-down flips, print variation,
                                  brightness match, placement with tolerance 0.5 and scale
                                  U(0.3, 0.5), resize + U(-0.1, 0.1) noise + brightness U(-0.3, 0.3),
                                  clip, pad -2, rotate U(±20°), where, clip, paste; target mask =
                                  original region - pasted region
  UNetBackBone / PatchNeutralizer generator.py:17-101 (n_filters 8, dropout 0.2, batchnorm)
  AttentionBlock                  generator.py:104-151
  Conv2DBlock                     generator.py:154-216
  Conv2DTransposeBlock            generator.py:219-266

Keras semantics restated: Conv2D 'same' (3x3, stride 1: pad 1), Conv2DTranspose 3x3 stride 2
'same' (TF pads the equivalent forward conv (0, 1): out[2i + k] += x[i] w[k], cropped to 2H),
BatchNormalization training mode (batch statistics, eps 1e-3, moving statistics momentum 0.99 with
the Bessel-corrected variance), leaky_relu alpha 0.2 [TF-recall: Keras 2.8 resolves the string
Activation('leaky_relu') of generator.py:120,173,179 to tf.nn.leaky_relu, whose default alpha is
0.2; no reference file pins the value], MaxPooling2D 2x2 valid, Dropout 0.2
(x * 1.25 * [u >= 0.2]).  Random draws are the product's Philox streams (oracle/philox.py).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import detector as D
from . import eot
from . import philox as ph
from . import postprocess as pp

f32 = np.float32
RNG_DSHUF, RNG_DFLIP, RNG_DROPOUT = 7, 8, 9
CROP = 240          # Masker patches: images[:, :240, :240] (attack_detection.py:487)
NF = 8              # n_filters (generator.py:20)
DROP = 0.2          # dropout (generator.py:20)


# ------------------------------------------------------------------------------------------
# parameters: the product's manifest order (phx_def_manifest)
# ------------------------------------------------------------------------------------------
def unet_layout(nf=NF):
    """[(name, shape)] of the trainable variables and [(bn name, channels)] of the BN layers."""
    params, bns = [], []

    def conv(name, k, ci, co):
        params.append((f"{name}/kernel", (k, k, ci, co)))
        params.append((f"{name}/bias", (co,)))

    def bn(name, c):
        params.append((f"{name}/gamma", (c,)))
        params.append((f"{name}/beta", (c,)))
        bns.append((name, c))

    def block(name, ci, n):
        conv(f"{name}/cnv1", 3, ci, n)
        bn(f"{name}/bn1", n)
        conv(f"{name}/cnv2", 3, n, n)
        bn(f"{name}/bn2", n)

    ci = 3
    for i in range(4):
        block(f"conv{i}", ci, nf * 2 ** i)
        ci = nf * 2 ** i
    block("conv4", ci, nf * 16)
    ci = nf * 16
    m = 8
    for i in range(4):
        n = nf * m
        params.append((f"deconv{i}/cnv/kernel", (3, 3, n, ci)))  # Conv2DTranspose: [k, k, out, in]
        params.append((f"deconv{i}/cnv/bias", (n,)))
        conv(f"deconv{i}/attention/cnv1", 1, n, n)
        bn(f"deconv{i}/attention/bn1", n)
        conv(f"deconv{i}/attention/cnv2", 1, n, n)
        bn(f"deconv{i}/attention/bn2", n)
        conv(f"deconv{i}/attention/conv3", 1, n, 1)
        bn(f"deconv{i}/attention/bn3", 1)
        block(f"deconv{i}/convblock", 2 * n, n)
        ci = n
        m //= 2
    conv("output", 1, nf, 3)
    return params, bns


def unpack(flat, layout):
    out, off = {}, 0
    for name, shape in layout:
        n = int(np.prod(shape))
        out[name] = flat[off:off + n].reshape(shape)
        off += n
    return out


# ------------------------------------------------------------------------------------------
# U-Net (torch, NCHW internally)
# ------------------------------------------------------------------------------------------
def dropout_mask(shape_nhwc, layer, seed, step, gimg0):
    """Keras Dropout(0.2) keep mask for one layer: element e of image b keeps when
    u01(philox(seed; e, layer, gimg0 + b, step << 8 | RNG_DROPOUT).x) >= 0.2."""
    B, H, W, C = shape_nhwc
    e = np.arange(H * W * C, dtype=np.uint32)
    keep = np.empty((B, H * W * C), bool)
    for b in range(B):
        r = ph.draw(seed, e, layer, gimg0 + b, step, RNG_DROPOUT)
        keep[b] = ph.u01(r[0]) >= f32(DROP)
    return keep.reshape(B, H, W, C)


class UNet:
    def __init__(self, params: dict, moving: dict, dtype=torch.float64, training=True, seed=0, step=0, gimg0=0):
        self.p = {k: torch.as_tensor(np.asarray(v, np.float64), dtype=dtype) for k, v in params.items()}
        for v in self.p.values():
            v.requires_grad_(True)
        self.moving = {k: (np.asarray(m, np.float64).copy(), np.asarray(v, np.float64).copy())
                       for k, (m, v) in moving.items()}
        self.dtype, self.training = dtype, training
        self.seed, self.step, self.gimg0 = seed, step, gimg0

    def conv(self, x, name, k):
        w = self.p[f"{name}/kernel"].permute(3, 2, 0, 1)  # [k,k,ci,co] -> [co,ci,k,k]
        return F.conv2d(x, w, self.p[f"{name}/bias"], padding=k // 2)

    def tconv(self, x, name):
        w = self.p[f"{name}/kernel"].permute(3, 2, 0, 1)  # [k,k,co,ci] -> [ci,co,k,k]
        H, W = x.shape[2], x.shape[3]
        y = F.conv_transpose2d(x, w, self.p[f"{name}/bias"], stride=2)
        return y[:, :, :2 * H, :2 * W]

    def bn(self, x, name):
        g, b = self.p[f"{name}/gamma"], self.p[f"{name}/beta"]
        if self.training:
            mean = x.mean(dim=(0, 2, 3))
            var = ((x - mean[None, :, None, None]) ** 2).mean(dim=(0, 2, 3))
            n = x.shape[0] * x.shape[2] * x.shape[3]
            mm, mv = self.moving[name]
            uvar = var.detach().numpy() * n / max(n - 1, 1)
            self.moving[name] = (mm - (mm - mean.detach().numpy()) * 0.01, mv - (mv - uvar) * 0.01)
        else:
            mean = torch.as_tensor(self.moving[name][0], dtype=x.dtype)
            var = torch.as_tensor(self.moving[name][1], dtype=x.dtype)
        inv = 1.0 / torch.sqrt(var + 1e-3)
        return (x - mean[None, :, None, None]) * (inv * g)[None, :, None, None] + b[None, :, None, None]

    @staticmethod
    def leaky(x):
        return F.leaky_relu(x, 0.2)

    def dropout(self, x, layer):
        if not self.training:
            return x
        keep = dropout_mask((x.shape[0], x.shape[2], x.shape[3], x.shape[1]), layer, self.seed, self.step,
                            self.gimg0)
        keep_t = torch.as_tensor(keep.transpose(0, 3, 1, 2), dtype=x.dtype)
        return x * 1.25 * keep_t

    def block(self, x, name):
        x = self.leaky(self.bn(self.conv(x, f"{name}/cnv1", 3), f"{name}/bn1"))
        return self.leaky(self.bn(self.conv(x, f"{name}/cnv2", 3), f"{name}/bn2"))

    def attention(self, up, skip, name):
        g = self.bn(self.conv(up, f"{name}/cnv1", 1), f"{name}/bn1")
        x = self.bn(self.conv(skip, f"{name}/cnv2", 1), f"{name}/bn2")
        s = self.leaky(g + x)
        a = torch.sigmoid(self.bn(self.conv(s, f"{name}/conv3", 1), f"{name}/bn3"))
        return skip * a

    def __call__(self, images_nhwc):
        x = images_nhwc.permute(0, 3, 1, 2)
        encs = []
        for i in range(4):
            x = self.block(x, f"conv{i}")
            encs.append(x)
            x = self.dropout(F.max_pool2d(x, 2), i)
        x = self.block(x, "conv4")
        for i, enc in enumerate(encs[::-1]):
            up = self.tconv(x, f"deconv{i}/cnv")
            skip = self.attention(up, enc, f"deconv{i}/attention")
            x = self.dropout(torch.cat([up, skip], 1), 4 + i)
            x = self.block(x, f"deconv{i}/convblock")
        out = torch.tanh(self.conv(x, "output", 1))
        return out.permute(0, 2, 3, 1)


# ------------------------------------------------------------------------------------------
# Masker (training mode)
# ------------------------------------------------------------------------------------------
def shuffle_perm(B, seed, step, gimg0):
    """tf.random.shuffle over the batch: sort by one Philox key per image (ties by index)."""
    keys = np.array([ph.draw(seed, 0, 0, gimg0 + b, step, RNG_DSHUF)[0] for b in range(B)], np.uint64)
    return np.argsort(keys, kind="stable")


def flips(seed, step, gimg):
    """random_flip_left_right / up_down of batch entry gimg: flip when u01 >= 0.5."""
    r = ph.draw(seed, 0, 0, gimg, step, RNG_DFLIP)
    return bool(ph.u01(r[0]) >= f32(0.5)), bool(ph.u01(r[1]) >= f32(0.5))


def train_patches(images, seed, step, gimg0):
    B = images.shape[0]
    perm = shuffle_perm(B, seed, step, gimg0)
    out = []
    for b in range(B):
        p = images[perm[b], :CROP, :CROP, :]
        lr, ud = flips(seed, step, gimg0 + b)
        if lr:
            p = p[:, ::-1]
        if ud:
            p = p[::-1]
        out.append(np.ascontiguousarray(p))
    return np.stack(out).astype(np.float32)


def placement(box, H, W, seed, step, gimg, k):
    """Masker.create (attack_detection.py:450-483), training: tolerance 0.5, scale U(0.3, 0.5)."""
    ymin, xmin, ymax, xmax = (f32(v) for v in box)
    h = f32(ymax - ymin)
    w = f32(xmax - xmin)
    longer = max(h, w)
    r = ph.draw(seed, 0, k, gimg, step, ph.RNG_PLACE)
    scale = ph.runif(r[2], 0.3, 0.5)
    psf = f32(np.floor(f32(longer * scale)))
    diag = min(f32(f32(1.41421354) * psf), f32(W))
    tol = f32(0.5)
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
                pad=int(np.floor((diag_i - ps_i) / 2)), angle=f32(angle), delta=f32(delta))


def noise(seed, step, gimg, k, ps, amp=0.1):
    px = np.arange(ps * ps, dtype=np.uint32)
    r = ph.draw(seed, px, k, gimg, step, ph.RNG_NOISE)
    return np.stack([ph.runif(r[0], -amp, amp), ph.runif(r[1], -amp, amp), ph.runif(r[2], -amp, amp)],
                    -1).reshape(ps, ps, 3)


def mask_image(image, patch, boxes, seed, step, gimg, eval_scale=None):
    """Masker.add_patches_to_image (attack_detection.py:362-396) for one image: returns (patched
    image, target mask), torch fp64 [H,W,3].  Training: `patch` is the image's 240^2 crop and the
    placement draws tolerance 0.5 / scale U(0.3, 0.5); evaluation (eval_scale given): `patch` is the
    attacker's 640^2 patch placed centred (tolerance 0) at eval_scale (:454-456)."""
    H, W = image.shape[0], image.shape[1]
    w, b = eot.print_params(seed, step, gimg)
    p = torch.clamp(torch.as_tensor(w.astype(np.float64)) * patch + torch.as_tensor(b.astype(np.float64)),
                    -1.0, 1.0)
    p = eot.brightness_match(p, image)
    img = image.clone()
    mask = torch.zeros_like(image)
    for k, box in enumerate(boxes):
        if eval_scale is None:
            pl = placement(box, H, W, seed, step, gimg, k)
        else:
            pl = eot.placement(box, eval_scale, H, W, seed, step, gimg, k, tol=0.0)
        if not pl["valid"]:
            continue
        ps, diag, pad = pl["ps"], pl["diag"], pl["pad"]
        Wy = torch.as_tensor(eot.resize_matrix(ps, p.shape[0]).astype(np.float64))
        Wx = torch.as_tensor(eot.resize_matrix(ps, p.shape[1]).astype(np.float64))
        im = torch.einsum("iy,yxc,jx->ijc", Wy, p, Wx)
        im = im + torch.as_tensor(noise(seed, step, gimg, k, ps).astype(np.float64))
        im = im + float(pl["delta"])
        im = torch.clamp(im, -1.0, 1.0)
        padded = torch.full((diag, diag, 3), -2.0, dtype=im.dtype)
        padded[pad:pad + ps, pad:pad + ps] = im
        t = eot.rotate_transform(pl["angle"], diag)
        im = eot.projective_bilinear(padded, t, -2.0)
        y0, x0 = pl["ymin"], pl["xmin"]
        bg = img[y0:y0 + diag, x0:x0 + diag]
        im = torch.where(im < -1.0, bg, im)
        im = torch.clamp(im, -1.0, 1.0)
        img[y0:y0 + diag, x0:x0 + diag] = im
        mask[y0:y0 + diag, x0:x0 + diag] = image[y0:y0 + diag, x0:x0 + diag] - im
    return img, mask


def masker(images, boxes, seed, step, gimg0):
    """Masker.call(training=True) over a batch: (patched images, targets), numpy float64."""
    pt = train_patches(np.asarray(images, np.float32), seed, step, gimg0)
    outs, masks = [], []
    for b in range(images.shape[0]):
        img = torch.as_tensor(np.asarray(images[b], np.float64))
        o, m = mask_image(img, torch.as_tensor(pt[b].astype(np.float64)), boxes[b], seed, step, gimg0 + b)
        outs.append(o.numpy())
        masks.append(m.numpy())
    return np.stack(outs), np.stack(masks)


def masker_eval(images, boxes, patch, scale, seed, step, gimg0):
    """Masker.call(training=False) over a batch with the attacker's patch: (patched, targets)."""
    outs, masks = [], []
    pt = torch.as_tensor(np.asarray(patch, np.float64))
    for b in range(images.shape[0]):
        img = torch.as_tensor(np.asarray(images[b], np.float64))
        o, m = mask_image(img, pt, boxes[b], seed, step, gimg0 + b, eval_scale=np.float32(scale))
        outs.append(o.numpy())
        masks.append(m.numpy())
    return np.stack(outs), np.stack(masks)


# ------------------------------------------------------------------------------------------
# first pass and the step
# ------------------------------------------------------------------------------------------
def first_pass(det, images_t, image_size, score_thresh=0.5, filter_thresh=None):
    """odet_model (attack_detection.py:96-127): person anchors -> soft-NMS -> clip -> valid.
    score_thresh sets the soft-NMS threshold (`or 0.001`); filter_valid_boxes reads the config's
    threshold, filter_thresh (default: score_thresh)."""
    filter_thresh = score_thresh if filter_thresh is None else filter_thresh
    with torch.no_grad():
        cls, box = det(images_t)
        scores, classes, boxes = D.pre_nms(cls, box, image_size, det.cfg["anchor_scale"])
    out = []
    for b in range(images_t.shape[0]):
        sc = scores[b].numpy().astype(np.float32)
        bx = boxes[b].numpy().astype(np.float32)
        keep = classes[b].numpy() == 0
        ob, os_, n = pp.nms_padded(bx[keep], sc[keep], image_size, 100, score_thresh or 0.001)
        ob, os_ = ob[:n], os_[:n]
        h = ob[:, 2] - ob[:, 0]
        w = ob[:, 3] - ob[:, 1]
        ok = ((w / f32(image_size) <= 1) & (h / f32(image_size) <= 1) & (f32(h * w) > f32(100.0))
              & (os_ >= f32(filter_thresh)))
        out.append((ob[ok], os_[ok]))
    return out


def defender_step(unet_params, moving, images, boxes=None, victim_weights=None, model="efficientdet-d0",
                  image_size=None, seed=0, step=0, gimg0=0, score_thresh=0.5, masked=None, dtype=torch.float64):
    """PatchAttackDefender.call(images, training=True): dict(loss, grad (flat, manifest order),
    patched, targets, updates, moving (updated), first_pass).  masked = (patched, targets) skips the
    Masker (the U-Net parity test feeds the product's own Masker outputs).  dtype: the detector's and
    U-Net's arithmetic (fp64 for parity; fp32 is the CPU baseline the defender bench times)."""
    layout, bns = unet_layout()
    images = np.asarray(images, np.float32)
    fp = None
    if boxes is None and masked is None:
        image_size = image_size or images.shape[1]
        det = D.Detector(victim_weights, model, image_size, dtype=dtype, training=False)
        fp = first_pass(det, torch.as_tensor(images.astype(np.float64), dtype=dtype), image_size, score_thresh)
        boxes = [b for b, _ in fp]
    if masked is not None:
        patched, targets = (np.asarray(a, np.float64) for a in masked)
    else:
        patched, targets = masker(images, boxes, seed, step, gimg0)
    net = UNet(unpack(unet_params, layout), moving, dtype=dtype, seed=seed, step=step, gimg0=gimg0)
    upd = 2.0 * net(torch.as_tensor(patched, dtype=dtype))
    t = torch.as_tensor(targets, dtype=dtype)
    B = images.shape[0]
    loss = ((t.reshape(B, -1) - upd.reshape(B, -1)) ** 2).mean(dim=1).sum()
    grads = torch.autograd.grad(loss, [net.p[n] for n, _ in layout])
    grad = np.concatenate([g.detach().numpy().reshape(-1) for g in grads])
    return dict(loss=loss.item(), grad=grad, patched=patched, targets=targets, updates=upd.detach().numpy(),
                moving=net.moving, first_pass=fp, boxes=boxes)


def adam(params, grad, m, v, lr, t):
    """Keras Adam (ResourceApplyAdam, b1 .9, b2 .999, eps 1e-7), float32, no constraints."""
    p = params.astype(np.float32).copy()
    g = grad.astype(np.float32)
    b1, b2, eps = np.float32(0.9), np.float32(0.999), np.float32(1e-7)
    alpha = np.float32(lr) * np.sqrt(np.float32(1) - np.float32(b2 ** t)) / (np.float32(1) - np.float32(b1 ** t))
    m = m + (g - m) * (np.float32(1) - b1)
    v = v + (g * g - v) * (np.float32(1) - b2)
    return p - (m * alpha) / (np.sqrt(v) + eps), m, v


def defender_eval(unet_params, moving, images, eval_patch, eval_scale, victim_weights, boxes=None,
                  model="efficientdet-d0", image_size=None, seed=0, step=0, gimg0=0, score_thresh=0.5,
                  masked=None):
    """PatchAttackDefender.call(images, training=False) (attack_detection.py:168-198) as test_step
    runs it: first pass (unless `boxes`), the Masker's evaluation branch with the attacker's patch,
    the second detector pass odet_model(images, score_thresh=0.) (soft-NMS at 0.001, valid filter at
    the config's score_thresh), updates = 2 * U-Net(images, training=False) and the loss.  Returns
    dict(loss, patched, targets, updates, second=[(boxes, scores)] per image, boxes).  masked =
    (patched, targets) skips the first pass and the Masker (the U-Net check feeds the product's own);
    victim_weights None skips the second pass (second = None)."""
    layout, _ = unet_layout()
    images = np.asarray(images, np.float32)
    image_size = image_size or images.shape[1]
    det = D.Detector(victim_weights, model, image_size, training=False)
    if masked is not None:
        patched, targets = (np.asarray(a, np.float64) for a in masked)
    else:
        if boxes is None:
            boxes = [b for b, _ in first_pass(det, torch.as_tensor(images.astype(np.float64)), image_size,
                                               score_thresh)]
        patched, targets = masker_eval(images, boxes, eval_patch, eval_scale, seed, step, gimg0)
    second = None if victim_weights is None else first_pass(det, torch.as_tensor(patched), image_size, 0.0,
                                                             filter_thresh=score_thresh)
    net = UNet(unpack(unet_params, layout), moving, training=False, seed=seed, step=step, gimg0=gimg0)
    with torch.no_grad():
        upd = 2.0 * net(torch.as_tensor(patched))
    t = torch.as_tensor(targets)
    B = images.shape[0]
    loss = ((t.reshape(B, -1) - upd.reshape(B, -1)) ** 2).mean(dim=1).sum()
    return dict(loss=loss.item(), patched=patched, targets=targets, updates=upd.numpy(), second=second,
                boxes=boxes)
