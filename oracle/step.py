"""The attack step restated end to end — PatchAttacker.call (attacker.py:172-219) + train_step's
Adam (attacker.py:307-316, Keras Adam lr 1e-2: attacker_train.py:38) — for the oracle.
"""
from __future__ import annotations

import numpy as np
import torch

from . import detector as D
from . import eot
from . import postprocess as pp


def _ragged_max(scores, mask):
    """tf.reduce_max over a ragged row (attacker.py:190): ties split equally; empty -> lowest."""
    s = scores[mask]
    if s.numel() == 0:
        return torch.tensor(-np.finfo(np.float32).max, dtype=scores.dtype)
    return D.TieMax.apply(s)


def nms_thresh(score_thresh):
    """postprocess.nms, method 'gaussian': score_threshold = score_thresh or 0.001 (postprocess.py:186-188)"""
    return score_thresh or 0.001


def first_pass(det, images_t, image_size, score_thresh=0.5):
    """PatchAttacker.first_pass (attacker.py:91-116): boxes per image after soft-NMS + clip."""
    with torch.no_grad():
        cls, box = det(images_t)
        scores, classes, boxes = D.pre_nms(cls, box, image_size, det.cfg["anchor_scale"])
    out = []
    H = W = image_size
    for b in range(images_t.shape[0]):
        sc = scores[b].numpy().astype(np.float32)
        bx = boxes[b].numpy().astype(np.float32)
        keep = (classes[b].numpy() == 0) & pp.valid_mask(bx, H, W, sc, score_thresh)
        ob, os_, n = pp.nms_padded(bx[keep], sc[keep], image_size, 100, nms_thresh(score_thresh))
        out.append((ob[:n], os_[:n]))
    return out


def asr_counts(first, second):
    """calc_asr (attacker.py:238-255) numerator / denominator: soft-NMS boxes with score >= 0.5
    after (second) and before (first) the patch."""
    num = sum(int((s >= np.float32(0.5)).sum()) for _, s in second)
    den = sum(int((s >= np.float32(0.5)).sum()) for _, s in first)
    return num, den


def calc_asr(num, den, coords=4):
    """calc_asr's value (attacker.py:253-255): 1 - tf.size(boxes_pred_filt.flat_values) /
    (tf.size(labels_filt.flat_values) + epsilon), in float32.  The ragged boxes are [B,(n),4], so
    each size counts 4 floats per box: 1 - 4n / (4d + 1e-7) (Keras epsilon 1e-7)."""
    n = np.float32(coords * num)
    d = np.float32(coords * den) + np.float32(1e-7)
    return float(np.float32(1.0) - n / d)


def attack_step(weights, images, patch, scale, boxes=None, seed=0, step=0, gimg0=0,
                model="efficientdet-d0", image_size=None, add_tv=True, score_thresh=0.5,
                dtype=torch.float64, training=True, image_grad=False, bn_frozen=False, bf16=False):
    """Returns dict(loss, grad (NPARAM float64: [patch | scale]), m (per image), patched, ...).

    boxes: None -> first-pass soft-NMS boxes (the reference); else a list per image of [n,4]
    arrays used for placement (the first pass still runs, as in the product).
    training=False: call(training=False) as test_step runs it (attacker.py:318-326): inference BN
    from the moving statistics, no drop connect; no gradient is taken (grad is None)."""
    image_size = image_size or D.MODELS[model]["image_size"]
    det = D.Detector(weights, model, image_size, dtype=dtype, training=training,
                     drop=dict(seed=seed, step=step, gimg0=gimg0, **{"pass": 0}), bn_frozen=bn_frozen)
    det.bf16 = bf16  # emulate the library's bf16 1x1-conv arithmetic
    images_t = torch.as_tensor(np.asarray(images, dtype=np.float64), dtype=dtype)
    B = images_t.shape[0]
    fp = first_pass(det, images_t, image_size, score_thresh)
    det.drop = dict(det.drop, **{"pass": 1})  # the second pass draws its own drop-connect masks
    place_boxes = [fp[b][0] for b in range(B)] if boxes is None else [np.asarray(bx, np.float32) for bx in boxes]
    patch_t = torch.as_tensor(np.asarray(patch, dtype=np.float64), dtype=dtype).requires_grad_(training)
    scale_t = torch.tensor(float(np.float32(scale)), dtype=dtype, requires_grad=training)
    patched, places = [], []
    for b in range(B):
        img, pl = eot.patch_image(images_t[b], patch_t, place_boxes[b], np.float32(scale), seed, step,
                                  gimg0 + b, return_places=True)
        patched.append(img)
        places.append(pl)
    patched = torch.stack(patched)
    cls, box = det(patched)
    scores, classes, dboxes = D.pre_nms(cls, box, image_size, det.cfg["anchor_scale"])
    m_raw, m, second = [], [], []
    for b in range(B):
        keep = torch.as_tensor((classes[b].numpy() == 0)
                               & pp.valid_mask(dboxes[b].numpy().astype(np.float32), image_size, image_size))
        # the ASR metric's soft-NMS of the second pass (attacker.py:203-205): person & valid only
        sb = scores[b].detach().numpy().astype(np.float32)[keep.numpy()]
        bb = dboxes[b].numpy().astype(np.float32)[keep.numpy()]
        ob, os_, n = pp.nms_padded(bb, sb, image_size, 100, nms_thresh(score_thresh))
        second.append((ob[:n], os_[:n]))
        r = _ragged_max(scores[b], keep)
        m_raw.append(r)
        m.append(torch.where(r >= 0, r, torch.zeros_like(r)))  # tf.maximum(x, 0): grad to x on ties
    m = torch.stack(m)
    scale_losses = (m - scale_t) ** 2
    tv = (patch_t[1:, :, :] - patch_t[:-1, :, :]).abs().sum() + (patch_t[:, 1:, :] - patch_t[:, :-1, :]).abs().sum()
    loss = (m ** 2 + scale_losses).sum()
    if add_tv:
        loss = loss + 1e-5 * tv
    grad = dimg = None
    if training:
        if image_grad:  # d loss / d patched images as well (diagnostics)
            gp, gs, gi = torch.autograd.grad(loss, [patch_t, scale_t, patched])
            dimg = gi.detach().numpy()
        else:
            gp, gs = torch.autograd.grad(loss, [patch_t, scale_t])
        grad = np.concatenate([gp.detach().numpy().reshape(-1), [gs.item()]])
    num, den = asr_counts(fp, second)
    return dict(loss=loss.item(), grad=grad, m=m.detach().numpy(), m_raw=np.array([float(v.detach()) for v in m_raw]),
                scale_loss=scale_losses.sum().item(), tv=tv.item(), patched=patched.detach().numpy(),
                places=places, first_pass=fp, second_nms=second, asr_num=num, asr_den=den,
                nbox=sum(int(p["valid"]) for pl in places for p in pl), det=det, dimg=dimg)


def adam_clip(params, grad, m, v, lr, t):
    """Keras Adam via ResourceApplyAdam (b1 .9, b2 .999, eps 1e-7) + clip constraints, float32."""
    params = params.astype(np.float32).copy()
    g = grad.astype(np.float32)
    b1, b2, eps = np.float32(0.9), np.float32(0.999), np.float32(1e-7)
    b1p, b2p = np.float32(b1 ** t), np.float32(b2 ** t)
    alpha = np.float32(lr) * np.sqrt(np.float32(1) - b2p) / (np.float32(1) - b1p)
    m = m + (g - m) * (np.float32(1) - b1)
    v = v + (g * g - v) * (np.float32(1) - b2)
    params = params - (m * alpha) / (np.sqrt(v) + eps)
    npatch = params.size - 1
    params[:npatch] = np.clip(params[:npatch], -1, 1)
    params[npatch:] = np.clip(params[npatch:], 0, 1)
    return params, m, v
