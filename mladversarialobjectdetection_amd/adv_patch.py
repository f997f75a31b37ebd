"""Inference-time patch compositor — mirror of the reference's adv_patch.py.

Reference: `AdversarialPatch` (adv_patch.py:16-201) pastes a printed, brightness-matched, resized and
noised copy of the adversarial patch onto every person box of an image with numpy + OpenCV on the
CPU (the demos call `add_adv_to_img(frame, boxes)`, demo.py:116, 177).  Here the same class drives
one HIP call, `phx_adv_patch` (csrc/kernels_advpatch.hip), over a whole batch of uint8 images on the
device; the arithmetic follows OpenCV's own fixed-point / float32 steps and numpy's float64 ones
(restated in oracle/adv_patch.py, the tests' checker).  No CPU fallback: the library must be present.

Random draws: the reference's random patch (np.random.rand, :31) and the per-pixel noise
(np.random.uniform, :147) are Philox draws keyed by the context seed here, so a run is reproducible
and independent of the batch split.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

PATCH_SIZE = 640


def _stream():
    return torch.cuda.current_stream().cuda_stream


class AdversarialPatch:
    """adv_patch.AdversarialPatch: same constructor arguments (scale, h, w, patch_file) and the
    methods a caller uses — print_patch, add_adv_to_img — plus add_adv_to_images for a device batch.
    `seed` keys the random patch (when patch_file is None) and the noise; `ctx` lets several objects
    share one library context."""

    def __init__(self, *, scale, h=PATCH_SIZE, w=PATCH_SIZE, patch_file=None, seed=0, ctx=None, device="cuda"):
        if patch_file is not None:
            from PIL import Image
            self._patch_img = np.asarray(Image.open(patch_file).convert("RGB"))
        else:
            rng = np.random.default_rng(seed)
            self._patch_img = (rng.random((h, w, 3)) * 255).astype("uint8")
        if self._patch_img.shape[0] != self._patch_img.shape[1]:
            raise ValueError("AdversarialPatch: the patch must be square (the attacker writes 640x640)")
        self.scale = float(scale)
        self.seed = seed  # keys the noise (the context's seed when ctx is given)
        self.output_size = int(h), int(w)
        self.mean_rgb, self.stddev_rgb = 127.0, 128.0
        self.device = torch.device(device)
        self._ctx = ctx or _lib.Context("efficientdet-d0", 0, 1, seed=seed)
        self._patch_dev = torch.as_tensor(np.ascontiguousarray(self._patch_img), device=self.device)
        self._calls = 0

    def print_patch(self):
        """The printed patch (adv_patch.py:40-58; the library applies it to the stored patch)."""
        p = self._patch_img.astype(np.int64)
        return ((p + 127) >> 1).astype(np.uint8)

    def add_adv_to_images(self, images: torch.Tensor, bboxes, step=None, global_image_offset=0):
        """add_adv_to_img for a batch: images [B,H,W,3] uint8 on the device (a patched copy is returned),
        bboxes[b] = the person boxes (ymin, xmin, ymax, xmax) of image b, taken as float32 (the
        detector's output dtype; _create's arithmetic then follows numpy's promotion of float32)."""
        if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[3] != 3:
            raise ValueError("add_adv_to_images: expected [B,H,W,3] uint8")
        B, H, W, _ = images.shape
        if len(bboxes) != B:
            raise ValueError("add_adv_to_images: one box list per image")
        out = images.contiguous().clone()
        counts = np.asarray([len(bb) for bb in bboxes], dtype=np.int32)
        maxb = max(1, int(counts.max()) if B else 1)
        boxes = np.zeros((B, maxb, 4), dtype=np.float32)
        for b, bb in enumerate(bboxes):
            if len(bb):
                boxes[b, :len(bb)] = np.asarray(bb, dtype=np.float32).reshape(-1, 4)
        if step is None:
            step = self._calls
        self._calls += 1
        oh, ow = self.output_size
        self._ctx.call("phx_adv_patch", out.data_ptr(), B, H, W, boxes.ctypes.data, counts.ctypes.data, maxb,
                       self._patch_dev.data_ptr(), int(self._patch_dev.shape[0]), self.scale, oh, ow, int(step),
                       int(global_image_offset), _stream())
        return out

    def add_adv_to_img(self, img: np.ndarray, bboxes, step=None):
        """adv_patch.py:189-201: the patched copy of one HxWx3 uint8 image (host in, host out)."""
        t = torch.as_tensor(np.ascontiguousarray(img), device=self.device)[None]
        return self.add_adv_to_images(t, [list(bboxes)], step=step)[0].cpu().numpy()
