"""Training input pipeline on the GPU — mirror of train_data_generator.py.

Reference: `DataSequence` (train_data_generator.py:26-118) decodes each image with PIL
(`_read_image`, :122-132), letterboxes it on the CPU in float64 with cv2 (`_map_fn`, :55-77) and
yields one image at a time; `partition` (:161-234) batches and applies the train-set augment maps
(:201-204, 222-225).  Here decoding stays on the host (PIL, as the reference), and a whole batch is
letterboxed (`phx_letterbox`) and augmented (`phx_augment`) by HIP kernels in libphx.so on the
caller's stream.  No CPU fallback: the library must be present.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .attacker import EfficientDetVictim, _stream


def _read_image(img_dir, filename):
    """train_data_generator.py:122-132: PIL decode, converted to RGB."""
    from PIL import Image
    im = Image.open(os.path.join(img_dir, filename))
    if im.mode != "RGB":
        im = im.convert("RGB")
    return np.asarray(im)


def pack_images(images_u8, device):
    """Pack decoded HWC uint8 images into one device buffer + offsets [B] + dims [B,2]."""
    sizes = [int(np.prod(im.shape)) for im in images_u8]
    for im in images_u8:
        if im.dtype != np.uint8 or im.ndim != 3 or im.shape[2] != 3:
            raise ValueError("pack_images: expected HxWx3 uint8 images")
    offsets = np.zeros(len(images_u8), dtype=np.int64)
    offsets[1:] = np.cumsum(sizes)[:-1]
    flat = np.concatenate([np.ascontiguousarray(im).reshape(-1) for im in images_u8])
    dims = np.asarray([im.shape[:2] for im in images_u8], dtype=np.int32)
    return (torch.as_tensor(flat, device=device), torch.as_tensor(offsets, device=device),
            torch.as_tensor(dims, device=device))


def letterbox(victim: EfficientDetVictim, src, offsets, dims, output_size, mean_rgb, stddev_rgb):
    """DataSequence._map_fn for a packed batch (device tensors from pack_images) -> [B,H,W,3] fp32."""
    B = int(offsets.numel())
    oh, ow = output_size
    out = torch.empty((B, oh, ow, 3), dtype=torch.float32, device=src.device)
    mean = np.ascontiguousarray(mean_rgb, dtype=np.float32)
    std = np.ascontiguousarray(stddev_rgb, dtype=np.float32)
    victim.ctx.call("phx_letterbox", src.data_ptr(), offsets.data_ptr(), dims.data_ptr(), B,
                    mean.ctypes.data, std.ctypes.data, oh, ow, out.data_ptr(), _stream())
    return out


def augment(victim: EfficientDetVictim, images, step, global_image_offset=0):
    """partition()'s train-set maps (train_data_generator.py:222-225) on a [B,H,W,3] batch:
    random_flip_left_right -> RandomFlip -> RandomContrast(.2) -> random_brightness(.2) -> clip."""
    images = images.contiguous().float()
    B, H, W, _ = images.shape
    out = torch.empty_like(images)
    victim.ctx.call("phx_augment", images.data_ptr(), B, H, W, int(step), int(global_image_offset),
                    out.data_ptr(), _stream())
    return out


class DataSequence:
    """train_data_generator.DataSequence: same constructor, length and indexing; `batch(i)` returns
    a letterboxed [B,H,W,3] device batch (the reference's `.batch(batch_size)` of yielded images)."""

    def __init__(self, victim: EfficientDetVictim, img_dir, output_size, mean_rgb, stddev_rgb, *,
                 file_list=None, shuffle=True, batch_size=2, seed=0):
        self._victim = victim
        self._img_dir = img_dir
        self._output_size = tuple(output_size)
        self._mean_rgb = mean_rgb
        self._stddev_rgb = stddev_rgb
        self._flist = list(file_list or os.listdir(img_dir))
        self._shuffle = shuffle
        self._batch_size = batch_size
        self._rng = np.random.default_rng(seed)
        if shuffle:
            self._rng.shuffle(self._flist)

    def __len__(self):
        return len(self._flist)

    def _map_batch(self, images_u8):
        dev = torch.device("cuda", self._victim.device)
        src, off, dims = pack_images(images_u8, dev)
        return letterbox(self._victim, src, off, dims, self._output_size, self._mean_rgb, self._stddev_rgb)

    def __getitem__(self, idx):
        return self._map_batch([_read_image(self._img_dir, self._flist[idx])])[0]

    def batch(self, i):
        names = [self._flist[(i * self._batch_size + k) % len(self)] for k in range(self._batch_size)]
        return self._map_batch([_read_image(self._img_dir, n) for n in names])

    def __call__(self):
        """Endless generator of batches; reshuffles at the end of each pass, as the reference."""
        i, n = 0, max(1, len(self) // self._batch_size)
        while True:
            yield self.batch(i)
            i += 1
            if i == n:
                if self._shuffle:
                    self._rng.shuffle(self._flist)
                i = 0
