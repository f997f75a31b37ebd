"""Host-side mirror of the reference's attack interface (attacker.py, brightness_matcher.py,
util.get_victim_model) over the libphx C ABI.

Same names, argument meaning and error behaviour as the reference where they exist:

  EfficientDetVictim       util.get_victim_model (util.py:177-189) + KerasDriver (infer_lib.py:383)
  BrightnessMatcher.call   brightness_matcher.py:43-73
  Patcher.call             attacker.py:490-498
  PatchAttacker            attacker.py:24-341: first_pass :91, second-pass loss and gradient in
                           call :172-219, calc_asr :238, train_step :307, save_weights :328

Every computation runs in the HIP kernels of libphx.so on PyTorch-ROCm device memory; PyTorch
provides only allocation, streams and torch.distributed (RCCL).  Data parallelism: one process per
GPU, each holding B/world images; the [patch | scale] gradient is SUM-all-reduced once per step
(bn=local: statistics per rank).
"""
from __future__ import annotations

import ctypes
import math
import os
from collections.abc import Mapping
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from . import distributed as ddp
from . import tiff
from . import weights as wmod

MEAN_RGB = {"efficientdet": [0.485 * 255, 0.456 * 255, 0.406 * 255], "lite": [127.0] * 3}
STDDEV_RGB = {"efficientdet": [0.229 * 255, 0.224 * 255, 0.225 * 255], "lite": [128.0] * 3}


def _stream():
    return torch.cuda.current_stream().cuda_stream


@dataclass
class NmsConfig:
    """hparams_config.py:258-266 (+ attacker_train.py:31 override)"""
    method: str = "gaussian"
    iou_thresh: float | None = None
    score_thresh: float = 0.0
    sigma: float | None = None
    max_output_size: int = 100


@dataclass
class VictimConfig:
    name: str
    image_size: int
    mean_rgb: list
    stddev_rgb: list
    nms_configs: NmsConfig = field(default_factory=NmsConfig)
    # the library context this config describes (set by EfficientDetVictim): overrides that change
    # the computation are forwarded to it, as the reference's model.config.override reaches the model
    ctx: object = field(default=None, repr=False, compare=False)

    def override(self, d: dict, ctx=None):
        """Config.override (hparams_config.py:91-109) for the keys the attack uses.  The values that
        change the computation are forwarded to the library context (score_thresh); overrides the
        library does not implement raise instead of diverging silently from the reference."""
        ctx = ctx if ctx is not None else self.ctx
        for k, v in d.items():
            if k != "nms_configs":
                raise ValueError(f"config_override: unsupported key {k!r} (only nms_configs)")
            for kk, vv in v.items():
                if kk == "score_thresh":
                    if ctx is None:
                        raise ValueError("config_override: score_thresh needs the victim's library context "
                                         "(a VictimConfig not owned by an EfficientDetVictim)")
                    ctx.set_score_thresh(float(vv))
                elif kk == "iou_thresh":
                    pass  # unused by the gaussian method: iou_thresh = 1.0 (postprocess.py:184-188)
                elif kk == "method" and vv != "gaussian":
                    raise ValueError("config_override: only nms method 'gaussian' (the reference's) is built")
                elif kk == "sigma" and vv not in (None, 0.5):
                    raise ValueError("config_override: soft-NMS sigma is fixed at the default 0.5")
                elif kk == "max_output_size" and vv != 100:
                    raise ValueError("config_override: max_output_size is fixed at 100")
                elif kk not in ("method", "sigma", "max_output_size", "pyfunc", "max_nms_inputs"):
                    raise ValueError(f"config_override: unsupported nms_configs key {kk!r}")
                elif kk in ("pyfunc", "max_nms_inputs") and vv:
                    raise ValueError(f"config_override: nms_configs.{kk} = {vv!r} is not built")
                setattr(self.nms_configs, kk, vv)


class EfficientDetVictim:
    """The victim detector held by a libphx context (one device)."""

    def __init__(self, model_name="efficientdet-d0", weights="synthetic", *, seed=0, image_size=0,
                 max_batch=16, bn_mode="local", score_thresh=0.5, rng_seed=0, device=None,
                 person_bias=0.0, dtype="f32"):
        if device is None:
            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        self.device = device
        if dtype not in ("f32", "bf16"):
            raise ValueError("dtype must be 'f32' (the reference's precision) or 'bf16'")
        modes = {"local": _lib.BN_LOCAL, "frozen": _lib.BN_FROZEN, "sync": _lib.BN_SYNC}
        if bn_mode not in modes:
            raise ValueError("bn_mode must be 'local', 'frozen' or 'sync'")
        self.ctx = _lib.Context(model_name, image_size, max_batch, modes[bn_mode], score_thresh, rng_seed, device,
                                _lib.DTYPE_BF16 if dtype == "bf16" else _lib.DTYPE_F32)
        self.bn_mode = bn_mode
        if bn_mode == "sync":
            # SyncBN: the library hands every BN's per-channel sums to this collective
            from .distributed import bn_sync_callback
            self._ar = bn_sync_callback()
            self.ctx.call("phx_set_allreduce", ctypes.cast(self._ar, ctypes.c_void_p), None)
        self.dtype = dtype
        self.manifest = self.ctx.manifest()
        if isinstance(weights, str) and weights == "synthetic":
            blob = wmod.synthetic_blob(self.manifest, seed=seed, person_bias=person_bias)
        elif isinstance(weights, (str, os.PathLike)):
            # a TensorFlow checkpoint (directory or prefix), restored as KerasDriver does
            # (util_keras.restore_ckpt with ema_decay 0.9998, skip_mismatch=False)
            from .ckpt import checkpoint_to_blob
            blob = np.ascontiguousarray(checkpoint_to_blob(os.fspath(weights), self.manifest, ema_decay=0.9998))
        else:
            blob = np.ascontiguousarray(np.asarray(weights, dtype=np.float32))
        self.load_weights(blob)
        fam = "lite" if "lite" in model_name else "efficientdet"
        self.config = VictimConfig(model_name, self.ctx.image_size, MEAN_RGB[fam], STDDEV_RGB[fam],
                                   NmsConfig(score_thresh=score_thresh), ctx=self.ctx)
        self.num_anchors = self.ctx.num_anchors
        self.max_batch = max_batch

    def load_weights(self, blob: np.ndarray):
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        if blob.size != self.ctx.weight_count():
            raise ValueError(f"weight blob has {blob.size} floats, manifest needs {self.ctx.weight_count()}")
        self.ctx.call("phx_load_weights", blob.ctypes.data, blob.size)
        self.blob = blob

    def read_weights(self) -> np.ndarray:
        out = np.empty(self.ctx.weight_count(), np.float32)
        self.ctx.call("phx_read_weights", out.ctypes.data, out.size)
        return out

    def _check_images(self, images):
        S = self.ctx.image_size
        if images.dim() != 4 or tuple(images.shape[1:]) != (S, S, 3) or images.dtype != torch.float32:
            raise ValueError(f"images must be float32 [B,{S},{S},3], got {tuple(images.shape)} {images.dtype}")
        if not images.is_cuda:
            raise ValueError("images must be a device tensor")
        if images.shape[0] > self.max_batch:
            raise ValueError("batch exceeds max_batch")
        return images.contiguous()

    def detect(self, images):
        """EfficientDetModel.call(pre_mode=None, post_mode=None) + postprocess.pre_nms."""
        images = self._check_images(images)
        B, A = images.shape[0], self.num_anchors
        scores = torch.empty(B, A, device=images.device)
        classes = torch.empty(B, A, dtype=torch.int32, device=images.device)
        boxes = torch.empty(B, A, 4, device=images.device)
        self.ctx.call("phx_detect", images.data_ptr(), B, scores.data_ptr(), classes.data_ptr(),
                      boxes.data_ptr(), _stream())
        return boxes, scores, classes

    def first_pass(self, images):
        images = self._check_images(images)
        B = images.shape[0]
        ob = torch.empty(B, _lib.MAX_OUT, 4, device=images.device)
        os_ = torch.empty(B, _lib.MAX_OUT, device=images.device)
        oc = torch.empty(B, dtype=torch.int32, device=images.device)
        self.ctx.call("phx_first_pass", images.data_ptr(), B, ob.data_ptr(), os_.data_ptr(), oc.data_ptr(),
                      _stream())
        return ob, os_, oc

    def soft_nms(self, boxes, scores, count=None):
        """postprocess.nms(padded=True) over [B,N,4] / [B,N] candidates."""
        boxes = boxes.contiguous().float()
        scores = scores.contiguous().float()
        B, N = scores.shape
        if count is None:
            count = torch.full((B,), N, dtype=torch.int32, device=scores.device)
        count = count.to(torch.int32).contiguous()
        ob = torch.empty(B, _lib.MAX_OUT, 4, device=scores.device)
        os_ = torch.empty(B, _lib.MAX_OUT, device=scores.device)
        oc = torch.empty(B, dtype=torch.int32, device=scores.device)
        self.ctx.call("phx_soft_nms", boxes.data_ptr(), scores.data_ptr(), count.data_ptr(), B, N,
                      ob.data_ptr(), os_.data_ptr(), oc.data_ptr(), _stream())
        return ob, os_, oc


class BrightnessMatcher:
    """brightness_matcher.BrightnessMatcher: Y-channel mean transfer patch -> scene."""

    def __init__(self, victim: EfficientDetVictim):
        self.victim = victim

    def __call__(self, inputs):
        src, tgt = inputs
        squeeze = src.dim() == 3
        if squeeze:
            src, tgt = src[None], tgt[None]
        src = src.contiguous().float()
        tgt = tgt.contiguous().float()
        B, Pp = src.shape[0], src.shape[1]
        out = torch.empty_like(src)
        self.victim.ctx.call("phx_brightness_match", src.data_ptr(), Pp, tgt.data_ptr(), tgt.shape[1],
                             tgt.shape[2], B, out.data_ptr(), _stream())
        return out[0] if squeeze else out

    call = __call__


def _withdraw_if_refilled(obj, withdraw):
    """The first pass prefetched for the next step (phx_set_next / phx_def_set_next) read that batch's
    buffer as it was then.  If the buffer has been written in place since — the tensor's version
    counter (shared with every view of it) moved, as a pinned-ring loader refilling one device buffer
    does — the prefetched detections are stale: withdraw them (set_next(NULL)), so the step runs its
    own first pass (attacker.py:172-184 computes it from the images the step gets)."""
    rec = getattr(obj, "_next_rec", None)
    if rec is not None and rec[0]._version != rec[1]:
        withdraw()


def _pad_boxes(boxes, B, device):
    """list of [n_b,4] (or a padded [B,maxb,4] + count) -> ([B,maxb,4], count[B])"""
    if isinstance(boxes, (tuple, list)) and len(boxes) == 2 and torch.is_tensor(boxes[0]) and boxes[0].dim() == 3:
        bx, cnt = boxes
        return bx.contiguous().float(), cnt.to(torch.int32).contiguous()
    maxb = max(1, max(len(b) for b in boxes))
    if maxb > _lib.MAX_OUT:
        raise ValueError("at most 100 boxes per image")
    # padded on the host, then one transfer: [B*maxb*4 boxes | B counts] as raw 32-bit words
    out = np.zeros((B, maxb, 4), np.float32)
    cnt = np.zeros(B, np.int32)
    for i, b in enumerate(boxes):
        b = np.asarray(b, dtype=np.float32).reshape(-1, 4)
        out[i, :len(b)] = b
        cnt[i] = len(b)
    flat = torch.as_tensor(np.concatenate([out.reshape(-1).view(np.int32), cnt])).to(device)
    return flat[:out.size].view(torch.float32).view(B, maxb, 4), flat[out.size:]


class Patcher:
    """attacker.Patcher: EOT paste of the current patch onto every box of every image."""

    def __init__(self, attacker: "PatchAttacker"):
        self.attacker = attacker

    def __call__(self, inputs, step=None):
        boxes, images = inputs
        a = self.attacker
        images = a.model._check_images(images)
        B = images.shape[0]
        bx, cnt = _pad_boxes(boxes, B, images.device)
        out = torch.empty_like(images)
        self.last_placements = torch.zeros(B, bx.shape[1], 8, device=images.device)
        a.model.ctx.call("phx_patch_images", images.data_ptr(), B, bx.data_ptr(), cnt.data_ptr(), bx.shape[1],
                         a.params.data_ptr(), int(a.cur_step if step is None else step), a.global_offset(B),
                         out.data_ptr(), self.last_placements.data_ptr(), _stream())
        return out

    call = __call__


class _Mean:
    """keras.metrics.Mean (what add_metric aggregates per epoch)."""

    def __init__(self):
        self.total, self.count = 0.0, 0

    def update(self, v):
        self.total += float(v)
        self.count += 1

    def result(self):
        return self.total / max(self.count, 1)


class _StepMetrics(Mapping):
    """The {name: running mean} dict train_step returns, evaluated on first access."""

    def __init__(self, attacker, sid):
        self._a, self._sid, self._d = attacker, sid, None

    def _get(self):
        if self._d is None:
            self._a._flush_metrics()
            snap = self._a._snapshots.get(self._sid)
            # a reset_metrics() after this step dropped its snapshot: report the current means
            self._d = dict(snap) if snap is not None else {k: m.result() for k, m in self._a.metrics.items()}
        return self._d

    def __getitem__(self, k):
        return self._get()[k]

    def __iter__(self):
        return iter(self._get())

    def __len__(self):
        return len(self._get())


class PatchAttacker:
    """attacker.PatchAttacker: trainable [patch | scale] optimised against the victim."""

    METRICS = ("loss", "scale", "scale_loss", "tv_loss", "mean_max_score", "std_max_score", "asr",
               "asr_to_scale")

    def __init__(self, model: EfficientDetVictim, initial_patch=None, config_override=None,
                 visualize_freq=200, *, seed=0, learning_rate=1e-2, device=None):
        self.model = model
        self.config = model.config
        if config_override:
            self.config.override(config_override, model.ctx)
        dev = torch.device("cuda", model.device) if device is None else torch.device(device)
        if initial_patch is None:
            # np.random.uniform(-1, 1, (640, 640, 3)), scale .4 (attacker.py:42-44)
            patch_img = np.random.default_rng(seed).uniform(-1.0, 1.0, size=(640, 640, 3))
            scale = 0.4
        else:
            patch_img, scale = load_patch(initial_patch)
        params = np.concatenate([np.asarray(patch_img, np.float32).reshape(-1), [np.float32(scale)]])
        self.params = torch.as_tensor(params, dtype=torch.float32, device=dev).contiguous()
        # [d patch | d scale | metric row]: one SUM all-reduce per step carries the gradient and the
        # per-rank metric sums (loss, counts, #images; TV only on the rank that adds it), so every
        # rank issues exactly the same collective at the same point of train_step
        self._red = torch.zeros(_lib.NPARAM + _lib.NMETRIC, device=dev)
        self.grad = self._red[:_lib.NPARAM]
        self.metrics_buf = self._red[_lib.NPARAM:]
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.learning_rate = learning_rate
        self.iterations = 0
        self.cur_step = 0
        self.visualize_freq = visualize_freq
        self._patcher = Patcher(self)
        self._matcher = BrightnessMatcher(model)
        self.metrics = {k: _Mean() for k in self.METRICS}
        self._pending = []      # (step id, device metric row) not yet folded into self.metrics
        self._snapshots = {}    # step id -> running-mean dict after that step
        self._step_id = 0
        self.bins = np.arange(self.config.nms_configs.score_thresh, .805, .01, dtype="float32")

    # ---- variables -----------------------------------------------------------------------------
    @property
    def patch(self):
        return self.params[:_lib.NPATCH].view(640, 640, 3)

    @property
    def scale(self):
        return self.params[_lib.NPATCH]

    @property
    def _trainable_variables(self):
        return [self.params[_lib.NPATCH:], self.patch]

    def global_offset(self, B):
        return ddp.global_offset(B)

    # ---- reference methods -------------------------------------------------------------------
    def first_pass(self, images):
        return self.model.first_pass(images)

    def call(self, images, *, training=True, boxes=None, add_tv=None):
        """PatchAttacker.call (attacker.py:172-219).  training=True: the attack step, returns
        [d scale, d patch] (attacker.py:217).  training=False: the victim in inference mode, returns
        the second pass's soft-NMS person detections (boxes_pred, scores_pred) as padded [B,100,4],
        [B,100] plus counts [B].  `boxes` optionally replaces the first-pass detections for
        placement (injected boxes).  The metric row of the step is left in metrics_buf."""
        images = self.model._check_images(images)
        B = images.shape[0]
        if add_tv is None:
            add_tv = ddp.rank() == 0  # TV counted once per global step
        if boxes is not None:
            bx, cnt = _pad_boxes(boxes, B, images.device)
            bp, cp, maxb = bx.data_ptr(), cnt.data_ptr(), bx.shape[1]
            self._keep = (bx, cnt)
        else:
            bp, cp, maxb = None, None, 0
        if not training:
            ob = torch.empty(B, _lib.MAX_OUT, 4, device=images.device)
            os_ = torch.empty(B, _lib.MAX_OUT, device=images.device)
            oc = torch.empty(B, dtype=torch.int32, device=images.device)
            self.model.ctx.call("phx_eval_step", images.data_ptr(), B, bp, cp, maxb, self.params.data_ptr(),
                                int(self.cur_step), self.global_offset(B), int(bool(add_tv)),
                                self.metrics_buf.data_ptr(), ob.data_ptr(), os_.data_ptr(), oc.data_ptr(),
                                _stream())
            return ob, os_, oc
        self.model.ctx.call("phx_step_grad", images.data_ptr(), B, bp, cp, maxb, self.params.data_ptr(),
                            int(self.cur_step), self.global_offset(B), int(bool(add_tv)), self.grad.data_ptr(),
                            self.metrics_buf.data_ptr(), _stream())
        return [self.grad[_lib.NPATCH:], self.grad[:_lib.NPATCH].view(640, 640, 3)]

    __call__ = call

    def sync(self):
        """Makes the current stream wait for a prefetched first pass (train_step(next_inputs=...))."""
        self.model.ctx.call("phx_sync", _stream())

    def apply_gradients(self):
        """optimizer.apply_gradients + variable constraints (attacker.py:315, :51-54)."""
        self.iterations += 1
        self.model.ctx.call("phx_adam_clip", self.params.data_ptr(), self.grad.data_ptr(), self.m.data_ptr(),
                            self.v.data_ptr(), float(self.learning_rate), int(self.iterations), _stream())

    def allreduce_gradients(self):
        """SUM over ranks of [d patch | d scale | metric row] (the step's one collective)."""
        ddp.allreduce_sum_(self._red)

    def _metric_row(self):
        """Device row [metric row | scale] of the step just run (scale before the update, as the
        reference's add_metric(self._scale_regressor) inside call, attacker.py:197)."""
        return torch.cat([self.metrics_buf, self.params[_lib.NPATCH:]])

    @staticmethod
    def _derive(v):
        """add_metric values (attacker.py:196-207) from a rank-summed [metrics | scale] row."""
        n, scale = float(v[_lib.M_NIMG]), float(v[_lib.NMETRIC])
        mean = v[_lib.M_SUM_M] / n
        var = max(v[_lib.M_SUM_M2] / n - mean * mean, 0.0)
        # calc_asr (attacker.py:253-255) divides tf.size of the flattened ragged [n,4] boxes, 4
        # floats per box, in float32: 1 - 4n / (4d + epsilon)
        asr = float(np.float32(1.0) - np.float32(4.0 * v[_lib.M_ASR_NUM])
                    / (np.float32(4.0 * v[_lib.M_ASR_DEN]) + np.float32(1e-7)))
        return {"loss": float(v[_lib.M_LOSS]), "scale": scale, "scale_loss": float(v[_lib.M_SCALE_LOSS]),
                "tv_loss": float(v[_lib.M_TV]), "mean_max_score": mean, "std_max_score": math.sqrt(var),
                "asr": asr, "asr_to_scale": asr / scale if scale else float("inf"),
                "patches": float(v[_lib.M_NBOX])}

    def step_metrics(self):
        """Per-step values of the reference's add_metric set (attacker.py:196-207) for the step
        just run: global over ranks after train_step (its all-reduce), this rank's after a bare
        call().  Synchronises with the device; issues no collective."""
        return self._derive(self._metric_row().cpu().numpy().astype(np.float64))

    def _flush_metrics(self):
        """Fold the queued per-step rows (already reduced by train_step's all-reduce) into the
        Keras-style running means with one device->host copy, so train_step never waits on the GPU
        and reading metrics never issues a collective (any rank may read them, or none)."""
        if not self._pending:
            return
        ids = [i for i, _ in self._pending]
        rows = torch.stack([r for _, r in self._pending]).cpu().numpy().astype(np.float64)
        self._pending.clear()
        for sid, v in zip(ids, rows):
            sm = self._derive(v)
            for k in self.METRICS:
                self.metrics[k].update(sm[k])
            self._snapshots[sid] = {k: m.result() for k, m in self.metrics.items()}
        for old in [k for k in self._snapshots if k < ids[-1] - 1024]:
            del self._snapshots[old]

    def train_step(self, inputs, boxes=None, next_inputs=None):
        """attacker.py:307-316: grads = self(inputs); apply_gradients; return metrics.  The metric
        dict is evaluated lazily (like the tensors Keras returns): reading it synchronises.
        next_inputs: the batch the next train_step will get (attacker_train.py's fit draws it from
        the generator).  With first-pass placement its clean first pass — a function of the images,
        not of the patch — then runs beside this step's second pass and backward (phx_set_next) and
        the next train_step places its patches by it; the results are the same either way."""
        # the batch the previous step prefetched, kept alive until this call (which joins its first
        # pass on the current stream) has been issued
        prev = getattr(self, "_next_keep", None)
        _withdraw_if_refilled(self, lambda: self.model.ctx.call("phx_set_next", None, 0, 0))
        self._next_keep = self._next_rec = None
        if next_inputs is not None and boxes is None:
            nx = self.model._check_images(next_inputs)
            self._next_keep = nx  # alive until the step that consumes it
            self._next_rec = (nx, nx._version)
            self.model.ctx.call("phx_set_next", nx.data_ptr(), nx.shape[0], self.global_offset(nx.shape[0]))
        self.call(inputs, boxes=boxes)
        del prev
        sid = self._step_id
        self._step_id += 1
        self.allreduce_gradients()
        self._pending.append((sid, self._metric_row()))
        if len(self._pending) >= 256:  # bound the queue when nobody reads the metrics
            self._flush_metrics()
        self.apply_gradients()
        self.cur_step += 1
        return _StepMetrics(self, sid)

    def test_step(self, inputs, boxes=None):
        """attacker.py:318-326: self(inputs, training=False) — the victim in inference mode (BN
        from the moving statistics, no drop connect), the same EOT paste, loss and metrics, no
        gradient and no update.  Returns (metrics, (boxes_pred, scores_pred, count)) where the
        predictions are call()'s soft-NMS person detections on the patched images."""
        preds = self.call(inputs, training=False, boxes=boxes)
        ddp.allreduce_sum_(self.metrics_buf)  # every rank, same point: the metric row's one collective
        return self.step_metrics(), preds

    def reset_metrics(self):
        """Keras reset at epoch boundaries: queued steps are folded first (they belong to the
        finished epoch)."""
        self._flush_metrics()
        for m in self.metrics.values():
            m.total, m.count = 0.0, 0
        self._snapshots = {}

    def save_weights(self, dirpath, **kwargs):
        """attacker.py:328-341, same three files: scale.txt (str of the float32 scale), patch.png
        (clip(patch*std + mean, 0, 255) as uint8) and patch.tiff (the raw float32 normalised patch,
        written by our own baseline-TIFF writer since tifffile is not installed)."""
        os.makedirs(dirpath)
        with open(os.path.join(dirpath, "scale.txt"), "w") as f:
            f.write(str(np.float32(self.scale.item())))
        patch = self.patch.detach().cpu().numpy()
        tiff.write_float_tiff(os.path.join(dirpath, "patch.tiff"), patch)
        img = np.clip(patch * np.asarray(self.config.stddev_rgb, np.float32)
                      + np.asarray(self.config.mean_rgb, np.float32), 0, 255)
        from PIL import Image
        Image.fromarray(img.astype(np.uint8)).save(os.path.join(dirpath, "patch.png"))


def load_patch(dirpath):
    """initial_patch=dir (attacker.py:46-48): tifffile.imread(patch.tiff) + float(scale.txt)."""
    import ast
    patch = tiff.read_float_tiff(os.path.join(dirpath, "patch.tiff"))
    if patch.shape != (640, 640, 3):
        raise ValueError(f"patch.tiff holds {patch.shape}, expected (640, 640, 3)")
    with open(os.path.join(dirpath, "scale.txt")) as f:
        scale = ast.literal_eval(f.read())
    return patch, float(scale)


class ReduceLROnPlateau:
    """keras ReduceLROnPlateau(monitor='loss', factor=.5, patience=50, min_lr=1e-4) used by
    attacker_train.py:70-71, stepped once per epoch."""

    def __init__(self, attacker: PatchAttacker, factor=0.5, patience=50, min_lr=1e-4, min_delta=1e-4):
        self.a, self.factor, self.patience, self.min_lr, self.min_delta = attacker, factor, patience, min_lr, min_delta
        self.best, self.wait = float("inf"), 0

    def on_epoch_end(self, loss):
        if loss < self.best - self.min_delta:
            self.best, self.wait = loss, 0
        else:
            self.wait += 1
            if self.wait >= self.patience and self.a.learning_rate > self.min_lr:
                self.a.learning_rate = max(self.a.learning_rate * self.factor, self.min_lr)
                self.wait = 0
