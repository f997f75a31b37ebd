"""Mirror of the reference's defender (attack_detection.PatchAttackDefender + generator.PatchNeutralizer)
over libphx: the U-Net variables and Adam state are caller-owned device tensors, every step runs in
the HIP library (phx_def_step_grad), and data parallelism is one SUM all-reduce of
[d variables | loss] per step (torch.distributed, RCCL on ROCm).

  PatchAttackDefender.__init__  attack_detection.py:34-71 (U-Net built at the protege's image size)
  PatchAttackDefender.call      attack_detection.py:168-206 (training=True, and training=False with the
                                attacker's eval patch)
  PatchAttackDefender.test_step attack_detection.py:320-326
  PatchAttackDefender.train_step attack_detection.py:327-336
  generator.define_model        generator.py:269-281 (Keras initialisers restated in numpy)
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib
from . import distributed as ddp
from .attacker import EfficientDetVictim, _pad_boxes, _stream, _withdraw_if_refilled
from .h5 import read_keras_weights, write_keras_weights

KERAS_MODEL = "patch_neutralizer"  # generator.py:80: PatchNeutralizer's name; its output conv is
                                   # Conv2D(name='patch_neutralizer/output') (generator.py:81)


def _keras_layer(name: str) -> str:
    """The top-level Keras layer of a manifest variable: PatchNeutralizer's tracked layers are the
    encoder blocks conv0..conv4, the decoder blocks deconv0..deconv3 (generator.py:30-41) and the
    output conv (generator.py:81)."""
    top = name.split("/")[0]
    return f"{KERAS_MODEL}/output" if top == "output" else top


def _keras_name(name: str) -> str:
    return (f"{KERAS_MODEL}/{name}" if name.split("/")[0] == "output" else name) + ":0"


def keras_weight_layers(manifest: dict, params: np.ndarray, moving: np.ndarray):
    """The U-Net's variables as Keras's HDF5 `save_weights` lays them out: one entry per top-level
    layer in PatchNeutralizer's order, each layer's weights as Keras's Layer.weights lists them —
    the trainable ones in build order (kernel, bias / gamma, beta), then the non-trainable BN moving
    mean / variance in build order."""
    order, by = [], {}
    for p in manifest["params"]:
        lay = _keras_layer(p["name"])
        if lay not in by:
            by[lay] = ([], [])
            order.append(lay)
        n = int(np.prod(p["shape"]))
        by[lay][0].append((_keras_name(p["name"]), params[p["offset"]:p["offset"] + n].reshape(p["shape"])))
    for b in manifest["bn"]:
        lay, c = _keras_layer(b["name"]), b["channels"]
        by[lay][1].append((_keras_name(b["name"] + "/moving_mean"), moving[b["moving_mean"]:b["moving_mean"] + c]))
        by[lay][1].append((_keras_name(b["name"] + "/moving_variance"),
                           moving[b["moving_variance"]:b["moving_variance"] + c]))
    return [(lay, by[lay][0] + by[lay][1]) for lay in order]


def from_keras_weight_layers(manifest: dict, layers):
    """(flat trainable variables, flat moving statistics) from read_keras_weights' layers.  A file
    weight (':0' dropped) matches the manifest variable whose name it equals or ends with after a
    '/' (Keras may prefix nested variable names with their outer layers' scopes); every manifest
    variable must be matched exactly once, with its shape."""
    want = {p["name"]: ("p", p["offset"], tuple(p["shape"])) for p in manifest["params"]}
    for b in manifest["bn"]:
        want[b["name"] + "/moving_mean"] = ("m", b["moving_mean"], (b["channels"],))
        want[b["name"] + "/moving_variance"] = ("m", b["moving_variance"], (b["channels"],))
    out = np.zeros(manifest["n_params"], np.float32)
    mv = np.zeros(manifest["n_moving"], np.float32)
    seen = set()
    for _, weights in layers:
        for wname, arr in weights:
            w = wname[:-2] if wname.endswith(":0") else wname
            if w.startswith(KERAS_MODEL + "/"):
                w = w[len(KERAS_MODEL) + 1:]
            hits = [m for m in want if w == m or w.endswith("/" + m)]
            if not hits:
                raise ValueError(f"antipatch: weight {wname!r} matches no U-Net variable")
            m = max(hits, key=len)
            if m in seen:
                raise ValueError(f"antipatch: {m} appears twice")
            kind, off, shape = want[m]
            a = np.asarray(arr, np.float32)
            if a.shape != shape:
                raise ValueError(f"antipatch: {wname} has shape {a.shape}, the U-Net needs {shape}")
            (out if kind == "p" else mv)[off:off + a.size] = a.reshape(-1)
            seen.add(m)
    missing = sorted(set(want) - seen)
    if missing:
        raise ValueError(f"antipatch: missing {missing[:4]}{' ...' if len(missing) > 4 else ''}")
    return out, mv


def _fans(shape, transpose=False):
    """keras compute_fans for a conv kernel [k, k, a, b]: fan_in = k*k*a, fan_out = k*k*b."""
    rf = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    return shape[-2] * rf, shape[-1] * rf


def init_unet_params(manifest: dict, seed: int = 0) -> np.ndarray:
    """generator.py initialisers: he_normal (truncated normal, stddev sqrt(2 / fan_in) / .87962566)
    for the encoder / decoder 3x3 convs, the transposed convs and the output conv; glorot_uniform for
    the attention 1x1 convs (Keras default); zero biases; BN gamma 1, beta 0."""
    rng = np.random.default_rng(seed)
    out = np.zeros(manifest["n_params"], np.float32)
    for p in manifest["params"]:
        name, shape, off = p["name"], tuple(p["shape"]), p["offset"]
        n = int(np.prod(shape))
        if name.endswith("/kernel"):
            fan_in, fan_out = _fans(shape)
            if "/attention/" in name:
                lim = np.sqrt(6.0 / (fan_in + fan_out))
                v = rng.uniform(-lim, lim, n)
            else:
                sd = np.sqrt(2.0 / fan_in) / 0.87962566103423978
                v = rng.standard_normal(n)
                bad = np.abs(v) > 2.0
                while bad.any():
                    v[bad] = rng.standard_normal(int(bad.sum()))
                    bad = np.abs(v) > 2.0
                v = v * sd
            out[off:off + n] = v.astype(np.float32)
        elif name.endswith("/gamma"):
            out[off:off + n] = 1.0
    return out


class PatchAttackDefender:
    """attack_detection.PatchAttackDefender (training path): the protege is frozen (inference BN),
    the trainable variables are the U-Net's."""

    def __init__(self, protege_model: EfficientDetVictim, initial_weights=None, protege_config_override=None, *,
                 eval_patch=None, seed=0, learning_rate=1e-2, max_batch=None, device=None):
        """eval_patch (attack_detection.py:33, 57-61): the attacker's trained patch for the evaluation
        branch — a directory holding patch.tiff / scale.txt (PatchAttacker.save_weights), a
        (patch [640,640,3], scale) pair, or a PatchAttacker (its current variables).  Only
        call(training=False) / test_step need it."""
        self.protege_model = protege_model
        self.config = protege_model.config
        if protege_config_override:
            self.config.override(protege_config_override, protege_model.ctx)
        dev = torch.device("cuda", protege_model.device) if device is None else torch.device(device)
        self.handle = _lib.Defender(protege_model.ctx, max_batch or protege_model.max_batch, seed)
        self.manifest = self.handle.manifest()
        n = self.handle.num_params
        if initial_weights is None:
            init = init_unet_params(self.manifest, seed)
        elif isinstance(initial_weights, (str, os.PathLike)):
            init = self._read_npz(initial_weights)
        else:
            init = np.asarray(initial_weights, np.float32).reshape(-1)
        if init.size != n:
            raise ValueError(f"U-Net variables: {init.size} floats, manifest needs {n}")
        self.params = torch.as_tensor(init, device=dev).contiguous()
        # [d variables | loss]: the step's one SUM all-reduce
        self._red = torch.zeros(n + 1, device=dev)
        self.grad = self._red[:n]
        self.loss_buf = self._red[n:]
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.learning_rate = learning_rate
        self.iterations = 0
        self.cur_step = 0
        self.eval_params = None if eval_patch is None else self._eval_params(eval_patch, dev)
        self.eval_loss = torch.zeros(1, device=dev)

    @staticmethod
    def _eval_params(eval_patch, dev):
        """[patch | scale] of the evaluation patch as one device vector (the layout phx_def_eval_step
        reads, the same as the attacker's parameters)."""
        from .attacker import PatchAttacker, load_patch
        if isinstance(eval_patch, PatchAttacker):
            return eval_patch.params.detach().clone().to(dev)
        if isinstance(eval_patch, (str, os.PathLike)):
            patch, scale = load_patch(eval_patch)
        else:
            patch, scale = eval_patch
        patch = np.asarray(patch, np.float32)
        if patch.shape != (_lib.PATCH_SIZE, _lib.PATCH_SIZE, 3):
            raise ValueError(f"eval patch must be [640,640,3], got {patch.shape}")
        return torch.as_tensor(np.concatenate([patch.reshape(-1), [np.float32(scale)]]), device=dev).contiguous()

    @property
    def _trainable_variables(self):
        return {p["name"]: self.params[p["offset"]:p["offset"] + int(np.prod(p["shape"]))].view(*p["shape"])
                for p in self.manifest["params"]}

    def moving_statistics(self, replica_mean: bool = False) -> np.ndarray:
        """The U-Net BN moving mean / variance.  Each rank updates its own copy from its shard (as
        each replica of a Keras MirroredStrategy does).  replica_mean=True returns what Keras reads
        from those ON_READ/MEAN variables — the mean over ranks — through one SUM all-reduce, so
        every rank must call it at the same point."""
        if not (replica_mean and ddp.is_dist()):
            out = np.empty(self.handle.num_moving, np.float32)
            self.handle.call("phx_def_moving", out.ctypes.data, None, None)
            return out
        t = torch.empty(self.handle.num_moving, device=self.params.device)
        self.handle.call("phx_def_moving", t.data_ptr(), None, _stream())
        ddp.allreduce_sum_(t)
        return (t / ddp.world()).cpu().numpy()

    def call(self, images, *, training=True, boxes=None):
        """PatchAttackDefender.call(images, training) (attack_detection.py:168-206).

        training=True: returns the gradient of the loss w.r.t. the U-Net variables (flat, manifest
        order); the loss of the step is left in loss_buf.
        training=False (test_step): the Masker pastes the attacker's eval patch at its trained scale,
        the protege makes a second pass at score_thresh 0 and the U-Net runs in inference mode;
        returns the second pass's detections (boxes [B,100,4], scores [B,100], count [B]) and leaves
        the loss in eval_loss.  `boxes` optionally replaces the first pass's detections for
        placement."""
        images = self.protege_model._check_images(images)
        B = images.shape[0]
        if boxes is not None:
            bx, cnt = _pad_boxes(boxes, B, images.device)
            if bx.shape[1] != _lib.MAX_OUT:
                pad = torch.zeros(B, _lib.MAX_OUT, 4, device=images.device)
                pad[:, :bx.shape[1]] = bx
                bx = pad.contiguous()
            self._keep = (bx, cnt)
            bp, cp = bx.data_ptr(), cnt.data_ptr()
        else:
            bp = cp = None
        if not training:
            if self.eval_params is None:
                raise ValueError("evaluation needs eval_patch (attack_detection.py:57-61)")
            ob = torch.empty(B, _lib.MAX_OUT, 4, device=images.device)
            os_ = torch.zeros(B, _lib.MAX_OUT, device=images.device)
            oc = torch.empty(B, dtype=torch.int32, device=images.device)
            self.handle.call("phx_def_eval_step", images.data_ptr(), B, bp, cp, self.params.data_ptr(),
                             self.eval_params.data_ptr(), self.eval_loss.data_ptr(), ob.data_ptr(), os_.data_ptr(),
                             oc.data_ptr(), int(self.cur_step), self.global_offset(B), _stream())
            return ob, os_, oc
        self.handle.call("phx_def_step_grad", images.data_ptr(), B, bp, cp, self.params.data_ptr(),
                         self._red.data_ptr(), int(self.cur_step), self.global_offset(B), _stream())
        return self.grad

    __call__ = call

    def sync(self):
        """Makes the current stream wait for a prefetched first pass (train_step(next_inputs=...))
        before other users of the protege's context run on it."""
        self.handle.call("phx_def_sync", _stream())

    def global_offset(self, B):
        """Global index of this rank's first image (RNG keys: draws do not depend on the GPU count)."""
        return ddp.global_offset(B)

    def apply_gradients(self):
        """Keras Adam (defender_train.py:35, lr 1e-2), no constraints."""
        self.iterations += 1
        rc = self.handle.lib.phx_adam(self.params.data_ptr(), self.grad.data_ptr(), self.m.data_ptr(),
                                      self.v.data_ptr(), self.params.numel(), float(self.learning_rate),
                                      int(self.iterations), _stream())
        if rc != 0:
            raise _lib.PhxError(f"phx_adam failed ({rc})")

    def train_step(self, inputs, boxes=None, next_inputs=None):
        """attack_detection.py:327-336: grads = self(inputs); apply_gradients.  Returns the loss as a
        device scalar (reading it synchronises).  next_inputs: the batch the next train_step will get
        (defender_train.py's fit draws it from the generator): its first pass (a function of the
        images alone: the protege is frozen) then runs beside this step's U-Net work
        (phx_def_set_next), and that train_step uses its boxes.  The result is the same either way."""
        prev = getattr(self, "_next_keep", None)  # alive until the call that joins its first pass
        _withdraw_if_refilled(self, lambda: self.handle.call("phx_def_set_next", None, 0, 0))
        self._next_keep = self._next_rec = None
        if next_inputs is not None:
            nx = self.protege_model._check_images(next_inputs)
            self._next_keep = nx  # alive until the step that consumes it
            self._next_rec = (nx, nx._version)
            self.handle.call("phx_def_set_next", nx.data_ptr(), nx.shape[0], self.global_offset(nx.shape[0]))
        self.call(inputs, boxes=boxes)
        del prev
        ddp.allreduce_sum_(self._red)
        self.apply_gradients()
        self.cur_step += 1
        return {"loss": self.loss_buf[0]}

    def test_step(self, inputs, boxes=None):
        """attack_detection.py:320-326: self(inputs, training=False); the loss metric summed over
        ranks (the one collective; every rank calls it).  Returns ({"loss": float}, detections)."""
        preds = self.call(inputs, training=False, boxes=boxes)
        ddp.allreduce_sum_(self.eval_loss)
        return {"loss": float(self.eval_loss.item())}, preds

    def debug(self, what: int, B: int):
        S = self.protege_model.ctx.image_size
        shape = {_lib.DEF_PATCHED: (B, S, S, 3), _lib.DEF_TARGETS: (B, S, S, 3), _lib.DEF_UPDATES: (B, S, S, 3),
                 _lib.DEF_BOXES: (B, _lib.MAX_OUT, 4), _lib.DEF_COUNTS: (B,)}[what]
        out = torch.empty(shape, device=self.params.device)
        self.handle.call("phx_def_debug", int(what), out.data_ptr(), out.numel(), _stream())
        if what == _lib.DEF_COUNTS:
            return out.view(torch.int32)
        return out

    def save_weights(self, dirpath, **kwargs):
        """attack_detection.py:300-308: `self._antipatch.save_weights(dirpath/antipatch.h5)` — the U-Net
        variables and BN moving statistics in Keras's HDF5 weights layout (h5.py; the moving
        statistics as their mean over ranks), plus the same variables in antipatch.npz under their
        Keras names.  Under data parallelism every rank calls it (the moving statistics are
        all-reduced) and rank 0 writes the files."""
        mv = self.moving_statistics(replica_mean=True)
        if ddp.rank() != 0:
            return
        os.makedirs(dirpath)
        params = self.params.detach().cpu().numpy()
        write_keras_weights(os.path.join(dirpath, "antipatch.h5"), keras_weight_layers(self.manifest, params, mv))
        arrs = {k: v.detach().cpu().numpy() for k, v in self._trainable_variables.items()}
        for b in self.manifest["bn"]:
            arrs[b["name"] + "/moving_mean"] = mv[b["moving_mean"]:b["moving_mean"] + b["channels"]]
            arrs[b["name"] + "/moving_variance"] = mv[b["moving_variance"]:b["moving_variance"] + b["channels"]]
        np.savez(os.path.join(dirpath, "antipatch.npz"), **arrs)

    def _read_npz(self, path):
        """initial_weights (attack_detection.py:54-55 `load_weights`): an .h5 Keras weights file, an
        .npz of this class's save_weights, or a directory holding antipatch.h5 (preferred) or
        antipatch.npz.  Sets the BN moving statistics; returns the flat trainable variables."""
        p = path
        if os.path.isdir(path):
            h5 = os.path.join(path, "antipatch.h5")
            p = h5 if os.path.exists(h5) else os.path.join(path, "antipatch.npz")
        if str(p).endswith((".h5", ".hdf5", ".keras")):
            out, mv = from_keras_weight_layers(self.manifest, read_keras_weights(p))
            self.handle.call("phx_def_moving", None, mv.ctypes.data, None)
            return out
        z = np.load(p)
        out = np.zeros(self.handle.num_params, np.float32)
        for q in self.manifest["params"]:
            out[q["offset"]:q["offset"] + int(np.prod(q["shape"]))] = z[q["name"]].reshape(-1)
        mv = np.zeros(self.handle.num_moving, np.float32)
        for b in self.manifest["bn"]:
            mv[b["moving_mean"]:b["moving_mean"] + b["channels"]] = z[b["name"] + "/moving_mean"]
            mv[b["moving_variance"]:b["moving_variance"] + b["channels"]] = z[b["name"] + "/moving_variance"]
        self.handle.call("phx_def_moving", None, mv.ctypes.data, None)
        return out
