"""ctypes binding of libphx.so (the C ABI declared in include/phx.h).

The shared library is built in-tree (``python -m mladversarialobjectdetection_amd.build`` or
``__graft_entry__.build()``) and loaded from this package directory.  There is deliberately no
fallback: if the library is missing every entry point raises, so a GPU run can never silently
execute anything but the HIP kernels.
"""
from __future__ import annotations

import ctypes
import json
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_size_t, c_uint64, c_void_p

ABI_VERSION = 2
PATCH_SIZE = 640
NPATCH = PATCH_SIZE * PATCH_SIZE * 3
NPARAM = NPATCH + 1
MAX_OUT = 100

# metric slots (phx.h PHX_M_*)
M_LOSS, M_SCALE_LOSS, M_TV, M_SUM_M, M_SUM_M2, M_ASR_NUM, M_ASR_DEN, M_NBOX, M_NIMG = range(9)
NMETRIC = 9

BN_LOCAL, BN_FROZEN, BN_SYNC = 0, 1, 2
DTYPE_F32, DTYPE_BF16 = 0, 1

_HERE = os.path.dirname(os.path.abspath(__file__))
# PHX_LIB selects another in-tree build (libphx*.so next to this file) for A/B timing runs
_ALT = os.environ.get("PHX_LIB", "")
LIB_PATH = os.path.join(_HERE, os.path.basename(_ALT) if _ALT.startswith("libphx") and _ALT.endswith(".so")
                        else "libphx.so")


class PhxError(RuntimeError):
    pass


class _Config(ctypes.Structure):
    _fields_ = [
        ("model_name", c_char_p),
        ("image_size", c_int),
        ("max_batch", c_int),
        ("bn_mode", c_int),
        ("score_thresh", c_float),
        ("seed", c_uint64),
        ("compute_dtype", c_int),
    ]


# (name, restype, argtypes) — one row per declaration in include/phx.h
_SIGS = [
    ("phx_abi_version", c_int, []),
    ("phx_create", c_int, [POINTER(_Config), c_int, POINTER(c_void_p)]),
    ("phx_destroy", None, [c_void_p]),
    ("phx_last_error", c_char_p, [c_void_p]),
    ("phx_model_info", c_int, [c_void_p, c_char_p, c_size_t, POINTER(c_size_t)]),
    ("phx_set_score_thresh", c_int, [c_void_p, c_float]),
    ("phx_weight_manifest", c_int, [c_void_p, c_char_p, c_size_t, POINTER(c_size_t)]),
    ("phx_weight_count", c_size_t, [c_void_p]),
    ("phx_load_weights", c_int, [c_void_p, c_void_p, c_size_t]),
    ("phx_read_weights", c_int, [c_void_p, c_void_p, c_size_t]),
    ("phx_detect", c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("phx_num_anchors", c_int, [c_void_p]),
    ("phx_workspace_bytes", c_int, [c_void_p, c_int, POINTER(c_size_t)]),
    ("phx_image_size", c_int, [c_void_p]),
    ("phx_first_pass", c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("phx_soft_nms", c_int,
     [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("phx_brightness_match", c_int,
     [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    ("phx_patch_images", c_int,
     [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_int, c_void_p,
      c_void_p, c_void_p]),
    ("phx_step_grad", c_int,
     [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_int, c_int,
      c_void_p, c_void_p, c_void_p]),
    ("phx_set_next", c_int, [c_void_p, c_void_p, c_int, c_int]),
    ("phx_sync", c_int, [c_void_p, c_void_p]),
    ("phx_eval_step", c_int,
     [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_int, c_int,
      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("phx_adam_clip", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int64, c_void_p]),
    ("phx_letterbox", c_int,
     [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    ("phx_augment", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int64, c_int, c_void_p, c_void_p]),
    ("phx_set_allreduce", c_int, [c_void_p, c_void_p, c_void_p]),
    ("phx_adv_patch", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_double, c_int, c_int,
      c_int64, c_int, c_void_p]),
    ("phx_profile", c_int, [c_void_p, c_int]),
    ("phx_profile_report", c_int, [c_void_p, c_char_p, c_size_t, POINTER(c_size_t)]),
    ("phx_debug_last_patched", c_int, [c_void_p, c_void_p, c_void_p]),
    ("phx_debug_last_maxscores", c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    ("phx_debug_last_detections", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("phx_debug_last_image_grad", c_int, [c_void_p, c_void_p, c_void_p]),
    ("phx_debug_tap", c_int, [c_void_p, c_char_p, c_int, c_void_p, c_size_t, c_void_p]),
    ("phx_debug_checksums", c_int, [c_void_p, c_int, c_char_p, c_size_t, POINTER(c_size_t)]),
    ("phx_debug_tensor", c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_size_t, c_void_p]),
    # defender step
    ("phx_def_create", c_int, [c_void_p, c_int, c_uint64, POINTER(c_void_p)]),
    ("phx_def_destroy", None, [c_void_p]),
    ("phx_def_last_error", c_char_p, [c_void_p]),
    ("phx_def_num_params", c_int64, [c_void_p]),
    ("phx_def_num_moving", c_int64, [c_void_p]),
    ("phx_def_manifest", c_int, [c_void_p, c_char_p, c_size_t, POINTER(c_size_t)]),
    ("phx_def_moving", c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    ("phx_def_workspace_bytes", c_int, [c_void_p, c_int, POINTER(c_size_t)]),
    ("phx_def_eval_workspace_bytes", c_int, [c_void_p, c_int, POINTER(c_size_t)]),
    ("phx_def_step_grad", c_int,
     [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    ("phx_def_set_next", c_int, [c_void_p, c_void_p, c_int, c_int]),
    ("phx_def_sync", c_int, [c_void_p, c_void_p]),
    ("phx_def_eval_step", c_int,
     [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
      c_void_p, c_int64, c_int, c_void_p]),
    ("phx_def_debug", c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p]),
    ("phx_adam", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_int64, c_void_p]),
]

# phx_def_debug tensors
DEF_PATCHED, DEF_TARGETS, DEF_UPDATES, DEF_BOXES, DEF_COUNTS = range(5)

EXPORTED = [s[0] for s in _SIGS]

_lib = None


def load(path: str | None = None):
    """Load libphx.so once; raise PhxError when it is missing (no CPU fallback exists)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise PhxError(
            f"{p} not found: build the HIP extension first (python -m "
            "mladversarialobjectdetection_amd.build)")
    lib = ctypes.CDLL(p)
    for name, res, args in _SIGS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.phx_abi_version() != ABI_VERSION:
        raise PhxError("libphx ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def check(ctx, rc: int, what: str):
    if rc != 0:
        msg = load().phx_last_error(ctx)
        raise PhxError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


class Context:
    """Owns one phx_ctx (one victim model on one device)."""

    def __init__(self, model_name="efficientdet-d0", image_size=0, max_batch=16,
                 bn_mode=BN_LOCAL, score_thresh=0.5, seed=0, device=0, compute_dtype=DTYPE_F32):
        lib = load()
        self.lib = lib
        cfg = _Config(model_name.encode(), int(image_size), int(max_batch), int(bn_mode),
                      float(score_thresh), int(seed) & ((1 << 64) - 1), int(compute_dtype))
        h = c_void_p()
        rc = lib.phx_create(ctypes.byref(cfg), int(device), ctypes.byref(h))
        if rc != 0:
            msg = lib.phx_last_error(None)
            raise PhxError(f"phx_create({model_name}) failed ({rc}): {msg.decode() if msg else ''}")
        self.h = h
        self.model_name = model_name
        self.max_batch = int(max_batch)
        self.image_size = lib.phx_image_size(h)
        self.num_anchors = lib.phx_num_anchors(h)

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.lib.phx_destroy(h)
            self.h = None

    def manifest(self):
        need = c_size_t()
        self.lib.phx_weight_manifest(self.h, None, 0, ctypes.byref(need))
        buf = ctypes.create_string_buffer(need.value)
        self.lib.phx_weight_manifest(self.h, buf, need.value, ctypes.byref(need))
        return json.loads(buf.value.decode())

    def model_info(self) -> dict:
        """The configuration the program was built from (hparams_config key names + fpn_nodes)."""
        need = c_size_t()
        self.lib.phx_model_info(self.h, None, 0, ctypes.byref(need))
        buf = ctypes.create_string_buffer(need.value)
        self.lib.phx_model_info(self.h, buf, need.value, ctypes.byref(need))
        return json.loads(buf.value.decode())

    def set_score_thresh(self, t: float):
        self.call("phx_set_score_thresh", float(t))

    def weight_count(self) -> int:
        return int(self.lib.phx_weight_count(self.h))

    def profile(self, enable: bool):
        self.lib.phx_profile(self.h, int(enable))

    def profile_report(self) -> dict:
        need = c_size_t()
        check(self.h, self.lib.phx_profile_report(self.h, None, 0, ctypes.byref(need)), "phx_profile_report")
        cap = need.value
        buf = ctypes.create_string_buffer(cap)
        check(self.h, self.lib.phx_profile_report(self.h, buf, cap, ctypes.byref(need)), "phx_profile_report")
        if need.value > cap:  # (a library without the size-query cache: the report grew)
            raise PhxError(f"phx_profile_report: {need.value} bytes needed, {cap} given")
        return json.loads(buf.value.decode())

    def workspace_bytes(self, batch: int) -> int:
        """Device bytes of the executor for `batch` images (builds it if needed)."""
        n = c_size_t(0)
        self.call("phx_workspace_bytes", int(batch), ctypes.byref(n))
        return int(n.value)

    def checksums(self, tag: int = 0) -> list:
        """PHX_CKSUM diagnostics: [(name, hash)] of the last step's writes, in launch order."""
        need = c_size_t()
        self.call("phx_debug_checksums", int(tag), None, 0, ctypes.byref(need))
        buf = ctypes.create_string_buffer(need.value)
        self.call("phx_debug_checksums", int(tag), buf, need.value, ctypes.byref(need))
        return [tuple(ln.split("\t")) for ln in buf.value.decode().splitlines() if ln]

    def call(self, name: str, *args):
        rc = getattr(self.lib, name)(self.h, *args)
        check(self.h, rc, name)


class Defender:
    """Owns one phx_def (the defender's U-Net + Masker) over a victim Context."""

    def __init__(self, ctx: Context, max_batch: int, seed: int = 0):
        self.lib = ctx.lib
        self.ctx = ctx  # keeps the victim alive
        h = c_void_p()
        rc = self.lib.phx_def_create(ctx.h, int(max_batch), int(seed) & ((1 << 64) - 1), ctypes.byref(h))
        if rc != 0:
            msg = self.lib.phx_def_last_error(None)
            raise PhxError(f"phx_def_create failed ({rc}): {msg.decode() if msg else ''}")
        self.h = h
        self.max_batch = int(max_batch)
        self.num_params = int(self.lib.phx_def_num_params(h))
        self.num_moving = int(self.lib.phx_def_num_moving(h))

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.lib.phx_def_destroy(h)
            self.h = None

    def manifest(self) -> dict:
        need = c_size_t()
        self.call("phx_def_manifest", None, 0, ctypes.byref(need))
        buf = ctypes.create_string_buffer(need.value)
        self.call("phx_def_manifest", buf, need.value, ctypes.byref(need))
        return json.loads(buf.value.decode())

    def call(self, name: str, *args):
        rc = getattr(self.lib, name)(self.h, *args)
        if rc != 0:
            msg = self.lib.phx_def_last_error(self.h)
            raise PhxError(f"{name} failed ({rc}): {msg.decode() if msg else ''}")
