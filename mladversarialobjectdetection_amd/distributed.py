"""Data parallelism for the attack step.

One process per GPU (torchrun; backend "nccl" = RCCL over xGMI on ROCm, "gloo" on CPU for tests).
The global batch is split contiguously: rank r holds global images [r*B, (r+1)*B), which also keys
the EOT RNG, so every image sees the same random draws at any GPU count.  Exactly one exchange per
step: a SUM all-reduce of the contiguous [d patch | d scale | metric row] buffer (4.9 MB) between
the victim dgrad and the Adam update; the 1e-5*TV term (and its metric) is added by rank 0 only, so
the reduced gradient equals the sum of per-shard reference gradients (bn=local: BN statistics per
shard), and reading the metrics issues no further collective.  The defender reduces
[d U-Net variables | loss] the same way.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def global_offset(local_batch: int) -> int:
    """First global image index of this rank's shard."""
    return rank() * local_batch


def allreduce_sum_(t: torch.Tensor) -> torch.Tensor:
    """In-place SUM over ranks (no-op at world size 1)."""
    if is_dist():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


class _CudaBuf:
    """A device buffer of the library seen as a torch tensor (__cuda_array_interface__)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (ptr, False), "version": 2,
                                         "strides": None}


ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


def bn_sync_callback():
    """The phx_allreduce_fn of bn=sync: SUM all-reduce of the library's fp64 BN sums over the process
    group, issued on the library's stream `stream` (phx.h: the callback is ordered on it).  The
    collective runs under that stream as torch's current stream, so RCCL orders it after the fold
    kernel that wrote the sums and before the kernel that reads them, whatever stream the caller
    made current; gloo reduces through the host and returns when done.  A no-op at world size 1.
    Errors are reported to the library as a non-zero return (the step then fails with a message)."""

    def fn(user, ptr, n, stream):
        try:
            if is_dist():
                t = torch.as_tensor(_CudaBuf(int(ptr), int(n)), device="cuda")
                if stream:
                    with torch.cuda.stream(torch.cuda.ExternalStream(int(stream), device=t.device)):
                        dist.all_reduce(t, op=dist.ReduceOp.SUM)
                else:
                    dist.all_reduce(t, op=dist.ReduceOp.SUM)
            return 0
        except Exception as e:  # noqa: BLE001 — surfaced through the library's return code
            import sys
            print(f"bn=sync all-reduce failed: {e!r}", file=sys.stderr)
            return 1

    return ALLREDUCE_FN(fn)


def init_from_env(backend: str | None = None):
    """Initialise the process group from torchrun's env (MASTER_ADDR must be 127.0.0.1 here)."""
    if not dist.is_available() or dist.is_initialized():
        return
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return
    if backend is None:
        # PHX_DIST_BACKEND=gloo: CUDA tensors reduced through the host (tests / one-GPU rehearsals)
        backend = os.environ.get("PHX_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
