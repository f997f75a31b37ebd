"""CPU, world size 2 over gloo: the data-parallel reduction used by PatchAttacker/bench
(mladversarialobjectdetection_amd.distributed) reproduces the single-process gradient of the
global batch (bn=local: per-shard statistics; TV once on rank 0; RNG keyed by global image)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

S = 64


def _case():
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd import weights as W
    man = _lib.Context("efficientdet-d0", S).manifest()
    wd = W.unpack(man, W.synthetic_blob(man, seed=0))
    imgs = np.random.default_rng(1).uniform(-1, 1, (2, S, S, 3)).astype(np.float32)
    patch = np.random.default_rng(7).uniform(-1, 1, (640, 640, 3)).astype(np.float32)
    boxes = [np.array([[4, 6, 50, 30]], np.float32), np.array([[10, 10, 60, 40]], np.float32)]
    return wd, imgs, patch, boxes


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from mladversarialobjectdetection_amd import distributed as ddp
    from oracle import step as ST
    wd, imgs, patch, boxes = _case()
    B = 1
    g0 = ddp.global_offset(B)
    r = ST.attack_step(wd, imgs[g0:g0 + B], patch, 0.4, boxes=boxes[g0:g0 + B], seed=5, step=2, gimg0=g0,
                       image_size=S, add_tv=(ddp.rank() == 0))
    grad = torch.as_tensor(r["grad"])
    ddp.allreduce_sum_(grad)
    if rank == 0:
        q.put((g0, grad.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gradient_equals_sum_of_shards():
    from oracle import step as ST
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    g0, reduced = q.get(timeout=600)
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    assert g0 == 0
    wd, imgs, patch, boxes = _case()
    ref = np.zeros_like(reduced)
    for b in range(2):
        r = ST.attack_step(wd, imgs[b:b + 1], patch, 0.4, boxes=boxes[b:b + 1], seed=5, step=2, gimg0=b,
                           image_size=S, add_tv=(b == 0))
        ref += r["grad"]
    np.testing.assert_allclose(reduced, ref, rtol=1e-10, atol=1e-15)


def test_metric_row_is_sum_reducible():
    """The metric row (phx.h PHX_M_*) of a global batch is the SUM of the per-rank rows: train_step
    all-reduces it together with the gradient (one collective), and _derive turns the sums into the
    reference's add_metric values (attacker.py:196-207) — mean / std over all images, ASR over all
    boxes, TV counted once (only rank 0 writes it)."""
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd.attacker import PatchAttacker
    m = np.array([[0.3, 0.1], [0.7, 0.2, 0.5]], dtype=object)
    rows = []
    for r, mb in enumerate(m):
        mb = np.asarray(mb, np.float64)
        row = np.zeros(_lib.NMETRIC + 1)
        row[_lib.M_SCALE_LOSS] = ((mb - 0.4) ** 2).sum()
        row[_lib.M_TV] = 123.0 if r == 0 else 0.0
        row[_lib.M_LOSS] = (mb ** 2).sum() + row[_lib.M_SCALE_LOSS] + 1e-5 * row[_lib.M_TV]
        row[_lib.M_SUM_M], row[_lib.M_SUM_M2] = mb.sum(), (mb ** 2).sum()
        row[_lib.M_ASR_NUM], row[_lib.M_ASR_DEN], row[_lib.M_NIMG] = r, 2 + r, len(mb)
        row[_lib.NMETRIC] = 0.4  # the replicated scale column is not summed
        rows.append(row)
    tot = rows[0] + rows[1]
    tot[_lib.NMETRIC] = 0.4
    d = PatchAttacker._derive(tot)
    allm = np.array([0.3, 0.1, 0.7, 0.2, 0.5])
    assert d["mean_max_score"] == pytest.approx(allm.mean())
    assert d["std_max_score"] == pytest.approx(allm.std())  # tf.math.reduce_std: population std
    assert d["tv_loss"] == 123.0
    assert d["asr"] == pytest.approx(1 - 4 / (20 + 1e-7))  # calc_asr counts 4 floats per box
    assert d["loss"] == pytest.approx((allm ** 2).sum() + ((allm - 0.4) ** 2).sum() + 1e-5 * 123)


def test_bn_sync_callback_contract():
    """bn=sync's collective (distributed.bn_sync_callback, registered through phx_set_allreduce):
    without a process group it is the identity and touches nothing; a failing collective is
    reported to the library as a non-zero return (the step then fails with a message), never
    raised through the C frame."""
    import ctypes

    from mladversarialobjectdetection_amd import distributed as D
    cb = D.bn_sync_callback()
    fn = ctypes.cast(cb, D.ALLREDUCE_FN)
    assert not dist.is_initialized()
    assert fn(None, None, 0, None) == 0
    # a world-1 group is still the identity; a failing collective (forced: a device view of a bogus
    # pointer on this CPU-only host) returns 1 instead of raising
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        assert fn(None, 64, 3, None) == 0
        real = D.is_dist
        D.is_dist = lambda: True
        try:
            assert fn(None, 64, 3, None) == 1
        finally:
            D.is_dist = real
    finally:
        dist.destroy_process_group()
