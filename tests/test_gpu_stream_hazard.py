"""Stream-hazard checker (GPU): the concurrent step against the one-stream step, launch by launch.

With PHX_CKSUM=1 every phx_step_grad hashes each tensor and statistics slot an op writes, on that
op's stream right after the op, and once more after the side stream has joined ("post" entries).
A cross-stream hazard — a side-pass launch writing what a main-pass launch reads or writes, or a
kernel whose result depends on what shares its CU — shows up as a launch whose hash differs from the
one-stream step's on the same inputs, or as a tensor whose hash changed after its producer.

Round 4 masked a C4 failure of this kind by forking the side pass late; scripts/diag_cksum.py
named the launch (the bf16 residual add, 16-lane groups of stale v_pk_add_f32 high halves while the
CU was shared) and the library is now built without packed-FP32 instructions (csrc/Makefile NOPK).
These cases fork at stage 6 again, for C2 (D0 512^2 x 16 fp32) and C4 (D4 1024^2 x 4 bf16), plus
the D0 bf16 1024^2 x 4 step that failed every time before the fix.
"""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_boxes, synth_images  # noqa: E402

pytestmark = pytest.mark.gpu


def _check(monkeypatch, model, S, B, dtype, weights, n_conc):
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    monkeypatch.setenv("PHX_CKSUM", "1")
    imgs = torch.as_tensor(synth_images(list(range(B)), S)).cuda()
    boxes = synth_boxes(list(range(B)), S)
    v = EfficientDetVictim(model, weights, max_batch=B, rng_seed=5, dtype=dtype, image_size=S)
    att = PatchAttacker(v, seed=7)

    def step(conc):
        monkeypatch.setenv("PHX_CONC", "1" if conc else "0")
        att.cur_step = 3
        att.call(imgs, boxes=boxes)
        torch.cuda.synchronize()
        ck = v.ctx.checksums(0) + (v.ctx.checksums(1) if conc else [])
        return ck, att.grad.clone()

    def changed_later(ck):
        post = {n[5:]: h for n, h in ck if n.startswith("post ")}
        return [n for n, h in ck if n in post and post[n] != h]

    ref, g0 = step(False)
    assert len(ref) > 500 and not changed_later(ref)
    rd = dict(ref)
    for k in range(n_conc):
        got, g = step(True)
        common = [(n, h) for n, h in got if n in rd]
        # every second-pass and backward launch, and the first pass's (on the side executor)
        assert len(common) >= len(ref) - 8, (len(common), len(ref))
        diffs = [n for n, h in common if rd[n] != h]
        assert not diffs, f"concurrent step {k}: {len(diffs)} launches differ, first {diffs[:3]}"
        assert not changed_later(got), f"concurrent step {k}: tensors rewritten after their producer"
        assert torch.equal(g, g0)
    del att, v
    torch.cuda.empty_cache()


def test_stream_hazard_c2(monkeypatch):
    _check(monkeypatch, "efficientdet-d0", 512, 16, "f32", "synthetic", 4)


def test_stream_hazard_c4(monkeypatch):
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd import weights as W
    wts = W.well_conditioned_blob(_lib.Context("efficientdet-d4", 1024, 1).manifest())
    _check(monkeypatch, "efficientdet-d4", 1024, 4, "bf16", wts, 6)


def test_stream_hazard_d0_bf16_1024(monkeypatch):
    _check(monkeypatch, "efficientdet-d0", 1024, 4, "bf16", "synthetic", 6)
