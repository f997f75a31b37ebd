"""GPU: the concurrent first pass of phx_step_grad.  With injected placement boxes the first (clean)
pass only feeds the ASR denominator and the moving statistics, so the library runs it on a second
stream beside the second pass and the backward (its own executor), deferring both passes'
moving-statistics updates and applying them in pass order after the join.  The result must equal
the one-stream order (PHX_CONC=0) bit for bit: gradient, parameters after Adam, the metric row and
the moving statistics after two steps — with and without drop connect (D1 draws per-pass masks).
The second pass's soft-NMS (ASR numerator) also runs on the side stream, in both placement flows."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(B, S):
    rng = np.random.default_rng(3)
    imgs = rng.uniform(-1, 1, (B, S, S, 3)).astype(np.float32)
    boxes = [np.array([[8 + 4 * b, 10, S * 0.6, S * 0.5]], np.float32) for b in range(B)]
    boxes[1] = np.array([[5, 5, S - 9, S // 2], [S // 3, S // 4, S - 20, S - 30]], np.float32)
    return imgs, boxes


def _run(conc, model, B, S, person_bias=0.0, inject=True):
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    old = os.environ.get("PHX_CONC")
    os.environ["PHX_CONC"] = "1" if conc else "0"
    try:
        v = EfficientDetVictim(model, "synthetic", seed=0, image_size=S, max_batch=B, rng_seed=5,
                               person_bias=person_bias)
        att = PatchAttacker(v, seed=7)
        imgs, boxes = _case(B, S)
        x = torch.as_tensor(imgs).cuda()
        rows = []
        for _ in range(2):
            att.train_step(x, boxes=boxes if inject else None)
            torch.cuda.synchronize()
            rows.append(att.metrics_buf.cpu().numpy().copy())
        return (att.grad.cpu().numpy().copy(), att.params.cpu().numpy().copy(), np.stack(rows),
                v.read_weights().copy(), v.ctx.workspace_bytes(B))
    finally:
        if old is None:
            os.environ.pop("PHX_CONC", None)
        else:
            os.environ["PHX_CONC"] = old


@pytest.mark.parametrize("model,S,B,pb", [("efficientdet-d0", 256, 4, 4.0), ("efficientdet-d1", 256, 3, 0.0)])
def test_concurrent_first_pass_equals_one_stream(model, S, B, pb):
    from mladversarialobjectdetection_amd import _lib
    g1, p1, m1, w1, ws1 = _run(False, model, B, S, pb)
    g2, p2, m2, w2, ws2 = _run(True, model, B, S, pb)
    assert np.isfinite(g1).all()
    assert np.array_equal(g1, g2)
    assert np.array_equal(p1, p2)
    assert np.array_equal(m1, m2)
    assert np.array_equal(w1, w2)  # moving statistics: both passes applied in pass order
    assert ws2 > ws1  # the first pass's own executor
    if pb:
        assert m2[:, _lib.M_ASR_DEN].min() > 0  # the first pass's metric (run on the side stream) is live


def test_side_stream_soft_nms_with_first_pass_placement():
    """boxes=None (the reference's flow): the first pass feeds the placement, so it stays on the
    step's stream; only the second pass's soft-NMS (the ASR numerator) runs beside the backward."""
    from mladversarialobjectdetection_amd import _lib
    g1, p1, m1, w1, _ = _run(False, "efficientdet-d0", 4, 256, 4.0, inject=False)
    g2, p2, m2, w2, _ = _run(True, "efficientdet-d0", 4, 256, 4.0, inject=False)
    assert np.array_equal(g1, g2) and np.array_equal(p1, p2) and np.array_equal(w1, w2)
    assert np.array_equal(m1, m2)
    assert m2[:, _lib.M_NBOX].min() > 0 and m2[:, _lib.M_ASR_NUM].max() > 0


@pytest.mark.parametrize("model,S,B,pb", [("efficientdet-d0", 256, 4, 4.0), ("efficientdet-d1", 256, 3, 4.0)])
def test_first_pass_prefetch_equals_in_step(model, S, B, pb):
    """train_step(next_inputs=...) with first-pass placement (phx_set_next): the next batch's first pass
    runs on its own stream beside the current step's second pass and backward, with its moving-statistics
    updates deferred to the step that uses it.  Three steps over three batches equal the in-step
    order bit for bit: per-step gradient and metric row (placement boxes, ASR denominator), the patch
    after Adam and the moving statistics — with drop connect (D1) keyed by the next step."""
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    rng = np.random.default_rng(9)
    xs = [torch.as_tensor(rng.uniform(-1, 1, (B, S, S, 3)).astype(np.float32)).cuda() for _ in range(3)]
    out = []
    for pf in (False, True):
        v = EfficientDetVictim(model, "synthetic", seed=0, image_size=S, max_batch=B, rng_seed=5, person_bias=pb)
        att = PatchAttacker(v, seed=7)
        grads, rows = [], []
        for k in range(3):
            att.train_step(xs[k], next_inputs=xs[k + 1] if pf and k < 2 else None)
            torch.cuda.synchronize()
            grads.append(att.grad.cpu().numpy().copy())
            rows.append(att.metrics_buf.cpu().numpy().copy())
        out.append((np.stack(grads), np.stack(rows), att.params.cpu().numpy().copy(), v.read_weights().copy()))
    (g1, m1, p1, w1), (g2, m2, p2, w2) = out
    assert np.isfinite(g1).all()
    assert np.array_equal(g1, g2)
    assert np.array_equal(m1, m2)
    assert np.array_equal(p1, p2)
    assert np.array_equal(w1, w2)
    assert m2[:, _lib.M_NBOX].min() > 0 and m2[:, _lib.M_ASR_DEN].min() > 0


def test_first_pass_prefetch_mismatch_and_weight_load():
    """A prefetched first pass is used only by the step for exactly its batch: a step on other images
    computes its own first pass (same result as without any prefetch), and a weight load in between
    drops the prefetch (the next step's first pass then sees the new weights)."""
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    B, S = 2, 256
    rng = np.random.default_rng(11)
    xs = [torch.as_tensor(rng.uniform(-1, 1, (B, S, S, 3)).astype(np.float32)).cuda() for _ in range(3)]

    def run(seq, reload=False):
        v = EfficientDetVictim("efficientdet-d0", "synthetic", seed=0, image_size=S, max_batch=B, rng_seed=5,
                               person_bias=4.0)
        att = PatchAttacker(v, seed=7)
        out = []
        for k, (x, nx) in enumerate(seq):
            if reload and k == 1:
                w = v.read_weights().copy()
                w[: w.size // 2] *= np.float32(0.5)  # other weights, so a stale first pass would show
                v.load_weights(w)
            att.train_step(xs[x], next_inputs=None if nx is None else xs[nx])
            torch.cuda.synchronize()
            out.append((att.grad.cpu().numpy().copy(), att.metrics_buf.cpu().numpy().copy()))
        return out

    ref = run([(0, None), (2, None)])
    got = run([(0, 1), (2, None)])  # prefetched batch 1, then stepped on batch 2
    for (g1, m1), (g2, m2) in zip(ref, got):
        assert np.array_equal(g1, g2) and np.array_equal(m1, m2)
    ref = run([(0, None), (1, None)], reload=True)
    got = run([(0, 1), (1, None)], reload=True)  # the reload drops the prefetch of batch 1
    for (g1, m1), (g2, m2) in zip(ref, got):
        assert np.array_equal(g1, g2) and np.array_equal(m1, m2)


def test_first_pass_prefetch_refilled_buffer():
    """The pinned-ring pattern: the caller hands the next batch's device buffer to train_step, then
    refills that same buffer in place with another batch before the next step.  The prefetched first
    pass read the old contents, so train_step withdraws it (the tensor's version counter moved) and
    the step equals the no-prefetch step on the new contents bit for bit."""
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    B, S = 2, 256
    rng = np.random.default_rng(12)
    xs = [torch.as_tensor(rng.uniform(-1, 1, (B, S, S, 3)).astype(np.float32)).cuda() for _ in range(3)]

    def run(prefetch):
        v = EfficientDetVictim("efficientdet-d0", "synthetic", seed=0, image_size=S, max_batch=B, rng_seed=5,
                               person_bias=4.0)
        att = PatchAttacker(v, seed=7)
        ring = xs[1].clone()
        att.train_step(xs[0], next_inputs=ring if prefetch else None)
        ring.copy_(xs[2])  # refilled in place: the prefetched pass saw xs[1]
        att.train_step(ring)
        torch.cuda.synchronize()
        return att.grad.cpu().numpy().copy(), att.metrics_buf.cpu().numpy().copy()

    g1, m1 = run(False)
    g2, m2 = run(True)
    assert np.array_equal(g1, g2) and np.array_equal(m1, m2)
