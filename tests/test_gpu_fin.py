"""In-launch BN finalize (GPU): a producer's last-arriving workgroup folds the BN partials itself
(common.hpp fin_arrive: write-through partial stores, an agent-scope ticket, one acquire) instead
of a k_bn_finalize launch.  The executor folds the BNs whose C * P <= PHX_FIN_MAX (default 0, off;
read per executor).  The fold adds the same fp64 partial sums in another order than the separate
launch, so the comparison is to rounding: loss, per-image max scores, the gradient and the moving
statistics of a D0 / D1 step with every eligible BN folded (PHX_FIN_MAX huge, so the multi-chunk
loads run too) against one with none (PHX_FIN_MAX=0); and the folded step is reproducible bit for
bit (the ticket's last arriver varies, the fold order does not).
"""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_boxes, synth_images  # noqa: E402

pytestmark = pytest.mark.gpu


def _step(monkeypatch, fin_max, model, S, B, repeat=1):
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    monkeypatch.setenv("PHX_FIN_MAX", str(fin_max))
    v = EfficientDetVictim(model, "synthetic", max_batch=B, rng_seed=5, image_size=S)
    att = PatchAttacker(v, seed=7)
    imgs = torch.as_tensor(synth_images(list(range(B)), S)).cuda()
    boxes = synth_boxes(list(range(B)), S)
    grads = []
    w_first = None
    for _ in range(repeat):
        att.cur_step = 3
        att.call(imgs, boxes=boxes)
        torch.cuda.synchronize()
        grads.append(att.grad.clone())
        if w_first is None:
            w_first = v.read_weights().copy()  # moving statistics after one step
    m = torch.empty(B, device="cuda")
    v.ctx.call("phx_debug_last_maxscores", m.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    out = (att.grad.cpu().numpy().astype(np.float64), att.metrics_buf.cpu().numpy().copy(), m.cpu().numpy(),
           w_first, grads)
    del att, v
    torch.cuda.empty_cache()
    return out


@pytest.mark.parametrize("model,S,B", [("efficientdet-d0", 256, 4), ("efficientdet-d1", 256, 2)])
def test_in_launch_finalize_matches_separate(monkeypatch, model, S, B):
    g1, m1, s1, w1, gs = _step(monkeypatch, 1 << 40, model, S, B, repeat=2)
    g0, m0, s0, w0, _ = _step(monkeypatch, 0, model, S, B)
    assert torch.equal(gs[0], gs[1])  # reproducible with the fold
    np.testing.assert_allclose(m1[0], m0[0], rtol=1e-5)
    np.testing.assert_allclose(s1, s0, rtol=5e-5, atol=1e-7)
    cos = float(g1 @ g0 / (np.linalg.norm(g1) * np.linalg.norm(g0)))
    assert cos >= 0.99999
    assert np.linalg.norm(g1 - g0) <= 1e-3 * np.linalg.norm(g0)
    assert abs(g1[-1] - g0[-1]) <= 1e-5 * abs(g0[-1])
    np.testing.assert_allclose(w1, w0, rtol=1e-4, atol=1e-6)
