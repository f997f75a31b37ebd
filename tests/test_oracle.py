"""CPU: the oracle against the committed golden vectors and against the TF op semantics it
restates (hand-derived cases)."""
import os

import numpy as np
import pytest
import torch

from oracle import eot, postprocess as pp, step as ST

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load_make_golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLD, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


def test_oracle_step_matches_golden():
    mg = _load_make_golden()
    g = np.load(os.path.join(GOLD, "d0_128_step.npz"))
    wd, imgs, patch, boxes = mg.case_inputs()
    c = mg.CASE
    r = ST.attack_step(wd, imgs, patch, c["scale"], boxes=boxes, seed=c["rng_seed"], step=c["step"],
                       image_size=c["image_size"])
    np.testing.assert_allclose(r["loss"], g["loss"], rtol=1e-9)
    np.testing.assert_allclose(r["m_raw"], g["m_raw"], rtol=1e-9)
    np.testing.assert_allclose(r["grad"][-1], g["dscale"], rtol=1e-9)
    blocks, idx, vals = mg.grad_summary(r["grad"])
    np.testing.assert_allclose(blocks, g["grad_blocks"], rtol=1e-7, atol=1e-14)
    np.testing.assert_allclose(vals, g["grad_vals"], rtol=1e-7, atol=1e-14)
    places = np.array([[p["ymin"], p["xmin"], p["ps"], p["diag"], int(p["valid"])] for pl in r["places"] for p in pl])
    np.testing.assert_array_equal(places, g["places"])


def test_soft_nms_golden():
    g = np.load(os.path.join(GOLD, "soft_nms.npz"))
    sel, ss = pp.soft_nms(g["boxes"], g["scores"], 100, 0.5, 0.25)
    np.testing.assert_array_equal(sel, g["sel"])
    np.testing.assert_array_equal(ss, g["sel_scores"])


def test_soft_nms_semantics():
    # disjoint boxes: nothing decays, selection in score order, ties -> lower index first
    bx = np.array([[0, 0, 10, 10], [20, 20, 30, 30], [40, 40, 50, 50]], np.float32)
    sel, ss = pp.soft_nms(bx, np.array([0.6, 0.9, 0.9], np.float32))
    assert sel.tolist() == [1, 2, 0]
    # identical box: iou = 1 -> score * exp(-0.5/0.25 * 1) = s * exp(-2)
    bx = np.array([[0, 0, 10, 10], [0, 0, 10, 10]], np.float32)
    sel, ss = pp.soft_nms(bx, np.array([0.95, 0.9], np.float32), score_threshold=0.1)
    assert sel.tolist() == [0, 1]
    np.testing.assert_allclose(ss[1], 0.9 * np.exp(-2.0), rtol=1e-6)
    # decayed below the threshold -> dropped; candidates must be strictly above the threshold
    sel, _ = pp.soft_nms(bx, np.array([0.95, 0.9], np.float32), score_threshold=0.5)
    assert sel.tolist() == [0]
    sel, _ = pp.soft_nms(bx[:1], np.array([0.5], np.float32), score_threshold=0.5)
    assert sel.tolist() == []
    # at most max_output_size
    bx = np.array([[i * 20, 0, i * 20 + 10, 10] for i in range(10)], np.float32)
    sel, _ = pp.soft_nms(bx, np.linspace(0.9, 0.6, 10).astype(np.float32), max_output_size=4)
    assert sel.tolist() == [0, 1, 2, 3]


def test_soft_nms_exact_duplicates_are_decayed_not_hard_suppressed():
    """postprocess.nms's gaussian branch passes iou_threshold = 1.0 to NonMaxSuppressionV5
    (postprocess.py:184-200).  TF's kernel (non_max_suppression_op.cc, DoNonMaxSuppressionOp)
    hard-suppresses only when soft_nms_sigma == 0 (`!is_soft_nms && similarity >
    similarity_threshold`); with sigma 0.25 every overlap, an exact duplicate at IoU 1.0 included,
    only scales the score by exp(-2 * iou^2) and the candidate is re-queued while above the
    threshold.  So at the NMS threshold 0.001 (score_thresh 0) duplicates are selected again with
    decayed scores, and at 0.5 they drop out."""
    bx = np.array([[0, 0, 10, 10]] * 3 + [[50, 50, 60, 60]], np.float32)
    sc = np.array([0.9, 0.8, 0.7, 0.6], np.float32)
    sel, ss = pp.soft_nms(bx, sc, 100, 0.001, 0.25)
    e2 = np.float32(np.exp(np.float32(-2.0)))
    assert sel.tolist() == [0, 3, 1, 2]
    np.testing.assert_array_equal(ss[1], sc[3])
    np.testing.assert_array_equal(ss[2], np.float32(sc[1] * e2))
    np.testing.assert_array_equal(ss[3], np.float32(np.float32(sc[2] * e2) * e2))
    sel, _ = pp.soft_nms(bx, sc, 100, 0.5, 0.25)
    assert sel.tolist() == [0, 3]


def test_valid_mask():
    bx = np.array([[0, 0, 20, 20], [0, 0, 5, 30], [-10, 0, 600, 20], [0, 0, 10, 10]], np.float32)
    m = pp.valid_mask(bx, 512, 512, np.array([0.9, 0.9, 0.9, 0.4], np.float32), 0.5)
    assert m.tolist() == [True, True, False, False]   # area 400 / 150 ok; h/H > 1; score < .5 & area 100


@pytest.mark.parametrize("ps", [3, 17, 200, 512, 640])
def test_resize_matrix_rows_normalised(ps):
    Wm = eot.resize_matrix(ps)
    np.testing.assert_allclose(Wm.sum(1), 1.0, rtol=2e-6)
    if ps == 640:
        np.testing.assert_array_equal(Wm, np.eye(640, dtype=np.float32))


def test_resize_gradient_is_exact_adjoint():
    Wm = torch.as_tensor(eot.resize_matrix(23).astype(np.float64))
    p = torch.randn(640, 640, 3, dtype=torch.float64, requires_grad=True)
    g = torch.randn(23, 23, 3, dtype=torch.float64)
    out = torch.einsum("iy,yxc,jx->ijc", Wm, p, Wm)
    (gp,) = torch.autograd.grad(out, p, g)
    np.testing.assert_allclose(gp.numpy(), torch.einsum("iy,ijc,jx->yxc", Wm, g, Wm).numpy(), rtol=1e-9, atol=1e-16)


def test_rotate_zero_angle_identity_and_tf_gradient_rule():
    img = torch.randn(31, 31, 3, dtype=torch.float64, requires_grad=True)
    out = eot.Rotate.apply(img, np.float32(0.0))
    np.testing.assert_allclose(out.detach().numpy(), img.detach().numpy(), atol=1e-12)
    # nonzero angle: gradient = inverse-transform warp of the upstream gradient with fill 0
    ang = np.float32(0.3)
    out = eot.Rotate.apply(img, ang)
    g = torch.randn_like(out)
    (gi,) = torch.autograd.grad(out, img, g)
    t = eot.rotate_transform(ang, 31)
    ref = eot.projective_bilinear(g, eot.inverse_transform(t), 0.0)
    np.testing.assert_allclose(gi.numpy(), ref.numpy(), rtol=1e-12)
    # inverse of the transform composes to identity
    a, b, tx, d, e, ty = t.astype(np.float64)
    M = np.array([[a, b, tx], [d, e, ty], [0, 0, 1]])
    ia, ib, itx, id_, ie, ity = eot.inverse_transform(t).astype(np.float64)
    Mi = np.array([[ia, ib, itx], [id_, ie, ity], [0, 0, 1]])
    np.testing.assert_allclose(M @ Mi, np.eye(3), atol=1e-6)


def test_brightness_matcher_on_reference_photos():
    """The reference's brightness-matcher test inputs (brightness_matcher.py:169-179): matching the
    day photo to the sunset photo transfers the Y mean when nothing clips."""
    ph = np.load(os.path.join(GOLD, "burj_khalifa_96.npz"))
    to_pm1 = lambda a: torch.as_tensor(a.astype(np.float64) / 127.0 - 1.0)
    src, tgt = to_pm1(ph["burj_khalifa_day"]), to_pm1(ph["burj_khalifa_sunset"])
    out = eot.brightness_match(src, tgt)
    Y = lambda x: (((x + 1.0) * float(np.float32(127 / 255))) @ eot.RGB2YUV)[..., 0]
    assert out.shape == src.shape
    assert float(out.min()) >= -1.0 - 1e-12 and float(out.max()) <= float(np.float32(255 / 127)) - 1 + 1e-9
    # Y mean moves from the source's towards the target's
    assert abs(float(Y(out).mean() - Y(tgt).mean())) < abs(float(Y(src).mean() - Y(tgt).mean()))


def test_placement_hand_computed():
    """Patcher.create for box [10,20,90,70], scale .4: ps = floor(80*.4) = 32, diag = int(32*sqrt 2) = 45."""
    p = eot.placement([10, 20, 90, 70], np.float32(0.4), 128, 128, 5, 3, 0, 0)
    assert (p["ps"], p["diag"], p["pad"], p["valid"]) == (32, 45, 6, True)
    assert 0 <= p["ymin"] <= 128 - 45 and 0 <= p["xmin"] <= 128 - 45
    # tiny box: ps*ps <= 4 -> dropped (attacker.py:391-394)
    assert not eot.placement([0, 0, 5, 5], np.float32(0.4), 128, 128, 5, 3, 0, 0)["valid"]
    # box larger than the image: diag capped by W, placement clamped inside
    p = eot.placement([0, 0, 128, 128], np.float32(1.0), 128, 128, 5, 3, 0, 1)
    assert p["diag"] == 128 and p["ymin"] == 0 and p["xmin"] == 0


def test_adam_reference_formula():
    p = np.array([0.5, -0.99, 0.2], np.float32)
    g = np.array([0.1, -0.2, 0.0], np.float32)
    out, m, v = ST.adam_clip(p, g, np.zeros(3, np.float32), np.zeros(3, np.float32), 1e-2, 1)
    # t=1: m = .1 g, v = .001 g^2, alpha = lr*sqrt(.001)/.1 -> step ~ lr * sign(g)
    np.testing.assert_allclose(out[:2], [0.5 - 0.01, -0.98], rtol=1e-5)
    assert out[2] == np.float32(0.2)   # scale slot untouched by a zero gradient, clip [0,1]


def test_drop_connect_draws():
    """Oracle drop connect (utils.py:329-344): per-image keep = floor(p + U) with the per-block
    survival p = 1 - 0.2*idx/N (efficientnet_model.py:752-755); the branch is x/p or exactly 0, and
    the two passes of a step draw independently."""
    import torch
    from oracle import detector as D
    det = D.Detector({}, "efficientdet-d1", 128, drop={"seed": 5, "step": 3, "gimg0": 0, "pass": 1})
    x = torch.ones(2, 4, 3, 3, dtype=torch.float64)
    y = det.drop_connect(x, 19, 23)  # both images dropped at step 3, pass 1 (see the GPU test)
    assert torch.equal(y, torch.zeros_like(x))
    p = float(np.float32(1.0 - 0.2 * 1 / 23))
    y = det.drop_connect(x, 1, 23)   # block 1 keeps both images
    assert torch.allclose(y, x / p)
    det.drop = {"seed": 5, "step": 3, "gimg0": 0, "pass": 0}
    assert torch.equal(det.drop_connect(x, 19, 23), x / float(np.float32(1.0 - 0.2 * 19 / 23)))
