"""GPU parity of the lite victims (the reference's default victim is efficientdet-lite4,
attacker_train.py:17): relu6 everywhere (Relu6Grad on the open interval), no SE, unscaled stem and
first/last block rows, BiFPN 'sum' fuse, mean/std 127/128, anchor scale 3 (lite0-2) or 4 (lite3-4),
drop connect with survival 0.8 (efficientnet_lite_builder.py:54-79, hparams_config.py:392-467).

Tolerance.  With synthetic weights the lite victims are numerically ill-conditioned in training-mode
BN: relu6 makes many activations exactly 0, so at the coarse pyramid levels whole BN channels are
nearly constant and each such BN multiplies rounding noise by up to 1/sqrt(eps) = 31.6.  The fp64
oracle evaluated in fp32 (same algorithm, PyTorch-CPU) already deviates from itself in fp64 by
1e-3 .. 1e-2 (lite4) in scores and gradients, so a fixed fp32-vs-fp64 bound would either fail a
correct kernel or be meaningless.  The bound is therefore relative to that intrinsic precision:
the GPU's deviation from fp64 must be within 4x the fp32 restatement's own deviation for scores and
loss, and within 16x for d patch (plus the D0 floors: scores 2e-5, loss 1e-5, d patch 1e-3 /
cosine 0.99999).  The gradient gets the wider factor because its error is dominated by discrete
events whose count grows with the rounding noise — relu6 kinks and max-pool taps whose order
flips — and the device's transcendentals (v_exp / v_rcp, 1 ulp) round differently from the CPU's;
measured: lite0 320^2 9x (3.7e-2 vs 4.2e-3), D4 256^2 4.1x (1.0e-2 vs 2.5e-3).  A real defect (a
wrong activation, fuse rule or gradient path) gives O(1) relative errors, far above these bounds.
Sizes: lite0 at its native 320^2, lite4 at 384^2 (P7 3x3: BN over 18 rows instead of 2).

lite4's gradient is not compared under this relative bound (at 8.8 % intrinsic deviation it would
admit almost anything); test_lite4_640_well_conditioned_step_matches_oracle checks it at a
well-conditioned point with a fixed tolerance instead.
"""
import numpy as np
import pytest
import torch

from bench import synth_boxes, synth_images

pytestmark = pytest.mark.gpu

# + EfficientDet-D4 (BASELINE config 4's victim, b4 backbone with drop connect, 224-channel BiFPN) at
# 256^2, compared the same way (its fp32 restatement deviates ~1e-4 in scores at this size)
CASES = [("efficientdet-lite0", 320), ("efficientdet-lite4", 384), ("efficientdet-d4", 256)]


def _victim(model, S):
    from mladversarialobjectdetection_amd import weights as W
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim
    v = EfficientDetVictim(model, "synthetic", seed=0, image_size=S, max_batch=2, rng_seed=5)
    return v, W.unpack(v.manifest, v.blob.copy())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,S", CASES)
def test_lite_detect_matches_oracle(model, S):
    from oracle import detector as D
    v, wd = _victim(model, S)
    imgs = synth_images([0, 1], S)
    _, scores, classes = v.detect(torch.as_tensor(imgs).cuda())
    torch.set_num_threads(16)
    ref = {}
    for dt in (torch.float64, torch.float32):
        # phx_detect keys drop connect as pass 2 (standalone detect), step 0, images 0..B-1
        det = D.Detector(wd, model, S, dtype=dt, drop=dict(seed=5, step=0, gimg0=0, **{"pass": 2}))
        with torch.no_grad():
            rs, rc, _ = D.pre_nms(*det(torch.as_tensor(imgs, dtype=dt)), S, D.MODELS[model]["anchor_scale"])
        ref[dt] = (rs.double().numpy(), rc.numpy())
    s64, c64 = ref[torch.float64]
    e32 = np.abs(ref[torch.float32][0] - s64).max()
    egpu = np.abs(scores.cpu().numpy() - s64).max()
    assert egpu <= max(2e-5, 4 * e32), (egpu, e32)
    assert (classes.cpu().numpy() == c64).mean() >= 0.995


@pytest.mark.timeout(600)
@pytest.mark.parametrize("model,S", [c for c in CASES if c[0] != "efficientdet-lite4"])
def test_lite_step_matches_oracle(model, S):
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd.attacker import PatchAttacker
    from oracle import step as ST
    v, wd = _victim(model, S)
    imgs = synth_images([0, 1], S)
    boxes = synth_boxes([0, 1], S)
    att = PatchAttacker(v, seed=7)
    att.cur_step = 3
    att.call(torch.as_tensor(imgs).cuda(), boxes=boxes)
    g = att.grad.cpu().numpy().astype(np.float64)
    met = att.metrics_buf.cpu().numpy()
    torch.set_num_threads(16)
    ref = {dt: ST.attack_step(wd, imgs, att.patch.cpu().numpy(), np.float32(0.4), boxes=boxes, seed=5, step=3,
                              model=model, image_size=S, dtype=dt) for dt in (torch.float64, torch.float32)}
    r64, r32 = ref[torch.float64], ref[torch.float32]

    def rel(a, b):
        return float(np.linalg.norm(a - b) / np.linalg.norm(b))

    def cos(a, b):
        return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))

    le32 = abs(r32["loss"] - r64["loss"]) / abs(r64["loss"])
    assert abs(met[_lib.M_LOSS] - r64["loss"]) / abs(r64["loss"]) <= max(1e-5, 4 * le32)
    gp, rp, p32 = g[:-1], r64["grad"][:-1], r32["grad"][:-1]
    assert rel(gp, rp) <= max(1e-3, 16 * rel(p32, rp)), (rel(gp, rp), rel(p32, rp))
    assert 1 - cos(gp, rp) <= max(1e-5, 256 * (1 - cos(p32, rp))), (cos(gp, rp), cos(p32, rp))
    assert abs(g[-1] - r64["grad"][-1]) <= max(1e-5, 4 * abs(r32["grad"][-1] - r64["grad"][-1])) * max(
        1.0, abs(r64["grad"][-1]))
    assert met[_lib.M_NBOX] == r64["nbox"] and met[_lib.M_NIMG] == 2


@pytest.mark.timeout(900)
def test_lite4_640_well_conditioned_step_matches_oracle():
    """The reference's default victim (efficientdet-lite4, attacker_train.py:17) at its native
    640^2 (hparams_config.py:457-467), at a well-conditioned point, against the fp64
    oracle with fixed tolerances: loss rel <= 1e-5, d scale rel <= 1e-5, d patch rel <= 1e-3 and
    cosine >= 0.99999.

    Why the point is chosen.  With SURVEY 8d's BN draw (gamma U(0.5, 1.5), beta N(0, 0.1)) half of
    every relu6 input sits near the kink at 0; the ~1e-3 forward rounding noise the 7-cell BiFPN
    accumulates then flips relu6 masks next to the loss anchor, where the backward support is a few
    hundred values, and the fp32 restatement itself deviates 8.8 % from fp64 in d patch (measured at
    640^2 and 384^2) — no fixed bound can tell a correct kernel from a wrong one there.  With gamma
    U(0.2, 0.4) and beta N(1, 0.1) relu6 inputs sit 2.5-6 sigma inside (0, 6), so masks do not flip;
    a person prior of 3 keeps the seed 4 m - 2 s away from 0.  The fp32 restatement then deviates
    6.9e-6 from fp64 (measured at 640^2 with 4 images; 2 here keep the fp64 oracle near a minute), so 1e-3 leaves two orders of margin while any
    wrong activation, fuse, drop-connect or gradient path gives O(1) errors.  The standard draw's
    relu6 kinks are still exercised by the lite0 case above."""
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd import weights as W
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    from oracle import step as ST
    model, S, B = "efficientdet-lite4", 640, 2
    v = EfficientDetVictim(model, W.synthetic_blob(
        _lib.Context(model, S, 1).manifest(), seed=0, person_bias=3.0, gamma=(0.2, 0.4), beta=(1.0, 0.1)),
        image_size=S, max_batch=B, rng_seed=5)
    wd = W.unpack(v.manifest, v.blob.copy())
    imgs = synth_images(list(range(B)), S)
    boxes = synth_boxes(list(range(B)), S)
    att = PatchAttacker(v, seed=7)
    att.cur_step = 3
    att.call(torch.as_tensor(imgs).cuda(), boxes=boxes)
    g = att.grad.cpu().numpy().astype(np.float64)
    met = att.metrics_buf.cpu().numpy()
    torch.set_num_threads(16)
    r64 = ST.attack_step(wd, imgs, att.patch.cpu().numpy(), np.float32(0.4), boxes=boxes, seed=5, step=3,
                         model=model, image_size=S)
    gp, rp = g[:-1], r64["grad"][:-1]
    rel = float(np.linalg.norm(gp - rp) / np.linalg.norm(rp))
    cos = float(gp @ rp / (np.linalg.norm(gp) * np.linalg.norm(rp)))
    assert abs(met[_lib.M_LOSS] - r64["loss"]) <= 1e-5 * abs(r64["loss"])
    assert abs(g[-1] - r64["grad"][-1]) <= 1e-5 * max(1.0, abs(r64["grad"][-1]))
    assert rel <= 1e-3, rel
    assert cos >= 0.99999, cos
    assert met[_lib.M_NBOX] == r64["nbox"] and met[_lib.M_NIMG] == B
    np.testing.assert_allclose(met[_lib.M_SUM_M], r64["m"].sum(), rtol=1e-5)
