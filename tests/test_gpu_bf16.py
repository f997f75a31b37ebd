"""GPU parity of the bf16 compute mode (PHX_DTYPE_BF16, BASELINE config 4 "bf16"): every 1x1 conv
with more than 16 output channels (and every data gradient with more than 16 input channels) runs on
v_mfma_f32_32x32x16_bf16 with its operands rounded to bf16 and fp32 accumulation; BN statistics,
depthwise convs, EOT, loss and the patch gradient stay fp32.

Two references:
  * the fp64 oracle (the reference's arithmetic): SURVEY.md 8c's C4 tolerance — loss rel <= 1e-2,
    d patch cosine >= 0.99;
  * the fp64 oracle with the same bf16 rounding points (oracle.detector.Bf16Conv1x1).  Layer by
    layer, where both sides still have fp32-exact inputs (the first bf16 convs), the GPU's outputs
    must equal the emulation 20x more closely than the emulation equals fp64 — this pins which
    operands are rounded.  Deeper, bf16 noise (~2^-9) is amplified like any perturbation of this
    synthetic-weight net (training-mode BN over a 2-image batch, P7 over 2 rows; max-pool and class
    maxima whose top taps are that close resolve differently in any two bf16 evaluations), so the
    end results are held to the same order as the bf16 arithmetic's own deviation from fp64: loss
    rel <= 1e-4, ||d - d_emul|| <= 2 ||d_emul - d_fp64||, cosine >= 0.99.
"""
import numpy as np
import pytest
import torch

from bench import synth_boxes, synth_images

pytestmark = pytest.mark.gpu

S = 128


def _rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def _cos(a, b):
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))


def test_bf16_gemm_rounding_points_match_emulation():
    """The first 1x1 convs of the second pass, whose inputs are still fp32-exact on both sides: the
    GPU's conv outputs (BN inputs, read back through phx_debug_tap) equal the emulated bf16
    arithmetic far more closely than that arithmetic equals fp64.  blocks_0's project conv (16
    outputs) runs on the fp32 register kernel, so there GPU and fp64 agree to fp32 precision."""
    from mladversarialobjectdetection_amd import weights as W
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    from oracle import detector as D
    from oracle import step as ST
    v = EfficientDetVictim("efficientdet-d0", "synthetic", seed=0, image_size=S, max_batch=2, rng_seed=5,
                           dtype="bf16")
    wd = W.unpack(v.manifest, v.blob.copy())
    imgs = np.random.default_rng(2).uniform(-1, 1, (2, S, S, 3)).astype(np.float32)
    boxes = [np.array([[10, 20, 90, 70]], np.float32), np.array([[5, 5, 120, 60]], np.float32)]
    att = PatchAttacker(v, seed=7)
    att.cur_step = 1
    att.call(torch.as_tensor(imgs).cuda(), boxes=boxes)
    taps = {}
    for bf in (False, True):
        orig = D.Detector.__init__

        def init(self, *a, **k):
            orig(self, *a, **k)
            self.taps = {}
        D.Detector.__init__ = init
        try:
            r = ST.attack_step(wd, imgs, att.patch.cpu().numpy(), np.float32(0.4), boxes=boxes, seed=5, step=1,
                               image_size=S, bf16=bf)
        finally:
            D.Detector.__init__ = orig
        taps[bf] = r["det"].taps
    b0 = "efficientnet-b0/blocks_0/tpu_batch_normalization_1"
    for name, bf_layer in ((b0, False), ("efficientnet-b0/blocks_1/tpu_batch_normalization", True),
                           ("efficientnet-b0/blocks_1/tpu_batch_normalization_2", True)):
        x_emul = taps[True][name][0].detach().permute(0, 2, 3, 1).numpy()
        x_64 = taps[False][name][0].detach().permute(0, 2, 3, 1).numpy()
        buf = torch.empty(x_emul.size, device="cuda")
        v.ctx.call("phx_debug_tap", name.encode(), 0, buf.data_ptr(), buf.numel(),
                   torch.cuda.current_stream().cuda_stream)
        x_gpu = buf.cpu().numpy().reshape(x_emul.shape).astype(np.float64)
        e_gpu, e_emul = _rel(x_gpu, x_emul), _rel(x_emul, x_64)
        if bf_layer:
            assert e_emul > 1e-4, (name, e_emul)  # visibly bf16
            assert e_gpu <= 0.05 * e_emul, (name, e_gpu, e_emul)
        else:
            assert e_emul == 0.0 and e_gpu <= 1e-5, (name, e_gpu)


def test_bf16_step_matches_oracle():
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd import weights as W
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    from oracle import step as ST
    v = EfficientDetVictim("efficientdet-d0", "synthetic", seed=0, image_size=S, max_batch=2, rng_seed=5,
                           dtype="bf16")
    assert v.ctx.model_info()["compute_dtype"] == "bf16"
    wd = W.unpack(v.manifest, v.blob.copy())
    imgs = np.random.default_rng(1).uniform(-1, 1, (2, S, S, 3)).astype(np.float32)
    boxes = [np.array([[10, 20, 90, 70]], np.float32),
             np.array([[5, 5, 120, 60], [30, 40, 100, 110]], np.float32)]
    att = PatchAttacker(v, seed=7)
    att.cur_step = 3
    att.call(torch.as_tensor(imgs).cuda(), boxes=boxes)
    g = att.grad.cpu().numpy().astype(np.float64)
    loss = float(att.metrics_buf.cpu().numpy()[_lib.M_LOSS])
    kw = dict(boxes=boxes, seed=5, step=3, image_size=S)
    r64 = ST.attack_step(wd, imgs, att.patch.cpu().numpy(), np.float32(0.4), **kw)
    rem = ST.attack_step(wd, imgs, att.patch.cpu().numpy(), np.float32(0.4), bf16=True, **kw)
    gp = g[:-1]
    # against the reference's arithmetic
    assert abs(loss - r64["loss"]) <= 1e-2 * abs(r64["loss"])
    assert _cos(gp, r64["grad"][:-1]) >= 0.99
    # against the same bf16 rounding points
    assert abs(loss - rem["loss"]) <= 1e-4 * abs(rem["loss"])
    e_gpu, e_emul = _rel(gp, rem["grad"][:-1]), _rel(rem["grad"][:-1], r64["grad"][:-1])
    assert e_gpu <= 2 * e_emul, (e_gpu, e_emul)
    assert _cos(gp, rem["grad"][:-1]) >= 0.99


def _well_conditioned_d4(S):
    """D4 weights at a well-conditioned point.  With SURVEY 8d's BN draw (gamma U(0.5, 1.5), beta
    N(0, 0.1)) the bf16 arithmetic itself is chaotic on synthetic D4 weights: the oracle's exact bf16
    emulation deviates from fp64 with d patch cosine 0.06 and max scores 0.53 -> 0.30 at 256^2
    (measured) — BN over 8 rows at P7 and 7 BiFPN cells amplify bf16's 2^-9 rounding to O(1), so no
    tolerance could separate a right kernel from a wrong one.  With gamma U(0.2, 0.4), beta N(1, 0.1)
    and a person prior of 3 the emulation deviates 4.8e-5 in loss and 1.9e-3 in d patch (cosine
    0.999998): there the C4 tolerance constrains the result."""
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd import weights as W
    return W.synthetic_blob(_lib.Context("efficientdet-d4", S, 1).manifest(), seed=0, person_bias=3.0,
                            gamma=(0.2, 0.4), beta=(1.0, 0.1))


@pytest.mark.timeout(900)
def test_bf16_d4_256_matches_emulation_oracle():
    """BASELINE C4's victim (EfficientDet-D4: b4 backbone with drop connect, 224-channel BiFPN x7)
    in bf16 against the fp64 oracle with and without the product's bf16 rounding points, at 256^2
    (the largest size whose fp64 oracle finishes in about a minute) and a well-conditioned weight
    draw.  SURVEY 8c's C4 tolerance vs fp64 (loss rel <= 1e-2, cosine >= 0.99), and against the
    emulation the same as D0's above."""
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd import weights as W
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    from oracle import step as ST
    S4 = 256
    v = EfficientDetVictim("efficientdet-d4", _well_conditioned_d4(S4), image_size=S4, max_batch=2, rng_seed=5,
                           dtype="bf16")
    wd = W.unpack(v.manifest, v.blob.copy())
    imgs = synth_images([0, 1], S4)
    boxes = synth_boxes([0, 1], S4)
    att = PatchAttacker(v, seed=7)
    att.cur_step = 3
    att.call(torch.as_tensor(imgs).cuda(), boxes=boxes)
    g = att.grad.cpu().numpy().astype(np.float64)
    loss = float(att.metrics_buf.cpu().numpy()[_lib.M_LOSS])
    torch.set_num_threads(16)
    kw = dict(boxes=boxes, seed=5, step=3, image_size=S4, model="efficientdet-d4")
    r64 = ST.attack_step(wd, imgs, att.patch.cpu().numpy(), np.float32(0.4), **kw)
    rem = ST.attack_step(wd, imgs, att.patch.cpu().numpy(), np.float32(0.4), bf16=True, **kw)
    gp = g[:-1]
    assert abs(loss - r64["loss"]) <= 1e-2 * abs(r64["loss"])
    assert _cos(gp, r64["grad"][:-1]) >= 0.99
    assert abs(loss - rem["loss"]) <= 1e-4 * abs(rem["loss"])
    e_gpu, e_emul = _rel(gp, rem["grad"][:-1]), _rel(rem["grad"][:-1], r64["grad"][:-1])
    assert e_gpu <= 2 * e_emul, (e_gpu, e_emul)
    assert _cos(gp, rem["grad"][:-1]) >= 0.99


@pytest.mark.timeout(600)
def test_bf16_d4_1024_four_images():
    """C4's model, size and per-GPU batch (D4 1024^2, 4 images, bf16): finite and non-trivial,
    bit-identical on rerun (step and detector), and the step agrees with the fp32 build of the same
    victim within SURVEY 8c's C4 tolerance (loss rel <= 1e-2, d patch cosine >= 0.99; per-image max
    scores within 2e-2), at the well-conditioned weight draw above.  The fp64 oracle at this size
    would need ~100 GB of host memory, so the fp32 build (parity-tested against it at 256^2 in
    test_gpu_deep.py) is the reference here.  (D4's drop connect keys its draws by batch position,
    so a permuted batch is not expected to give permuted outputs; D0's equivariance is tested in
    test_gpu_fullsize.py.)"""
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker
    B4 = 4
    imgs = torch.as_tensor(synth_images(list(range(B4)), 1024)).cuda()
    boxes = synth_boxes(list(range(B4)), 1024)
    res = {}
    for dt in ("bf16", "f32"):
        v = EfficientDetVictim("efficientdet-d4", _well_conditioned_d4(1024), max_batch=B4, rng_seed=5,
                               dtype=dt)
        att = PatchAttacker(v, seed=7)
        att.cur_step = 3
        att.call(imgs, boxes=boxes)
        g1 = att.grad.clone()
        met = att.metrics_buf.cpu().numpy().copy()
        m = torch.empty(B4, device="cuda")
        v.ctx.call("phx_debug_last_maxscores", m.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
        if dt == "bf16":
            att.call(imgs, boxes=boxes)
            torch.cuda.synchronize()
            assert torch.isfinite(g1).all()
            assert g1[:-1].abs().sum() > 0
            assert torch.equal(att.grad, g1)
            _, s0, c0 = v.detect(imgs)
            _, s1, c1 = v.detect(imgs)
            assert torch.equal(s0, s1) and torch.equal(c0, c1)
        res[dt] = (g1.cpu().numpy().astype(np.float64), met, m.cpu().numpy())
        del att, v
        torch.cuda.empty_cache()
    (gb, mb, sb), (gf, mf, sf) = res["bf16"], res["f32"]
    assert abs(mb[_lib.M_LOSS] - mf[_lib.M_LOSS]) <= 1e-2 * abs(mf[_lib.M_LOSS])
    assert np.abs(sb - sf).max() <= 2e-2, (sb, sf)
    assert _cos(gb[:-1], gf[:-1]) >= 0.99, _cos(gb[:-1], gf[:-1])
    assert mb[_lib.M_NBOX] == mf[_lib.M_NBOX] and mb[_lib.M_NIMG] == B4
