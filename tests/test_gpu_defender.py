"""GPU parity of the defender step (BASELINE C5) against the CPU oracle
(oracle/defender.py, fp64):

  odet_model       attack_detection.py:96-166: the frozen victim's person anchors -> soft-NMS ->
                   clip -> filter_valid_boxes (area > 100, score >= 0.5), exact against the oracle's
                   NMS + filter over the product's own detections
  Masker           attack_detection.py:321-498 (training): shuffled / flipped 240^2 crops, print,
                   brightness match, placement (tolerance 0.5, scale U(0.3, 0.5)), resize + noise,
                   rotate, paste; target = original - pasted
  PatchNeutralizer generator.py:17-277: attention U-Net forward (training BN, Dropout) and the
                   gradient of sum_b mean((t - 2 u)^2) w.r.t. every variable; BN moving statistics
  Adam             Keras Adam, no constraints

The victim is D0 at 256^2 (the U-Net needs a multiple of 16, >= 240) with inference BN (the
protege's layers are frozen, attack_detection.py:46-47) and the person prior (person_bias) so the
first pass yields boxes.
Tolerances: first-pass counts / boxes exact; patched pixels and targets 99.99 % within 1e-4 (the
bilinear rotation's floor boundaries, as the attacker's EOT test); loss rel <= 1e-5; gradient cosine
>= 0.99999 and |d|/|ref| <= 1e-3 overall; moving statistics rel <= 1e-5.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

S = 256
B = 2


def _stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.fixture(scope="module")
def victim():
    from mladversarialobjectdetection_amd.attacker import EfficientDetVictim
    return EfficientDetVictim("efficientdet-d0", "synthetic", seed=0, image_size=S, max_batch=B, rng_seed=5,
                              person_bias=4.0, bn_mode="frozen")


@pytest.fixture(scope="module")
def defender(victim):
    from mladversarialobjectdetection_amd.defender import PatchAttackDefender
    return PatchAttackDefender(victim, protege_config_override={"nms_configs": {"iou_thresh": .5, "score_thresh": .5}},
                               seed=9)


def _images(seed=1):
    return np.random.default_rng(seed).uniform(-1, 1, (B, S, S, 3)).astype(np.float32)


def _boxes():
    return [np.array([[20, 30, 200, 120], [100, 100, 250, 250]], np.float32),
            np.array([[5, 5, 240, 140]], np.float32)]


def _moving0(defender):
    mv = defender.moving_statistics()
    return {b["name"]: (mv[b["moving_mean"]:b["moving_mean"] + b["channels"]].astype(np.float64),
                        mv[b["moving_variance"]:b["moving_variance"] + b["channels"]].astype(np.float64))
            for b in defender.manifest["bn"]}


def test_manifest_matches_oracle(defender):
    from oracle import defender as DF
    layout, bns = DF.unet_layout()
    man = defender.manifest
    assert man["n_params"] == sum(int(np.prod(s)) for _, s in layout) == 553439
    off = 0
    for (name, shape), p in zip(layout, man["params"]):
        assert p["name"] == name and tuple(p["shape"]) == tuple(shape) and p["offset"] == off
        off += int(np.prod(shape))
    assert [(b["name"], b["channels"]) for b in man["bn"]] == bns


def test_first_pass_matches_oracle_nms(victim, defender):
    from oracle import postprocess as pp
    imgs = torch.as_tensor(_images()).cuda()
    defender.call(imgs)
    torch.cuda.synchronize()
    cnt = defender.debug(4, B).cpu().numpy()
    gbx = defender.debug(3, B).cpu().numpy()
    boxes, scores, classes = (t.cpu().numpy() for t in victim.detect(imgs))
    tot = 0
    for b in range(B):
        keep = classes[b] == 0
        ob, os_, n = pp.nms_padded(boxes[b][keep], scores[b][keep], S, 100, 0.5)
        ob, os_ = ob[:n], os_[:n]
        h, w = ob[:, 2] - ob[:, 0], ob[:, 3] - ob[:, 1]
        ok = (w / np.float32(S) <= 1) & (h / np.float32(S) <= 1) & (h * w > np.float32(100)) & (os_ >= np.float32(.5))
        assert cnt[b] == ok.sum()
        np.testing.assert_array_equal(gbx[b, :cnt[b]], ob[ok])
        tot += cnt[b]
    assert tot > 0


def test_masker_matches_oracle(defender):
    from oracle import defender as DF
    imgs = _images(2)
    defender.cur_step = 3
    defender.call(torch.as_tensor(imgs).cuda(), boxes=_boxes())
    torch.cuda.synchronize()
    patched = defender.debug(0, B).cpu().numpy()
    targets = defender.debug(1, B).cpu().numpy()
    rp, rt = DF.masker(imgs, _boxes(), 9, 3, 0)
    for got, ref in ((patched, rp), (targets, rt)):
        d = np.abs(got - ref)
        assert (d <= 1e-4).mean() >= 0.9999, f"{(d > 1e-4).mean():.2e} off, max {d.max():.3e}"
    assert np.abs(rt).max() > 0.1  # patches were pasted


def test_unet_step_matches_oracle(defender):
    from oracle import defender as DF
    imgs = _images(3)
    mv0 = _moving0(defender)
    params = defender.params.cpu().numpy().copy()
    defender.cur_step = 5
    defender.call(torch.as_tensor(imgs).cuda(), boxes=_boxes())
    torch.cuda.synchronize()
    g = defender.grad.cpu().numpy().astype(np.float64)
    loss = float(defender.loss_buf.item())
    patched = defender.debug(0, B).cpu().numpy()
    targets = defender.debug(1, B).cpu().numpy()
    upd = defender.debug(2, B).cpu().numpy()
    ref = DF.defender_step(params, mv0, imgs, boxes=_boxes(), seed=9, step=5, masked=(patched, targets))
    assert abs(loss - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    assert np.abs(upd - ref["updates"]).max() <= 1e-4
    rg = ref["grad"]
    cos = g @ rg / (np.linalg.norm(g) * np.linalg.norm(rg))
    assert cos >= 0.99999, cos
    assert np.linalg.norm(g - rg) <= 1e-3 * np.linalg.norm(rg)
    # per variable: every variable's gradient is produced (no stale or missing writes)
    for p in defender.manifest["params"]:
        sl = slice(p["offset"], p["offset"] + int(np.prod(p["shape"])))
        nr = np.linalg.norm(rg[sl])
        if nr > 1e-6:
            assert np.linalg.norm(g[sl] - rg[sl]) <= 2e-2 * nr, p["name"]
    mv = defender.moving_statistics()
    for b in defender.manifest["bn"]:
        rm, rv = ref["moving"][b["name"]]
        gm = mv[b["moving_mean"]:b["moving_mean"] + b["channels"]]
        gv = mv[b["moving_variance"]:b["moving_variance"] + b["channels"]]
        np.testing.assert_allclose(gm, rm, rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(gv, rv, rtol=1e-4, atol=1e-6)


def test_adam_matches_oracle(defender):
    from oracle import defender as DF
    from mladversarialobjectdetection_amd import _lib
    rng = np.random.default_rng(4)
    n = 1000
    p = rng.normal(0, 1, n).astype(np.float32)
    g = rng.normal(0, 1, n).astype(np.float32)
    m = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    tp, tg, tm, tv = (torch.as_tensor(a).cuda() for a in (p, g, m, v))
    for t in (1, 2):
        rc = _lib.load().phx_adam(tp.data_ptr(), tg.data_ptr(), tm.data_ptr(), tv.data_ptr(), n, 1e-2, t, _stream())
        assert rc == 0
        p, m, v = DF.adam(p, g, m, v, 1e-2, t)
    np.testing.assert_allclose(tp.cpu().numpy(), p, rtol=1e-6, atol=1e-7)


def test_train_step_deterministic(victim):
    from mladversarialobjectdetection_amd.defender import PatchAttackDefender
    imgs = torch.as_tensor(_images(5)).cuda()
    out = []
    for _ in range(2):
        d = PatchAttackDefender(victim, seed=11)
        for _ in range(2):
            d.train_step(imgs)
        torch.cuda.synchronize()
        out.append((d.params.cpu().numpy().copy(), float(d.loss_buf.item())))
    assert np.isfinite(out[0][1])
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


def test_unet_implicit_im2col_matches_column_matrix(victim, monkeypatch):
    """The U-Net's wide 3x3 convs (more than 32 outputs or K > 288: the 64- and 128-channel levels,
    their data gradients, the transposed convs and theirs) gather the column matrix inside the GEMM
    (k_gemm2 MODE 4, no column matrix in HBM); PHX_UN_GATHER=0 writes it with k_im2col and runs the
    GEMM over it.  The products and their order are the same, so two training steps are bit-identical
    (variables and loss)."""
    from mladversarialobjectdetection_amd.defender import PatchAttackDefender
    imgs = torch.as_tensor(_images(6)).cuda()
    out = []
    for g in ("1", "0"):
        monkeypatch.setenv("PHX_UN_GATHER", g)
        d = PatchAttackDefender(victim, seed=11)
        for _ in range(2):
            d.train_step(imgs)
        torch.cuda.synchronize()
        out.append((d.params.cpu().numpy().copy(), float(d.loss_buf.item())))
    assert np.isfinite(out[0][1])
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


def test_eval_step_matches_oracle(victim):
    """PatchAttackDefender.call(training=False) / test_step (attack_detection.py:168-198, 320-326):
    the Masker's evaluation branch pastes the attacker's patch (print, brightness match, centred
    placement at the fixed scale, resize + noise, rotate), the protege's second pass at
    score_thresh 0 (soft-NMS at 0.001, valid filter at the config's 0.5), the U-Net in inference
    mode (moving statistics, no Dropout) and the loss.  Nothing may change: variables and moving
    statistics are checked bit for bit."""
    from oracle import defender as DF
    from oracle import postprocess as pp
    from mladversarialobjectdetection_amd import weights as W
    from mladversarialobjectdetection_amd.defender import PatchAttackDefender
    rng = np.random.default_rng(12)
    epatch = rng.uniform(-1, 1, (640, 640, 3)).astype(np.float32)
    d = PatchAttackDefender(victim, protege_config_override={"nms_configs": {"iou_thresh": .5, "score_thresh": .5}},
                            seed=9, eval_patch=(epatch, 0.4))
    d.cur_step = 4
    # non-trivial moving statistics: two training steps first
    for _ in range(2):
        d.train_step(torch.as_tensor(_images(6)).cuda(), boxes=_boxes())
    torch.cuda.synchronize()
    params = d.params.cpu().numpy().copy()
    mv_before = d.moving_statistics()
    mv0 = _moving0(d)
    imgs = _images(7)
    ob, os_, oc = d.call(torch.as_tensor(imgs).cuda(), training=False, boxes=_boxes())
    torch.cuda.synchronize()
    loss = float(d.eval_loss.item())
    patched = d.debug(0, B).cpu().numpy()
    targets = d.debug(1, B).cpu().numpy()
    upd = d.debug(2, B).cpu().numpy()
    assert np.array_equal(d.params.cpu().numpy(), params)
    assert np.array_equal(d.moving_statistics(), mv_before)
    # Masker evaluation branch
    rp, rt = DF.masker_eval(imgs, _boxes(), epatch, 0.4, 9, d.cur_step, 0)
    for got, ref in ((patched, rp), (targets, rt)):
        dd = np.abs(got - ref)
        assert (dd <= 1e-4).mean() >= 0.9999, f"{(dd > 1e-4).mean():.2e} off, max {dd.max():.3e}"
    assert np.abs(rt).max() > 0.1
    # second pass: the oracle's NMS (threshold 0.001) + valid filter (0.5) over the protege's own
    # detections of the product's patched images, exactly
    boxes, scores, classes = (t.cpu().numpy() for t in victim.detect(torch.as_tensor(patched).cuda()))
    oc, ob, os_ = oc.cpu().numpy(), ob.cpu().numpy(), os_.cpu().numpy()
    for b in range(B):
        keep = classes[b] == 0
        nb, ns, n = pp.nms_padded(boxes[b][keep], scores[b][keep], S, 100, 0.001)
        nb, ns = nb[:n], ns[:n]
        h, w = nb[:, 2] - nb[:, 0], nb[:, 3] - nb[:, 1]
        ok = (w / np.float32(S) <= 1) & (h / np.float32(S) <= 1) & (h * w > np.float32(100)) & (ns >= np.float32(.5))
        assert oc[b] == ok.sum()
        np.testing.assert_array_equal(ob[b, :oc[b]], nb[ok])
        # decayed scores: the device expf and numpy's exp may differ by an ulp (test_gpu_parity.py)
        np.testing.assert_allclose(os_[b, :oc[b]], ns[ok], rtol=2e-6, atol=0)
    # the U-Net in inference mode on the product's patched images
    ref = DF.defender_eval(params, mv0, imgs, epatch, 0.4, None, masked=(patched, targets), seed=9, step=d.cur_step)
    assert abs(loss - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    # two training steps leave the moving statistics near their initial (0, 1), so the inference-mode
    # U-Net's pre-tanh values are large and most outputs saturate at +-2; where they do not, the
    # fp32 rounding of those large values shows (measured max 3e-3).  Hence the pixel criterion of
    # the Masker checks rather than a max bound.
    du = np.abs(upd - ref["updates"])
    assert (du <= 1e-4).mean() >= 0.9999 and du.max() <= 1e-2, (du > 1e-4).mean()
    # test_step: the same call, the loss as the metric
    m, _ = d.test_step(torch.as_tensor(imgs).cuda(), boxes=_boxes())
    assert m["loss"] == pytest.approx(ref["loss"], rel=1e-5)


def test_eval_after_batch_size_switch(victim):
    """The fit-then-validate cycle with a partial batch: eval(B), train(B-1), train(B), eval(B).
    Every batch-size switch rebuilds the defender's workspace; the evaluation buffers belong to it
    and are rebuilt with it, so the second evaluation of the same inputs (same step, same parameters)
    equals the first bit for bit (freed evaluation buffers must never be reused)."""
    from mladversarialobjectdetection_amd.defender import PatchAttackDefender
    rng = np.random.default_rng(13)
    epatch = rng.uniform(-1, 1, (640, 640, 3)).astype(np.float32)
    d = PatchAttackDefender(victim, seed=9, eval_patch=(epatch, 0.4))
    imgs = torch.as_tensor(_images(8)).cuda()

    def evaluate():
        d.cur_step = 6
        ob, os_, oc = d.call(imgs, training=False, boxes=_boxes())
        torch.cuda.synchronize()
        return (ob.cpu().numpy(), os_.cpu().numpy(), oc.cpu().numpy(), float(d.eval_loss.item()),
                d.debug(0, B).cpu().numpy())

    first = evaluate()
    params = d.params.clone()
    moving = d.moving_statistics()
    d.train_step(imgs[:B - 1], boxes=_boxes()[:B - 1])
    d.train_step(imgs, boxes=_boxes())
    torch.cuda.synchronize()
    assert not np.array_equal(d.moving_statistics(), moving)
    # evaluate with the same variables and moving statistics as the first time
    d.params.copy_(params)
    d.handle.call("phx_def_moving", None, moving.ctypes.data, None)
    second = evaluate()
    for a, b in zip(first, second):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    assert first[2].sum() >= 0 and np.isfinite(first[3])


def test_save_weights_h5_roundtrip(victim, tmp_path):
    """save_weights writes antipatch.h5 in Keras's HDF5 weights layout (attack_detection.py:300-318) and
    PatchAttackDefender(initial_weights=dir or the .h5 path) restores the same variables and BN moving
    statistics (attack_detection.py:54-55), after a training step has moved them."""
    from mladversarialobjectdetection_amd import h5
    from mladversarialobjectdetection_amd.defender import PatchAttackDefender
    ov = {"nms_configs": {"iou_thresh": .5, "score_thresh": .5}}
    d = PatchAttackDefender(victim, protege_config_override=ov, seed=3)
    d.train_step(torch.as_tensor(_images(4)).cuda(), boxes=_boxes())
    torch.cuda.synchronize()
    params, moving = d.params.cpu().numpy(), d.moving_statistics()
    out = tmp_path / "save"
    d.save_weights(str(out))
    assert (out / "antipatch.h5").exists() and (out / "antipatch.npz").exists()
    names = [n for n, _ in h5.read_keras_weights(str(out / "antipatch.h5"))]
    assert names[0] == "conv0" and names[-1] == "patch_neutralizer/output"
    for src in (str(out), str(out / "antipatch.h5")):
        e = PatchAttackDefender(victim, initial_weights=src, protege_config_override=ov, seed=11)
        assert np.array_equal(e.params.cpu().numpy(), params)
        assert np.array_equal(e.moving_statistics(), moving)


def test_first_pass_prefetch_matches_in_step(victim):
    """train_step(next_inputs=...) (phx_def_set_next): the next batch's first pass runs on the
    defender's stream beside the current step's U-Net work and the next step uses its boxes.  The
    first pass depends only on the images, the step (drop connect) and the image offset, so three
    steps with the prefetch equal three without it bit for bit: variables, U-Net moving statistics,
    losses and the placement boxes."""
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd.defender import PatchAttackDefender
    ov = {"nms_configs": {"iou_thresh": .5, "score_thresh": .5}}
    batches = [torch.as_tensor(_images(20 + j)).cuda() for j in range(3)]
    res = []
    for pf in (False, True):
        d = PatchAttackDefender(victim, protege_config_override=ov, seed=13)
        losses, boxes = [], []
        for k in range(3):
            nx = batches[k + 1] if pf and k + 1 < 3 else None
            out = d.train_step(batches[k], next_inputs=nx)
            losses.append(float(out["loss"].item()))
            boxes.append(d.debug(_lib.DEF_BOXES, B).cpu().numpy())
        d.sync()
        torch.cuda.synchronize()
        res.append((d.params.cpu().numpy(), d.moving_statistics(), losses, boxes))
    (p0, m0, l0, b0), (p1, m1, l1, b1) = res
    assert np.array_equal(p0, p1) and np.array_equal(m0, m1)
    assert l0 == l1
    for a, b in zip(b0, b1):
        assert np.array_equal(a, b)
    assert any(np.abs(b).sum() > 0 for b in b0)  # the first passes found boxes


def test_first_pass_prefetch_refilled_buffer(victim):
    """A next batch refilled in place after train_step handed it over: the defender withdraws the
    prefetched first pass (version counter) and places by the new contents, as without a prefetch."""
    from mladversarialobjectdetection_amd import _lib
    from mladversarialobjectdetection_amd.defender import PatchAttackDefender
    ov = {"nms_configs": {"iou_thresh": .5, "score_thresh": .5}}
    batches = [torch.as_tensor(_images(30 + j)).cuda() for j in range(3)]
    res = []
    for pf in (False, True):
        d = PatchAttackDefender(victim, protege_config_override=ov, seed=13)
        ring = batches[1].clone()
        d.train_step(batches[0], next_inputs=ring if pf else None)
        ring.copy_(batches[2])
        out = d.train_step(ring)
        res.append((float(out["loss"].item()), d.debug(_lib.DEF_BOXES, B).cpu().numpy(), d.params.cpu().numpy()))
    (l0, b0, p0), (l1, b1, p1) = res
    assert l0 == l1 and np.array_equal(b0, b1) and np.array_equal(p0, p1)
