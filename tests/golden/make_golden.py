"""Generate the committed golden fixtures from the CPU oracle (fp64).

    python tests/golden/make_golden.py

Fixtures are data only: seeds/config + expected outputs.  Inputs are regenerated from the seeds
(numpy default_rng), weights from the manifest + seed (mladversarialobjectdetection_amd.weights).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from mladversarialobjectdetection_amd import _lib  # noqa: E402
from mladversarialobjectdetection_amd import weights as W  # noqa: E402
from oracle import postprocess as pp  # noqa: E402
from oracle import step as ST  # noqa: E402

CASE = dict(model="efficientdet-d0", image_size=128, batch=2, weight_seed=0, image_seed=1, patch_seed=7,
            scale=0.4, rng_seed=5, step=3)
BOXES = [[[10, 20, 90, 70]], [[5, 5, 120, 60], [30, 40, 100, 110]]]


def case_inputs(c=CASE):
    man = _lib.Context(c["model"], c["image_size"]).manifest()
    wd = W.unpack(man, W.synthetic_blob(man, seed=c["weight_seed"]))
    S = c["image_size"]
    imgs = np.random.default_rng(c["image_seed"]).uniform(-1, 1, (c["batch"], S, S, 3)).astype(np.float32)
    patch = np.random.default_rng(c["patch_seed"]).uniform(-1, 1, (640, 640, 3)).astype(np.float32)
    boxes = [np.asarray(b, np.float32) for b in BOXES]
    return wd, imgs, patch, boxes


def grad_summary(g):
    gp = g[:-1].reshape(640, 640, 3)
    blocks = gp.reshape(40, 16, 40, 16, 3).sum(axis=(1, 3))
    idx = np.random.default_rng(0).choice(gp.size, 2000, replace=False)
    return blocks, idx, gp.reshape(-1)[idx]


def main():
    wd, imgs, patch, boxes = case_inputs()
    c = CASE
    r = ST.attack_step(wd, imgs, patch, c["scale"], boxes=boxes, seed=c["rng_seed"], step=c["step"],
                       image_size=c["image_size"])
    blocks, idx, vals = grad_summary(r["grad"])
    places = np.array([[p["ymin"], p["xmin"], p["ps"], p["diag"], int(p["valid"])] for pl in r["places"] for p in pl],
                      np.int64)
    np.savez_compressed(os.path.join(HERE, "d0_128_step.npz"), loss=r["loss"], m_raw=r["m_raw"],
                        dscale=r["grad"][-1], grad_norm=np.linalg.norm(r["grad"][:-1]), grad_blocks=blocks,
                        grad_idx=idx, grad_vals=vals, places=places, tv=r["tv"], scale_loss=r["scale_loss"],
                        patched_sum=r["patched"].sum(axis=(1, 2)), case=str(CASE))
    # soft-NMS golden: random candidates -> selected indices / scores
    rng = np.random.default_rng(3)
    yx = rng.uniform(0, 100, (300, 2))
    hw = rng.uniform(8, 40, (300, 2))
    bx = np.concatenate([yx, yx + hw], -1).astype(np.float32)
    sc = rng.uniform(0.3, 1.0, 300).astype(np.float32)
    sel, ss = pp.soft_nms(bx, sc, 100, 0.5, 0.25)
    np.savez_compressed(os.path.join(HERE, "soft_nms.npz"), boxes=bx, scores=sc, sel=sel, sel_scores=ss)
    print("loss", r["loss"], "grad_norm", np.linalg.norm(r["grad"][:-1]), "nms selected", len(sel))


if __name__ == "__main__":
    main()

# burj_khalifa_96.npz: the reference's brightness-matcher test photos (burj_khalifa_day.jpg,
# burj_khalifa_sunset.jpg, used by brightness_matcher.py:169-179) resized to 96x96 RGB uint8 with
# PIL bilinear — generated once in the survey container (the reference is absent on the GPU box):
#   Image.open(path).convert("RGB").resize((96, 96), Image.BILINEAR)
