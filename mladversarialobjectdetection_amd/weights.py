"""Victim weights: a flat float32 blob laid out by the library's manifest.

No pretrained checkpoint exists offline (util.download, util.py:76-87, needs the network), so the
benchmark and parity tests use deterministic synthetic weights drawn with the reference's own
initialisers where they are defined:

* conv kernels: N(0, sqrt(2 / fan_out)), fan_out = kh*kw*out  (efficientnet_model.py:53-74;
  depthwise kernels [k,k,C,1] -> fan_out = k*k);
* class-predict bias: -log((1 - 0.01) / 0.01)  (efficientdet_keras.py:464-471);
* BN: gamma ~ U(0.5, 1.5), beta ~ N(0, 0.1), moving mean ~ N(0, 0.1), moving var ~ U(0.5, 1.5)
  (SURVEY.md 8(d));  other biases ~ N(0, 0.05) so every bias path is exercised;
* BiFPN fastattn weights ~ U(0.5, 1.5) (the reference initialises them to ones).

A converter from the reference's TF checkpoints (util_keras.restore_ckpt, util_keras.py:108-203)
only needs to fill the same manifest names.
"""
from __future__ import annotations

import math

import numpy as np


def synthetic_blob(manifest, seed: int = 0, person_bias: float = 0.0, gamma=(0.5, 1.5),
                   beta=(0.0, 0.1)) -> np.ndarray:
    """Return the float32 weight blob for `manifest` (list of {name, shape, offset, kind}).

    gamma = (lo, hi) of the BN scale's uniform draw, beta = (mean, std) of the BN shift's normal
    draw.  The defaults are SURVEY.md 8(d)'s; a narrower gamma with a positive beta keeps most
    relu6 inputs inside (0, 6), away from the kinks (a well-conditioned lite point for parity)."""
    total = 0
    for e in manifest:
        total = max(total, e["offset"] + int(np.prod(e["shape"])))
    blob = np.zeros(total, dtype=np.float32)
    rng = np.random.default_rng(seed)
    prior = -math.log((1 - 0.01) / 0.01)
    for e in manifest:
        shape = tuple(e["shape"])
        n = int(np.prod(shape))
        kind = e["kind"]
        name = e["name"]
        if kind == "kernel":
            if len(shape) == 4:
                kh, kw, _, out = shape
                fan_out = kh * kw * out
            else:
                fan_out = shape[-1]
            v = rng.normal(0.0, math.sqrt(2.0 / fan_out), size=n)
        elif kind == "bias":
            if name.startswith("class_net/class-predict"):
                v = np.full(n, prior) + rng.normal(0.0, 0.05, size=n)
                if person_bias:
                    # raise the person logit of every anchor (class 0 of each 90-block)
                    v = v.reshape(-1, 90)
                    v[:, 0] += person_bias
                    v = v.reshape(-1)
            else:
                v = rng.normal(0.0, 0.05, size=n)
        elif kind == "gamma":
            v = rng.uniform(gamma[0], gamma[1], size=n)
        elif kind == "beta":
            v = rng.normal(beta[0], beta[1], size=n)
        elif kind == "moving_mean":
            v = rng.normal(0.0, 0.1, size=n)
        elif kind == "moving_variance":
            v = rng.uniform(0.5, 1.5, size=n)
        elif kind == "wsm":
            v = rng.uniform(0.5, 1.5, size=n)
        else:
            raise ValueError(f"unknown weight kind {kind}")
        blob[e["offset"]:e["offset"] + n] = np.asarray(v, dtype=np.float32)
    return blob


def unpack(manifest, blob: np.ndarray) -> dict:
    """name -> array view (HWIO kernels as in TF)."""
    out = {}
    for e in manifest:
        n = int(np.prod(e["shape"]))
        out[e["name"]] = blob[e["offset"]:e["offset"] + n].reshape(e["shape"])
    return out


def trainable_count(manifest) -> int:
    """Trainable parameter count as TF reports it (kernels, biases, gamma, beta, WSM)."""
    return int(sum(int(np.prod(e["shape"])) for e in manifest
                   if e["kind"] in ("kernel", "bias", "gamma", "beta", "wsm")))


# The well-conditioned synthetic draw for bf16 parity (BASELINE C4): gamma U(0.2, 0.4), beta N(1, 0.1),
# person prior 3.  At SURVEY 8d's standard draw (gamma U(0.5, 1.5), beta N(0, 0.1)) bf16 rounding on
# synthetic D4 weights is amplified to O(1) by the BN chains (tests/test_gpu_bf16.py), so the C4 bench
# line and its parity test (test_bf16_d4_1024_four_images) both run this draw.
WELL_CONDITIONED = {"seed": 0, "person_bias": 3.0, "gamma": (0.2, 0.4), "beta": (1.0, 0.1)}


def well_conditioned_blob(manifest) -> np.ndarray:
    return synthetic_blob(manifest, **WELL_CONDITIONED)

