"""Diagnostic: per-anchor score agreement of the bf16 (bf16 activations + bf16 GEMMs) and fp32 builds
of one victim — D4 1024^2 at the well-conditioned weight draw of test_gpu_bf16.py.  Prints, per image,
the largest and the 99.9th-percentile |score difference| over anchors, and where each build's top anchor
scores in the other build."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import synth_images  # noqa: E402
from mladversarialobjectdetection_amd.attacker import EfficientDetVictim  # noqa: E402
from tests.test_gpu_bf16 import _well_conditioned_d4  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
B = 4
imgs = torch.as_tensor(synth_images(list(range(B)), S)).cuda()
out = {}
for dt in ("bf16", "f32"):
    v = EfficientDetVictim("efficientdet-d4", _well_conditioned_d4(S), image_size=S, max_batch=B, rng_seed=5, dtype=dt)
    _, s, c = v.detect(imgs)
    out[dt] = (s.cpu().numpy(), c.cpu().numpy())
    del v
    torch.cuda.empty_cache()
sb, cb = out["bf16"]
sf, cf = out["f32"]
for b in range(B):
    d = np.abs(sb[b] - sf[b])
    ib, jf = int(np.argmax(sb[b] * (cb[b] == 0))), int(np.argmax(sf[b] * (cf[b] == 0)))
    print(f"image {b}: max|ds| {d.max():.4f} p99.9 {np.quantile(d, 0.999):.5f} median {np.median(d):.6f}; "
          f"class agree {np.mean(cb[b] == cf[b]):.5f}; top person anchor bf16 {ib} ({sb[b, ib]:.4f} / f32 {sf[b, ib]:.4f}), "
          f"f32 {jf} ({sf[b, jf]:.4f} / bf16 {sb[b, jf]:.4f} class {cb[b, jf]})")
