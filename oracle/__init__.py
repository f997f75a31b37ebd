"""CPU oracle for the adversarial-patch optimisation step — TEST INFRASTRUCTURE ONLY.

A line-by-line restatement of the reference's hot path (tiiuae/MLAdversarialObjectDetection,
attacker.py / brightness_matcher.py and the vendored automl EfficientDet) in PyTorch-CPU fp64
(detector, EOT, loss, gradients) and numpy fp32 (discrete geometry, soft-NMS), each function
citing the reference file:line it follows.  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s cpu_baseline leg may import it, and only as the checker / CPU baseline: the product
path (mladversarialobjectdetection_amd + libphx.so) never calls into it.

Pinning.  TensorFlow 2.8.1 / TFA 0.17 are not installed and no reference checkpoint exists
(SURVEY.md 8c), so the reference's own TF path cannot run here.  The oracle is pinned by the
reference's own known-answer tests wherever they touch this path — parameter counts of every
EfficientDet variant (efficientdet_arch_test.py:47-114), BiFPN node lists
(tf2/fpn_configs_test.py:23-58), feature sizes (utils_test.py:71-95), activation values
(utils_test.py:113-141), the fastattn fuse fixture (efficientdet_arch_test.py:207-215), anchor
normalisation (tf2/postprocess_test.py:205-229) — plus Random123's Philox known-answer vectors
for the RNG.  The TF/TFA op semantics it restates (ScaleAndTranslate, ImageProjectiveTransformV3
and its registered gradient, NonMaxSuppressionV5, FusedBatchNorm, rgb_to_yuv) are not covered by
any reference test: for those ops parity is "unpinned" beyond this restatement.
"""
