"""Attack-path post-processing restated for the oracle.

  filter_valid_boxes       attacker.py:69-89
  person mask              attacker.py:105-108, 132-135 (classes == 0, CLASS_OFFSET=1)
  soft-NMS                 postprocess.nms (postprocess.py:159-205) -> NonMaxSuppressionV5 with
                           method 'gaussian' (hparams_config.py:258-266): iou_thresh 1.0,
                           soft_nms_sigma = 0.5 / 2, score_thresh from config_override (0.5).
                           The op's algorithm (lazy priority queue) is restated from TensorFlow's
                           non_max_suppression_op.cc [TF-recall], in float32.
  clip_boxes               postprocess.py:61-64
"""
from __future__ import annotations

import heapq

import numpy as np


def valid_mask(boxes, h, w, scores=None, thresh=0.5):
    """filter_valid_boxes: w/W<=1, h/H<=1, area>100 (and score>=thresh when given), fp32."""
    boxes = np.asarray(boxes, dtype=np.float32)
    bh = boxes[..., 2] - boxes[..., 0]
    bw = boxes[..., 3] - boxes[..., 1]
    area = bh * bw
    m = (bw / np.float32(w) <= 1.0) & (bh / np.float32(h) <= 1.0) & (area > np.float32(100.0))
    if scores is not None:
        m &= np.asarray(scores, dtype=np.float32) >= np.float32(thresh)
    return m


def _iou(bi, bj):
    ymin_i, xmin_i = min(bi[0], bi[2]), min(bi[1], bi[3])
    ymax_i, xmax_i = max(bi[0], bi[2]), max(bi[1], bi[3])
    ymin_j, xmin_j = min(bj[0], bj[2]), min(bj[1], bj[3])
    ymax_j, xmax_j = max(bj[0], bj[2]), max(bj[1], bj[3])
    f = np.float32
    area_i = f(f(ymax_i - ymin_i) * f(xmax_i - xmin_i))
    area_j = f(f(ymax_j - ymin_j) * f(xmax_j - xmin_j))
    if area_i <= 0 or area_j <= 0:
        return f(0.0)
    iy0, ix0 = max(ymin_i, ymin_j), max(xmin_i, xmin_j)
    iy1, ix1 = min(ymax_i, ymax_j), min(xmax_i, xmax_j)
    inter = f(max(f(iy1 - iy0), f(0.0)) * max(f(ix1 - ix0), f(0.0)))
    return f(inter / f(f(area_i + area_j) - inter))


def soft_nms(boxes, scores, max_output_size=100, score_threshold=0.5, soft_nms_sigma=0.25):
    """NonMaxSuppressionV5 (iou_threshold = 1.0, soft) over one image; float32 arithmetic.
    Returns (selected_indices, selected_scores)."""
    boxes = np.asarray(boxes, dtype=np.float32)
    scores = np.asarray(scores, dtype=np.float32)
    thr = np.float32(score_threshold)
    scale = np.float32(-0.5) / np.float32(soft_nms_sigma) if soft_nms_sigma > 0 else np.float32(0)
    # max-heap on (score desc, index asc)
    heap = [(-scores[i], i, 0) for i in range(len(scores)) if scores[i] > thr]
    heapq.heapify(heap)
    cur = {i: scores[i] for _, i, _ in heap}
    selected, sel_scores = [], []
    while len(selected) < max_output_size and heap:
        negs, idx, sb = heapq.heappop(heap)
        score = np.float32(-negs)
        orig = score
        for j in range(len(selected) - 1, sb - 1, -1):
            sim = _iou(boxes[idx], boxes[selected[j]])
            score = np.float32(score * np.float32(np.exp(np.float32(np.float32(scale * sim) * sim))))
            if score <= thr:
                break
        sb = len(selected)
        if score == orig:
            selected.append(idx)
            sel_scores.append(score)
            continue
        if score > thr:
            heapq.heappush(heap, (-score, idx, sb))
    return np.asarray(selected, dtype=np.int64), np.asarray(sel_scores, dtype=np.float32)


def nms_padded(boxes, scores, image_size, max_output_size=100, score_threshold=0.5):
    """postprocess.nms(..., padded=True) + clip_boxes for one image: boxes [100,4], scores [100], n."""
    idx, sc = soft_nms(boxes, scores, max_output_size, score_threshold, 0.5 / 2)
    out_b = np.zeros((max_output_size, 4), np.float32)
    out_s = np.zeros((max_output_size,), np.float32)
    n = len(idx)
    if n:
        out_b[:n] = np.clip(np.asarray(boxes, np.float32)[idx], 0, image_size)
        out_s[:n] = sc
    return out_b, out_s, n
