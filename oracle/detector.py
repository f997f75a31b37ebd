"""EfficientDet victim restated in PyTorch (CPU, fp64 by default) — oracle only.

Follows the reference's vendored automl TF2 Keras model:
  backbone   backbone/efficientnet_model.py:129-151 (round_filters/round_repeats), :154-196 (SE),
             :224-417 (MBConvBlock), :507-528 (Stem), :711-780 (Model.call, reductions)
             backbone/efficientnet_builder.py:31-46, 163-168 ; efficientnet_lite_builder.py:28-79
  FPN        tf2/efficientdet_keras.py:42-172 (FNode), :175-221 (OpAfterCombine),
             :224-324 (ResampleFeatureMap), :700-775 (FPNCells / FPNCell), tf2/fpn_configs.py:24-72
  heads      tf2/efficientdet_keras.py:327-471 (ClassNet), :474-632 (BoxNet)
  assembly   tf2/efficientdet_keras.py:884-906 (EfficientDetNet.call)
  BN         utils.py:244-266 / tf2/util_keras.py:29-66 — Keras BatchNormalization, eps 1e-3; with
             training=True (the attack step, attacker.py:172) it normalises with the batch's biased
             mean/variance over (N, H, W).
Tensors are NCHW internally; weights come in TF HWIO layout from the manifest blob.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from . import philox as ph

# hparams_config.py:301-467 (checked against the reference's own config module by
# tests/test_kats.py::test_oracle_model_table_matches_reference_configs via
# tests/golden/hparams_configs.json); backbone width/depth: efficientnet_builder.py:31-46,
# efficientnet_lite_builder.py:31-41.  lite: lite_common_param (hparams_config.py:392-397) —
# relu6 everywhere, BiFPN fuse 'sum', mean/std 127/128; backbone without SE and with the stem and the
# first/last block rows unscaled (efficientnet_lite_builder.py:54-79, fix_head_stem in
# efficientnet_model.py:643-662).
_D = dict(act="swish", fuse="fastattn", anchor_scale=4.0, lite=False)
_L = dict(act="relu6", fuse="sum", anchor_scale=4.0, lite=True)
MODELS = {
    "efficientdet-d0": dict(_D, backbone="efficientnet-b0", image_size=512, fpn=64, cells=3, rep=3, w=1.0, d=1.0),
    "efficientdet-d1": dict(_D, backbone="efficientnet-b1", image_size=640, fpn=88, cells=4, rep=3, w=1.0, d=1.1),
    "efficientdet-d2": dict(_D, backbone="efficientnet-b2", image_size=768, fpn=112, cells=5, rep=3, w=1.1, d=1.2),
    "efficientdet-d3": dict(_D, backbone="efficientnet-b3", image_size=896, fpn=160, cells=6, rep=4, w=1.2, d=1.4),
    "efficientdet-d4": dict(_D, backbone="efficientnet-b4", image_size=1024, fpn=224, cells=7, rep=4, w=1.4, d=1.8),
    "efficientdet-lite0": dict(_L, backbone="efficientnet-lite0", image_size=320, fpn=64, cells=3, rep=3, w=1.0, d=1.0,
                               anchor_scale=3.0),
    "efficientdet-lite1": dict(_L, backbone="efficientnet-lite1", image_size=384, fpn=88, cells=4, rep=3, w=1.0, d=1.1,
                               anchor_scale=3.0),
    "efficientdet-lite2": dict(_L, backbone="efficientnet-lite2", image_size=448, fpn=112, cells=5, rep=3, w=1.1,
                               d=1.2, anchor_scale=3.0),
    "efficientdet-lite3": dict(_L, backbone="efficientnet-lite3", image_size=512, fpn=160, cells=6, rep=4, w=1.2,
                               d=1.4),
    "efficientdet-lite4": dict(_L, backbone="efficientnet-lite4", image_size=640, fpn=224, cells=7, rep=4, w=1.4,
                               d=1.8),
}
BLOCKS = [  # efficientnet_builder.py:163-168: (r, k, s, e, i, o, se)
    (1, 3, 1, 1, 32, 16, 0.25), (2, 3, 2, 6, 16, 24, 0.25), (2, 5, 2, 6, 24, 40, 0.25),
    (3, 3, 2, 6, 40, 80, 0.25), (3, 5, 1, 6, 80, 112, 0.25), (4, 5, 2, 6, 112, 192, 0.25),
    (1, 3, 1, 6, 192, 320, 0.25),
]
BN_EPS = 1e-3
MIN_LEVEL, MAX_LEVEL = 3, 7
NUM_CLASSES = 90
NUM_ANCHORS = 9


def round_filters(filters, mult, skip=False):
    """efficientnet_model.py:129-143"""
    if skip or not mult:
        return filters
    divisor = 8
    filters *= mult
    new = max(divisor, int(filters + divisor / 2) // divisor * divisor)
    if new < 0.9 * filters:
        new += divisor
    return int(new)


def round_repeats(r, mult):
    return int(math.ceil(mult * r))


def same_pads(size, k, s):
    """TF 'SAME': total = max((ceil(in/s)-1)*s + k - in, 0), before = total // 2."""
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


def bifpn_nodes(min_level=MIN_LEVEL, max_level=MAX_LEVEL):
    """tf2/fpn_configs.py:24-72"""
    num_levels = max_level - min_level + 1
    node_ids = {min_level + i: [i] for i in range(num_levels)}
    cnt = num_levels
    nodes = []
    for i in range(max_level - 1, min_level - 1, -1):
        nodes.append({"feat_level": i, "inputs_offsets": [node_ids[i][-1], node_ids[i + 1][-1]]})
        node_ids[i].append(cnt)
        cnt += 1
    for i in range(min_level + 1, max_level + 1):
        nodes.append({"feat_level": i, "inputs_offsets": node_ids[i] + [node_ids[i - 1][-1]]})
        node_ids[i].append(cnt)
        cnt += 1
    return nodes


def feat_sizes(image_size, max_level=MAX_LEVEL):
    """utils.py:506-526"""
    out = [image_size]
    s = image_size
    for _ in range(max_level):
        s = (s - 1) // 2 + 1
        out.append(s)
    return out


class TieMax(torch.autograd.Function):
    """reduce_max over the last axis with TF's gradient: split equally among ties (_MaxGrad)."""

    @staticmethod
    def forward(ctx, x):
        m = x.max(dim=-1).values
        ctx.save_for_backward(x, m)
        return m

    @staticmethod
    def backward(ctx, g):
        x, m = ctx.saved_tensors
        mask = (x == m.unsqueeze(-1)).to(x.dtype)
        return g.unsqueeze(-1) * mask / mask.sum(-1, keepdim=True)


def fuse_nodes(nodes, wsm, method):
    """FNode.fuse_features (efficientdet_keras.py:75-110): 'fastattn' = sum_i x_i * relu(w_i) /
    (sum_j relu(w_j) + 1e-4) accumulated in input order (tf.add_n); 'sum' = add_n(nodes)."""
    if method == "sum":
        out = nodes[0]
        for v in nodes[1:]:
            out = out + v
        return out
    ws = [torch.relu(w) for w in wsm]
    wsum = ws[0]
    for v in ws[1:]:
        wsum = wsum + v
    out = nodes[0] * ws[0] / (wsum + 0.0001)
    for i in range(1, len(nodes)):
        out = out + nodes[i] * ws[i] / (wsum + 0.0001)
    return out


def _rbf16(t):
    """round to bf16 (nearest even) and back"""
    return t.to(torch.bfloat16).to(t.dtype)


class Bf16Store(torch.autograd.Function):
    """A tensor as a PHX_DTYPE_BF16 context stores it (SURVEY.md 8a R4 "C4: bf16 act"): every
    activation the library writes — conv / depthwise / stem outputs (BN inputs), fuse, add and
    resample outputs, the class / box head outputs — is rounded to bf16; BN outputs are computed on
    load in fp32 and never stored.  Gradients stay fp32, so the backward is the identity."""

    @staticmethod
    def forward(ctx, x):
        return _rbf16(x)

    @staticmethod
    def backward(ctx, g):
        return g


class Bf16Conv1x1(torch.autograd.Function):
    """A 1x1 convolution as the library's bf16 GEMM computes it (PHX_DTYPE_BF16, SURVEY.md 8a R4
    "C4: bf16 act, fp32 acc"): operands rounded to bf16, products accumulated in full precision.
    Forward rounds x and w when the GEMM's N (output channels) > 16; the data gradient rounds dy and
    w when its N (input channels) > 16 — smaller GEMMs run on the fp32 register kernel."""

    @staticmethod
    def forward(ctx, x, w, rnd_fwd, rnd_bwd):
        ctx.save_for_backward(w)
        ctx.rnd_bwd = rnd_bwd
        if rnd_fwd:
            x, w = _rbf16(x), _rbf16(w)
        return F.conv2d(x, w)

    @staticmethod
    def backward(ctx, g):
        (w,) = ctx.saved_tensors
        if ctx.rnd_bwd:
            g, w = _rbf16(g), _rbf16(w)
        return torch.einsum("nohw,oi->nihw", g, w[:, :, 0, 0]), None, None, None


class Relu6(torch.autograd.Function):
    """tf.nn.relu6 with TF's Relu6Grad: the gradient passes on the open interval (0, 6)."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.clamp(x, 0.0, 6.0)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * ((x > 0) & (x < 6)).to(g.dtype)


class Detector:
    """EfficientDetNet.call(images, training) restated; weights: name -> HWIO array."""

    def __init__(self, weights: dict, model="efficientdet-d0", image_size=None, dtype=torch.float64,
                 training=True, drop=None, bn_frozen=False):
        self.W = weights
        self.cfg = MODELS[model]
        self.image_size = image_size or self.cfg["image_size"]
        self.dtype = dtype
        self.training = training
        # bn_frozen: inference BN (moving statistics) even in a training pass — Keras BN layers with
        # trainable=False (attack_detection.py:46-47; the library's bn=frozen mode); drop connect
        # still follows `training`
        self.bn_frozen = bn_frozen
        # bf16: emulate the library's PHX_DTYPE_BF16 arithmetic — bf16 1x1-conv operands
        # (Bf16Conv1x1) and bf16 activation storage (Bf16Store)
        self.bf16 = False
        # drop-connect draws: dict(seed, step, gimg0, pass) — pass 0 first, 1 second, 2 detect
        self.drop = drop
        self._cache = {}
        self.taps = None
        self.bn_stats = {}   # BN prefix -> list of (batch mean, biased batch var), one per training pass

    # ---- weights -----------------------------------------------------------------------------
    def w(self, name):
        t = self._cache.get(name)
        if t is None:
            t = torch.as_tensor(np.asarray(self.W[name], dtype=np.float64), dtype=self.dtype)
            self._cache[name] = t
        return t

    # ---- layers ------------------------------------------------------------------------------
    def conv(self, x, kname, stride=1, bias=None):
        k = self.w(kname)  # HWIO
        kh, kw = k.shape[0], k.shape[1]
        wt = k.permute(3, 2, 0, 1)
        pt, pb = same_pads(x.shape[2], kh, stride)
        pl, pr = same_pads(x.shape[3], kw, stride)
        if pt or pb or pl or pr:
            x = F.pad(x, (pl, pr, pt, pb))
        if self.bf16 and kh == 1 and kw == 1 and "/se/" not in kname:
            cin, cout = wt.shape[1], wt.shape[0]
            # the class-predict conv's data gradient is the library's sparse fp32 scatter
            y = Bf16Conv1x1.apply(x, wt, cout > 16, cin > 16 and "class-predict" not in kname)
        else:
            y = F.conv2d(x, wt, stride=stride)
        if bias is not None:
            y = y + self.w(bias).view(1, -1, 1, 1)
        if "/se/" in kname:  # the SE MLP runs on pooled vectors, nothing is stored
            return y
        return self.store(y)

    def store(self, t):
        """a tensor the library writes to its activation arena (bf16 storage in bf16 mode)"""
        return Bf16Store.apply(t) if self.bf16 else t

    def dwconv(self, x, kname, stride=1):
        k = self.w(kname)  # [k,k,C,1]
        kk = k.shape[0]
        wt = k.permute(2, 3, 0, 1)  # [C,1,k,k]
        pt, pb = same_pads(x.shape[2], kk, stride)
        pl, pr = same_pads(x.shape[3], kk, stride)
        x = F.pad(x, (pl, pr, pt, pb))
        return self.store(F.conv2d(x, wt, stride=stride, groups=x.shape[1]))

    def bn(self, x, pfx, act=False):
        """BatchNormalization (+ the activation that follows it when act=True).  With
        self.taps = {} it records (BN input, output) per prefix, the output retaining its gradient
        (per-layer diagnostics against the product's debug hook)."""
        y = self._bn(x, pfx)
        if act:
            y = self.act(y)
        if self.taps is not None:
            if y.requires_grad:
                y.retain_grad()
            self.taps[pfx] = (x, y)
        return y

    def _tap(self, name, y):
        if self.taps is not None:
            if y.requires_grad:
                y.retain_grad()
            self.taps[name] = (y, y)
        return y

    def _bn(self, x, pfx):
        g, b = self.w(pfx + "/gamma"), self.w(pfx + "/beta")
        if self.training and not self.bn_frozen:
            mean = x.mean(dim=(0, 2, 3), keepdim=True)
            var = ((x - mean) ** 2).mean(dim=(0, 2, 3), keepdim=True)
            self.bn_stats.setdefault(pfx, []).append((mean.detach().flatten(), var.detach().flatten(),
                                                      x.shape[0] * x.shape[2] * x.shape[3]))
        else:
            mean = self.w(pfx + "/moving_mean").view(1, -1, 1, 1)
            var = self.w(pfx + "/moving_variance").view(1, -1, 1, 1)
        xh = (x - mean) / torch.sqrt(var + BN_EPS)
        return xh * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)

    def act(self, x):
        """utils.activation_fn (utils.py:36-53): swish = x*sigmoid(x) (tf.nn.swish), relu6 (lite)"""
        if self.cfg["act"] == "relu6":
            return Relu6.apply(x)
        return x * torch.sigmoid(x)

    def moving_stats(self, pfx, mean0, var0):
        """Moving statistics after this detector's training passes (Keras BN, momentum 0.99,
        util_keras.py:33-35: moving -= (moving - batch) * 0.01; the fused op hands the
        Bessel-corrected variance to the update [TF-recall])."""
        m = np.asarray(mean0, np.float64).copy()
        v = np.asarray(var0, np.float64).copy()
        for mu, var, n in self.bn_stats.get(pfx, []):
            uv = var.numpy() * n / (n - 1) if n > 1 else var.numpy()
            m = m - (m - mu.numpy()) * 0.01
            v = v - (v - uv) * 0.01
        return m, v

    def sepconv(self, x, pfx):
        """keras SeparableConv2D(depth_multiplier=1, 3x3, same, bias)"""
        x = self.dwconv(x, pfx + "/depthwise_kernel")
        return self.conv(x, pfx + "/pointwise_kernel", bias=pfx + "/bias")

    def drop_connect(self, x, idx, nb):
        """utils.py:329-344 with the per-block survival of efficientnet_model.py:752-755 (global
        survival 0.8, efficientnet_builder.py:174; b0 overrides it to 0, efficientdet_keras.py:803-804).
        TF draws U[0,1) per image; here U = u01(Philox(seed; block, pass, global image, step, RNG_DROP))
        so the product's draws are reproduced: keep = floor(p + U) in fp32, x / p * keep."""
        if self.drop is None:
            raise ValueError("drop connect is active (non-b0 backbone, training): pass drop=dict(...)")
        d = self.drop
        p = np.float32(1.0 - (1.0 - 0.8) * float(idx) / nb)
        B = x.shape[0]
        u = ph.u01(ph.draw(d["seed"], idx, d["pass"], np.arange(B) + d["gimg0"], d["step"], ph.RNG_DROP)[0])
        keep = np.floor((p + u).astype(np.float32))
        k = torch.as_tensor(keep.astype(np.float64), dtype=x.dtype).view(-1, 1, 1, 1)
        return x / float(p) * k

    # ---- backbone ----------------------------------------------------------------------------
    def backbone(self, x):
        bb = self.cfg["backbone"]
        wc, dc = self.cfg["w"], self.cfg["d"]
        lite = self.cfg["lite"]
        x = self.bn(self.conv(x, bb + "/stem/conv2d/kernel", 2), bb + "/stem/tpu_batch_normalization", act=True)
        blocks = []
        for a, (r, k, s, e, i, o, se) in enumerate(BLOCKS):
            inf, outf = round_filters(i, wc), round_filters(o, wc)
            if lite:
                se = 0  # use_se=False (efficientnet_lite_builder.py:79)
            blocks.append((k, s, e, inf, outf, se))
            reps = r if lite and a in (0, len(BLOCKS) - 1) else round_repeats(r, dc)
            for _ in range(reps - 1):
                blocks.append((k, 1, e, outf, outf, se))
        reductions = []
        for idx, (k, s, e, inf, outf, se) in enumerate(blocks):
            pfx = f"{bb}/blocks_{idx}"
            inputs = x
            cid = bid = 0

            def cname(i):
                return "conv2d" if i == 0 else f"conv2d_{i}"

            def bname(i):
                return "tpu_batch_normalization" if i == 0 else f"tpu_batch_normalization_{i}"

            if e != 1:
                x = self.bn(self.conv(x, f"{pfx}/{cname(cid)}/kernel"), f"{pfx}/{bname(bid)}", act=True)
                cid += 1
                bid += 1
            x = self.bn(self.dwconv(x, f"{pfx}/depthwise_conv2d/depthwise_kernel", s),
                                 f"{pfx}/{bname(bid)}", act=True)
            bid += 1
            if se:  # SE (efficientnet_model.py:184-196)
                sq = x.mean(dim=(2, 3), keepdim=True)
                sq = self.act(self.conv(sq, f"{pfx}/se/conv2d/kernel", bias=f"{pfx}/se/conv2d/bias"))
                sq = self.conv(sq, f"{pfx}/se/conv2d_1/kernel", bias=f"{pfx}/se/conv2d_1/bias")
                x = torch.sigmoid(sq) * x
            x = self.bn(self.conv(x, f"{pfx}/{cname(cid)}/kernel"), f"{pfx}/{bname(bid)}")
            if s == 1 and inf == outf:
                if self.training and "b0" not in bb:
                    x = self.drop_connect(x, idx, len(blocks))
                x = self.store(x + inputs)
            if idx == len(blocks) - 1 or blocks[idx + 1][1] > 1:
                reductions.append(x)
        return reductions[MIN_LEVEL - 1:MIN_LEVEL + 2]  # P3..P5 = reduction_3..5

    # ---- resampling ---------------------------------------------------------------------------
    def maxpool(self, x, k, s):
        pt, pb = same_pads(x.shape[2], k, s)
        pl, pr = same_pads(x.shape[3], k, s)
        x = F.pad(x, (pl, pr, pt, pb), value=-math.inf)
        return F.max_pool2d(x, k, s)

    @staticmethod
    def upsample(x, th, tw):
        """tf.compat.v1.image.resize_nearest_neighbor (legacy): src = min(floor(dst*in/out), in-1)"""
        h, w = x.shape[2], x.shape[3]
        sy = np.float32(h) / np.float32(th)
        sx = np.float32(w) / np.float32(tw)
        iy = np.minimum(np.floor(np.arange(th, dtype=np.float32) * sy).astype(np.int64), h - 1)
        ix = np.minimum(np.floor(np.arange(tw, dtype=np.float32) * sx).astype(np.int64), w - 1)
        return x[:, :, torch.as_tensor(iy)][:, :, :, torch.as_tensor(ix)]

    def resample(self, x, th, tw, pfx):
        """ResampleFeatureMap.call (efficientdet_keras.py:297-324)"""
        fpn = self.cfg["fpn"]
        h, w, c = x.shape[2], x.shape[3], x.shape[1]

        def maybe_1x1(v):
            if c != fpn:
                v = self.bn(self.conv(v, pfx + "/conv2d/kernel", bias=pfx + "/conv2d/bias"), pfx + "/bn")
            return v

        if h > th and w > tw:
            x = maybe_1x1(x)
            sh = (h - 1) // th + 1
            x = self._tap(pfx + "/max_pool", self.store(self.maxpool(x, sh + 1, sh)))
        else:
            x = maybe_1x1(x)
            if h < th or w < tw:
                x = self._tap(pfx + "/upsample", self.store(self.upsample(x, th, tw)))
        return x

    # ---- full network ---------------------------------------------------------------------------
    def __call__(self, images_nhwc):
        """images [B,H,W,3] -> (cls [5 x B,810,h,w], box [5 x B,36,h,w]) (NCHW)"""
        x = images_nhwc.permute(0, 3, 1, 2)
        feats = self.backbone(x)
        for level in range(6, MAX_LEVEL + 1):
            last = feats[-1]
            th, tw = (last.shape[2] + 1) // 2, (last.shape[3] + 1) // 2
            feats.append(self.resample(last, th, tw, f"resample_p{level}"))
        nodes = bifpn_nodes()
        fpn = self.cfg["fpn"]
        for cell in range(self.cfg["cells"]):
            allf = list(feats)
            for ni, nd in enumerate(nodes):
                npfx = f"fpn_cells/cell_{cell}/fnode{ni}"
                target = allf[nd["feat_level"] - MIN_LEVEL]
                ins = []
                for i, off in enumerate(nd["inputs_offsets"]):
                    ins.append(self.resample(allf[off], target.shape[2], target.shape[3],
                                             f"{npfx}/resample_{i}_{off}_{len(allf)}"))
                wsm = None
                if self.cfg["fuse"] != "sum":
                    wsm = [self.w(f"{npfx}/WSM" + ("" if i == 0 else f"_{i}")).reshape(()) for i in range(len(ins))]
                nd_out = fuse_nodes(ins, wsm, self.cfg["fuse"])
                oac = f"{npfx}/op_after_combine{len(allf)}"
                v = self._tap(f"{npfx}/fuse", self.store(self.act(nd_out)))
                v = self.sepconv(v, oac + "/conv")
                v = self.bn(v, oac + "/bn")
                allf.append(v)
            nf = []
            for level in range(MIN_LEVEL, MAX_LEVEL + 1):
                for i, nd in enumerate(reversed(nodes)):
                    if nd["feat_level"] == level:
                        nf.append(allf[-1 - i])
                        break
            feats = nf

        def head(net, tag):
            outs = []
            for li, v in enumerate(feats):
                for i in range(self.cfg["rep"]):
                    v = self.sepconv(v, f"{net}/{tag}-{i}")
                    v = self.bn(v, f"{net}/{tag}-{i}-bn-{MIN_LEVEL + li}", act=True)
                outs.append(self.sepconv(v, f"{net}/{tag}-predict"))
            return outs

        return head("class_net", "class"), head("box_net", "box")


def anchors(image_size, anchor_scale=4.0, num_scales=3, aspect_ratios=(1.0, 2.0, 0.5),
            min_level=MIN_LEVEL, max_level=MAX_LEVEL):
    """anchors.py:83-165 (Anchors._generate_boxes), float64 then float32."""
    fs = feat_sizes(image_size, max_level)
    boxes_all = []
    for level in range(min_level, max_level + 1):
        stride = fs[0] / float(fs[level])
        boxes_level = []
        for octave in range(num_scales):
            for aspect in aspect_ratios:
                base = anchor_scale * stride * 2 ** (octave / float(num_scales))
                ax = np.sqrt(aspect)
                ay = 1.0 / ax
                sx2, sy2 = base * ax / 2.0, base * ay / 2.0
                x = np.arange(stride / 2, image_size, stride)
                y = np.arange(stride / 2, image_size, stride)
                xv, yv = np.meshgrid(x, y)
                xv, yv = xv.reshape(-1), yv.reshape(-1)
                b = np.vstack((yv - sy2, xv - sx2, yv + sy2, xv + sx2)).swapaxes(0, 1)
                boxes_level.append(np.expand_dims(b, axis=1))
        boxes_all.append(np.concatenate(boxes_level, axis=1).reshape([-1, 4]))
    return np.vstack(boxes_all).astype(np.float32)


def pre_nms(cls_outs, box_outs, image_size, anchor_scale=4.0):
    """postprocess.pre_nms (postprocess.py:119-156) with max_nms_inputs = 0:
    returns scores [B,A] (differentiable), classes [B,A] (argmax), boxes [B,A,4] (decoded)."""
    B = cls_outs[0].shape[0]
    cls = torch.cat([c.permute(0, 2, 3, 1).reshape(B, -1, NUM_CLASSES) for c in cls_outs], 1)
    box = torch.cat([b.permute(0, 2, 3, 1).reshape(B, -1, 4) for b in box_outs], 1)
    classes = torch.argmax(cls, dim=-1)
    logit = TieMax.apply(cls)
    an = torch.as_tensor(anchors(image_size, anchor_scale), dtype=box.dtype)
    yca = (an[:, 0] + an[:, 2]) / 2
    xca = (an[:, 1] + an[:, 3]) / 2
    ha = an[:, 2] - an[:, 0]
    wa = an[:, 3] - an[:, 1]
    bd = box.detach()
    ty, tx, th, tw = bd.unbind(-1)
    w = torch.exp(tw) * wa
    h = torch.exp(th) * ha
    yc = ty * ha + yca
    xc = tx * wa + xca
    boxes = torch.stack([yc - h / 2.0, xc - w / 2.0, yc + h / 2.0, xc + w / 2.0], -1)
    return torch.sigmoid(logit), classes, boxes
