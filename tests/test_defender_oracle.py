"""CPU checks of the defender restatement (oracle/defender.py) itself: the Keras layer conventions
it encodes and its autograd gradient.  No GPU."""
import numpy as np
import torch

from oracle import defender as DF


def _flat_params(seed=0, scale=0.2):
    layout, bns = DF.unet_layout()
    rng = np.random.default_rng(seed)
    parts = []
    for name, shape in layout:
        n = int(np.prod(shape))
        parts.append(np.ones(n) if name.endswith("gamma") else rng.normal(0, scale, n))
    return np.concatenate(parts), {nm: (np.zeros(c), np.ones(c)) for nm, c in bns}


def test_layout_matches_generator_definition():
    """generator.py: 4 encoder blocks of 8*2^i filters, a 128-filter bottleneck, 4 attention decoder
    blocks (64, 32, 16, 8) and a 3-channel 1x1 output: 553,439 variables, 30 batch norms."""
    layout, bns = DF.unet_layout()
    assert sum(int(np.prod(s)) for _, s in layout) == 553439
    assert len(bns) == 30
    d = dict(layout)
    assert d["conv0/cnv1/kernel"] == (3, 3, 3, 8)
    assert d["conv4/cnv2/kernel"] == (3, 3, 128, 128)
    assert d["deconv0/cnv/kernel"] == (3, 3, 64, 128)  # Conv2DTranspose: [k, k, out, in]
    assert d["deconv3/convblock/cnv1/kernel"] == (3, 3, 16, 8)
    assert d["deconv2/attention/conv3/kernel"] == (1, 1, 16, 1)
    assert d["output/kernel"] == (1, 1, 8, 3)


def test_transposed_conv_is_tf_same_stride2():
    """Conv2DTranspose(3, strides 2, 'same'): out[2i + k] += x[i] w[k] (TF pads the equivalent
    forward conv (0, 1)), output 2H x 2W — checked against the direct definition."""
    rng = np.random.default_rng(1)
    H, W, ci, co = 3, 4, 2, 3
    x = rng.normal(size=(1, H, W, ci))
    w = rng.normal(size=(3, 3, co, ci))
    b = rng.normal(size=co)
    ref = np.zeros((1, 2 * H + 2, 2 * W + 2, co))
    for i in range(H):
        for j in range(W):
            for ky in range(3):
                for kx in range(3):
                    ref[0, 2 * i + ky, 2 * j + kx] += w[ky, kx] @ x[0, i, j]
    ref = ref[:, :2 * H, :2 * W] + b
    net = DF.UNet({"t/kernel": w, "t/bias": b}, {})
    got = net.tconv(torch.as_tensor(x).permute(0, 3, 1, 2), "t").permute(0, 2, 3, 1).detach().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)


def test_unet_gradient_matches_finite_differences():
    """Directional derivatives of the restated loss along single variables, central differences at
    eps 1e-7 in fp64 (the leaky kinks and max-pool switches make larger steps non-smooth)."""
    flat, moving = _flat_params()
    layout, _ = DF.unet_layout()
    rng = np.random.default_rng(2)
    x = torch.as_tensor(rng.uniform(-1, 1, (2, 64, 64, 3)))
    t = torch.as_tensor(rng.uniform(-0.5, 0.5, (2, 64, 64, 3)))

    def loss_of(f):
        net = DF.UNet(DF.unpack(f, layout), moving, seed=3, step=1)
        u = 2.0 * net(x)
        return ((t.reshape(2, -1) - u.reshape(2, -1)) ** 2).mean(1).sum(), net

    loss, net = loss_of(flat)
    grads = torch.autograd.grad(loss, [net.p[n] for n, _ in layout])
    g = np.concatenate([q.detach().numpy().reshape(-1) for q in grads])
    offs = {}
    off = 0
    for name, shape in layout:
        offs[name] = (off, int(np.prod(shape)))
        off += int(np.prod(shape))
    for name in ("output/kernel", "deconv1/attention/conv3/kernel", "conv3/bn2/gamma", "deconv2/cnv/kernel"):
        o, n = offs[name]
        d = np.zeros_like(flat)
        d[o:o + n] = rng.normal(size=n)
        eps = 1e-7
        fd = (loss_of(flat + eps * d)[0].item() - loss_of(flat - eps * d)[0].item()) / (2 * eps)
        assert abs(fd - g @ d) <= 2e-3 * abs(g @ d) + 1e-7, name


def test_masker_targets_are_original_minus_patched():
    rng = np.random.default_rng(5)
    imgs = rng.uniform(-1, 1, (2, 256, 256, 3)).astype(np.float32)
    boxes = [np.array([[20, 30, 200, 120]], np.float32), np.array([[5, 5, 240, 140], [50, 50, 90, 90]], np.float32)]
    patched, targets = DF.masker(imgs, boxes, 9, 0, 0)
    np.testing.assert_allclose(imgs - patched, targets, atol=1e-12)
    assert (targets != 0).mean() > 0.01
    # the crops are a permutation of the batch's own top-left 240 x 240 regions (flipped)
    pt = DF.train_patches(imgs, 9, 0, 0)
    for b in range(2):
        src = DF.shuffle_perm(2, 9, 0, 0)[b]
        lr, ud = DF.flips(9, 0, b)
        p = imgs[src, :240, :240]
        p = p[:, ::-1] if lr else p
        p = p[::-1] if ud else p
        np.testing.assert_array_equal(pt[b], p)


def test_dropout_mask_rate():
    keep = DF.dropout_mask((2, 64, 64, 8), 0, 3, 1, 0)
    assert abs(keep.mean() - 0.8) < 0.01
    assert not np.array_equal(keep[0], keep[1])
