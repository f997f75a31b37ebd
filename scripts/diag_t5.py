"""GPU diagnostic: decompose the gradient of one tensor (the output of a given BN) into its
consumers' contributions and compare with the product's."""
import sys
import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from bench import synth_boxes, synth_images  # noqa: E402
from mladversarialobjectdetection_amd import weights as W  # noqa: E402
from mladversarialobjectdetection_amd.attacker import EfficientDetVictim, PatchAttacker  # noqa: E402
from oracle import step as ST  # noqa: E402
from oracle import detector as D  # noqa: E402

torch.set_num_threads(16)
S, B = (int(v) for v in sys.argv[1].split("x"))
cell = sys.argv[2] if len(sys.argv) > 2 else "0"
v = EfficientDetVictim("efficientdet-d0", "synthetic", seed=0, image_size=S, max_batch=B, rng_seed=0)
wd = W.unpack(v.manifest, v.blob.copy())
idx = list(range(B))
imgs = synth_images(idx, S)
boxes = synth_boxes(idx, S)
att = PatchAttacker(v, seed=7)
att.cur_step = 1
att.call(torch.as_tensor(imgs).cuda(), boxes=boxes)
torch.cuda.synchronize()
orig_init = D.Detector.__init__


def init(self, *a, **k):
    orig_init(self, *a, **k)
    self.taps = {}


D.Detector.__init__ = init
ref = ST.attack_step(wd, imgs, att.patch.cpu().numpy(), np.float32(0.4), boxes=boxes, seed=0, step=1, image_size=S)
taps = ref["det"].taps


def gpu(name, which, shape):
    buf = torch.empty(int(np.prod(shape)), device="cuda")
    v.ctx.call("phx_debug_tap", name.encode(), which, buf.data_ptr(), buf.numel(), torch.cuda.current_stream().cuda_stream)
    return buf.cpu().numpy().reshape(shape).astype(np.float64)


def nhwc(t):
    return t.detach().permute(0, 2, 3, 1).contiguous().numpy()


t5 = f"fpn_cells/cell_{cell}/fnode5/op_after_combine10/bn"
mp = f"fpn_cells/cell_{cell}/fnode6/resample_2_10_11/max_pool"
x5, y5 = taps[t5]
R = nhwc(y5.grad)
G = gpu(t5, 1, R.shape)
Rm = nhwc(taps[mp][1].grad)
Gm = gpu(mp, 1, Rm.shape)
# maxpool contribution through the oracle's routing
yy = y5.detach().clone().requires_grad_(True)
pt, pb = D.same_pads(yy.shape[2], 3, 2)
out = F.max_pool2d(F.pad(yy, (pt, pb, pt, pb), value=-float("inf")), 3, 2)
out.backward(taps[mp][1].grad)
C = nhwc(yy.grad)
n = np.linalg.norm
print("t5 grad rel", n(G - R) / n(R), "|R|", n(R), "|C|", n(C))
print("maxpool-out grad rel", n(Gm - Rm) / n(Rm))
for lab, H in [("R-C", R - C), ("R+C", R + C)]:
    print(lab, n(G - H) / n(R))
E = G - R
print("error per image", [n(E[b]) for b in range(B)])
print("error per row (img0)", [round(n(E[0, i]), 6) for i in range(E.shape[1])])
print("error per col (img0)", [round(n(E[0, :, j]), 6) for j in range(E.shape[2])])
ch = [n(E[..., c]) for c in range(E.shape[3])]
print("top channels", np.argsort(ch)[::-1][:8], sorted(ch)[::-1][:8])
b, c = 0, int(np.argmax(ch))
print("oracle BN-out window (rows 5..9, cols 5..9):")
print(nhwc(y5)[b, 5:10, 5:10, c])
print("oracle maxpool out", nhwc(taps[mp][0])[b, 2:5, 2:5, c])
print("gpu    maxpool out", gpu(mp, 0, Rm.shape)[b, 2:5, 2:5, c])
