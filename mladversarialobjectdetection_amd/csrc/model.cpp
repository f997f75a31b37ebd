// model.cpp — victim architecture walk (see model.hpp for the reference map).
#include "model.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <stdexcept>

namespace phx {

namespace {

struct BlockArgs {
  int r, k, s, e, i, o;
  float se;
};

// efficientnet_builder.py:163-168 (== efficientnet_lite_builder.py:46-51)
const BlockArgs kBlocks[] = {
    {1, 3, 1, 1, 32, 16, 0.25f}, {2, 3, 2, 6, 16, 24, 0.25f},  {2, 5, 2, 6, 24, 40, 0.25f},
    {3, 3, 2, 6, 40, 80, 0.25f}, {3, 5, 1, 6, 80, 112, 0.25f}, {4, 5, 2, 6, 112, 192, 0.25f},
    {1, 3, 1, 6, 192, 320, 0.25f},
};

// efficientnet_model.py:129-143
int round_filters(int filters, double mult, bool skip) {
  if (skip || mult == 0.0) return filters;
  const int divisor = 8;
  double f = filters * mult;
  int nf = std::max(divisor, (int)(f + divisor / 2.0) / divisor * divisor);
  if (nf < 0.9 * f) nf += divisor;
  return nf;
}

// efficientnet_model.py:146-151
int round_repeats(int r, double mult) { return (int)std::ceil(mult * r); }

// TF 'SAME' padding: total = max((ceil(in/s)-1)*s + k - in, 0), top = total/2.
void same_pad(int in, int k, int s, int* out, int* pad_before) {
  int o = (in + s - 1) / s;
  int total = std::max((o - 1) * s + k - in, 0);
  *out = o;
  *pad_before = total / 2;
}

std::string fmt(const char* f, int a) {
  char buf[256];
  snprintf(buf, sizeof buf, f, a);
  return buf;
}
std::string fmt2(const char* f, int a, int b) {
  char buf[256];
  snprintf(buf, sizeof buf, f, a, b);
  return buf;
}

}  // namespace

bool get_model_config(const std::string& name, ModelConfig* c) {
  *c = ModelConfig();
  c->name = name;
  // hparams_config.py:301-389 (efficientdet_model_param_dict)
  struct D { const char* n; const char* bb; int img, fpn, cells, rep; double w, d; };
  static const D dtab[] = {
      {"efficientdet-d0", "efficientnet-b0", 512, 64, 3, 3, 1.0, 1.0},
      {"efficientdet-d1", "efficientnet-b1", 640, 88, 4, 3, 1.0, 1.1},
      {"efficientdet-d2", "efficientnet-b2", 768, 112, 5, 3, 1.1, 1.2},
      {"efficientdet-d3", "efficientnet-b3", 896, 160, 6, 4, 1.2, 1.4},
      {"efficientdet-d4", "efficientnet-b4", 1024, 224, 7, 4, 1.4, 1.8},
      {"efficientdet-d5", "efficientnet-b5", 1280, 288, 7, 4, 1.6, 2.2},
      {"efficientdet-d6", "efficientnet-b6", 1280, 384, 8, 5, 1.8, 2.6},
      {"efficientdet-d7", "efficientnet-b6", 1536, 384, 8, 5, 1.8, 2.6},
  };
  for (const D& d : dtab) {
    if (name == d.n) {
      c->backbone = d.bb;
      c->image_size = d.img;
      c->fpn_num_filters = d.fpn;
      c->fpn_cell_repeats = d.cells;
      c->box_class_repeats = d.rep;
      c->width_coefficient = d.w;
      c->depth_coefficient = d.d;
      if (name == "efficientdet-d6" || name == "efficientdet-d7") c->fpn_weight_method = 1;  // 'sum'
      if (name == "efficientdet-d7") c->anchor_scale = 5.0f;
      // b0 disables drop connect (efficientdet_keras.py:803-804); others keep 0.8
      // (efficientnet_builder.py:174).
      c->survival_prob = (std::string(d.bb) == "efficientnet-b0") ? 0.0 : 0.8;
      return true;
    }
  }
  // hparams_config.py:392-467 (efficientdet_lite_param_dict), lite_common_param :392-397
  struct L { const char* n; const char* bb; int img, fpn, cells, rep; float as; double w, d; };
  static const L ltab[] = {
      {"efficientdet-lite0", "efficientnet-lite0", 320, 64, 3, 3, 3.0f, 1.0, 1.0},
      {"efficientdet-lite1", "efficientnet-lite1", 384, 88, 4, 3, 3.0f, 1.0, 1.1},
      {"efficientdet-lite2", "efficientnet-lite2", 448, 112, 5, 3, 3.0f, 1.1, 1.2},
      {"efficientdet-lite3", "efficientnet-lite3", 512, 160, 6, 4, 4.0f, 1.2, 1.4},
      {"efficientdet-lite4", "efficientnet-lite4", 640, 224, 7, 4, 4.0f, 1.4, 1.8},
  };
  for (const L& d : ltab) {
    if (name == d.n) {
      c->backbone = d.bb;
      c->image_size = d.img;
      c->fpn_num_filters = d.fpn;
      c->fpn_cell_repeats = d.cells;
      c->box_class_repeats = d.rep;
      c->anchor_scale = d.as;
      c->width_coefficient = d.w;
      c->depth_coefficient = d.d;
      c->lite = true;
      c->act = ACT_RELU6;
      c->fpn_weight_method = 1;
      for (int i = 0; i < 3; ++i) { c->mean_rgb[i] = 127.0f; c->stddev_rgb[i] = 128.0f; }
      c->survival_prob = 0.8;
      return true;
    }
  }
  return false;
}

NetBuilder::NetBuilder(const ModelConfig& cfg, int batch, bool training)
    : cfg_(cfg), batch_(batch), training_(training) {
  prog_.batch = batch;
}

int NetBuilder::new_tensor(int n, int h, int w, int c) {
  Tensor t;
  t.n = n; t.h = h; t.w = w; t.c = c;
  t.off = prog_.act_floats;
  // keep every tensor 64-byte aligned
  prog_.act_floats += (t.numel() + 15) / 16 * 16;
  prog_.tensors.push_back(t);
  return (int)prog_.tensors.size() - 1;
}

long NetBuilder::wref(const std::string& name, std::vector<int> shape, const std::string& kind) {
  auto it = wmap_.find(name);
  if (it != wmap_.end()) return it->second;
  size_t n = 1;
  for (int s : shape) n *= (size_t)s;
  WeightEntry e{name, shape, wfloats_, kind};
  weights_.push_back(e);
  long off = (long)wfloats_;
  wfloats_ += n;
  wmap_[name] = off;
  return off;
}

int NetBuilder::op_stem(int x, const std::string& pfx, int cout) {
  const Tensor tx = prog_.tensors[x];
  Op op;
  op.t = OP_STEM;
  op.k = 3; op.stride = 2;
  int oh, ow;
  same_pad(tx.h, 3, 2, &oh, &op.pad_t);
  same_pad(tx.w, 3, 2, &ow, &op.pad_l);
  op.w = wref(pfx + "/conv2d/kernel", {3, 3, tx.c, cout}, "kernel");
  op.in[0] = x; op.nin = 1;
  op.out = new_tensor(tx.n, oh, ow, cout);
  op.name = pfx + "/conv2d";
  prog_.ops.push_back(op);
  return op.out;
}

int NetBuilder::op_pw(int x, const std::string& wname, int cout, bool bias) {
  const Tensor tx = prog_.tensors[x];
  Op op;
  op.t = OP_PW;
  op.w = wref(wname + "/kernel", {1, 1, tx.c, cout}, "kernel");
  if (bias) op.b = wref(wname + "/bias", {cout}, "bias");
  op.in[0] = x; op.nin = 1;
  op.out = new_tensor(tx.n, tx.h, tx.w, cout);
  op.name = wname;
  prog_.ops.push_back(op);
  return op.out;
}

int NetBuilder::op_dw(int x, const std::string& wname, int k, int stride) {
  const Tensor tx = prog_.tensors[x];
  Op op;
  op.t = OP_DW;
  op.k = k; op.stride = stride;
  int oh, ow;
  same_pad(tx.h, k, stride, &oh, &op.pad_t);
  same_pad(tx.w, k, stride, &ow, &op.pad_l);
  op.w = wref(wname, {k, k, tx.c, 1}, "kernel");
  op.in[0] = x; op.nin = 1;
  op.out = new_tensor(tx.n, oh, ow, tx.c);
  op.name = wname;
  prog_.ops.push_back(op);
  return op.out;
}

int NetBuilder::op_bn(int x, const std::string& pfx, int act) {
  const Tensor tx = prog_.tensors[x];
  Op op;
  op.t = OP_BN;
  op.act = act;
  op.gamma = wref(pfx + "/gamma", {tx.c}, "gamma");
  op.beta = wref(pfx + "/beta", {tx.c}, "beta");
  op.mmean = wref(pfx + "/moving_mean", {tx.c}, "moving_mean");
  op.mvar = wref(pfx + "/moving_variance", {tx.c}, "moving_variance");
  op.slot = prog_.n_slots++;
  prog_.slot_channels.push_back(tx.c);
  op.in[0] = x; op.nin = 1;
  op.out = new_tensor(tx.n, tx.h, tx.w, tx.c);
  prog_.tensors[op.out].level = tx.level;
  op.name = pfx;
  prog_.ops.push_back(op);
  return op.out;
}

int NetBuilder::op_se(int x, const std::string& pfx, int cse) {
  const Tensor tx = prog_.tensors[x];
  Op op;
  op.t = OP_SE;
  op.cse = cse;
  op.w1 = wref(pfx + "/conv2d/kernel", {1, 1, tx.c, cse}, "kernel");
  op.b1 = wref(pfx + "/conv2d/bias", {cse}, "bias");
  op.w2 = wref(pfx + "/conv2d_1/kernel", {1, 1, cse, tx.c}, "kernel");
  op.b2 = wref(pfx + "/conv2d_1/bias", {tx.c}, "bias");
  op.act = cfg_.act;
  op.slot = prog_.n_slots++;
  prog_.slot_channels.push_back(tx.c);
  op.in[0] = x; op.nin = 1;
  op.out = new_tensor(tx.n, tx.h, tx.w, tx.c);
  op.name = pfx;
  prog_.ops.push_back(op);
  return op.out;
}

int NetBuilder::op_add(int a, int b) {
  const Tensor ta = prog_.tensors[a];
  Op op;
  op.t = OP_ADD;
  op.in[0] = a; op.in[1] = b; op.nin = 2;
  op.out = new_tensor(ta.n, ta.h, ta.w, ta.c);
  op.name = "add";
  prog_.ops.push_back(op);
  return op.out;
}

int NetBuilder::op_maxpool(int x, int k, int stride, int oh, int ow) {
  const Tensor tx = prog_.tensors[x];
  Op op;
  op.t = OP_MAXPOOL;
  op.k = k; op.stride = stride;
  int o1, o2;
  same_pad(tx.h, k, stride, &o1, &op.pad_t);
  same_pad(tx.w, k, stride, &o2, &op.pad_l);
  if (o1 != oh || o2 != ow) throw std::runtime_error("maxpool output size mismatch");
  op.in[0] = x; op.nin = 1;
  op.out = new_tensor(tx.n, oh, ow, tx.c);
  op.name = "max_pool";  // renamed by resample() to <prefix>/max_pool
  prog_.ops.push_back(op);
  return op.out;
}

int NetBuilder::op_upsample(int x, int oh, int ow) {
  const Tensor tx = prog_.tensors[x];
  Op op;
  op.t = OP_UPSAMPLE;
  op.in[0] = x; op.nin = 1;
  op.out = new_tensor(tx.n, oh, ow, tx.c);
  op.name = "upsample";
  prog_.ops.push_back(op);
  return op.out;
}

int NetBuilder::op_fuse(const std::vector<int>& xs, const std::string& pfx, int act) {
  const Tensor t0 = prog_.tensors[xs[0]];
  Op op;
  op.t = OP_FUSE;
  op.act = act;
  op.fuse_method = cfg_.fpn_weight_method;
  op.nin = (int)xs.size();
  for (int i = 0; i < op.nin; ++i) {
    op.in[i] = xs[i];
    if (op.fuse_method == 0)
      op.wsm[i] = wref(pfx + (i == 0 ? std::string("/WSM") : "/WSM_" + std::to_string(i)), {1},
                       "wsm");
  }
  op.out = new_tensor(t0.n, t0.h, t0.w, t0.c);
  op.name = pfx + "/fuse";
  prog_.ops.push_back(op);
  return op.out;
}

// keras SeparableConv2D(depth_multiplier=1, 3x3, same, bias): depthwise -> pointwise -> bias
int NetBuilder::sepconv(int x, const std::string& pfx, int cout) {
  int y = op_dw(x, pfx + "/depthwise_kernel", 3, 1);
  // pointwise kernel registered under the separable layer's name
  const Tensor ty = prog_.tensors[y];
  Op op;
  op.t = OP_PW;
  op.w = wref(pfx + "/pointwise_kernel", {1, 1, ty.c, cout}, "kernel");
  op.b = wref(pfx + "/bias", {cout}, "bias");
  op.in[0] = y; op.nin = 1;
  op.out = new_tensor(ty.n, ty.h, ty.w, cout);
  prog_.tensors[op.out].level = ty.level;
  op.name = pfx + "/pointwise";
  prog_.ops.push_back(op);
  return op.out;
}

void NetBuilder::build_backbone(std::vector<int>* feats) {
  const std::string bb = cfg_.backbone;
  const bool fix = cfg_.lite;
  const double wc = cfg_.width_coefficient, dc = cfg_.depth_coefficient;
  const int act = cfg_.act;
  // Stem: efficientnet_model.py:507-528
  int x = op_stem(prog_.input, bb + "/stem", round_filters(32, wc, fix));
  x = op_bn(x, bb + "/stem/tpu_batch_normalization", act);

  // Expand the block list: efficientnet_model.py:645-703
  struct B { int k, s, e, i, o; float se; };
  std::vector<B> blocks;
  const int nargs = (int)(sizeof(kBlocks) / sizeof(kBlocks[0]));
  for (int a = 0; a < nargs; ++a) {
    const BlockArgs& ba = kBlocks[a];
    int inf = round_filters(ba.i, wc, false);
    int outf = round_filters(ba.o, wc, false);
    int rep = (fix && (a == 0 || a == nargs - 1)) ? ba.r : round_repeats(ba.r, dc);
    blocks.push_back({ba.k, ba.s, ba.e, inf, outf, ba.se});
    for (int r = 1; r < rep; ++r) blocks.push_back({ba.k, 1, ba.e, outf, outf, ba.se});
  }
  const int nb = (int)blocks.size();
  std::vector<int> reductions;
  for (int idx = 0; idx < nb; ++idx) {
    const B& b = blocks[idx];
    const std::string pfx = bb + fmt("/blocks_%d", idx);
    const int xin = x;
    const int cin = prog_.tensors[x].c;
    int cid = 0, bid = 0;
    auto conv_name = [&]() { int i = cid++; return i == 0 ? std::string("conv2d") : fmt("conv2d_%d", i); };
    auto bn_name = [&]() {
      int i = bid++;
      return i == 0 ? std::string("tpu_batch_normalization") : fmt("tpu_batch_normalization_%d", i);
    };
    int filters = b.i * b.e;
    if (b.e != 1) {  // expand: efficientnet_model.py:295-311, 388
      x = op_pw(x, pfx + "/" + conv_name(), filters, false);
      x = op_bn(x, pfx + "/" + bn_name(), act);
    }
    // depthwise: :321-328, 390
    x = op_dw(x, pfx + "/depthwise_conv2d/depthwise_kernel", b.k, b.s);
    x = op_bn(x, pfx + "/" + bn_name(), act);
    if (!cfg_.lite && b.se > 0) {  // SE: :337-341, :154-196
      int cse = std::max(1, (int)(b.i * b.se));
      x = op_se(x, pfx + "/se", cse);
    }
    // project: :344-359, 397
    x = op_pw(x, pfx + "/" + conv_name(), b.o, false);
    x = op_bn(x, pfx + "/" + bn_name(), ACT_NONE);
    if (b.s == 1 && b.i == b.o) {  // id_skip: :406-413
      x = op_add(x, xin);
      // drop connect on the block branch before the add (:411-412, utils.py:329-344) with the
      // survival probability decayed per block (efficientnet_model.py:752-755); training only
      if (cfg_.survival_prob > 0.0 && batch_ > 0 && training_) {
        const double drop_rate = 1.0 - cfg_.survival_prob;
        prog_.ops.back().survival = (float)(1.0 - drop_rate * (double)idx / (double)nb);
        prog_.ops.back().drop_block = idx;
      }
    }
    (void)cin;
    // reduction endpoints: :751-762
    bool is_red = (idx == nb - 1) || (blocks[idx + 1].s > 1);
    if (is_red) reductions.push_back(x);
  }
  // all_feats[min_level:max_level+1] with all_feats = [features, reduction_1..5]
  // (efficientdet_keras.py:887-888): P3..P5 = reduction_3..5
  for (int l = cfg_.min_level; l <= std::min(cfg_.max_level, 5); ++l) feats->push_back(reductions[l - 1]);
}

// ResampleFeatureMap.call, efficientdet_keras.py:297-324 (apply_bn=True, conv_after_downsample=False)
int NetBuilder::resample(int x, int th, int tw, const std::string& pfx) {
  const int target_c = cfg_.fpn_num_filters;
  Tensor t = prog_.tensors[x];
  auto maybe_1x1 = [&](int v) {
    if (prog_.tensors[v].c != target_c) {
      v = op_pw(v, pfx + "/conv2d", target_c, true);
      v = op_bn(v, pfx + "/bn", ACT_NONE);
    }
    return v;
  };
  if (t.h > th && t.w > tw) {
    x = maybe_1x1(x);
    int sh = (t.h - 1) / th + 1;
    int sw = (t.w - 1) / tw + 1;
    if (sh != sw) throw std::runtime_error("non-square pooling unsupported");
    x = op_maxpool(x, sh + 1, sh, th, tw);
    prog_.ops.back().name = pfx + "/max_pool";
  } else if (t.h <= th && t.w <= tw) {
    x = maybe_1x1(x);
    if (t.h < th || t.w < tw) {
      x = op_upsample(x, th, tw);
      prog_.ops.back().name = pfx + "/upsample";
    }
  } else {
    throw std::runtime_error("incompatible resampling");
  }
  return x;
}

void NetBuilder::build() {
  const int n = batch_ > 0 ? batch_ : 1;
  const int S = cfg_.image_size;
  prog_.input = new_tensor(n, S, S, 3);
  std::vector<int> feats;
  build_backbone(&feats);
  // P6, P7: efficientdet_keras.py:815-827, 890-892
  for (int level = 6; level <= cfg_.max_level; ++level) {
    const Tensor t = prog_.tensors[feats.back()];
    int th = (t.h + 1) / 2, tw = (t.w + 1) / 2;
    feats.push_back(resample(feats.back(), th, tw, fmt("resample_p%d", level)));
  }
  const int nlev = cfg_.max_level - cfg_.min_level + 1;
  // BiFPN node list: fpn_configs.py:24-72
  struct N { int level; std::vector<int> inputs; };
  std::vector<N> nodes;
  {
    std::map<int, std::vector<int>> ids;
    for (int i = 0; i < nlev; ++i) ids[cfg_.min_level + i] = {i};
    int cnt = nlev;
    for (int i = cfg_.max_level - 1; i >= cfg_.min_level; --i) {
      nodes.push_back({i, {ids[i].back(), ids[i + 1].back()}});
      ids[i].push_back(cnt++);
    }
    for (int i = cfg_.min_level + 1; i <= cfg_.max_level; ++i) {
      std::vector<int> in = ids[i];
      in.push_back(ids[i - 1].back());
      nodes.push_back({i, in});
      ids[i].push_back(cnt++);
    }
  }
  // FPNCells.call / FPNCell / FNode: efficientdet_keras.py:720-775, 164-172
  for (int cell = 0; cell < cfg_.fpn_cell_repeats; ++cell) {
    std::vector<int> all = feats;
    for (size_t ni = 0; ni < nodes.size(); ++ni) {
      const N& nd = nodes[ni];
      const std::string npfx = fmt2("fpn_cells/cell_%d/fnode%d", cell, (int)ni);
      const Tensor target = prog_.tensors[all[nd.level - cfg_.min_level]];
      std::vector<int> ins;
      for (size_t i = 0; i < nd.inputs.size(); ++i) {
        int off = nd.inputs[i];
        char rn[64];
        snprintf(rn, sizeof rn, "/resample_%d_%d_%d", (int)i, off, (int)all.size());
        ins.push_back(resample(all[off], target.h, target.w, npfx + rn));
      }
      char on[64];
      snprintf(on, sizeof on, "/op_after_combine%d", (int)all.size());
      // OpAfterCombine (conv_bn_act_pattern=False): act -> separable conv -> bn (:214-221)
      int v = op_fuse(ins, npfx, cfg_.act);
      v = sepconv(v, npfx + on + "/conv", cfg_.fpn_num_filters);
      v = op_bn(v, npfx + on + "/bn", ACT_NONE);
      prog_.tensors[v].level = nd.level;
      all.push_back(v);
    }
    std::vector<int> nf;
    for (int level = cfg_.min_level; level <= cfg_.max_level; ++level) {
      for (int i = (int)nodes.size() - 1; i >= 0; --i) {
        if (nodes[i].level == level) {
          nf.push_back(all[feats.size() + i]);
          break;
        }
      }
    }
    feats = nf;
  }
  // ClassNet / BoxNet: efficientdet_keras.py:414-471, 576-632
  const int na = cfg_.num_anchors();
  auto head = [&](const std::string& net, const std::string& tag, int nout, std::vector<int>* outs) {
    for (int l = 0; l < nlev; ++l) {
      int v = feats[l];
      for (int i = 0; i < cfg_.box_class_repeats; ++i) {
        v = sepconv(v, net + "/" + tag + fmt("-%d", i), cfg_.fpn_num_filters);
        v = op_bn(v, net + "/" + tag + fmt2("-%d-bn-%d", i, cfg_.min_level + l), cfg_.act);
      }
      v = sepconv(v, net + "/" + tag + "-predict", nout);
      prog_.tensors[v].level = cfg_.min_level + l;
      outs->push_back(v);
    }
  };
  head("class_net", "class", cfg_.num_classes * na, &prog_.cls_out);
  head("box_net", "box", 4 * na, &prog_.box_out);
  if (batch_ > 0) plan_backward();
}

// Static backward plan: which ops run, which input grads are overwritten vs accumulated.
// Only the class head carries a loss gradient (the box outputs feed non-differentiable
// masks, attacker.py:132-140), so the box head and everything reachable only through it is
// pruned.
void NetBuilder::plan_backward() {
  auto& T = prog_.tensors;
  std::vector<char> has(T.size(), 0);
  for (int t : prog_.cls_out) has[t] = 1;
  // reverse sweep: an op runs backward iff its output receives a gradient
  for (int i = (int)prog_.ops.size() - 1; i >= 0; --i) {
    Op& op = prog_.ops[i];
    op.bwd = has[op.out] != 0;
    if (!op.bwd) continue;
    for (int j = 0; j < op.nin; ++j) {
      int t = op.in[j];
      op.acc[j] = has[t] != 0;  // a later op (earlier in this sweep) already wrote it
      has[t] = 1;
    }
  }
  // Residual adds: both input gradients equal the output's.  When the add is the last consumer
  // of both inputs (nothing accumulated into them yet) and has no drop connect, both inputs take
  // the output's gradient buffer instead of copies of it.  Later accumulations into the skip input
  // (the block's expand conv) happen after every reader of the branch gradient (project dgrad,
  // BN sums) in the reverse sweep.  Aliases are resolved last-op-first so chains of blocks share.
  std::vector<char> alias(T.size(), 0);
  std::vector<int> alias_ops;
  for (int i = (int)prog_.ops.size() - 1; i >= 0; --i) {
    const Op& op = prog_.ops[i];
    if (op.t != OP_ADD || !op.bwd || op.survival > 0.f || op.in[0] == op.in[1]) continue;
    if (op.acc[0] || op.acc[1] || alias[op.in[0]] || alias[op.in[1]]) continue;
    alias[op.in[0]] = alias[op.in[1]] = 1;
    alias_ops.push_back(i);
  }
  size_t g = 0;
  for (size_t t = 0; t < T.size(); ++t) {
    if (has[t] && !alias[t]) {
      T[t].goff = (long)g;
      g += (T[t].numel() + 15) / 16 * 16;
    }
  }
  for (int i : alias_ops) {  // last op first: an add's output may itself alias a later add's
    const Op& op = prog_.ops[i];
    T[op.in[0]].goff = T[op.in[1]].goff = T[op.out].goff;
  }
  prog_.grad_floats = g;
}

}  // namespace phx
