// defender.cpp — the defender step (BASELINE C5):
//   PatchAttackDefender.call(images, training=True)   attack_detection.py:168-206
//     first pass (frozen protege)                      :96-166 -> def_first_pass (api.cpp)
//     Masker (training: self-supervised patches)       :321-498 -> EOT kernels (kernels_eot.hip)
//     updates = 2 * PatchNeutralizer(images)           generator.py:17-277 -> kernels_unet.hip + GEMM
//     loss = sum_b mean((targets - updates)^2)         :194-198
//     tape.gradient(loss, U-Net variables)             :202-206
// The U-Net is hand-scheduled here (it is fixed: n_filters 8, four encoder blocks, a bottleneck,
// four attention decoder blocks, a 1x1 tanh output); every tensor lives at a per-batch-size arena
// offset, and the backward walks the same layers in reverse writing each variable's gradient once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"
#include "phx.h"
#include "post.hpp"
#include "unet.hpp"

using namespace phx;

namespace {

struct DevFree {
  void operator()(void* p) const { (void)hipFree(p); }
};
using DBuf = std::unique_ptr<void, DevFree>;

inline int r4(int k) { return (k + 3) / 4 * 4; }

struct UConv {
  std::string name;
  int k = 3, ci = 0, co = 0;
  int kind = 0;          // 0 conv 3x3, 2 transposed conv 3x3 s2, 4 1x1
  long w = 0, b = 0;     // offsets in the flat parameters
  int kp_f = 0, kp_d = 0;
  long bt_f = -1, bt_d = -1;  // offsets of the GEMM B operands in the Bt arena (-1: none)
};

struct UBn {
  std::string name;
  int c = 0;
  long gamma = 0, beta = 0;  // flat parameters
  long mm = 0, mv = 0;       // moving statistics buffer
  float *mean = nullptr, *rstd = nullptr, *sc = nullptr, *mdz = nullptr, *mdzx = nullptr;
};

struct Block {
  int c1, b1, c2, b2;  // conv / bn indices
};

struct Att {
  int up, cnv1, bn1, cnv2, bn2, conv3, bn3;
  Block blk;
};

// one level's tensors
struct Lvl {
  int B = 0, H = 0, W = 0, C = 0;
  long M() const { return (long)B * H * W; }
};

}  // namespace

struct phx_def {
  phx_ctx* victim = nullptr;
  int device = 0, max_batch = 0, S = 0;
  uint64_t seed = 0;
  std::string err;
  std::vector<std::pair<std::string, std::vector<int>>> manifest;
  std::vector<UConv> convs;
  std::vector<UBn> bns;
  Block enc[4], c4;
  Att dec[4];
  int out_conv = -1;
  long nparams = 0, nmoving = 0, nbt = 0;
  DBuf moving;  // [mean | var] per BN
  // cross-step first-pass prefetch (phx_def_set_next): the next batch's first pass runs on `side`
  // beside this step's U-Net work, into pboxes / pcount[slot]
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_done = nullptr;
  struct Next {
    const float* images = nullptr;
    int B = 0, gimg0 = 0;
  } next;
  struct Pre {
    const float* images = nullptr;
    int B = 0, gimg0 = 0, slot = 0;
    int64_t step = -1;
    bool pending = false;
    uint64_t gen = 0;  // the victim's generation (ctx_generation) it was made at
  } pre;
  float* pboxes[2] = {nullptr, nullptr};
  int* pcount[2] = {nullptr, nullptr};
  const float* last_boxes = nullptr;  // the boxes the last step placed its patches by (phx_def_debug)
  const int* last_count = nullptr;
  // `s` waits for the prefetch in flight (the victim ctx and its executor are in use until then)
  void join(hipStream_t s) {
    if (pre.pending) PHX_HIP(hipStreamWaitEvent(s, ev_done, 0));
  }
  ~phx_def() {
    if (side) {
      (void)hipStreamSynchronize(side);
      (void)hipStreamDestroy(side);
      (void)hipEventDestroy(ev_fork);
      (void)hipEventDestroy(ev_done);
    }
  }
  // per batch-size workspace
  int wsB = 0;
  std::vector<DBuf> owned;
  template <class T>
  T* alloc(size_t n) {
    void* p = nullptr;
    PHX_HIP(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
    owned.emplace_back(p);
    return reinterpret_cast<T*>(p);
  }
  // workspace tensors
  float* bt = nullptr;
  struct EncT { float *y1, *a1, *y2, *a2, *p, *denc; uint8_t* arg; } et[4];
  struct C4T { float *y1, *a1, *y2, *a2; } c4t;
  struct DecT { float *up, *g, *xs, *s, *t, *cat, *y1, *a1, *y2, *a2; } dt[4];
  float *upd = nullptr, *dz = nullptr, *tmpX = nullptr, *tmpY = nullptr, *tmpT = nullptr, *col = nullptr;
  float *gpart = nullptr, *wpart = nullptr, *d1 = nullptr, *d2 = nullptr;
  double *cpart = nullptr, *lpart = nullptr;
  // Masker
  EotDims ed{};
  ImgParams* img = nullptr;
  BoxPlace* place = nullptr;
  SpanEntry* spans = nullptr;
  double* ysum = nullptr;
  float *ymean = nullptr, *matched = nullptr, *rstore = nullptr, *crops = nullptr, *patched = nullptr, *mask = nullptr;
  float* boxes = nullptr;
  int *count = nullptr, *info = nullptr, *eerr = nullptr;
  size_t ws_bytes = 0;

  int add_conv(const std::string& name, int k, int ci, int co, int kind) {
    UConv c;
    c.name = name;
    c.k = k; c.ci = ci; c.co = co; c.kind = kind;
    c.w = nparams;
    if (kind == 2) manifest.push_back({name + "/kernel", {k, k, co, ci}});
    else manifest.push_back({name + "/kernel", {k, k, ci, co}});
    nparams += (long)k * k * ci * co;
    c.b = nparams;
    manifest.push_back({name + "/bias", {co}});
    nparams += co;
    if (kind == 0) { c.kp_f = r4(9 * ci); c.kp_d = r4(9 * co); }
    else if (kind == 2) { c.kp_f = r4(9 * ci); c.kp_d = r4(9 * co); }
    else { c.kp_f = ci; c.kp_d = co; }
    if (co >= 4 || kind != 4) {  // the 1-channel attention conv and the 3-channel output have own kernels
      c.bt_f = nbt;
      nbt += (long)co * c.kp_f;
      c.bt_d = nbt;
      nbt += (long)ci * c.kp_d;
    }
    convs.push_back(c);
    return (int)convs.size() - 1;
  }
  int add_bn(const std::string& name, int c) {
    UBn b;
    b.name = name;
    b.c = c;
    b.gamma = nparams;
    manifest.push_back({name + "/gamma", {c}});
    nparams += c;
    b.beta = nparams;
    manifest.push_back({name + "/beta", {c}});
    nparams += c;
    b.mm = nmoving;
    b.mv = nmoving + c;
    nmoving += 2 * c;
    bns.push_back(b);
    return (int)bns.size() - 1;
  }
  Block add_block(const std::string& name, int ci, int n) {
    Block k;
    k.c1 = add_conv(name + "/cnv1", 3, ci, n, 0);
    k.b1 = add_bn(name + "/bn1", n);
    k.c2 = add_conv(name + "/cnv2", 3, n, n, 0);
    k.b2 = add_bn(name + "/bn2", n);
    return k;
  }
  // generator.py:17-101 (n_filters 8) in the oracle's manifest order
  void build() {
    const int nf = 8;
    int ci = 3;
    for (int i = 0; i < 4; ++i) {
      enc[i] = add_block("conv" + std::to_string(i), ci, nf << i);
      ci = nf << i;
    }
    c4 = add_block("conv4", ci, nf * 16);
    ci = nf * 16;
    int m = 8;
    for (int i = 0; i < 4; ++i) {
      const int n = nf * m;
      const std::string p = "deconv" + std::to_string(i);
      Att& a = dec[i];
      a.up = add_conv(p + "/cnv", 3, ci, n, 2);
      a.cnv1 = add_conv(p + "/attention/cnv1", 1, n, n, 4);
      a.bn1 = add_bn(p + "/attention/bn1", n);
      a.cnv2 = add_conv(p + "/attention/cnv2", 1, n, n, 4);
      a.bn2 = add_bn(p + "/attention/bn2", n);
      a.conv3 = add_conv(p + "/attention/conv3", 1, n, 1, 4);
      a.bn3 = add_bn(p + "/attention/bn3", 1);
      a.blk = add_block(p + "/convblock", 2 * n, n);
      ci = n;
      m /= 2;
    }
    out_conv = add_conv("output", 1, nf, 3, 4);
  }
  std::string manifest_json() const {
    std::ostringstream js;
    js << "{\"n_params\":" << nparams << ",\"n_moving\":" << nmoving << ",\"params\":[";
    long off = 0;
    for (size_t i = 0; i < manifest.size(); ++i) {
      long n = 1;
      js << (i ? "," : "") << "{\"name\":\"" << manifest[i].first << "\",\"shape\":[";
      for (size_t j = 0; j < manifest[i].second.size(); ++j) {
        js << (j ? "," : "") << manifest[i].second[j];
        n *= manifest[i].second[j];
      }
      js << "],\"offset\":" << off << "}";
      off += n;
    }
    js << "],\"bn\":[";
    for (size_t i = 0; i < bns.size(); ++i)
      js << (i ? "," : "") << "{\"name\":\"" << bns[i].name << "\",\"channels\":" << bns[i].c
         << ",\"moving_mean\":" << bns[i].mm << ",\"moving_variance\":" << bns[i].mv << "}";
    js << "]}";
    return js.str();
  }
  // evaluation Masker (the attacker's 640^2 patch): reserved by the first evaluation of a workspace
  // (eval_reserve), freed with it
  float *ematched = nullptr, *erstore = nullptr;
  int eB = 0;
  size_t eval_bytes(int B) const;
  void eval_reserve(int B);

  void workspace(int B);
  void prep_weights(const float* W, hipStream_t s);
  // U-Net forward on `patched` (train: batch-statistics BN with moving-statistics update and
  // Dropout; else inference BN from the moving statistics, no Dropout), then the output layer and
  // loss against `mask` into *loss (and dz, its gradient)
  void unet_forward(int B, const float* W, bool train, int64_t stp, int gimg0, float* loss, hipStream_t s);
  void step(const float* images, int B, const float* boxes_in, const int* count_in, const float* params,
            float* grad, int64_t step, int gimg0, hipStream_t s);
  void eval(const float* images, int B, const float* boxes_in, const int* count_in, const float* params,
            const float* eval_patch, float* metrics, float* out_boxes, float* out_scores, int* out_count,
            int64_t stp, int gimg0, hipStream_t s);
};

namespace {

// a launch group on the victim context's profiler (phx_profile): kind, algorithmic FLOPs and bytes
struct DScope {
  ProfScope r;
  DScope(phx_ctx* v, const char* kind, double flops, double bytes, hipStream_t s)
      : r(prof_begin(v, kind, flops, bytes, s)) {}
  ~DScope() noexcept(false) { prof_end(r); }
};

void gemm(const float* A, const float* Bt, const float* bias, float* C, long M, int N, int K, bool acc, float* part,
          hipStream_t s) {
  launch_gemm(InX{A, nullptr, nullptr, nullptr, 0}, Bt, bias, C, (int)M, N, K, acc, nullptr, 1, s, part);
}

// PHX_UN_GATHER=0: the U-Net's wide 3x3 convs write their column matrix (k_im2col) and run the plain
// GEMM over it instead of gathering it inside the GEMM (read on every call: tests compare the two)
bool un_gather_on() {
  const char* e = std::getenv("PHX_UN_GATHER");
  return !(e && e[0] == '0');
}

// a 3x3 conv of more than kConvMaxN outputs (or K > kConvMaxKp): the GEMM over the gathered column
// matrix (k_im2col's gathers), implicit when the geometry allows it
void conv3_gemm(const float* x, float* col, const float* Bt, const float* bias, float* out, int B, int H, int W, int C,
                int Ho, int Wo, int N, int Kp, int mode, int st, int pt, int pl, float* part, hipStream_t s) {
  if (un_gather_on() && gemm_gather_ok(B, H, W, C, Ho, Wo, Kp, mode, st, pt, pl)) {
    launch_gemm_gather(x, B, H, W, C, Ho, Wo, mode, st, pt, pl, Bt, bias, out, N, Kp, s, part);
    return;
  }
  un_im2col(x, col, B, H, W, C, Ho, Wo, Kp, mode, st, pt, pl, s);
  // the implicit im2col's plan (no wave-split K), so both forms multiply in the same order
  if (gemm_impl_for(N) == 2)
    gemm2_run(0, InX{col, nullptr, nullptr, nullptr, 0}, GradX{}, Bt, bias, out, (int)((long)B * Ho * Wo), N, Kp, false,
              nullptr, 1, s, part, StatSink{}, gemm2_target_wgs(), GradSink{}, false, false);
  else
    gemm(col, Bt, bias, out, (long)B * Ho * Wo, N, Kp, false, part, s);
}

}  // namespace

void phx_def::workspace(int B) {
  if (B == wsB) return;
  PHX_HIP(hipDeviceSynchronize());
  pre = Pre{};  // (its buffers go with the old workspace)
  owned.clear();
  ws_bytes = 0;
  wsB = B;
  const int S_ = S;
  auto F = [&](size_t n) {
    ws_bytes += n * 4;
    return alloc<float>(n);
  };
  bt = F(nbt);
  size_t maxMC = 0, maxcol = 0, maxpart = 1, maxw = 1, maxcr = 1;
  auto note_gemm = [&](long M, int N, int K) { maxpart = std::max(maxpart, gemm_partial_floats((int)M, N, K)); };
  auto note_w = [&](long M, int Co, int Kp) { maxw = std::max(maxw, (size_t)un_wgrad_slices(M, Co, Kp) * Co * Kp); };
  auto note_cr = [&](long M, int C) { maxcr = std::max(maxcr, un_colred_doubles(M, C)); };
  auto note_conv = [&](const UConv& c, long M_out, long M_in) {
    maxcol = std::max(maxcol, (size_t)std::max(M_out * c.kp_f, M_in * (long)c.kp_d));
    note_gemm(M_out, c.co, c.kp_f);
    note_gemm(M_in, c.ci, c.kp_d);
    note_w(M_out, c.co, c.kp_f);
    note_cr(M_out, c.co);
  };
  for (int i = 0; i < 4; ++i) {
    const int H = S_ >> i, n = convs[enc[i].c1].co;
    const long M = (long)B * H * H;
    et[i].y1 = F(M * n); et[i].a1 = F(M * n); et[i].y2 = F(M * n); et[i].a2 = F(M * n);
    et[i].denc = F(M * n);
    et[i].p = F(M / 4 * n);
    ws_bytes += M / 4 * n;
    et[i].arg = alloc<uint8_t>(M / 4 * n);
    maxMC = std::max(maxMC, (size_t)M * convs[enc[i].c1].ci);
    maxMC = std::max(maxMC, (size_t)M * n);
    note_conv(convs[enc[i].c1], M, M);
    note_conv(convs[enc[i].c2], M, M);
  }
  {
    const int H = S_ >> 4, n = convs[c4.c1].co;
    const long M = (long)B * H * H;
    c4t.y1 = F(M * n); c4t.a1 = F(M * n); c4t.y2 = F(M * n); c4t.a2 = F(M * n);
    maxMC = std::max(maxMC, (size_t)M * n);
    note_conv(convs[c4.c1], M, M);
    note_conv(convs[c4.c2], M, M);
  }
  for (int i = 0; i < 4; ++i) {
    const int H = S_ >> (3 - i), n = convs[dec[i].up].co, hin = H / 2;
    const long M = (long)B * H * H, Min = (long)B * hin * hin;
    DecT& d = dt[i];
    d.up = F(M * n); d.g = F(M * n); d.xs = F(M * n); d.s = F(M * n); d.t = F(M);
    d.cat = F(M * 2 * n);
    d.y1 = F(M * n); d.a1 = F(M * n); d.y2 = F(M * n); d.a2 = F(M * n);
    maxMC = std::max(maxMC, (size_t)M * 2 * n);
    note_conv(convs[dec[i].up], M, Min);
    for (int c : {dec[i].cnv1, dec[i].cnv2}) note_conv(convs[c], M, M);
    note_w(M, 1, n);
    note_cr(M, n);
    note_conv(convs[dec[i].blk.c1], M, M);
    note_conv(convs[dec[i].blk.c2], M, M);
  }
  const long Mf = (long)B * S_ * S_;
  note_w(Mf, 3, 8);
  note_cr(Mf, 3);
  upd = F(Mf * 3);
  dz = F(Mf * 3);
  tmpX = F(maxMC);
  tmpY = F(maxMC);
  tmpT = F(maxMC);
  col = F(maxcol);
  gpart = F(maxpart);
  wpart = F(maxw);
  d1 = F(Mf);
  d2 = F(Mf);
  cpart = alloc<double>(maxcr);
  ws_bytes += maxcr * 8;
  lpart = alloc<double>(un_loss_blocks(Mf));
  for (UBn& b : bns) {
    b.mean = F(b.c); b.rstd = F(b.c); b.sc = F(b.c); b.mdz = F(b.c); b.mdzx = F(b.c);
  }
  // Masker (the EOT kernels with the defender's placement rule and printed per-image sources)
  ed.B = B;
  ed.H = ed.W = S_;
  ed.maxb = PHX_MAX_OUT;
  ed.P = std::min(240, S_);
  ed.span_stride = S_;
  const long psmax = S_ / 2 + 1;  // floor(longer side * 0.5) with boxes clipped to the image
  ed.rcap = (long)B * PHX_MAX_OUT * psmax * psmax * 3;
  const long nslot = (long)B * PHX_MAX_OUT;
  img = alloc<ImgParams>(B);
  place = reinterpret_cast<BoxPlace*>(alloc<char>(nslot * sizeof(BoxPlace) + (4 + 2 * B + 3 * nslot + 2 + 8 * B + 8 * nslot) * sizeof(int)));
  spans = alloc<SpanEntry>(nslot * S_);
  ysum = alloc<double>((size_t)B * 2 * 64);
  ymean = F((size_t)B * 2);
  matched = F((size_t)B * ed.P * ed.P * 3);
  crops = F((size_t)B * ed.P * ed.P * 3);
  rstore = F(ed.rcap);
  patched = F(Mf * 3);
  mask = F(Mf * 3);
  boxes = F((size_t)B * PHX_MAX_OUT * 4);
  count = alloc<int>(B);
  for (int k = 0; k < 2; ++k) {
    pboxes[k] = F((size_t)B * PHX_MAX_OUT * 4);
    pcount[k] = alloc<int>(B);
  }
  last_boxes = boxes;
  last_count = count;
  info = alloc<int>((size_t)B * 3);
  eerr = alloc<int>(1);
  // the evaluation Masker's buffers are reserved by the first evaluation (eval_reserve): a run that
  // only trains never holds them; this rebuild freed any earlier ones with the rest of `owned`
  ematched = erstore = nullptr;
  eB = 0;
}

// evaluation Masker (the attacker's 640^2 patch) buffers for the current workspace batch size.
// Placement side <= floor(longer side * scale) <= S for scale in [0, 1] (the attacker's clip);
// soft-NMS may return 100 overlapping image-sized boxes, so the R store keeps the worst case.
size_t phx_def::eval_bytes(int B) const {
  return ((size_t)B * PHX_PATCH_SIZE * PHX_PATCH_SIZE * 3 + (size_t)B * PHX_MAX_OUT * S * S * 3) * sizeof(float);
}

void phx_def::eval_reserve(int B) {
  if (eB == B && ematched && erstore) return;
  ematched = alloc<float>((size_t)B * PHX_PATCH_SIZE * PHX_PATCH_SIZE * 3);
  erstore = alloc<float>((size_t)B * PHX_MAX_OUT * S * S * 3);
  eB = B;
}

// ---- U-Net forward (generator.py:17-101) + output layer and loss ----
void phx_def::unet_forward(int B, const float* W, bool train, int64_t stp, int gimg0, float* loss, hipStream_t s) {
  auto conv3_fwd = [&](const float* x, int H, const UConv& c, float* y) {
    const long M = (long)B * H * H;
    DScope g(victim, "unet_conv", 2.0 * M * c.co * 9 * c.ci, 4.0 * M * (c.ci + c.co), s);
    if (un_conv3_small(x, bt + c.bt_f, W + c.b, y, B, H, H, c.ci, H, H, c.co, c.kp_f, 0, 1, 1, 1, s)) return;
    conv3_gemm(x, col, bt + c.bt_f, W + c.b, y, B, H, H, c.ci, H, H, c.co, c.kp_f, 0, 1, 1, 1, gpart, s);
  };
  auto bn_fwd = [&](UBn& b, const float* y, long M, float* a, int act) {
    DScope g(victim, "unet_bn", 0.0, (train ? 4.0 : 0.0) * M * b.c + (a ? 8.0 * M * b.c : 0.0), s);
    float* mv = reinterpret_cast<float*>(moving.get());
    if (train) un_bn_stats(y, M, b.c, W + b.gamma, b.mean, b.rstd, b.sc, mv + b.mm, mv + b.mv, cpart, s);
    else launch_bn_frozen_stats(mv + b.mm, mv + b.mv, b.mean, b.rstd, W + b.gamma, b.sc, b.c, 1e-3f, s);
    if (a) un_bnact(y, b.mean, b.sc, W + b.beta, a, M, b.c, act, s);
  };
  auto block_fwd = [&](const Block& k, const float* x, int H, float* y1, float* a1, float* y2, float* a2) {
    const long M = (long)B * H * H;
    conv3_fwd(x, H, convs[k.c1], y1);
    bn_fwd(bns[k.b1], y1, M, a1, 1);
    conv3_fwd(a1, H, convs[k.c2], y2);
    bn_fwd(bns[k.b2], y2, M, a2, 1);
  };
  const float* x = patched;
  for (int i = 0; i < 4; ++i) {
    const int H = S >> i;
    block_fwd(enc[i], x, H, et[i].y1, et[i].a1, et[i].y2, et[i].a2);
    DScope g(victim, "unet_other", 0.0, 5.0 * B * H * H * convs[enc[i].c2].co, s);
    un_pool_drop(et[i].a2, et[i].p, et[i].arg, B, H, H, convs[enc[i].c2].co, seed, stp, gimg0, train ? i : -1, s);
    x = et[i].p;
  }
  block_fwd(c4, x, S >> 4, c4t.y1, c4t.a1, c4t.y2, c4t.a2);
  x = c4t.a2;
  for (int i = 0; i < 4; ++i) {
    const Att& a = dec[i];
    const int H = S >> (3 - i), hin = H / 2;
    const long M = (long)B * H * H;
    const UConv& up = convs[a.up];
    const int n = up.co;
    DecT& d = dt[i];
    {
      const long Min = (long)B * hin * hin;
      DScope g(victim, "unet_conv", 2.0 * Min * 9 * up.ci * n, 4.0 * (Min * up.ci + M * n), s);
      if (!un_conv3_small(x, bt + up.bt_f, W + up.b, d.up, B, hin, hin, up.ci, H, H, n, up.kp_f, 1, 2, 0, 0, s)) {
        conv3_gemm(x, col, bt + up.bt_f, W + up.b, d.up, B, hin, hin, up.ci, H, H, n, up.kp_f, 1, 2, 0, 0, gpart, s);
      }
    }
    const float* skip = et[3 - i].a2;
    {
      DScope g(victim, "unet_gemm", 2.0 * M * n * n, 8.0 * M * n, s);
      gemm(d.up, bt + convs[a.cnv1].bt_f, W + convs[a.cnv1].b, d.g, M, n, n, false, gpart, s);
    }
    bn_fwd(bns[a.bn1], d.g, M, nullptr, 0);
    {
      DScope g(victim, "unet_gemm", 2.0 * M * n * n, 8.0 * M * n, s);
      gemm(skip, bt + convs[a.cnv2].bt_f, W + convs[a.cnv2].b, d.xs, M, n, n, false, gpart, s);
    }
    bn_fwd(bns[a.bn2], d.xs, M, nullptr, 0);
    const UBn &b1 = bns[a.bn1], &b2 = bns[a.bn2];
    {
      DScope g(victim, "unet_other", 2.0 * M * n, 4.0 * M * (3 * n + 1), s);
      un_att_s(d.g, d.xs, b1.mean, b1.sc, W + b1.beta, b2.mean, b2.sc, W + b2.beta, d.s, M, n, s);
      un_att_t(d.s, W + convs[a.conv3].w, W + convs[a.conv3].b, d.t, M, n, s);
    }
    UBn& b3 = bns[a.bn3];
    bn_fwd(b3, d.t, M, nullptr, 0);
    {
      DScope g(victim, "unet_other", 0.0, 4.0 * M * (2 * n + 1 + 2 * n), s);
      un_att_cat(d.up, skip, d.t, b3.mean, b3.sc, W + b3.beta, d.cat, B, (long)H * H, n, seed, stp, gimg0,
                 train ? 4 + i : -1, s);
    }
    block_fwd(a.blk, d.cat, H, d.y1, d.a1, d.y2, d.a2);
    x = d.a2;
  }
  const long Mf = (long)B * S * S;
  const UConv& oc = convs[out_conv];
  DScope g(victim, "unet_other", 2.0 * Mf * 3 * oc.ci, 4.0 * Mf * (oc.ci + 9), s);
  un_out_loss(x, W + oc.w, W + oc.b, mask, upd, dz, lpart, loss, Mf, (long)S * S, oc.ci, s);
}

// derived GEMM operands of this step's weights
void phx_def::prep_weights(const float* W, hipStream_t s) {
  for (const UConv& c : convs) {
    if (c.bt_f < 0) continue;
    const int kf = c.kind == 0 ? 0 : c.kind == 2 ? 2 : 4;
    un_wprep(W + c.w, bt + c.bt_f, kf, c.ci, c.co, c.kp_f, s);
    un_wprep(W + c.w, bt + c.bt_d, kf + 1, c.ci, c.co, c.kp_d, s);
  }
}

void phx_def::step(const float* images, int B, const float* boxes_in, const int* count_in, const float* params,
                   float* grad, int64_t stp, int gimg0, hipStream_t s) {
  workspace(B);
  const float* W = params;
  float* G = grad;
  // a first pass prefetched by the previous step for exactly this batch (phx_def_set_next)
  // (and the victim unchanged since: a weight load, a training pass or new score thresholds on the
  // protege's context make its detections stale)
  const bool use_pre = pre.pending && !boxes_in && pre.images == images && pre.B == B && pre.step == stp &&
                       pre.gimg0 == gimg0 && pre.gen == ctx_generation(victim);
  join(s);
  pre.pending = false;
  prep_weights(W, s);
  // ---- first pass + Masker ----
  const float* bx = boxes_in;
  const int* cn = count_in;
  int used_slot = -1;
  if (use_pre) {
    used_slot = pre.slot;
    bx = pboxes[used_slot];
    cn = pcount[used_slot];
  } else if (!bx) {
    def_first_pass(victim, images, B, stp, gimg0, boxes, count, s);
    bx = boxes;
    cn = count;
  }
  last_boxes = bx == boxes_in ? boxes : bx;
  last_count = cn == count_in ? count : cn;
  DScope gm(victim, "masker", 0.0, 4.0 * B * ((double)S * S * 3 * 3 + 2.0 * ed.P * ed.P * 3), s);
  def_perm_crops(images, info, crops, B, S, S, ed.P, seed, stp, gimg0, s);
  PlaceRule rule;
  rule.tol = 0.5f;
  rule.random_scale = 1;
  rule.scale_lo = 0.3f;
  rule.scale_hi = 0.5f;
  launch_eot_place(ed, bx, cn, nullptr, seed, stp, gimg0, img, place, spans, eerr, s, rule);
  launch_eot_match_batch(ed, crops, img, images, matched, ysum, ymean, s);
  launch_eot_resize(ed, matched, place, spans, seed, stp, gimg0, rstore, s, 0.1f);
  launch_eot_composite(ed, images, place, rstore, patched, nullptr, s, mask);
  prof_end(gm.r);
  gm.r.p = nullptr;
  // the next batch's first pass (the step after this one) on the side stream, beside the U-Net work
  // below: it starts once this step's own first pass and Masker are done with the victim executor
  // and the boxes, and writes the slot this step did not read
  // (not while the victim is profiled: a profiled step runs its launch groups one at a time, as the
  // attacker's prefetch_ok keeps a profiled step on one stream)
  if (next.images) {
    if (next.B == B && !ctx_profiling(victim)) {
      const int slot = used_slot == 0 ? 1 : 0;
      PHX_HIP(hipEventRecord(ev_fork, s));
      PHX_HIP(hipStreamWaitEvent(side, ev_fork, 0));
      def_first_pass(victim, next.images, B, stp + 1, next.gimg0, pboxes[slot], pcount[slot], side);
      PHX_HIP(hipEventRecord(ev_done, side));
      pre = Pre{next.images, B, next.gimg0, slot, stp + 1, true, ctx_generation(victim)};
    }
    next = Next{};
  }

  unet_forward(B, W, true, stp, gimg0, G + nparams, s);
  const float* x = dt[3].a2;
  const UConv& oc = convs[out_conv];
  const long Mf = (long)B * S * S;

  // ---- backward ----
  auto bias_grad = [&](const float* dy, long M, const UConv& c, hipStream_t st) {
    un_colsum(dy, M, c.co, G + c.b, cpart, st);
  };
  auto bn_bwd = [&](UBn& b, const float* da, const float* y, long M, int act, float* dy) {
    DScope g(victim, "unet_bn", 0.0, 12.0 * M * b.c, s);
    un_bn_bwd(da, y, M, b.c, b.mean, b.rstd, b.sc, W + b.beta, act, b.mdz, b.mdzx, G + b.gamma, G + b.beta, dy, cpart,
              s);
  };
  auto conv3_wgrad = [&](const float* xin, int H, const UConv& c, const float* dy, hipStream_t st) {
    const long M = (long)B * H * H;
    DScope g(victim, "unet_wgrad", 2.0 * M * c.co * 9 * c.ci, 4.0 * M * (c.co + c.ci), st);
    un_wgrad(dy, c.co, xin, c.ci, 1, B, H, H, c.ci, M, c.co, c.kp_f, c.ci, 9, 0, wpart, G + c.w, st);
    bias_grad(dy, M, c, st);
  };
  auto conv3_dgrad = [&](const float* dy, int H, const UConv& c, float* dx) {
    const long M = (long)B * H * H;
    DScope g(victim, "unet_conv", 2.0 * M * c.ci * 9 * c.co, 4.0 * M * (c.co + c.ci), s);
    if (un_conv3_small(dy, bt + c.bt_d, nullptr, dx, B, H, H, c.co, H, H, c.ci, c.kp_d, 0, 1, 1, 1, s)) return;
    conv3_gemm(dy, col, bt + c.bt_d, nullptr, dx, B, H, H, c.co, H, H, c.ci, c.kp_d, 0, 1, 1, 1, gpart, s);
  };
  // da2 (clobbered) -> dx of the block input (when dx != nullptr)
  auto block_bwd = [&](const Block& k, const float* xin, int H, const float* y1, const float* a1, const float* y2,
                       float* da2, float* tmp, float* dx) {
    const long M = (long)B * H * H;
    bn_bwd(bns[k.b2], da2, y2, M, 1, tmp);
    conv3_wgrad(a1, H, convs[k.c2], tmp, s);
    conv3_dgrad(tmp, H, convs[k.c2], da2);
    bn_bwd(bns[k.b1], da2, y1, M, 1, tmp);
    conv3_wgrad(xin, H, convs[k.c1], tmp, s);
    if (dx) conv3_dgrad(tmp, H, convs[k.c1], dx);
  };
  // output layer: dz [Mf,3]
  {
    DScope g(victim, "unet_other", 4.0 * Mf * 3 * oc.ci, 4.0 * Mf * (6 + 2 * oc.ci), s);
    un_wgrad(dz, 3, x, oc.ci, 0, 1, 1, 1, 1, Mf, 3, oc.ci, oc.ci, 1, 4, wpart, G + oc.w, s);
    un_colsum(dz, Mf, 3, G + oc.b, cpart, s);
    un_small_dgrad(dz, W + oc.w, tmpX, Mf, oc.ci, 3, false, s);
  }
  // decoders, last first: tmpX holds the gradient of the decoder block's output
  for (int i = 3; i >= 0; --i) {
    const Att& a = dec[i];
    const int H = S >> (3 - i), hin = H / 2;
    const long M = (long)B * H * H;
    const UConv& up = convs[a.up];
    const int n = up.co;
    DecT& d = dt[i];
    float* denc = et[3 - i].denc;
    const float* skip = et[3 - i].a2;
    block_bwd(a.blk, d.cat, H, d.y1, d.a1, d.y2, tmpX, tmpT, tmpY);  // tmpY = d cat
    UBn& b3 = bns[a.bn3];
    {
      DScope g(victim, "unet_other", 0.0, 4.0 * M * (2 * n + n + 1 + 2 * n + 1), s);
      un_att_cat_bwd(tmpY, skip, d.t, b3.mean, b3.sc, W + b3.beta, tmpX, denc, d1, B, (long)H * H, n, seed, stp,
                     gimg0, 4 + i, s);  // tmpX = d up, denc = d skip (direct), d1 = d bn3 output
    }
    bn_bwd(b3, d1, d.t, M, 0, d2);  // d2 = d t
    const UConv& c3 = convs[a.conv3];
    UBn &b1 = bns[a.bn1], &b2 = bns[a.bn2];
    {
      DScope g(victim, "unet_other", 4.0 * M * n, 4.0 * M * (2 * n + 1 + 2 * n + n), s);
      un_wgrad(d2, 1, d.s, n, 0, 1, 1, 1, 1, M, 1, n, n, 1, 4, wpart, G + c3.w, s);
      un_colsum(d2, M, 1, G + c3.b, cpart, s);
      un_att_s_bwd(d2, W + c3.w, d.g, d.xs, b1.mean, b1.sc, W + b1.beta, b2.mean, b2.sc, W + b2.beta, tmpY, M, n,
                   s);
    }
    // bn1 / cnv1 on up
    bn_bwd(b1, tmpY, d.g, M, 0, tmpT);
    const UConv& k1 = convs[a.cnv1];
    {
      DScope g(victim, "unet_wgrad", 2.0 * M * n * n, 8.0 * M * n, s);
      un_wgrad(tmpT, n, d.up, n, 0, 1, 1, 1, 1, M, n, n, n, 1, 4, wpart, G + k1.w, s);
      bias_grad(tmpT, M, k1, s);
    }
    {
      DScope g(victim, "unet_gemm", 2.0 * M * n * n, 12.0 * M * n, s);
      gemm(tmpT, bt + k1.bt_d, nullptr, tmpX, M, n, n, true, gpart, s);
    }
    // bn2 / cnv2 on skip
    bn_bwd(b2, tmpY, d.xs, M, 0, tmpT);
    const UConv& k2 = convs[a.cnv2];
    {
      DScope g(victim, "unet_wgrad", 2.0 * M * n * n, 8.0 * M * n, s);
      un_wgrad(tmpT, n, skip, n, 0, 1, 1, 1, 1, M, n, n, n, 1, 4, wpart, G + k2.w, s);
      bias_grad(tmpT, M, k2, s);
    }
    {
      DScope g(victim, "unet_gemm", 2.0 * M * n * n, 12.0 * M * n, s);
      gemm(tmpT, bt + k2.bt_d, nullptr, denc, M, n, n, true, gpart, s);
    }
    // transposed conv: input = the previous decoder's output (or the bottleneck's)
    const float* xin = i == 0 ? c4t.a2 : dt[i - 1].a2;
    const long Min = (long)B * hin * hin;
    {
      DScope g(victim, "unet_wgrad", 2.0 * Min * 9 * up.ci * n, 4.0 * (M * n + Min * up.ci), s);
      un_wgrad(tmpX, n, xin, up.ci, 2, B, H, H, up.ci, M, n, up.kp_f, up.ci, 9, 2, wpart, G + up.w, s);
      bias_grad(tmpX, M, up, s);
    }
    {
      DScope g(victim, "unet_conv", 2.0 * Min * 9 * up.ci * n, 4.0 * (M * n + Min * up.ci), s);
      if (!un_conv3_small(tmpX, bt + up.bt_d, nullptr, tmpY, B, H, H, n, hin, hin, up.ci, up.kp_d, 0, 2, 0, 0, s)) {
        conv3_gemm(tmpX, col, bt + up.bt_d, nullptr, tmpY, B, H, H, n, hin, hin, up.ci, up.kp_d, 0, 2, 0, 0, gpart, s);
      }
    }
    std::swap(tmpX, tmpY);  // tmpX = gradient of the next (earlier) block's output
  }
  // bottleneck: tmpX = d c4 output
  block_bwd(c4, et[3].p, S >> 4, c4t.y1, c4t.a1, c4t.y2, tmpX, tmpT, tmpY);  // tmpY = d p3
  for (int i = 3; i >= 0; --i) {
    const int H = S >> i;
    const int n = convs[enc[i].c2].co;
    {
      DScope g(victim, "unet_other", 0.0, 4.0 * B * H * H * n * 2.25, s);
      un_pool_drop_bwd(tmpY, et[i].arg, et[i].denc, B, H, H, n, seed, stp, gimg0, i, true, s);
    }
    const float* xin = i == 0 ? patched : et[i - 1].p;
    block_bwd(enc[i], xin, H, et[i].y1, et[i].a1, et[i].y2, et[i].denc, tmpT, i == 0 ? nullptr : tmpY);
  }
}

// PatchAttackDefender.call(images, training=False) as test_step runs it (attack_detection.py:168-198,
// 320-326): the first pass; the Masker's evaluation branch — the attacker's trained patch and scale
// (eval_patch, the [patch | scale] of patch.tiff / scale.txt, :57-61), print variation, brightness
// match, centred placement (tolerance 0) at the fixed scale, resize + U(-0.1, 0.1) noise + brightness,
// rotate, paste (:366-370, 454-456); the second detector pass odet_model(images, score_thresh=0.)
// (:185-187); updates = 2 * PatchNeutralizer(images, training=False) (inference BN, no Dropout) and the
// loss.  Nothing is updated (the BN moving statistics stay as they are).
void phx_def::eval(const float* images, int B, const float* boxes_in, const int* count_in, const float* W,
                   const float* eval_patch, float* metrics, float* out_boxes, float* out_scores, int* out_count,
                   int64_t stp, int gimg0, hipStream_t s) {
  workspace(B);
  EotDims e2 = ed;
  e2.P = PHX_PATCH_SIZE;
  // placement side <= floor(longer side * scale) <= S for scale in [0, 1] (the attacker's clip)
  e2.rcap = (long)B * PHX_MAX_OUT * S * S * 3;
  eval_reserve(B);
  join(s);  // (a prefetched first pass stays valid: this call only shares the victim executor)
  prep_weights(W, s);
  const float* bx = boxes_in;
  const int* cn = count_in;
  if (!bx) {
    def_first_pass(victim, images, B, stp, gimg0, boxes, count, s, false, 0);
    bx = boxes;
    cn = count;
  }
  PlaceRule rule;
  rule.tol = 0.f;  // Masker.create, evaluation: tolerance 0, scale = the attacker's (attack_detection.py:454-456)
  launch_eot_place(e2, bx, cn, eval_patch, seed, stp, gimg0, img, place, spans, eerr, s, rule);
  launch_eot_match(e2, eval_patch, img, images, ematched, ysum, ymean, true, s);
  launch_eot_resize(e2, ematched, place, spans, seed, stp, gimg0, erstore, s, 0.1f);
  launch_eot_composite(e2, images, place, erstore, patched, nullptr, s, mask);
  // the second pass on the patched images (its detections are the evaluation's output)
  float* ob = out_boxes ? out_boxes : boxes;
  int* oc = out_count ? out_count : count;
  def_first_pass(victim, patched, B, stp, gimg0, ob, oc, s, false, 1, 0.f, out_scores);
  unet_forward(B, W, false, stp, gimg0, metrics, s);
}

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
#define DEF_TRY try {
#define DEF_CATCH(d)                                                              \
  }                                                                               \
  catch (const std::out_of_range& e) { if (d) d->err = e.what(); return PHX_ECAP; } \
  catch (const std::invalid_argument& e) { if (d) d->err = e.what(); return PHX_EINVAL; } \
  catch (const std::logic_error& e) { if (d) d->err = e.what(); return PHX_ESTATE; } \
  catch (const HipError& e) { if (d) d->err = e.what(); return PHX_EHIP; }        \
  catch (const std::exception& e) { if (d) d->err = e.what(); return PHX_EINVAL; }

extern "C" {

namespace {
thread_local std::string g_def_create_err;  // phx_def_last_error(NULL): the last failed phx_def_create
}

int phx_def_create(phx_ctx* victim, int max_batch, uint64_t seed, phx_def** out) {
  g_def_create_err.clear();
  if (!victim || !out || max_batch <= 0) {
    g_def_create_err = "phx_def_create: null victim / output pointer or max_batch <= 0";
    return PHX_EINVAL;
  }
  *out = nullptr;
  phx_def* d = nullptr;
  DEF_TRY
  const int S = ctx_image_size(victim);
  if (S % 16 != 0 || S < 240) throw std::invalid_argument("defender: image size must be a multiple of 16 and >= 240");
  d = new phx_def();
  d->victim = victim;
  d->device = ctx_device(victim);
  d->max_batch = max_batch;
  d->S = S;
  d->seed = seed;
  PHX_HIP(hipSetDevice(d->device));
  d->build();
  void* p = nullptr;
  PHX_HIP(hipMalloc(&p, d->nmoving * sizeof(float)));
  d->moving.reset(p);
  // Keras BatchNormalization: moving mean 0, moving variance 1
  std::vector<float> mv(d->nmoving, 0.f);
  for (const UBn& b : d->bns)
    for (int c = 0; c < b.c; ++c) mv[b.mv + c] = 1.f;
  PHX_HIP(hipMemcpy(p, mv.data(), mv.size() * sizeof(float), hipMemcpyHostToDevice));
  *out = d;
  return PHX_OK;
  }
  catch (const std::exception& e) {
    delete d;
    g_def_create_err = std::string("phx_def_create: ") + e.what();
    return dynamic_cast<const HipError*>(&e) ? PHX_EHIP : PHX_EINVAL;
  }
}

void phx_def_destroy(phx_def* d) { delete d; }

const char* phx_def_last_error(phx_def* d) { return d ? d->err.c_str() : g_def_create_err.c_str(); }

int64_t phx_def_num_params(phx_def* d) { return d ? d->nparams : -1; }
int64_t phx_def_num_moving(phx_def* d) { return d ? d->nmoving : -1; }

int phx_def_manifest(phx_def* d, char* buf, size_t cap, size_t* need) {
  if (!d) return PHX_EINVAL;
  const std::string js = d->manifest_json();
  if (need) *need = js.size() + 1;
  if (buf && cap) {
    if (cap < js.size() + 1) return PHX_ECAP;
    std::memcpy(buf, js.c_str(), js.size() + 1);
  }
  return PHX_OK;
}

int phx_def_moving(phx_def* d, float* dst, const float* src, void* stream) {
  if (!d) return PHX_EINVAL;
  DEF_TRY
  hipStream_t s = (hipStream_t)stream;
  if (src) PHX_HIP(hipMemcpyAsync(d->moving.get(), src, d->nmoving * sizeof(float), hipMemcpyDefault, s));
  if (dst) PHX_HIP(hipMemcpyAsync(dst, d->moving.get(), d->nmoving * sizeof(float), hipMemcpyDefault, s));
  return PHX_OK;
  DEF_CATCH(d)
}

int phx_def_workspace_bytes(phx_def* d, int B, size_t* bytes) {
  if (!d || !bytes || B <= 0 || B > d->max_batch) return PHX_EINVAL;
  DEF_TRY
  d->workspace(B);
  *bytes = d->ws_bytes;
  return PHX_OK;
  DEF_CATCH(d)
}

int phx_def_eval_workspace_bytes(phx_def* d, int B, size_t* bytes) {
  if (!d || !bytes || B <= 0 || B > d->max_batch) return PHX_EINVAL;
  *bytes = d->eval_bytes(B);
  return PHX_OK;
}

int phx_def_step_grad(phx_def* d, const float* images, int B, const float* boxes, const int32_t* count,
                      const float* params, float* grad, int64_t step, int32_t global_image_offset, void* stream) {
  if (!d || !images || !params || !grad || B <= 0) return PHX_EINVAL;
  if (B > d->max_batch) return PHX_ECAP;
  if ((boxes == nullptr) != (count == nullptr)) return PHX_EINVAL;
  DEF_TRY
  PHX_HIP(hipSetDevice(d->device));
  d->step(images, B, boxes, count, params, grad, step, global_image_offset, (hipStream_t)stream);
  return PHX_OK;
  DEF_CATCH(d)
}

int phx_def_set_next(phx_def* d, const float* next_images, int B, int32_t global_image_offset) {
  if (!d) return PHX_EINVAL;
  if (next_images && (B <= 0 || B > d->max_batch)) return B <= 0 ? PHX_EINVAL : PHX_ECAP;
  DEF_TRY
  PHX_HIP(hipSetDevice(d->device));
  if (next_images && !d->side) {
    PHX_HIP(hipStreamCreateWithFlags(&d->side, hipStreamNonBlocking));
    PHX_HIP(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
    PHX_HIP(hipEventCreateWithFlags(&d->ev_done, hipEventDisableTiming));
  }
  d->next = next_images ? phx_def::Next{next_images, B, global_image_offset} : phx_def::Next{};
  // NULL also withdraws a prefetched first pass (the caller refilled that batch's buffer in place)
  if (!next_images && d->pre.pending) {
    PHX_HIP(hipStreamSynchronize(d->side));
    d->pre = phx_def::Pre{};
  }
  return PHX_OK;
  DEF_CATCH(d)
}

int phx_def_sync(phx_def* d, void* stream) {
  if (!d) return PHX_EINVAL;
  DEF_TRY
  PHX_HIP(hipSetDevice(d->device));
  d->join((hipStream_t)stream);
  return PHX_OK;
  DEF_CATCH(d)
}

int phx_def_eval_step(phx_def* d, const float* images, int B, const float* boxes, const int32_t* count,
                      const float* params, const float* eval_patch, float* metrics, float* out_boxes,
                      float* out_scores, int32_t* out_count, int64_t step, int32_t global_image_offset, void* stream) {
  if (!d || !images || !params || !eval_patch || !metrics || B <= 0) return PHX_EINVAL;
  if (B > d->max_batch) return PHX_ECAP;
  if ((boxes == nullptr) != (count == nullptr)) return PHX_EINVAL;
  DEF_TRY
  PHX_HIP(hipSetDevice(d->device));
  d->eval(images, B, boxes, count, params, eval_patch, metrics, out_boxes, out_scores, out_count, step,
          global_image_offset, (hipStream_t)stream);
  return PHX_OK;
  DEF_CATCH(d)
}

int phx_def_debug(phx_def* d, int what, float* dst, size_t n, void* stream) {
  if (!d || !dst || d->wsB == 0) return PHX_EINVAL;
  DEF_TRY
  const long Mf = (long)d->wsB * d->S * d->S;
  const float* src = nullptr;
  size_t have = 0;
  switch (what) {
    case PHX_DEF_PATCHED: src = d->patched; have = Mf * 3; break;
    case PHX_DEF_TARGETS: src = d->mask; have = Mf * 3; break;
    case PHX_DEF_UPDATES: src = d->upd; have = Mf * 3; break;
    case PHX_DEF_BOXES: src = d->last_boxes; have = (size_t)d->wsB * PHX_MAX_OUT * 4; break;
    case PHX_DEF_COUNTS: src = reinterpret_cast<const float*>(d->last_count); have = d->wsB; break;
    default: throw std::invalid_argument("phx_def_debug: unknown tensor");
  }
  if (n < have) throw std::out_of_range("phx_def_debug: destination too small");
  PHX_HIP(hipMemcpyAsync(dst, src, have * sizeof(float), hipMemcpyDefault, (hipStream_t)stream));
  return PHX_OK;
  DEF_CATCH(d)
}

int phx_adam(float* params, const float* grad, float* m, float* v, int64_t n, float lr, int64_t t, void* stream) {
  if (!params || !grad || !m || !v || n <= 0 || t <= 0) return PHX_EINVAL;
  try {
    launch_adam(params, grad, m, v, n, lr, t, (hipStream_t)stream);
  } catch (const std::exception&) {
    return PHX_EHIP;
  }
  return PHX_OK;
}

}  // extern "C"
