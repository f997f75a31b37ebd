// api.cpp — libphx C ABI: context, weight management, the program executor (victim forward
// and data-gradient), and the attack step that strings the kernels together on one stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <functional>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"
#include "model.hpp"
#include "phx.h"
#include "post.hpp"
#include "unet.hpp"

using namespace phx;

namespace {

constexpr float kBnEps = 1e-3f;  // efficientnet_builder.py:179, util_keras.py:35

template <typename T>
T* dalloc(size_t n) {
  if (n == 0) n = 1;
  void* p = nullptr;
  PHX_HIP(hipMalloc(&p, n * sizeof(T)));
  static const bool log = [] {
    const char* e = std::getenv("PHX_ALLOC_LOG");
    return e && e[0] == '1';
  }();
  if (log) fprintf(stderr, "phx alloc %p %zu\n", p, n * sizeof(T));
  return reinterpret_cast<T*>(p);
}

// PHX_GUARD_BYTES=n (diagnostics): every executor allocation gets n guard bytes of 0xA5 after its
// end, and phx_step_grad checks them after the step (synchronising), reporting any overwrite on
// stderr — an out-of-bounds write past a buffer shows up even when it corrupts nothing visible.
// (rounded up to a multiple of 256 so every buffer keeps the 256-B alignment its 16-B vector loads
// and the GEMM planner assume; counted in Exec::bytes)
size_t guard_bytes() {
  static const size_t g = [] {
    const char* e = std::getenv("PHX_GUARD_BYTES");
    const long v = e ? std::atol(e) : 0;
    const size_t r = v > 0 ? ((size_t)v + 255) / 256 * 256 : 0;
    if (r) fprintf(stderr, "phx: PHX_GUARD_BYTES: %zu-byte guard bands around every executor buffer\n", r);
    return r;
  }();
  return g;
}
struct Guard {
  const char* base;
  size_t size;  // the buffer's own bytes (the guard follows)
};

struct DevFree {
  void operator()(void* p) const {
    if (p) (void)hipFree(p);
  }
};
using DPtr = std::unique_ptr<void, DevFree>;

// Per-batch-size executable state: program + arenas + step buffers.
struct Exec {
  Program prog;
  int B = 0;
  std::vector<DPtr> owned;
  float* act = nullptr;
  float* grad = nullptr;
  std::vector<float*> slot_a, slot_b, slot_c;  // BN: mean,rstd ; SE: pool(+part),hidden,scale
  double* red = nullptr;                       // BN partial sums
  float* coef = nullptr;                       // BN backward coefficients
  float* se_g = nullptr;                       // SE backward scratch
  float* gpart = nullptr;                      // split-K GEMM partial slabs
  std::vector<int> se_of_tensor;               // tensor id -> SE op index producing it (-1)
  // BiFPN node fuse folded into the depthwise conv after it (computed on load, never written)
  std::vector<char> fuse_folded;               // op id of the fuse -> 1
  // fused separable convs (kernels_sep.hip): sep[i] = 1 for a 3x3 depthwise op i whose output only the
  // pointwise op i + 1 reads; one launch computes both and the depthwise output is never stored
  std::vector<char> sep;
  // sepb[i]: the fused sepconv at depthwise op i also runs its backward in one launch (the pointwise
  // data gradient never stored)
  std::vector<char> sepb;
  // expand -> BN -> act -> depthwise fused (kernels_dw.hip): op id of the expand
  // conv -> 1; the expand output is never stored in a training pass (ops i, i+1, i+2)
  std::vector<int> bn_of_tensor;               // tensor id -> BN op index producing it (-1)
  std::vector<int> bn_consumer;                // tensor id -> BN op index reading it (-1)
  std::vector<float*> slot_d, slot_e;          // BN backward: mean(dz), mean(dz*xhat)
  // BN statistics fused into the producing kernel (StatSink): channel-major partials and their
  // row counts; fused_bn[i]: BN op i takes its statistics from its producer
  float2* spart = nullptr;
  float* scnt = nullptr;
  std::vector<char> fused_bn;
  std::vector<int> stat_P;                     // tensor id -> partial rows written by its producer
  std::vector<uint8_t*> pool_amax;             // op id -> max-pool argmax taps (MAXPOOL ops)
  // BN backward sums fused into the dgrad of the BN output's first consumer (op i+1), which is the
  // last writer of the BN output's gradient in the reverse sweep (GradSink)
  std::vector<char> gfused_bn;
  std::vector<int> gstat_P;                    // op id of the BN -> partial rows
  // Level-batched heads: the per-level members of a class/box-head conv share their weights, so
  // each (head, position) runs as ONE grouped launch (members = levels), and so do the BNs after
  // them.  grp_of: op id -> group (-1); a group runs at its first member in the forward sweep and
  // at its last in the reverse sweep.  Member r of a group keeps its statistics partials in
  // region r of spart / scnt (region strides sp_region / sc_region).
  std::vector<int> grp_of;
  std::vector<std::vector<int>> groups;
  size_t sp_region = 0, sc_region = 0;
  std::vector<int> stat_region;                // tensor id -> region of its producer's partials
  std::vector<int> gstat_region;               // BN op id -> region of its backward partials
  LevelDesc* lev_dev = nullptr;
  std::vector<LevelDesc> lev;
  long* dxoff_dev = nullptr;
  std::vector<long> dxoff;
  bool cls_contig = true;
  int ntiles = 0;
  // pre_nms / nms / loss
  float *scores = nullptr, *boxes = nullptr;
  int* classes = nullptr;
  uint8_t* keep = nullptr;
  int* cand_list = nullptr;   // soft-NMS candidates appended by pre_nms [B][A] + counts [B]
  int* cand_count = nullptr;
  float* nms_ws = nullptr;
  float *nms1_boxes = nullptr, *nms1_scores = nullptr;
  int* nms1_count = nullptr;
  float *nms2_boxes = nullptr, *nms2_scores = nullptr;
  int* nms2_count = nullptr;
  float *mraw = nullptr, *dm = nullptr;
  int *argm = nullptr, *nties = nullptr;
  int* imax_scratch = nullptr;
  // EOT
  EotDims ed{};
  ImgParams* img = nullptr;
  BoxPlace* place = nullptr;  // followed by the int lists
  SpanEntry* spans = nullptr;
  double* ysum = nullptr;
  float* ymean = nullptr;
  float *rstore = nullptr, *dstore = nullptr;
  float *matched = nullptr, *dmatched = nullptr;
  double* dsum = nullptr;
  double* tvs = nullptr;
  int* err = nullptr;
  float* patched = nullptr;
  int16_t* owner = nullptr;
  // drop connect (non-b0 backbones, training): per drop op its block id and survival, and the
  // per-image keep flags of the current pass [ndrop][B]
  int ndrop = 0;
  int* drop_block = nullptr;
  float* drop_p = nullptr;
  float* drop_keep = nullptr;
  std::vector<int> drop_slot;                  // op id -> row of drop_keep (-1)
  // caller-injected placement boxes ([B,100,4] slot layout + counts)
  float* inj_boxes = nullptr;
  int* inj_count = nullptr;
  float* dscale_scratch = nullptr;  // dL/dscale of a gradient-free (eval) step
  double* sync_sums = nullptr;      // bn=sync: [member][C][3] per-channel sums to all-reduce

  int tag = 0;        // 0: the step's executor; 1: the concurrent first pass's (forward only)
  // deferred moving statistics (a step whose first pass runs beside the second): while defer_mov
  // the BN finalizes leave the moving statistics alone and write (batch mean, variance) of their
  // slot to side + 2 * side_off[slot]; launch_bn_moving_apply then applies both passes in order
  bool defer_mov = false;
  double* side = nullptr;
  std::vector<int> side_off;
  MovEntry* mov_tab = nullptr;
  int n_mov = 0, mov_cmax = 1;
  double* side_for(int slot) const { return defer_mov ? side + 2 * (size_t)side_off[slot] : nullptr; }
  bool bf16 = false;  // the context's compute dtype (GEMM plans depend on it)
  // activations (the arena tensors) stored as bf16: PHX_DTYPE_BF16, SURVEY.md 8a R4 "C4: bf16 act";
  // the program input (the images) and every gradient stay fp32
  bool abf = false;
  uint64_t frozen_ver = 0;  // ctx->w_ver whose inference-BN statistics the BN slots hold (0: none)
  size_t bytes = 0;  // device bytes owned by this executor
  uint64_t used = 0;  // phx_ctx::clock at the last use
  std::vector<Guard> guards;  // PHX_GUARD_BYTES
  // PHX_CKSUM=1 (diagnostics): a hash of every tensor / statistics slot an op writes, taken on the
  // op's stream right after it, in launch order (phx_debug_checksums)
  unsigned long long* ck = nullptr;
  size_t ck_cap = 0;
  bool ck_on = false;
  std::vector<std::string> ck_names;
  template <typename T>
  T* alloc(size_t n) {
    const size_t gb = guard_bytes();
    if (n == 0) n = 1;
    // [gb guard][buffer][gb guard] (gb a multiple of 256 keeps the buffer's alignment)
    char* q = dalloc<char>(n * sizeof(T) + 2 * gb);
    owned.emplace_back(q);
    if (gb) {
      PHX_HIP(hipMemset(q, 0xA5, gb));
      PHX_HIP(hipMemset(q + gb + n * sizeof(T), 0xA5, gb));
      guards.push_back(Guard{q + gb, n * sizeof(T)});
    }
    bytes += n * sizeof(T) + 2 * gb;
    return reinterpret_cast<T*>(q + gb);
  }
  // base pointer of tensor t (bf16 elements when tbf(t): kernels index it as such)
  float* tptr(int t, const float* input) const {
    if (t == prog.input) return const_cast<float*>(input);
    if (abf) return reinterpret_cast<float*>(reinterpret_cast<uint16_t*>(act) + prog.tensors[t].off);
    return act + prog.tensors[t].off;
  }
  int tbf(int t) const { return abf && t != prog.input ? 1 : 0; }
  float* gptr(int t) const {
    long g = prog.tensors[t].goff;
    return g < 0 ? nullptr : grad + g;
  }
};

}  // namespace

// Per-launch-group timing with HIP events on the launch stream (phx_profile): used by bench.py
// to time the dominant kernel live; off by default (no events on the timed path).
struct Prof {
  struct Rec {
    std::string kind;
    hipEvent_t a, b;
    double flops, bytes;
    double peak_tflops;  // the matrix-core peak the launch's FLOPs run at
  };
  bool on = false;
  std::vector<Rec> recs;
  std::string report;  // the report a size query (buf == NULL) built: the copy call returns it verbatim
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  hipEvent_t ev() {
    if (used == pool.size()) {
      hipEvent_t e;
      PHX_HIP(hipEventCreate(&e));
      pool.push_back(e);
    }
    return pool[used++];
  }
  ~Prof() {
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

struct phx_ctx {
  Prof prof;
  ModelConfig mc;
  int device = 0;
  int max_batch = 0;
  int bn_mode = PHX_BN_LOCAL;
  // bn=sync: the caller's SUM all-reduce of the BN sums (phx_set_allreduce)
  phx_allreduce_fn ar_fn = nullptr;
  void* ar_user = nullptr;
  bool batch_bn() const { return bn_mode != PHX_BN_FROZEN; }  // training-mode batch statistics
  bool bf16 = false;  // PHX_DTYPE_BF16: bf16 matrix cores for the 1x1 convs
  // nms_configs.score_thresh: the first pass keeps scores >= filter_thresh (attacker.py:83-84);
  // gaussian soft-NMS keeps scores > nms_thresh = score_thresh or 0.001 (postprocess.py:186-188)
  float score_thresh = 0.f;
  float filter_thresh = 0.f, nms_thresh = 0.001f;
  uint64_t seed = 0;
  std::vector<WeightEntry> weights;
  size_t wfloats = 0;
  std::string manifest_json;
  DPtr d_w, d_wt;
  // version of the weights and moving statistics: bumped by every load and every training-mode
  // forward (it may update the moving statistics); an executor's inference-BN statistics computed
  // at this version are reused (Exec::frozen_ver)
  uint64_t w_ver = 1;
  std::vector<long> wt_map;  // weight offset -> offset in d_wt (dense map over kernel entries)
  std::vector<std::pair<long, long>> wt_pairs;
  bool weights_loaded = false;
  DPtr d_anchors;
  int A = 0;
  std::vector<std::unique_ptr<Exec>> execs;
  Exec* last = nullptr;
  std::string err;
  // scratch for phx_soft_nms standalone
  DPtr sn_ws;
  size_t sn_cap = 0;
  // scratch for phx_augment (per-image channel-sum partials)
  DPtr aug_ws;
  size_t aug_cap = 0;
  DPtr ap_ws;          // inference compositor scratch (phx_adv_patch)
  size_t ap_cap = 0;
  // scratch for phx_brightness_match (Y-mean partials), grown on demand
  DPtr bm_ws;
  size_t bm_cap = 0;
  // executor use clock (least-recently-used eviction, see exec_for)
  uint64_t clock = 0;

  void set_score_thresh(float t) {
    score_thresh = t;
    filter_thresh = t;
    nms_thresh = t != 0.f ? t : 0.001f;
  }

  float* w() const { return reinterpret_cast<float*>(d_w.get()); }
  const float* wt_of(long off) const {
    for (auto& p : wt_pairs)
      if (p.first == off) return reinterpret_cast<const float*>(d_wt.get()) + p.second;
    throw std::runtime_error("no transposed kernel for weight offset");
  }
  Exec& exec_for(int B, int tag = 0);
  std::string model_info() const;
  // issued by run_forward once it has issued op fwd_hook_at (the second pass starts the concurrent
  // first pass part-way through its own forward, §12 of DESIGN.md)
  std::function<void()> fwd_hook;
  size_t fwd_hook_at = 0;
  // concurrent first pass (injected placement): its own stream and fork / join events
  hipStream_t s1 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // cross-step first-pass prefetch (phx_set_next, first-pass placement): the next batch's first pass
  // on s2 and the side executor (tag 1), beside the current step's second pass and backward
  hipStream_t s2 = nullptr;
  hipEvent_t ev_pfork = nullptr, ev_pdone = nullptr;
  struct Next {
    const float* images = nullptr;
    int B = 0, gimg0 = 0;
  } next;
  struct Pre {
    const float* images = nullptr;
    int B = 0, gimg0 = 0;
    int64_t step = -1;
    bool pending = false;
  } pre;
  // `s` waits for a prefetch in flight (it holds the side executor and its deferred statistics)
  void pre_join(hipStream_t s) {
    if (pre.pending) PHX_HIP(hipStreamWaitEvent(s, ev_pdone, 0));
  }
  // new weights or thresholds: a prefetched first pass no longer matches what the step would compute
  void pre_drop() {
    if (pre.pending) PHX_HIP(hipStreamSynchronize(s2));
    pre = Pre{};
  }
  ~phx_ctx() {
    if (s2) (void)hipStreamSynchronize(s2);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (s1) (void)hipStreamDestroy(s1);
    if (ev_pfork) (void)hipEventDestroy(ev_pfork);
    if (ev_pdone) (void)hipEventDestroy(ev_pdone);
    if (s2) (void)hipStreamDestroy(s2);
  }
};

namespace {

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o.push_back('\\');
    o.push_back(c);
  }
  return o;
}

// anchors.py:83-165 in float64, cast to float32
std::vector<float> make_anchors(const ModelConfig& mc) {
  std::vector<int> fs{mc.image_size};
  int f = mc.image_size;
  for (int l = 1; l <= mc.max_level; ++l) {
    f = (f - 1) / 2 + 1;
    fs.push_back(f);
  }
  std::vector<float> out;
  for (int level = mc.min_level; level <= mc.max_level; ++level) {
    const double stride = (double)fs[0] / (double)fs[level];
    struct C { double base_x, base_y, ax, ay; };
    std::vector<C> cs;
    for (int o = 0; o < mc.num_scales; ++o) {
      for (float ar : mc.aspect_ratios) {
        double octave = (double)o / (double)mc.num_scales;
        double base = (double)mc.anchor_scale * stride * std::pow(2.0, octave);
        double ax = std::sqrt((double)ar);
        double ay = 1.0 / ax;
        cs.push_back({base, base, ax, ay});
      }
    }
    std::vector<double> xs, ys;
    // numpy arange: start + i*step
    for (int i = 0;; ++i) {
      double v = stride / 2 + i * stride;
      if (v >= mc.image_size) break;
      xs.push_back(v);
    }
    ys = xs;
    for (double yv : ys) {
      for (double xv : xs) {
        for (const C& c : cs) {
          double sx2 = c.base_x * c.ax / 2.0, sy2 = c.base_y * c.ay / 2.0;
          out.push_back((float)(yv - sy2));
          out.push_back((float)(xv - sx2));
          out.push_back((float)(yv + sy2));
          out.push_back((float)(xv + sx2));
        }
      }
    }
  }
  return out;
}

thread_local std::string g_create_err;  // phx_last_error(NULL): the last failed phx_create

}  // namespace

// phx_model_info: the configuration the program builder used (model.cpp get_model_config) in
// hparams_config's key names, plus the BiFPN node list (fpn_configs.py:24-72)
std::string phx_ctx::model_info() const {
  const ModelConfig& c = mc;
  std::ostringstream js;
  js.precision(9);
  auto arr3 = [&](const float* v) {
    std::ostringstream o;
    o.precision(9);
    o << "[" << v[0] << "," << v[1] << "," << v[2] << "]";
    return o.str();
  };
  js << "{\"name\":\"" << json_escape(c.name) << "\",\"backbone_name\":\"" << json_escape(c.backbone)
     << "\",\"image_size\":" << c.image_size << ",\"fpn_num_filters\":" << c.fpn_num_filters
     << ",\"fpn_cell_repeats\":" << c.fpn_cell_repeats << ",\"box_class_repeats\":" << c.box_class_repeats
     << ",\"anchor_scale\":" << c.anchor_scale << ",\"num_scales\":" << c.num_scales << ",\"aspect_ratios\":[";
  for (size_t i = 0; i < c.aspect_ratios.size(); ++i) js << (i ? "," : "") << c.aspect_ratios[i];
  js << "],\"min_level\":" << c.min_level << ",\"max_level\":" << c.max_level << ",\"act_type\":\""
     << (c.act == ACT_RELU6 ? "relu6" : c.act == ACT_SWISH ? "swish" : "none") << "\",\"fpn_weight_method\":\""
     << (c.fpn_weight_method == 1 ? "sum" : "fastattn") << "\",\"mean_rgb\":" << arr3(c.mean_rgb)
     << ",\"stddev_rgb\":" << arr3(c.stddev_rgb) << ",\"num_classes\":" << c.num_classes
     << ",\"survival_prob\":" << c.survival_prob << ",\"width_coefficient\":" << c.width_coefficient
     << ",\"depth_coefficient\":" << c.depth_coefficient << ",\"score_thresh\":" << filter_thresh
     << ",\"nms_score_thresh\":" << nms_thresh << ",\"compute_dtype\":\"" << (bf16 ? "bf16" : "f32")
     << "\",\"fpn_nodes\":[";
  const int nlev = c.max_level - c.min_level + 1;
  std::map<int, std::vector<int>> ids;
  for (int i = 0; i < nlev; ++i) ids[c.min_level + i] = {i};
  int cnt = nlev;
  bool first = true;
  auto node = [&](int level, const std::vector<int>& in) {
    js << (first ? "" : ",") << "{\"feat_level\":" << level << ",\"inputs_offsets\":[";
    for (size_t k = 0; k < in.size(); ++k) js << (k ? "," : "") << in[k];
    js << "]}";
    first = false;
  };
  for (int i = c.max_level - 1; i >= c.min_level; --i) {
    node(i, {ids[i].back(), ids[i + 1].back()});
    ids[i].push_back(cnt++);
  }
  for (int i = c.min_level + 1; i <= c.max_level; ++i) {
    std::vector<int> in = ids[i];
    in.push_back(ids[i - 1].back());
    node(i, in);
    ids[i].push_back(cnt++);
  }
  js << "]}";
  return js.str();
}

namespace {

int fail(phx_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

// PHX_PROF_DETAIL=1: launch groups are split by shape ("gemm fwd M=.. N=.. K=..") for tuning
bool prof_detail() {
  static const bool on = [] {
    const char* e = std::getenv("PHX_PROF_DETAIL");
    return e && e[0] == '1';
  }();
  return on;
}

std::string op_tag(const Program& P, const Op& op, bool bwd) {
  const Tensor& ti = P.tensors[op.in[0]];
  const Tensor& to = P.tensors[op.out];
  char b[160];
  if (op.t == OP_PW)
    snprintf(b, sizeof b, " %s M=%zu N=%d K=%d", bwd ? "dgrad" : "fwd", ti.rows(), bwd ? ti.c : to.c,
             bwd ? to.c : ti.c);
  else if (op.t == OP_DW)
    snprintf(b, sizeof b, " %dx%dx%d k%d s%d", ti.h, ti.w, ti.c, op.k, op.stride);
  else
    snprintf(b, sizeof b, " %dx%dx%dx%d", ti.n, ti.h, ti.w, ti.c);
  return b;
}

// PHX_DEBUG_SYNC=1: synchronise and check for a device error after every launch group, naming it
// in the exception (fault localisation; never on the timed path)
bool debug_sync() {
  static const bool on = [] {
    const char* e = std::getenv("PHX_DEBUG_SYNC");
    return e && e[0] == '1';
  }();
  return on;
}

struct Scope {
  Prof* p;
  size_t idx;
  hipStream_t s;
  std::string dbg;
  ExtTiming ext;  // GEMM groups: timed by the kernels' own dispatch timestamps (PHX_TLAUNCH)
  Scope(phx_ctx* ctx, const char* kind, double flops, double bytes, hipStream_t st, const std::string& tag = "")
      : p(ctx->prof.on ? &ctx->prof : nullptr), s(st) {
    if (debug_sync()) {
      dbg = std::string(kind) + tag;
      PHX_HIP(hipStreamSynchronize(s));
    }
    if (!p) return;
    // GEMMs of a bf16 context run on the bf16 matrix cores; everything else at the fp32 rate
    const double peak = (ctx->bf16 && std::string(kind) == "gemm") ? 2500.0 : 157.3;
    Prof::Rec r{std::string(kind) + (prof_detail() ? tag : std::string()), p->ev(), p->ev(), flops, bytes, peak};
    PHX_HIP(hipEventRecord(r.a, s));  // (re-recorded by the group's first timed kernel)
    p->recs.push_back(r);
    idx = p->recs.size() - 1;
    if (std::string(kind) == "gemm") {
      ext = ExtTiming{r.a, r.b, false};
      ext_timing() = &ext;
    }
  }
  ~Scope() noexcept(false) {
    if (p) {
      if (ext_timing() == &ext) ext_timing() = nullptr;
      if (!ext.used) (void)hipEventRecord(p->recs[idx].b, s);
    }
    if (!dbg.empty() && std::uncaught_exceptions() == 0) {
      const hipError_t e = hipStreamSynchronize(s);
      if (e != hipSuccess) throw HipError(std::string("device error after ") + dbg + ": " + hipGetErrorString(e));
    }
  }
};

}  // namespace

// ------------------------------------------------------------------------------------------
// executor
// ------------------------------------------------------------------------------------------
namespace {
void plan_groups(Exec& E, bool local_bn);
bool is_cls_out(const Program& P, int t);
}  // namespace

// One executor per (batch size, tag) (the program and its arenas are shaped by B; tag 1 is the
// concurrent first pass's forward-only executor, §12 of DESIGN.md).  At most kMaxExecs stay
// alive, two per batch size for two batch sizes, so a driver that mixes batch sizes (a last
// partial batch, validation) keeps both sizes' step and side executors without evicting at every
// switch.  A third batch size evicts (after the device has drained, so no queued kernel still
// reads its memory) a forward-only executor first — the smaller, cheaper one to rebuild — and
// the least recently used among those.
constexpr size_t kMaxExecs = 4;

Exec& phx_ctx::exec_for(int B, int tag) {
  ++clock;
  for (auto& e : execs)
    if (e->B == B && e->tag == tag) {
      e->used = clock;
      return *e;
    }
  if (execs.size() >= kMaxExecs) {
    size_t lru = 0;
    auto older = [&](size_t i, size_t j) {
      if (execs[i]->tag != execs[j]->tag) return execs[i]->tag > execs[j]->tag;
      return execs[i]->used < execs[j]->used;
    };
    for (size_t i = 1; i < execs.size(); ++i)
      if (older(i, lru)) lru = i;
    PHX_HIP(hipDeviceSynchronize());
    if (last == execs[lru].get()) last = nullptr;
    if (execs[lru]->tag == 1) pre = Pre{};  // a prefetched first pass lives in the side executor
    execs.erase(execs.begin() + (long)lru);
  }
  auto ex = std::make_unique<Exec>();
  Exec& E = *ex;
  E.B = B;
  E.tag = tag;
  E.bf16 = bf16;
  E.abf = bf16;
  NetBuilder nb(mc, B, batch_bn());
  nb.build();
  E.prog = nb.program();
  Program& P = E.prog;
  E.act = E.alloc<float>(E.abf ? (P.act_floats + 1) / 2 : P.act_floats);
  // the concurrent first pass's executor (tag 1) runs forwards only: no gradient arena
  E.grad = E.alloc<float>(tag == 1 ? 1 : P.grad_floats);
  // statistics slots and scratch
  E.slot_a.assign(P.n_slots, nullptr);
  E.slot_b.assign(P.n_slots, nullptr);
  E.slot_c.assign(P.n_slots, nullptr);
  size_t red_need = 1, coef_need = 1, seg_need = 1;
  E.se_of_tensor.assign(P.tensors.size(), -1);
  E.bn_of_tensor.assign(P.tensors.size(), -1);
  E.bn_consumer.assign(P.tensors.size(), -1);
  E.slot_d.assign(P.n_slots, nullptr);
  E.slot_e.assign(P.n_slots, nullptr);
  for (size_t i = 0; i < P.ops.size(); ++i) {
    const Op& op = P.ops[i];
    const Tensor& ti = P.tensors[op.in[0]];
    if (op.t == OP_BN) {
      E.slot_a[op.slot] = E.alloc<float>(ti.c);
      E.slot_b[op.slot] = E.alloc<float>(ti.c);
      E.slot_c[op.slot] = E.alloc<float>(ti.c);
      E.slot_d[op.slot] = E.alloc<float>(ti.c);
      E.slot_e[op.slot] = E.alloc<float>(ti.c);
      PHX_HIP(hipMemset(E.slot_d[op.slot], 0, ti.c * sizeof(float)));
      PHX_HIP(hipMemset(E.slot_e[op.slot], 0, ti.c * sizeof(float)));
      E.bn_of_tensor[op.out] = (int)i;
      E.bn_consumer[op.in[0]] = (int)i;
      red_need = std::max(red_need, bn_stats_scratch_doubles((long)ti.rows(), ti.c));
      coef_need = std::max(coef_need, (size_t)ti.c * 3);
    } else if (op.t == OP_SE) {
      E.slot_a[op.slot] = E.alloc<float>((size_t)B * ti.c * 2);
      E.slot_b[op.slot] = E.alloc<float>((size_t)B * op.cse);
      E.slot_c[op.slot] = E.alloc<float>((size_t)B * ti.c);
      seg_need = std::max(seg_need, (size_t)B * ti.c * 2);
      red_need = std::max(red_need, colred_scratch_doubles((long)ti.h * ti.w, ti.c, B));
      E.se_of_tensor[op.out] = (int)i;
    }
  }
  {
    std::vector<MovEntry> tab;
    int off = 0;
    E.side_off.assign(P.n_slots, 0);
    for (const Op& op : P.ops)
      if (op.t == OP_BN) {
        const int C = P.tensors[op.in[0]].c;
        E.side_off[op.slot] = off;
        tab.push_back(MovEntry{op.mmean, op.mvar, C, off});
        off += C;
        E.mov_cmax = std::max(E.mov_cmax, C);
      }
    E.side = E.alloc<double>(2 * (size_t)std::max(off, 1));
    E.n_mov = (int)tab.size();
    E.mov_tab = E.alloc<MovEntry>(std::max<size_t>(tab.size(), 1));
    if (!tab.empty()) PHX_HIP(hipMemcpy(E.mov_tab, tab.data(), sizeof(MovEntry) * tab.size(), hipMemcpyHostToDevice));
  }
  // fused statistics: a BN whose input is produced by the op right before it (stem, 1x1 conv,
  // depthwise conv) gets its batch statistics from that producer's epilogue
  E.fused_bn.assign(P.ops.size(), 0);
  E.stat_P.assign(P.tensors.size(), 0);
  size_t sp_need = 1, sc_need = 1;
  if (batch_bn()) {
    for (size_t i = 1; i < P.ops.size(); ++i) {
      const Op& op = P.ops[i];
      const Op& pr = P.ops[i - 1];
      if (op.t != OP_BN || pr.out != op.in[0]) continue;
      const Tensor& ti = P.tensors[pr.in[0]];
      const Tensor& to = P.tensors[pr.out];
      int np = 0;
      if (pr.t == OP_STEM) np = cdiv((long)to.rows(), 256);
      else if (pr.t == OP_PW && to.c % 4 == 0) np = gemm_stat_partials((int)ti.rows(), to.c, ti.c, bf16);
      else if (pr.t == OP_DW) np = dw_stat_partials(ti.n, ti.h, ti.w, ti.c, to.h, to.w, pr.k, pr.stride, pr.pad_t, pr.pad_l);
      if (np <= 0) continue;
      E.fused_bn[i] = 1;
      sp_need = std::max(sp_need, (size_t)np * to.c);
      sc_need = std::max(sc_need, (size_t)np);
    }
  }
  E.gfused_bn.assign(P.ops.size(), 0);
  E.gstat_P.assign(P.ops.size(), 0);
  if (batch_bn()) {
    for (size_t i = 0; i + 1 < P.ops.size(); ++i) {
      const Op& bn = P.ops[i];
      const Op& L = P.ops[i + 1];
      if (bn.t != OP_BN || !bn.bwd || !L.bwd) continue;
      const Tensor& tz = P.tensors[bn.out];
      int np = 0;
      const Tensor& li = P.tensors[L.in[0]];
      const Tensor& lo = P.tensors[L.out];
      if (L.t == OP_DW && L.in[0] == bn.out)
        np = dw_bwd_partials(li.n, li.h, li.w, li.c, lo.h, lo.w, L.k, L.stride, L.pad_t, L.pad_l);
      else if (L.t == OP_SE && L.in[0] == bn.out)
        np = ew_gstats_partials((long)li.h * li.w, li.c, li.n);
      else if (L.t == OP_PW && L.in[0] == bn.out && std::find(P.cls_out.begin(), P.cls_out.end(), L.out) == P.cls_out.end())
        np = gemm_dgrad_gsink_partials((int)li.rows(), li.c, lo.c, bf16);
      else if (L.t == OP_ADD && (L.in[0] == bn.out || L.in[1] == bn.out) && L.in[0] != L.in[1])
        np = ew_gstats_partials((long)tz.rows(), tz.c, 1);
      if (np <= 0 || tz.c % 4) continue;
      E.gfused_bn[i] = 1;
      E.gstat_P[i] = np;
      sp_need = std::max(sp_need, (size_t)np * tz.c);
    }
  }
  plan_groups(E, batch_bn());
  if (bn_mode == PHX_BN_SYNC) {
    int cmax = 1;
    for (const Tensor& t : P.tensors) cmax = std::max(cmax, t.c);
    E.sync_sums = E.alloc<double>((size_t)kMaxSeg * cmax * 3);
  }
  E.fuse_folded.assign(P.ops.size(), 0);
  {
    static const bool fold = [] {
      const char* e = std::getenv("PHX_FOLD");
      return !(e && e[0] == '0');
    }();
    std::vector<int> nuse(P.tensors.size(), 0);
    for (const Op& op : P.ops)
      for (int j = 0; j < op.nin; ++j) ++nuse[op.in[j]];
    for (size_t i = 0; fold && i + 1 < P.ops.size(); ++i) {
      const Op& f = P.ops[i];
      const Op& d = P.ops[i + 1];
      if (f.t != OP_FUSE || d.t != OP_DW || d.in[0] != f.out || nuse[f.out] != 1) continue;
      if (d.k != 3 || d.stride != 1 || E.grp_of[i + 1] >= 0 || P.tensors[f.out].c % 4) continue;
      if (i + 2 < P.ops.size() && E.fused_bn[i + 2]) continue;
      E.fuse_folded[i] = 1;
    }
  }
  // fused separable convs: a 3x3 stride-1 depthwise op whose output feeds only the next op's
  // pointwise conv (keras SeparableConv2D of the BiFPN nodes and both heads, model.cpp sepconv), fp32,
  // both ungrouped or grouped member for member (the heads' per-level copies).  PHX_SEP=0 keeps the
  // two launches (A/B; read per executor).
  E.sep.assign(P.ops.size(), 0);
  {
    const char* se = std::getenv("PHX_SEP");
    const bool on = !(se && se[0] == '0');
    const char* sr = std::getenv("PHX_SEP_MINROWS");
    const long sep_min_rows = sr ? atol(sr) : 32768;
    std::vector<int> nuse(P.tensors.size(), 0);
    for (const Op& op : P.ops)
      for (int j = 0; j < op.nin; ++j) ++nuse[op.in[j]];
    for (size_t i = 0; on && i + 1 < P.ops.size(); ++i) {
      const Op& d = P.ops[i];
      const Op& pw = P.ops[i + 1];
      if (d.t != OP_DW || pw.t != OP_PW || pw.in[0] != d.out || pw.nin != 1 || nuse[d.out] != 1) continue;
      if (d.k != 3 || d.stride != 1 || d.in[0] == P.input) continue;
      const Tensor& ti = P.tensors[d.in[0]];
      const Tensor& to = P.tensors[pw.out];
      if (!sep_supported(ti.c, to.c, E.bf16 || E.abf) || E.se_of_tensor[d.out] >= 0) continue;
      // the fused launch is a latency chain per 8 x 16 tile (window, depthwise, MFMAs, stores): it wins
      // where there are enough tiles to fill the chip (the P3 level; a head group, whose P3 member
      // dominates) and loses to the two launches on the small levels (tools/sep_probe: 4 x 4 to
      // 32 x 32 levels of 16 images 1-5 us slower fused)
      if ((long)ti.rows() < sep_min_rows) continue;
      const int gd = E.grp_of[i], gp = E.grp_of[i + 1];
      if (gd < 0 && gp >= 0) continue;
      if (gd >= 0) {
        // the pointwise members: the depthwise group's, member for member — or ungrouped copies of one
        // kernel (the class head's predict conv: N = 810 is not grouped as a GEMM)
        const std::vector<int>& a = E.groups[gd];
        bool ok = a[0] == (int)i;
        for (size_t r = 0; ok && r < a.size(); ++r) {
          const Op& pr = P.ops[a[r] + 1];
          ok = pr.t == OP_PW && pr.in[0] == P.ops[a[r]].out && pr.w == pw.w && pr.b == pw.b &&
               (gp >= 0 ? E.grp_of[a[r] + 1] == gp && E.groups[gp][r] == a[r] + 1 : E.grp_of[a[r] + 1] < 0);
        }
        if (gp >= 0) ok = ok && E.groups[gp].size() == a.size();
        if (!ok) continue;
      }
      if (i > 0 && E.fuse_folded[i - 1] && gd >= 0) continue;  // (a fuse view is never grouped)
      const std::vector<int> mem = gd >= 0 ? E.groups[gd] : std::vector<int>{(int)i};
      for (int di : mem) {
        E.sep[di] = 1;
        const Tensor& tm = P.tensors[P.ops[di].in[0]];
        if (di + 2 < (int)P.ops.size() && E.fused_bn[di + 2] && P.ops[di + 2].in[0] == P.ops[di + 1].out) {
          const int np = sep_stat_partials(tm.n, tm.h, tm.w);
          sp_need = std::max(sp_need, (size_t)np * to.c);
          sc_need = std::max(sc_need, (size_t)np);
        }
      }
    }
  }
  // the fused sepconvs' backward: pointwise dgrad through the consumer BN's gradient view and the
  // depthwise transpose in one launch (not the class-predict conv: its input gradient is the sparse
  // scatter's).  PHX_SEPB=0 keeps the two launches.
  E.sepb.assign(P.ops.size(), 0);
  {
    const char* sb = std::getenv("PHX_SEPB");
    const bool on = !(sb && sb[0] == '0') && batch_bn();
    for (size_t i = 0; on && i + 1 < P.ops.size(); ++i) {
      if (!E.sep[i]) continue;
      const int gd = E.grp_of[i];
      if (gd >= 0 && E.groups[gd][0] != (int)i) continue;  // (decided per group, at its first member)
      const std::vector<int> mem = gd >= 0 ? E.groups[gd] : std::vector<int>{(int)i};
      bool ok = true;
      for (int di : mem) {
        const Op& d = P.ops[di];
        const Op& pw = P.ops[di + 1];
        const int bi = E.bn_consumer[pw.out];
        ok = ok && d.bwd && pw.bwd && !is_cls_out(P, pw.out) && bi >= 0 && P.ops[bi].bwd &&
             sep_bwd_supported(P.tensors[d.in[0]].c, P.tensors[pw.out].c, E.bf16 || E.abf);
        ok = ok && (di > 0 && E.gfused_bn[di - 1]) == (mem[0] > 0 && E.gfused_bn[mem[0] - 1]);
      }
      // a grouped pointwise dgrad must be the depthwise group's twin (the launch replaces both)
      if (gd >= 0 && E.grp_of[i + 1] < 0) ok = false;
      if (!ok) continue;
      for (int di : mem) {
        E.sepb[di] = 1;
        if (di > 0 && E.gfused_bn[di - 1]) {
          const Tensor& tm = P.tensors[P.ops[di].in[0]];
          const int np = sep_stat_partials(tm.n, tm.h, tm.w);
          E.gstat_P[di - 1] = np;
          sp_need = std::max(sp_need, (size_t)np * tm.c);
        }
      }
    }
  }
  const size_t nreg = E.groups.empty() ? 1 : kMaxSeg;
  E.sp_region = sp_need;
  E.sc_region = sc_need;
  E.spart = E.alloc<float2>(sp_need * nreg);
  E.scnt = E.alloc<float>(sc_need * nreg);
  E.stat_region.assign(P.tensors.size(), 0);
  E.gstat_region.assign(P.ops.size(), 0);
  E.pool_amax.assign(P.ops.size(), nullptr);
  for (size_t i = 0; i < P.ops.size(); ++i)
    if (P.ops[i].t == OP_MAXPOOL) E.pool_amax[i] = E.alloc<uint8_t>(P.tensors[P.ops[i].out].numel());
  size_t gp_need = 1;
  for (const Op& op : P.ops) {
    if (op.t != OP_PW) continue;
    const Tensor& ti = P.tensors[op.in[0]];
    const Tensor& to = P.tensors[op.out];
    gp_need = std::max(gp_need, gemm_partial_floats((int)ti.rows(), to.c, ti.c, bf16));  // forward
    gp_need = std::max(gp_need, gemm_partial_floats((int)ti.rows(), ti.c, to.c, bf16));  // dgrad
  }
  E.gpart = E.alloc<float>(gp_need);
  E.red = E.alloc<double>(red_need);
  E.coef = E.alloc<float>(coef_need);
  E.se_g = E.alloc<float>(seg_need);
  // level tables (class / box outputs)
  const int nlev = (int)P.cls_out.size();
  const int na = mc.num_anchors();
  int a0 = 0;
  for (int l = 0; l < nlev; ++l) {
    const Tensor& tc = P.tensors[P.cls_out[l]];
    const Tensor& tb = P.tensors[P.box_out[l]];
    LevelDesc d;
    d.cls_off = (long)tc.off - (long)P.tensors[P.cls_out[0]].off;
    d.box_off = (long)tb.off - (long)P.tensors[P.box_out[0]].off;
    d.h = tc.h;
    d.w = tc.w;
    d.anchor0 = a0;
    d.tile0 = E.ntiles;
    E.ntiles += pre_nms_tiles(tc.h, tc.w, na);
    a0 += tc.h * tc.w * na;
    E.lev.push_back(d);
    // input of the class-predict pointwise conv
    for (const Op& op : P.ops)
      if (op.out == P.cls_out[l]) E.dxoff.push_back(P.tensors[op.in[0]].goff);
  }
  if (a0 != A) throw std::runtime_error("anchor count mismatch");
  E.lev_dev = E.alloc<LevelDesc>(nlev);
  PHX_HIP(hipMemcpy(E.lev_dev, E.lev.data(), nlev * sizeof(LevelDesc), hipMemcpyHostToDevice));
  E.dxoff_dev = E.alloc<long>(nlev);
  PHX_HIP(hipMemcpy(E.dxoff_dev, E.dxoff.data(), nlev * sizeof(long), hipMemcpyHostToDevice));
  // post-processing buffers
  const long BA = (long)B * A;
  E.scores = E.alloc<float>(BA);
  E.classes = E.alloc<int>(BA);
  E.boxes = E.alloc<float>(BA * 4);
  E.keep = E.alloc<uint8_t>(BA);
  E.cand_list = E.alloc<int>(BA);
  E.cand_count = E.alloc<int>(B);
  PHX_HIP(hipMemset(E.cand_count, 0, (size_t)B * sizeof(int)));
  E.nms_ws = E.alloc<float>(soft_nms_work_floats(B, A));
  E.nms1_boxes = E.alloc<float>((size_t)B * PHX_MAX_OUT * 4);
  E.nms1_scores = E.alloc<float>((size_t)B * PHX_MAX_OUT);
  E.nms1_count = E.alloc<int>(B);
  E.nms2_boxes = E.alloc<float>((size_t)B * PHX_MAX_OUT * 4);
  E.nms2_scores = E.alloc<float>((size_t)B * PHX_MAX_OUT);
  E.nms2_count = E.alloc<int>(B);
  E.mraw = E.alloc<float>(B);
  E.dm = E.alloc<float>(B);
  E.argm = E.alloc<int>(B);
  E.nties = E.alloc<int>(B);
  E.imax_scratch = E.alloc<int>(image_max_scratch_ints(B));
  // EOT
  const int S = mc.image_size;
  E.ed.B = B;
  E.ed.H = S;
  E.ed.W = S;
  E.ed.maxb = PHX_MAX_OUT;
  E.ed.P = PHX_PATCH_SIZE;
  E.ed.span_stride = S;
  // worst case: every slot holds a full-image patch
  E.ed.rcap = (long)B * PHX_MAX_OUT * S * S * 3;
  const long nslot = (long)B * PHX_MAX_OUT;
  E.img = E.alloc<ImgParams>(B);
  {
    size_t bytes = nslot * sizeof(BoxPlace) + (4 + 2 * B + 3 * nslot + 2 + 8 * B + 8 * nslot) * sizeof(int);
    E.place = reinterpret_cast<BoxPlace*>(E.alloc<char>(bytes));
  }
  E.spans = E.alloc<SpanEntry>(nslot * S);
  E.ysum = E.alloc<double>((size_t)B * 2 * 64);
  E.ymean = E.alloc<float>((size_t)B * 2);
  // the resized patches; reused by the resize adjoint's row buffer once the rotation backward
  // has consumed them
  // (the concurrent first pass's executor runs no EOT: its patch stores stay one element)
  const bool eot = tag != 1;
  E.rstore = E.alloc<float>(eot ? std::max(E.ed.rcap, eot_resize_scratch_floats(E.ed)) : 1);
  E.dstore = E.alloc<float>(eot ? E.ed.rcap : 1);
  const size_t np = (size_t)PHX_PATCH_SIZE * PHX_PATCH_SIZE * 3;
  E.matched = E.alloc<float>(eot ? np * B : 1);
  E.dmatched = E.alloc<float>(eot ? np * B : 1);
  E.dsum = E.alloc<double>((size_t)B * 64);
  E.tvs = E.alloc<double>(256);
  E.err = E.alloc<int>(1);
  E.patched = E.alloc<float>(eot ? (size_t)B * S * S * 3 : 1);
  E.owner = E.alloc<int16_t>(eot ? (size_t)B * S * S * 3 : 1);
  {
    std::vector<int> blk;
    std::vector<float> pr;
    E.drop_slot.assign(P.ops.size(), -1);
    for (size_t i = 0; i < P.ops.size(); ++i)
      if (P.ops[i].t == OP_ADD && P.ops[i].survival > 0.f) {
        E.drop_slot[i] = (int)blk.size();
        blk.push_back(P.ops[i].drop_block);
        pr.push_back(P.ops[i].survival);
      }
    E.ndrop = (int)blk.size();
    if (E.ndrop) {
      E.drop_block = E.alloc<int>(E.ndrop);
      E.drop_p = E.alloc<float>(E.ndrop);
      E.drop_keep = E.alloc<float>((size_t)E.ndrop * B);
      PHX_HIP(hipMemcpy(E.drop_block, blk.data(), blk.size() * sizeof(int), hipMemcpyHostToDevice));
      PHX_HIP(hipMemcpy(E.drop_p, pr.data(), pr.size() * sizeof(float), hipMemcpyHostToDevice));
    }
  }
  E.inj_boxes = E.alloc<float>((size_t)B * PHX_MAX_OUT * 4);
  E.inj_count = E.alloc<int>(B);
  E.dscale_scratch = E.alloc<float>(1);
  E.used = clock;
  execs.push_back(std::move(ex));
  return *execs.back();
}

namespace {

// How consumers see tensor t: BN outputs are virtual (BN input + per-channel transform).
InX view(phx_ctx* ctx, const Exec& E, int t, const float* input) {
  int bi = E.bn_of_tensor[t];
  if (bi < 0) return InX{E.tptr(t, input), nullptr, nullptr, nullptr, 0, E.tbf(t)};
  const Op& op = E.prog.ops[bi];
  return InX{E.tptr(op.in[0], input), E.slot_a[op.slot], E.slot_c[op.slot], ctx->w() + op.beta, op.act,
             E.tbf(op.in[0])};
}

// The gradient w.r.t. tensor t as its producer's dgrad sees it: for a BN input the BN backward
// is applied on load (GradX); otherwise the materialised gradient.
GradX gview(phx_ctx* ctx, const Exec& E, int t, const float* input) {
  int bi = E.bn_consumer[t];
  if (bi >= 0 && E.prog.ops[bi].bwd) {
    const Op& op = E.prog.ops[bi];
    return GradX{E.gptr(op.out), E.tptr(t, input), E.slot_a[op.slot], E.slot_b[op.slot],
                 E.slot_c[op.slot], ctx->w() + op.beta, E.slot_d[op.slot], E.slot_e[op.slot], op.act, E.tbf(t)};
  }
  return GradX{E.gptr(t), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
}

// Work-skipping timing diagnostics (wrong results), compiled in only with -DPHX_DEBUG_KNOBS=1 (make
// DEBUG_KNOBS=1): the shipped library ignores PHX_SKIP_TIMING / PHX_SKIP_KINDS / PHX_NO_DROP, so no
// environment can make a measured step skip work (bench.py also refuses to run with them set).
#if defined(PHX_DEBUG_KNOBS) && PHX_DEBUG_KNOBS
// PHX_SKIP_TIMING=f,b,s (timing experiments only: wrong results): skip the forward BN finalizes (f),
// the backward ones (b), the SE MLP launches (s) — what removing them would be worth at most
bool skip_timing(char k) {
  static const std::string v = [] {
    const char* e = std::getenv("PHX_SKIP_TIMING");
    return std::string(e ? e : "");
  }();
  return v.find(k) != std::string::npos;
}

// PHX_SKIP_KINDS=f:gemm,b:dw_bwd,...|name1,name2 (timing experiments only: wrong results): skip the
// ungrouped launches of those kinds (f: forward, b: backward), or of ops whose name contains one of
// the names after '|'
bool skip_kind(const std::string& kind, const std::string& name) {
  static const std::pair<std::vector<std::string>, std::vector<std::string>> v = [] {
    std::pair<std::vector<std::string>, std::vector<std::string>> r;
    const char* e = std::getenv("PHX_SKIP_KINDS");
    std::string t = e ? e : "";
    const size_t bar = t.find('|');
    auto split = [](const std::string& x, std::vector<std::string>& out) {
      size_t a = 0;
      while (a < x.size()) {
        size_t b = x.find(',', a);
        if (b == std::string::npos) b = x.size();
        if (b > a) out.push_back(x.substr(a, b - a));
        a = b + 1;
      }
    };
    split(t.substr(0, bar), r.first);
    if (bar != std::string::npos) split(t.substr(bar + 1), r.second);
    return r;
  }();
  if (v.first.empty() && v.second.empty()) return false;
  for (const auto& k : v.first)
    if (k == kind) return true;
  for (const auto& n : v.second)
    if (name.find(n) != std::string::npos) return true;
  return false;
}
#else
bool skip_timing(char) { return false; }
bool skip_kind(const std::string&, const std::string&) { return false; }
#endif

// ---- PHX_CKSUM diagnostics -----------------------------------------------------------------
// Read per call, so one process can compare a one-stream step with concurrent ones op by op: the
// first checksum that differs between two steps on the same inputs names the launch whose inputs
// still agreed and whose output did not.
bool cksum_env() {
  const char* e = std::getenv("PHX_CKSUM");
  return e && e[0] == '1';
}

void ck_begin(Exec& E, hipStream_t s) {
  E.ck_on = cksum_env();
  E.ck_names.clear();
  if (!E.ck_on) return;
  if (!E.ck) {
    E.ck_cap = 8 * E.prog.ops.size() + 256;
    E.ck = E.alloc<unsigned long long>(E.ck_cap);
  }
  PHX_HIP(hipMemsetAsync(E.ck, 0, E.ck_cap * sizeof(unsigned long long), s));
}

void ck_note(Exec& E, const std::string& name, const void* p, size_t bytes, hipStream_t s) {
  if (!E.ck_on || !p || E.ck_names.size() >= E.ck_cap) return;
  launch_cksum(p, bytes, E.ck + E.ck_names.size(), s);
  E.ck_names.push_back(name);
}

// what forward op i wrote (every member, for a grouped launch)
void ck_fwd(Exec& E, int i, int pass, hipStream_t s) {
  if (!E.ck_on) return;
  const Program& P = E.prog;
  const Op& op = P.ops[i];
  if (E.fuse_folded[i] || E.sep[i]) return;  // (never stored)
  const std::string nm = "p" + std::to_string(pass) + " f " + std::to_string(i) + " " + op.name;
  const Tensor& ti = P.tensors[op.in[0]];
  if (op.t == OP_BN) {
    ck_note(E, nm + " mean", E.slot_a[op.slot], ti.c * 4, s);
    ck_note(E, nm + " rstd", E.slot_b[op.slot], ti.c * 4, s);
    ck_note(E, nm + " scale", E.slot_c[op.slot], ti.c * 4, s);
  } else if (op.t == OP_SE) {
    ck_note(E, nm + " excite", E.slot_c[op.slot], (size_t)E.B * ti.c * 4, s);
  } else {
    const Tensor& to = P.tensors[op.out];
    ck_note(E, nm + " out", E.tptr(op.out, nullptr), to.numel() * (E.tbf(op.out) ? 2 : 4), s);
  }
}

// the forward outputs of pass `pass` once more, as "post <name>" (after the step's join)
void ck_post(Exec& E, int pass, hipStream_t s) {
  const size_t n0 = E.ck_names.size();
  for (size_t i = 0; i < E.prog.ops.size(); ++i) ck_fwd(E, (int)i, pass, s);
  for (size_t k = n0; k < E.ck_names.size(); ++k) E.ck_names[k] = "post " + E.ck_names[k];
}

// what backward op i wrote: its inputs' gradients (BN: the backward means)
void ck_bwd(Exec& E, int i, hipStream_t s) {
  if (!E.ck_on) return;
  const Program& P = E.prog;
  const Op& op = P.ops[i];
  const std::string nm = "b " + std::to_string(i) + " " + op.name;
  if (op.t == OP_BN) {
    const int C = P.tensors[op.in[0]].c;
    ck_note(E, nm + " mdz", E.slot_d[op.slot], C * 4, s);
    ck_note(E, nm + " mdzx", E.slot_e[op.slot], C * 4, s);
    return;
  }
  for (int k = 0; k < op.nin; ++k)
    if (const float* g = E.gptr(op.in[k])) ck_note(E, nm + " d" + std::to_string(k), g, P.tensors[op.in[k]].numel() * 4, s);
}

// ---- level-batched heads -----------------------------------------------------------------
bool grouping_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("PHX_GROUP");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Members of a candidate group must be interchangeable launches: same op kind and geometry, same
// statistics / gradient-sink wiring, no SE row scale; grouped GEMMs must not need split-K.
bool group_uniform(const Exec& E, const std::vector<int>& v) {
  const Program& P = E.prog;
  const Op& a = P.ops[v[0]];
  const int n = (int)P.ops.size();
  auto fused_next = [&](int i) { return i + 1 < n && E.fused_bn[i + 1]; };
  auto gfused_prev = [&](int i) { return i > 0 && E.gfused_bn[i - 1]; };
  auto has_gx = [&](int i) {
    const int bi = E.bn_consumer[P.ops[i].out];
    return bi >= 0 && P.ops[bi].bwd;
  };
  std::vector<int> M;
  for (int i : v) {
    const Op& b = P.ops[i];
    const Tensor& ti = P.tensors[b.in[0]];
    const Tensor& to = P.tensors[b.out];
    const Tensor& ta = P.tensors[a.in[0]];
    const Tensor& tb = P.tensors[a.out];
    if (b.t != a.t || b.k != a.k || b.stride != a.stride || b.nin != 1 || ti.c != ta.c || to.c != tb.c ||
        ti.n != ta.n)
      return false;
    if (b.bwd != a.bwd || b.acc[0] != a.acc[0] || fused_next(i) != fused_next(v[0]) ||
        gfused_prev(i) != gfused_prev(v[0]) || has_gx(i) != has_gx(v[0]))
      return false;
    if ((E.bn_of_tensor[b.in[0]] >= 0) != (E.bn_of_tensor[a.in[0]] >= 0)) return false;
    if (E.se_of_tensor[b.in[0]] >= 0 || b.in[0] == P.input) return false;
    if (gfused_prev(i) && P.ops[i - 1].out != b.in[0]) return false;
    M.push_back((int)ti.rows());
  }
  if (a.t == OP_PW) {
    const Tensor& ta = P.tensors[a.in[0]];
    const Tensor& tb = P.tensors[a.out];
    if (!gemm_group_ok(M.data(), (int)M.size(), tb.c, ta.c, E.bf16)) return false;  // forward
    if (a.bwd && !gemm_group_ok(M.data(), (int)M.size(), ta.c, tb.c, E.bf16)) return false;  // dgrad
  }
  return true;
}

// Groups: convs sharing a weight tensor (the per-level copies of a head conv) and the BNs right
// after them.  The schedule is then checked; any violation disables grouping for this executor.
void plan_groups(Exec& E, bool local_bn) {
  const Program& P = E.prog;
  const int n = (int)P.ops.size();
  E.grp_of.assign(n, -1);
  E.groups.clear();
  if (!grouping_enabled() || !local_bn) return;
  std::map<long, std::vector<int>> byw;
  for (int i = 0; i < n; ++i)
    if ((P.ops[i].t == OP_DW || P.ops[i].t == OP_PW) && P.ops[i].w >= 0) byw[P.ops[i].w].push_back(i);
  for (auto& kv : byw) {
    const std::vector<int>& v = kv.second;
    if (v.size() < 2 || v.size() > (size_t)kMaxSeg || !group_uniform(E, v)) continue;
    const int g = (int)E.groups.size();
    E.groups.push_back(v);
    for (int i : v) E.grp_of[i] = g;
    std::vector<int> bn;
    for (int i : v)
      if (i + 1 < n && P.ops[i + 1].t == OP_BN && P.ops[i + 1].in[0] == P.ops[i].out && E.fused_bn[i + 1] &&
          !P.ops[i + 1].acc[0])
        bn.push_back(i + 1);
    if (bn.size() != v.size()) continue;
    bool ok = true;
    for (int b : bn)
      ok = ok && P.ops[b].bwd == P.ops[bn[0]].bwd && E.gfused_bn[b] == E.gfused_bn[bn[0]] &&
           P.ops[b].act == P.ops[bn[0]].act;
    if (!ok || (P.ops[bn[0]].bwd && !E.gfused_bn[bn[0]])) continue;
    const int gb = (int)E.groups.size();
    E.groups.push_back(bn);
    for (int b : bn) E.grp_of[b] = gb;
  }
  if (E.groups.empty()) return;
  // schedule checks: forward position = first member, reverse position = last member
  auto fpos = [&](int i) { return E.grp_of[i] >= 0 ? E.groups[E.grp_of[i]].front() : i; };
  auto bpos = [&](int i) { return E.grp_of[i] >= 0 ? E.groups[E.grp_of[i]].back() : i; };
  std::vector<int> producer(P.tensors.size(), -1);
  for (int i = 0; i < n; ++i) producer[P.ops[i].out] = i;
  bool ok = true;
  for (int i = 0; i < n && ok; ++i) {
    const Op& op = P.ops[i];
    for (int j = 0; j < op.nin; ++j) {
      const int p = producer[op.in[j]];
      if (p >= 0 && (fpos(p) >= fpos(i) || (E.grp_of[i] >= 0 && E.grp_of[p] == E.grp_of[i]))) ok = false;
    }
    // statistics partials: producer launch immediately before its BN's finalize
    if (op.t == OP_BN && E.fused_bn[i] && fpos(i) != fpos(i - 1) + 1) ok = false;
    if (op.t == OP_BN && E.gfused_bn[i] && op.bwd && bpos(i + 1) != bpos(i) + 1) ok = false;
  }
  // reverse sweep: every consumer's backward before its producer's; writers of one gradient keep
  // their program order and never share a launch
  for (int i = 0; i < n && ok; ++i) {
    if (!P.ops[i].bwd) continue;
    for (int c = i + 1; c < n && ok; ++c) {
      const Op& oc = P.ops[c];
      if (!oc.bwd || (oc.t == OP_PW && is_cls_out(P, oc.out))) continue;
      for (int j = 0; j < oc.nin; ++j) {
        if (oc.in[j] == P.ops[i].out && bpos(c) <= bpos(i)) ok = false;
        for (int k = 0; k < P.ops[i].nin; ++k)
          if (oc.in[j] == P.ops[i].in[k] && (bpos(c) <= bpos(i))) ok = false;
      }
    }
  }
  if (!ok) {
    E.grp_of.assign(n, -1);
    E.groups.clear();
  }
}

// PHX_FROZEN_REUSE=0: every inference pass recomputes its BN statistics (A/B; read per call)
bool frozen_reuse_off() {
  const char* e = std::getenv("PHX_FROZEN_REUSE");
  return e && e[0] == '0';
}


// bn=sync: the BN sums of `segs` (fold -> the caller's all-reduce -> statistics from the global sums)
// bn=sync: all-reduce the sums of `n` members already in E.sync_sums, then their statistics
void sync_reduce_apply(phx_ctx* ctx, Exec& E, const BnFinSeg* segs, int n, int C, bool bwd, hipStream_t s) {
  if (!ctx->ar_fn) throw std::logic_error("bn=sync: no collective registered (phx_set_allreduce)");
  if (ctx->ar_fn(ctx->ar_user, E.sync_sums, (size_t)n * C * 3, s) != 0)
    throw std::runtime_error("bn=sync: the all-reduce callback failed");
  launch_bn_from_sums(segs, n, C, bwd, E.sync_sums, kBnEps, s);
}

void sync_finalize(phx_ctx* ctx, Exec& E, const BnFinSeg* segs, int n, int C, bool bwd, hipStream_t s) {
  if (!ctx->ar_fn) throw std::logic_error("bn=sync: no collective registered (phx_set_allreduce)");
  launch_bn_fold_sums(segs, n, C, bwd, E.sync_sums, s);
  sync_reduce_apply(ctx, E, segs, n, C, bwd, s);
}

void run_group_fwd(phx_ctx* ctx, Exec& E, int gid, const float* input, hipStream_t s, bool frozen) {
  const Program& P = E.prog;
  const std::vector<int>& g = E.groups[gid];
  const int n = (int)g.size();
  const Op& o0 = P.ops[g[0]];
  const Tensor& ti0 = P.tensors[o0.in[0]];
  const Tensor& to0 = P.tensors[o0.out];
  float* W = ctx->w();
  const bool sink_on = !frozen && g[0] + 1 < (int)P.ops.size() && E.fused_bn[g[0] + 1];
  auto sink_of = [&](int r) {
    return sink_on ? StatSink{E.spart + (size_t)r * E.sp_region, E.scnt + (size_t)r * E.sc_region, to0.c, 0}
                   : StatSink{};
  };
  double fl = 0, by = 0;
  for (int i : g) {
    const Tensor& ti = P.tensors[P.ops[i].in[0]];
    const Tensor& to = P.tensors[P.ops[i].out];
    if (o0.t == OP_PW) fl += 2.0 * ti.rows() * ti.c * to.c;
    if (o0.t == OP_DW) fl += 2.0 * to.numel() * o0.k * o0.k;
    by += o0.t == OP_BN ? 8.0 * (double)E.stat_P[P.ops[i].in[0]] * ti.c : 4.0 * (double)(ti.numel() + to.numel());
  }
  if (o0.t == OP_PW) by += 4.0 * ti0.c * to0.c;
  Scope scope(ctx, o0.t == OP_PW ? "gemm" : o0.t == OP_DW ? "dw_fwd" : "bn_stats", fl, by, s,
              prof_detail() ? " group" + op_tag(P, o0, false) : std::string());
  switch (o0.t) {
    case OP_DW: {
      DwSeg segs[kMaxSeg];
      int nps[kMaxSeg];
      for (int r = 0; r < n; ++r) {
        const Op& op = P.ops[g[r]];
        const Tensor& ti = P.tensors[op.in[0]];
        const Tensor& to = P.tensors[op.out];
        segs[r] = DwSeg{view(ctx, E, op.in[0], input), GradX{}, E.tptr(op.out, input), ti.h, ti.w, to.h, to.w,
                        op.pad_t, op.pad_l, false, sink_of(r), GradSink{}};
      }
      launch_dw_fwd_group(segs, n, ti0.n, ti0.c, W + o0.w, o0.k, o0.stride, s, nps);
      if (sink_on)
        for (int r = 0; r < n; ++r) {
          E.stat_P[P.ops[g[r]].out] = nps[r];
          E.stat_region[P.ops[g[r]].out] = r;
        }
      break;
    }
    case OP_PW: {
      GemmSeg segs[kMaxSeg];
      const int mode = view(ctx, E, o0.in[0], input).mu ? 1 : 0;
      for (int r = 0; r < n; ++r) {
        const Op& op = P.ops[g[r]];
        segs[r] = GemmSeg{view(ctx, E, op.in[0], input), GradX{}, op.b >= 0 ? W + op.b : nullptr,
                          E.tptr(op.out, input), (int)P.tensors[op.in[0]].rows(), false, sink_of(r), GradSink{}};
      }
      int np[kMaxSeg];  // each member's statistics partial rows
      gemm_group_run(mode, segs, n, ctx->wt_of(o0.w), to0.c, ti0.c, s, E.bf16, np,
                     std::min<long>((long)(E.sp_region / to0.c), (long)E.sc_region));
      if (sink_on)
        for (int r = 0; r < n; ++r) {
          E.stat_P[P.ops[g[r]].out] = np[r];
          E.stat_region[P.ops[g[r]].out] = r;
        }
      break;
    }
    case OP_BN: {
      if (frozen) {  // inference BN (test_step): statistics from the moving averages
        if (E.frozen_ver == ctx->w_ver && !frozen_reuse_off()) break;  // (kept from the last inference pass)
        for (int r = 0; r < n; ++r) {
          const Op& op = P.ops[g[r]];
          launch_bn_frozen_stats(W + op.mmean, W + op.mvar, E.slot_a[op.slot], E.slot_b[op.slot],
                                 W + op.gamma, E.slot_c[op.slot], ti0.c, kBnEps, s);
        }
        break;
      }
      BnFinSeg segs[kMaxSeg];
      for (int r = 0; r < n; ++r) {
        const Op& op = P.ops[g[r]];
        const int reg = E.stat_region[op.in[0]];
        segs[r] = BnFinSeg{E.spart + (size_t)reg * E.sp_region, E.scnt + (size_t)reg * E.sc_region,
                           E.stat_P[op.in[0]], (long)P.tensors[op.in[0]].rows(), E.slot_a[op.slot],
                           E.slot_b[op.slot], W + op.gamma, E.slot_c[op.slot], W + op.mmean, W + op.mvar,
                           nullptr, nullptr, E.side_for(op.slot)};
      }
      if (ctx->bn_mode == PHX_BN_SYNC) sync_finalize(ctx, E, segs, n, ti0.c, false, s);
      else if (!skip_timing('f')) launch_bn_finalize_group(segs, n, ti0.c, kBnEps, s);
      break;
    }
    default:
      throw std::logic_error("grouped launch of an unsupported op");
  }
}

void run_group_bwd(phx_ctx* ctx, Exec& E, int gid, const float* input, hipStream_t s) {
  const Program& P = E.prog;
  const std::vector<int>& g = E.groups[gid];
  const int n = (int)g.size();
  const Op& o0 = P.ops[g[0]];
  const Tensor& ti0 = P.tensors[o0.in[0]];
  const Tensor& to0 = P.tensors[o0.out];
  float* W = ctx->w();
  const bool gs_on = g[0] > 0 && E.gfused_bn[g[0] - 1];
  auto gsk_of = [&](int r) {
    if (!gs_on) return GradSink{};
    const Op& bn = P.ops[g[r] - 1];
    return GradSink{E.spart + (size_t)r * E.sp_region, P.tensors[bn.out].c, 0, E.tptr(bn.in[0], input),
                    E.slot_a[bn.slot], E.slot_b[bn.slot], E.slot_c[bn.slot], W + bn.beta, bn.act, E.tbf(bn.in[0])};
  };
  double fl = 0, by = 0;
  for (int i : g) {
    const Tensor& ti = P.tensors[P.ops[i].in[0]];
    const Tensor& to = P.tensors[P.ops[i].out];
    if (o0.t == OP_PW) fl += 2.0 * ti.rows() * ti.c * to.c;
    if (o0.t == OP_DW) fl += 2.0 * to.numel() * o0.k * o0.k;
    by += o0.t == OP_BN ? 8.0 * (double)E.gstat_P[i] * ti.c : 4.0 * (double)(ti.numel() + to.numel());
    if (o0.t != OP_BN) {
      const int bi = E.bn_consumer[P.ops[i].out];
      if (bi >= 0 && P.ops[bi].bwd) by += 4.0 * (double)to.numel();
      if (P.ops[i].acc[0]) by += 4.0 * (double)ti.numel();
    }
  }
  if (o0.t == OP_PW) by += 4.0 * ti0.c * to0.c;
  Scope scope(ctx, o0.t == OP_PW ? "gemm" : o0.t == OP_DW ? "dw_bwd" : "bn_bwd_reduce", fl, by, s,
              prof_detail() ? " group" + op_tag(P, o0, true) : std::string());
  switch (o0.t) {
    case OP_DW: {
      DwSeg segs[kMaxSeg];
      int nps[kMaxSeg];
      for (int r = 0; r < n; ++r) {
        const Op& op = P.ops[g[r]];
        const Tensor& ti = P.tensors[op.in[0]];
        const Tensor& to = P.tensors[op.out];
        segs[r] = DwSeg{InX{}, gview(ctx, E, op.out, input), E.gptr(op.in[0]), ti.h, ti.w, to.h, to.w, op.pad_t,
                        op.pad_l, op.acc[0], StatSink{}, gsk_of(r)};
      }
      launch_dw_bwd_group(segs, n, ti0.n, ti0.c, W + o0.w, o0.k, o0.stride, s, nps);
      if (gs_on)
        for (int r = 0; r < n; ++r) {
          E.gstat_P[g[r] - 1] = nps[r];
          E.gstat_region[g[r] - 1] = r;
        }
      break;
    }
    case OP_PW: {
      GemmSeg segs[kMaxSeg];
      const GradX gx0 = gview(ctx, E, o0.out, input);
      const int mode = gx0.y ? 3 : 0;
      for (int r = 0; r < n; ++r) {
        const Op& op = P.ops[g[r]];
        const GradX gv = gview(ctx, E, op.out, input);
        segs[r] = GemmSeg{InX{gv.da, nullptr, nullptr, nullptr, 0}, gv, nullptr, E.gptr(op.in[0]),
                          (int)P.tensors[op.in[0]].rows(), op.acc[0], StatSink{}, gsk_of(r)};
      }
      // dX[M,Cin] = dY[M,Cout] * W^T : Bt = W in HWIO layout [Cin][Cout]
      int np[kMaxSeg];  // each member's BN-backward-sum partial rows
      gemm_group_run(mode, segs, n, W + o0.w, ti0.c, to0.c, s, E.bf16, np, (long)(E.sp_region / ti0.c));
      if (gs_on)
        for (int r = 0; r < n; ++r) {
          E.gstat_P[g[r] - 1] = np[r];
          E.gstat_region[g[r] - 1] = r;
        }
      break;
    }
    case OP_BN: {
      if (ctx->bn_mode == PHX_BN_FROZEN) break;
      BnFinSeg segs[kMaxSeg];
      for (int r = 0; r < n; ++r) {
        const int i = g[r];
        const Op& op = P.ops[i];
        segs[r] = BnFinSeg{E.spart + (size_t)E.gstat_region[i] * E.sp_region, nullptr, E.gstat_P[i],
                           (long)P.tensors[op.in[0]].rows(), nullptr, nullptr, nullptr, nullptr, nullptr,
                           nullptr, E.slot_d[op.slot], E.slot_e[op.slot]};
      }
      if (ctx->bn_mode == PHX_BN_SYNC) sync_finalize(ctx, E, segs, n, ti0.c, true, s);
      else if (!skip_timing('b')) launch_bn_bwd_finalize_group(segs, n, ti0.c, s);
      break;
    }
    default:
      throw std::logic_error("grouped launch of an unsupported op");
  }
}

// the fused separable conv whose depthwise op is i (its group's members when grouped): the depthwise
// op's input view — the BiFPN node fuse computed on load when that fuse is folded — the pointwise op's
// weights and output, and the BN after it takes its statistics from this launch
void run_sep(phx_ctx* ctx, Exec& E, int i, const float* input, hipStream_t s, bool frozen) {
  const Program& P = E.prog;
  float* W = ctx->w();
  const int gd = E.grp_of[i];
  const std::vector<int> mem = gd >= 0 ? E.groups[gd] : std::vector<int>{i};
  const int n = (int)mem.size();
  const Op& d0 = P.ops[mem[0]];
  const Op& p0 = P.ops[mem[0] + 1];
  const int C = P.tensors[d0.in[0]].c, N = P.tensors[p0.out].c;
  const bool sink_on = !frozen && mem[0] + 2 < (int)P.ops.size() && E.fused_bn[mem[0] + 2];
  SepMember m[kMaxSeg];
  double fl = 0, by = 4.0 * (9.0 * C + (double)N * C + N);
  for (int r = 0; r < n; ++r) {
    const int di = mem[r];
    const Op& d = P.ops[di];
    const Op& pw = P.ops[di + 1];
    const Tensor& ti = P.tensors[d.in[0]];
    SepMember& mm = m[r];
    mm = SepMember{};
    if (di > 0 && E.fuse_folded[di - 1]) {
      const Op& f = P.ops[di - 1];
      mm.fuse = true;
      mm.f.nin = f.nin;
      for (int k = 0; k < f.nin; ++k) {
        mm.f.x[k] = view(ctx, E, f.in[k], input);
        mm.f.w[k] = f.wsm[k] >= 0 ? W + f.wsm[k] : nullptr;
      }
      mm.f.method = f.fuse_method;
      mm.f.act = f.act;
      by += 4.0 * (double)ti.numel() * (f.nin - 1);
    } else {
      mm.x = view(ctx, E, d.in[0], input);
    }
    mm.y = E.tptr(pw.out, input);
    mm.H = ti.h;
    mm.W = ti.w;
    if (sink_on)
      mm.sink = StatSink{E.spart + (size_t)(gd >= 0 ? r : 0) * E.sp_region, E.scnt + (size_t)(gd >= 0 ? r : 0) * E.sc_region,
                         N, 0};
    fl += 2.0 * ti.numel() * 9.0 + 2.0 * (double)ti.rows() * C * N;
    by += 4.0 * ((double)ti.numel() + (double)ti.rows() * N);
  }
  Scope scope(ctx, "sep_fwd", fl, by, s,
              prof_detail() ? std::string(n > 1 ? " group" : "") + op_tag(P, p0, false) : std::string());
  int nps[kMaxSeg];
  launch_sep_fwd(m, n, E.B, C, N, W + d0.w, ctx->wt_of(p0.w), p0.b >= 0 ? W + p0.b : nullptr, s, nps);
  if (sink_on)
    for (int r = 0; r < n; ++r) {
      E.stat_P[P.ops[mem[r] + 1].out] = nps[r];
      E.stat_region[P.ops[mem[r] + 1].out] = gd >= 0 ? r : 0;
    }
}

// victim forward over the program (EfficientDetNet.call, efficientdet_keras.py:884-906)
// pass: 0 first (clean) pass, 1 second (patched) pass, 2 standalone detect — with `step` and the
// global index of the first image it keys the drop-connect draws
DropView drop_view(const Exec& E, int op) {
  const int d = E.drop_slot.empty() ? -1 : E.drop_slot[op];
  if (d < 0) return DropView{};
  const Tensor& t = E.prog.tensors[E.prog.ops[op].out];
  return DropView{E.drop_keep + (long)d * E.B, E.prog.ops[op].survival, (long)t.h * t.w};
}

// train = false: Keras training=False (test_step, attacker.py:325) — inference BN from the moving
// statistics (not updated) and no drop connect, whatever the context's BN mode
// force_frozen: inference BN in a training pass (a victim whose layers are not trainable, as the
// defender's protege, attack_detection.py:46-47); drop connect still follows `train`
void run_forward(phx_ctx* ctx, Exec& E, const float* input, hipStream_t s, int pass, int64_t step,
                 int gimg0, bool train = true, bool force_frozen = false) {
  const Program& P = E.prog;
  float* W = ctx->w();
  const bool frozen = ctx->bn_mode == PHX_BN_FROZEN || !train || force_frozen;
  // inference BN: the statistics from the moving averages are a function of the weights, so the
  // slots keep them from the last inference pass at the same weights version (the frozen protege of
  // the defender: 108 launches per step saved); a training pass overwrites the slots and may move
  // the moving statistics
  const bool frozen_reuse = frozen && E.frozen_ver == ctx->w_ver && !frozen_reuse_off();
  if (!frozen) {
    E.frozen_ver = 0;
    ++ctx->w_ver;
  }
  if (E.ndrop && train)
    launch_drop_keep(E.drop_block, E.drop_p, E.ndrop, E.B, ctx->seed, step, gimg0, pass, E.drop_keep, s);
  if (E.ndrop && train) ck_note(E, "p" + std::to_string(pass) + " drop keep", E.drop_keep, (size_t)E.ndrop * E.B * 4, s);
  for (size_t i = 0; i < P.ops.size(); ++i) {
    if (ctx->fwd_hook && i == ctx->fwd_hook_at) {
      auto h = std::move(ctx->fwd_hook);
      ctx->fwd_hook = nullptr;
      h();
    }
    if (E.grp_of[i] >= 0) {
      if (E.groups[E.grp_of[i]].front() == (int)i) {
        if (E.sep[i]) {
          run_sep(ctx, E, (int)i, input, s, frozen);
          for (int m : E.groups[E.grp_of[i]]) ck_fwd(E, m + 1, pass, s);
        } else if (!(i > 0 && E.sep[i - 1])) {  // (a fused sepconv's pointwise group: done above)
          run_group_fwd(ctx, E, E.grp_of[i], input, s, frozen);
          for (int m : E.groups[E.grp_of[i]]) ck_fwd(E, m, pass, s);
        }
      }
      continue;
    }
    if (E.fuse_folded[i]) continue;  // computed by the depthwise conv that follows
    if (E.sep[i]) {  // depthwise + pointwise in one launch
      run_sep(ctx, E, (int)i, input, s, frozen);
      ck_fwd(E, (int)i + 1, pass, s);
      continue;
    }
    if (i > 0 && E.sep[i - 1]) continue;  // (the pointwise half of the fused sepconv above)
    const Op& op = P.ops[i];
    const Tensor& ti = P.tensors[op.in[0]];
    const Tensor& to = P.tensors[op.out];
    float* x = E.tptr(op.in[0], input);
    float* y = E.tptr(op.out, input);
    double fl = 0, by = 4.0 * (double)(ti.numel() + to.numel());
    const char* kind = "fwd_other";
    switch (op.t) {
      case OP_STEM: kind = "stem_fwd"; fl = 2.0 * to.numel() * 27; break;
      case OP_PW: kind = "gemm"; fl = 2.0 * ti.rows() * ti.c * to.c; by += 4.0 * ti.c * to.c; break;
      case OP_DW: kind = "dw_fwd"; fl = 2.0 * to.numel() * op.k * op.k; break;
      case OP_BN: kind = "bn_stats"; by = 4.0 * ti.numel(); break;
      case OP_SE: kind = "se_fwd"; by = 4.0 * ti.numel(); break;
      default: break;
    }
    // the BN right after this op takes its statistics from this launch (StatSink)
    const bool sink_on = !frozen && i + 1 < P.ops.size() && E.fused_bn[i + 1];
    const StatSink sink = sink_on ? StatSink{E.spart, E.scnt, to.c, 0}
                                  : StatSink{};
    if (op.t == OP_BN && E.fused_bn[i]) by = 8.0 * (double)E.stat_P[op.in[0]] * ti.c;
    if (skip_kind(std::string("f:") + kind, op.name)) continue;
    Scope scope(ctx, kind, fl, by, s, (prof_detail() || debug_sync()) ? op_tag(P, op, false) : std::string());
    int np = 0;
    switch (op.t) {
      case OP_STEM:
        np = launch_stem_fwd(x, W + op.w, y, ti.n, ti.h, ti.w, to.h, to.w, to.c, op.pad_t, op.pad_l, s, sink,
                             E.tbf(op.out) != 0);
        break;
      case OP_PW: {
        InX A = view(ctx, E, op.in[0], input);
        const float* rs = nullptr;
        int rpi = 1;
        int se = E.se_of_tensor[op.in[0]];
        if (se >= 0) {  // SE excitation folded into the GEMM's A load
          const Op& sop = P.ops[se];
          A = view(ctx, E, sop.in[0], input);
          rs = E.slot_c[sop.slot];
          rpi = ti.h * ti.w;
        }
        np = launch_gemm(A, ctx->wt_of(op.w), op.b >= 0 ? W + op.b : nullptr, y, (int)ti.rows(), to.c,
                         ti.c, false, rs, rpi, s, E.gpart, sink, E.bf16);
        break;
      }
      case OP_DW:
        if (i > 0 && E.fuse_folded[i - 1]) {
          const Op& f = P.ops[i - 1];
          FuseView fv{};
          fv.nin = f.nin;
          for (int k = 0; k < f.nin; ++k) {
            fv.x[k] = view(ctx, E, f.in[k], input);
            fv.w[k] = f.wsm[k] >= 0 ? W + f.wsm[k] : nullptr;
          }
          fv.method = f.fuse_method;
          fv.act = f.act;
          launch_dw_fwd_fused(fv, W + op.w, y, ti.n, ti.h, ti.w, ti.c, to.h, to.w, op.k, op.stride, op.pad_t,
                              op.pad_l, s);
          break;
        }
        np = launch_dw_fwd(view(ctx, E, op.in[0], input), W + op.w, y, ti.n, ti.h, ti.w, ti.c, to.h, to.w, op.k,
                           op.stride, op.pad_t, op.pad_l, s, sink);
        break;
      case OP_BN: {
        float* mean = E.slot_a[op.slot];
        float* rstd = E.slot_b[op.slot];
        // statistics only: the normalised output is applied by every consumer on load (InX)
        if (frozen && frozen_reuse) {
        } else if (frozen)
          launch_bn_frozen_stats(W + op.mmean, W + op.mvar, mean, rstd, W + op.gamma,
                                 E.slot_c[op.slot], ti.c, kBnEps, s);
        else if (E.fused_bn[i] && ctx->bn_mode == PHX_BN_SYNC) {
          const BnFinSeg sg{E.spart + E.stat_region[op.in[0]] * E.sp_region,
                            E.scnt + E.stat_region[op.in[0]] * E.sc_region, E.stat_P[op.in[0]], (long)ti.rows(),
                            mean, rstd, W + op.gamma, E.slot_c[op.slot], W + op.mmean, W + op.mvar, nullptr, nullptr,
                            E.side_for(op.slot)};
          sync_finalize(ctx, E, &sg, 1, ti.c, false, s);
        } else if (E.fused_bn[i] && skip_timing('f')) {  // (timing diagnostics)
        } else if (E.fused_bn[i])
          launch_bn_finalize(E.spart + E.stat_region[op.in[0]] * E.sp_region,
                             E.scnt + E.stat_region[op.in[0]] * E.sc_region, E.stat_P[op.in[0]],
                             (long)ti.rows(), ti.c, mean, rstd,
                             W + op.gamma, E.slot_c[op.slot], W + op.mmean, W + op.mvar, kBnEps, s,
                             E.side_for(op.slot));
        else if (ctx->bn_mode == PHX_BN_SYNC) {
          launch_bn_stats_sums(x, (long)ti.rows(), ti.c, E.red, E.sync_sums, s, E.tbf(op.in[0]) != 0);
          const BnFinSeg sg{nullptr, nullptr, 0, (long)ti.rows(), mean, rstd, W + op.gamma, E.slot_c[op.slot],
                            W + op.mmean, W + op.mvar, nullptr, nullptr, E.side_for(op.slot)};
          sync_reduce_apply(ctx, E, &sg, 1, ti.c, false, s);
        }
        else
          launch_bn_stats(x, (long)ti.rows(), ti.c, E.red, mean, rstd, W + op.gamma,
                          E.slot_c[op.slot], W + op.mmean, W + op.mvar, kBnEps, s, E.tbf(op.in[0]) != 0,
                          E.side_for(op.slot));
        (void)y;
        break;
      }
      case OP_SE:
        if (skip_timing('s')) break;
        launch_se_fwd(view(ctx, E, op.in[0], input), nullptr, ti.n, ti.h * ti.w, ti.c, op.cse, W + op.w1, W + op.b1, W + op.w2,
                      W + op.b2, op.act, E.slot_a[op.slot], E.slot_b[op.slot], E.slot_c[op.slot], s,
                      E.red);
        break;
      case OP_ADD: {
#if defined(PHX_DEBUG_KNOBS) && PHX_DEBUG_KNOBS
        static const bool no_drop = [] {  // PHX_NO_DROP=1: diagnostics only (not the reference's step)
          const char* e = std::getenv("PHX_NO_DROP");
          return e && e[0] == '1';
        }();
#else
        constexpr bool no_drop = false;
#endif
        const DropView dv = (train && !no_drop) ? drop_view(E, (int)i) : DropView{};
        if (E.ck_on) {  // what the add is about to read (PHX_CKSUM)
          const std::string nm = "p" + std::to_string(pass) + " f " + std::to_string(i) + " add in ";
          for (int k = 0; k < 2; ++k) {
            const Tensor& tk = P.tensors[op.in[k]];
            ck_note(E, nm + std::to_string(k), E.tptr(op.in[k], input), tk.numel() * (E.tbf(op.in[k]) ? 2 : 4), s);
          }
          if (dv.keep) ck_note(E, nm + "keep", dv.keep, (size_t)E.B * 4, s);
        }
        launch_add(view(ctx, E, op.in[0], input), view(ctx, E, op.in[1], input), y,
                   (long)to.numel(), to.c, s, dv);
        break;
      }
      case OP_MAXPOOL:
        launch_maxpool_fwd(view(ctx, E, op.in[0], input), y, E.pool_amax[i], ti.n, ti.h, ti.w, ti.c, to.h, to.w, op.k, op.stride, op.pad_t,
                           op.pad_l, s);
        break;
      case OP_UPSAMPLE:
        launch_upsample_fwd(view(ctx, E, op.in[0], input), y, ti.n, ti.h, ti.w, ti.c, to.h, to.w, s);
        break;
      case OP_FUSE: {
        InX xs[3] = {};
        for (int k = 0; k < op.nin; ++k) xs[k] = view(ctx, E, op.in[k], input);
        launch_fuse_fwd(xs, op.nin, op.wsm[0] >= 0 ? W + op.wsm[0] : nullptr,
                        op.wsm[1] >= 0 ? W + op.wsm[1] : nullptr,
                        op.wsm[2] >= 0 ? W + op.wsm[2] : nullptr, op.fuse_method, op.act, y,
                        (long)to.numel(), to.c, s);
        break;
      }
    }
    if (sink_on) {
      E.stat_P[op.out] = np;
      E.stat_region[op.out] = 0;
    }
    ck_fwd(E, (int)i, pass, s);
  }
  if (frozen) E.frozen_ver = ctx->w_ver;
}

bool is_cls_out(const Program& P, int t) {
  return std::find(P.cls_out.begin(), P.cls_out.end(), t) != P.cls_out.end();
}

// the fused backward of the sepconv whose depthwise op is i (its group's members when grouped): dx of
// the depthwise input from the pointwise output's gradient view, and the BN-backward sums of the BN
// the depthwise conv reads
void run_sep_bwd(phx_ctx* ctx, Exec& E, int i, const float* input, hipStream_t s) {
  const Program& P = E.prog;
  float* W = ctx->w();
  const int gd = E.grp_of[i];
  const std::vector<int> mem = gd >= 0 ? E.groups[gd] : std::vector<int>{i};
  const int n = (int)mem.size();
  const Op& d0 = P.ops[mem[0]];
  const Op& p0 = P.ops[mem[0] + 1];
  const int C = P.tensors[d0.in[0]].c, N = P.tensors[p0.out].c;
  const bool gs_on = mem[0] > 0 && E.gfused_bn[mem[0] - 1];
  SepBwdMember m[kMaxSeg];
  double fl = 0, by = 4.0 * (9.0 * C + (double)N * C);
  for (int r = 0; r < n; ++r) {
    const int di = mem[r];
    const Op& d = P.ops[di];
    const Op& pw = P.ops[di + 1];
    const Tensor& ti = P.tensors[d.in[0]];
    SepBwdMember& mm = m[r];
    mm = SepBwdMember{};
    mm.gv = gview(ctx, E, pw.out, input);
    mm.dx = E.gptr(d.in[0]);
    mm.H = ti.h;
    mm.W = ti.w;
    mm.acc = d.acc[0];
    if (gs_on) {
      const Op& bn = P.ops[di - 1];
      mm.gs = GradSink{E.spart + (size_t)(gd >= 0 ? r : 0) * E.sp_region, P.tensors[bn.out].c, 0, E.tptr(bn.in[0], input),
                       E.slot_a[bn.slot], E.slot_b[bn.slot], E.slot_c[bn.slot], W + bn.beta, bn.act, E.tbf(bn.in[0])};
    }
    fl += 2.0 * (double)ti.rows() * C * N + 2.0 * ti.numel() * 9.0;
    by += 4.0 * (3.0 * (double)ti.rows() * N + (d.acc[0] ? 2.0 : 1.0) * ti.numel() + (gs_on ? ti.numel() : 0.0));
  }
  Scope scope(ctx, "sep_bwd", fl, by, s,
              prof_detail() ? std::string(n > 1 ? " group" : "") + op_tag(P, p0, true) : std::string());
  int nps[kMaxSeg];
  launch_sep_bwd(m, n, E.B, C, N, W + d0.w, W + p0.w, s, nps);
  if (gs_on)
    for (int r = 0; r < n; ++r) {
      if (nps[r] != E.gstat_P[mem[r] - 1]) throw std::logic_error("sep bwd: planned and launched partial counts differ");
      E.gstat_region[mem[r] - 1] = gd >= 0 ? r : 0;
    }
}

// data-gradient of the victim from the sparse class-logit gradient (attacker.py:217)
void run_backward(phx_ctx* ctx, Exec& E, const float* input, hipStream_t s) {
  const Program& P = E.prog;
  float* W = ctx->w();
  const bool frozen = ctx->bn_mode == PHX_BN_FROZEN;
  const int na = ctx->mc.num_anchors();
  // 1. sparse class-head gradient into the inputs of the class-predict pointwise convs
  int K = 0;
  long wpred = -1;
  std::vector<std::pair<char*, size_t>> zero;  // the levels' gradient buffers, merged where adjacent
  for (int l = 0; l < (int)P.cls_out.size(); ++l) {
    for (const Op& op : P.ops) {
      if (op.out != P.cls_out[l]) continue;
      const Tensor& ti = P.tensors[op.in[0]];
      zero.emplace_back(reinterpret_cast<char*>(E.gptr(op.in[0])), ti.numel() * sizeof(float));
      K = ti.c;
      wpred = op.w;
    }
  }
  std::sort(zero.begin(), zero.end());
  std::vector<char*> zp;
  std::vector<size_t> zb;
  for (size_t i = 0; i < zero.size();) {
    char* p0 = zero[i].first;
    char* p1 = p0 + zero[i].second;
    size_t j = i + 1;
    for (; j < zero.size() && zero[j].first <= p1; ++j) p1 = std::max(p1, zero[j].first + zero[j].second);
    zp.push_back(p0);
    zb.push_back((size_t)(p1 - p0));
    i = j;
  }
  // one launch for all of them (was one memset packet per level)
  bool aligned = zp.size() <= (size_t)kZeroSegs;
  for (size_t k = 0; k < zp.size(); ++k) aligned = aligned && ((reinterpret_cast<uintptr_t>(zp[k]) | zb[k]) & 15) == 0;
  if (aligned) launch_zero_segs(zp.data(), zb.data(), (int)zp.size(), s);
  else
    for (size_t k = 0; k < zp.size(); ++k) PHX_HIP(hipMemsetAsync(zp[k], 0, zb[k], s));
  launch_cls_scatter(E.scores, E.keep, E.mraw, E.nties, E.dm, E.tptr(P.cls_out[0], input),
                     E.lev_dev, (int)E.lev.size(), ctx->A, E.B, ctx->mc.num_classes, na,
                     W + wpred, K, E.grad, E.dxoff_dev, s, E.tbf(P.cls_out[0]));
  // 2. reverse sweep
  for (int i = (int)P.ops.size() - 1; i >= 0; --i) {
    const Op& op = P.ops[i];
    if (!op.bwd) continue;
    if (op.t == OP_PW && is_cls_out(P, op.out)) continue;  // handled by the scatter
    if (i > 0 && E.sepb[i - 1]) continue;  // (the pointwise half of a fused sepconv: with its depthwise op)
    if (E.grp_of[i] >= 0) {
      if (E.groups[E.grp_of[i]].back() == i) {
        if (E.sepb[i]) run_sep_bwd(ctx, E, i, input, s);
        else run_group_bwd(ctx, E, E.grp_of[i], input, s);
        for (int m : E.groups[E.grp_of[i]]) ck_bwd(E, m, s);
      }
      continue;
    }
    if (E.sepb[i]) {
      run_sep_bwd(ctx, E, i, input, s);
      ck_bwd(E, i, s);
      continue;
    }
    const Tensor& ti = P.tensors[op.in[0]];
    const Tensor& to = P.tensors[op.out];
    const float* dy = E.gptr(op.out);
    float* dx = E.gptr(op.in[0]);
    double fl = 0, by = 4.0 * (double)(ti.numel() + to.numel());
    const char* kind = "bwd_other";
    switch (op.t) {
      case OP_STEM: kind = "stem_bwd"; fl = 2.0 * to.numel() * 27; break;
      case OP_PW: kind = "gemm"; fl = 2.0 * ti.rows() * ti.c * to.c; by += 4.0 * ti.c * to.c; break;
      case OP_DW: kind = "dw_bwd"; fl = 2.0 * to.numel() * op.k * op.k; break;
      case OP_BN: kind = "bn_bwd_reduce"; by = 4.0 * 2.0 * ti.numel(); break;
      case OP_SE: kind = "se_bwd"; by = 4.0 * 3.0 * ti.numel(); break;
      default: break;
    }
    // algorithmic bytes of a dgrad: a gradient view also reads the BN input; accumulation
    // re-reads the destination
    if (op.t == OP_PW || op.t == OP_DW) {
      const int bi = E.bn_consumer[op.out];
      if (bi >= 0 && P.ops[bi].bwd) by += 4.0 * (double)to.numel();
      if (op.acc[0]) by += 4.0 * (double)ti.numel();
    }
    // the BN right before this op takes its backward sums from this op's dgrad (GradSink)
    GradSink gsk{};
    int gsk_in = -1;  // which input's gradient carries them
    if (i > 0 && E.gfused_bn[i - 1]) {
      const Op& bn = P.ops[i - 1];
      gsk = GradSink{E.spart, P.tensors[bn.out].c, 0, E.tptr(bn.in[0], input), E.slot_a[bn.slot],
                     E.slot_b[bn.slot], E.slot_c[bn.slot], W + bn.beta, bn.act, E.tbf(bn.in[0])};
      gsk_in = op.in[0] == bn.out ? 0 : 1;
    }
    if (op.t == OP_BN && E.gfused_bn[i]) by = 8.0 * (double)E.gstat_P[i] * ti.c;
    if (skip_kind(std::string("b:") + kind, op.name)) continue;
    Scope scope(ctx, kind, fl, by, s, (prof_detail() || debug_sync()) ? op_tag(P, op, true) : std::string());
    int np = -1;
    switch (op.t) {
      case OP_STEM: {
        GradX g = gview(ctx, E, op.out, input);
        // the image gradient feeds only the EOT backward, which reads it at owned pixels
        if (!op.acc[0] && stem_bwd_gx_supported(to.c)) {
          launch_stem_bwd_gx(g, W + op.w, E.owner, dx, ti.n, ti.h, ti.w, to.h, to.w, to.c, op.pad_t,
                             op.pad_l, s);
          break;
        }
        // the stem dgrad reads each dy element up to 4x: materialise the BN-backward output once
        float* gy = E.gptr(op.out);
        if (g.y) launch_bn_bwd_apply2(g, gy, (long)to.rows(), to.c, s);
        launch_stem_bwd(g.y ? gy : g.da, W + op.w, dx, ti.n, ti.h, ti.w, to.h, to.w, to.c, op.pad_t, op.pad_l,
                        op.acc[0], s);
        break;
      }
      case OP_PW:
        // dX[M,Cin] = dY[M,Cout] * W^T : Bt = W in HWIO layout [Cin][Cout]
        np = launch_gemm_dgrad(gview(ctx, E, op.out, input), W + op.w, dx, (int)ti.rows(), ti.c, to.c,
                               op.acc[0], s, E.gpart, gsk, E.bf16);
        break;
      case OP_DW:
        np = launch_dw_bwd(gview(ctx, E, op.out, input), W + op.w, dx, ti.n, ti.h, ti.w, ti.c, to.h, to.w, op.k,
                           op.stride, op.pad_t, op.pad_l, op.acc[0], s, gsk);
        break;
      case OP_BN:
        // reduction only; the apply half runs in the producer's dgrad (gview)
        if (op.acc[0]) throw std::runtime_error("BN input with several consumers");
        if (!frozen && E.gfused_bn[i] && ctx->bn_mode == PHX_BN_SYNC) {
          const BnFinSeg sg{E.spart + E.gstat_region[i] * E.sp_region, nullptr, E.gstat_P[i], (long)ti.rows(),
                            nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, E.slot_d[op.slot], E.slot_e[op.slot]};
          sync_finalize(ctx, E, &sg, 1, ti.c, true, s);
        } else if (!frozen && E.gfused_bn[i] && skip_timing('b')) {  // (timing diagnostics)
        } else if (!frozen && E.gfused_bn[i])
          launch_bn_bwd_finalize(E.spart + E.gstat_region[i] * E.sp_region, E.gstat_P[i], (long)ti.rows(),
                                 ti.c, E.slot_d[op.slot],
                                 E.slot_e[op.slot], s);
        else if (!frozen && ctx->bn_mode == PHX_BN_SYNC) {
          launch_bn_bwd_reduce_sums(dy, E.tptr(op.in[0], input), E.slot_a[op.slot], E.slot_b[op.slot], W + op.gamma,
                                    W + op.beta, (long)ti.rows(), ti.c, op.act, E.red, E.sync_sums, s,
                                    E.tbf(op.in[0]) != 0);
          const BnFinSeg sg{nullptr, nullptr, 0, (long)ti.rows(), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                            E.slot_d[op.slot], E.slot_e[op.slot]};
          sync_reduce_apply(ctx, E, &sg, 1, ti.c, true, s);
        }
        else if (!frozen)
          launch_bn_bwd_reduce(dy, E.tptr(op.in[0], input), E.slot_a[op.slot], E.slot_b[op.slot],
                               W + op.gamma, W + op.beta, (long)ti.rows(), ti.c, op.act, E.red,
                               E.slot_d[op.slot], E.slot_e[op.slot], s, E.tbf(op.in[0]) != 0);
        (void)dx;
        break;
      case OP_SE:
        np = launch_se_bwd(dy, view(ctx, E, op.in[0], input), dx, ti.n, ti.h * ti.w, ti.c, op.cse, W + op.w1,
                           W + op.b1, ctx->wt_of(op.w2), W + op.b2, op.act, E.slot_a[op.slot],
                           E.slot_b[op.slot], E.slot_c[op.slot], E.se_g, op.acc[0], s, E.red, gsk);
        break;
      case OP_ADD: {
        // inputs whose gradient buffer aliases the output's (model.cpp: plan_backward) need no
        // copy, only the BN-backward sums when they are a BN output
        int n0 = 0, n1 = 0;
        if (dx == dy) {
          if (gsk_in == 0) n0 = launch_grad_sums(dy, (long)to.numel(), to.c, gsk, s);
        } else {
          n0 = launch_copy_grad(dy, dx, (long)to.numel(), op.acc[0], s, to.c,
                                gsk_in == 0 ? gsk : GradSink{}, drop_view(E, i));
        }
        if (E.gptr(op.in[1]) == dy) {
          if (gsk_in == 1) n1 = launch_grad_sums(dy, (long)to.numel(), to.c, gsk, s);
        } else {
          n1 = launch_copy_grad(dy, E.gptr(op.in[1]), (long)to.numel(), op.acc[1], s, to.c,
                                gsk_in == 1 ? gsk : GradSink{});
        }
        np = gsk_in == 0 ? n0 : n1;
        break;
      }
      case OP_MAXPOOL:
        launch_maxpool_bwd(E.pool_amax[i], dy, dx, ti.n, ti.h, ti.w, ti.c, to.h, to.w,
                           op.k, op.stride, op.pad_t, op.pad_l, op.acc[0], s);
        break;
      case OP_UPSAMPLE:
        launch_upsample_bwd(dy, dx, ti.n, ti.h, ti.w, ti.c, to.h, to.w, op.acc[0], s);
        break;
      case OP_FUSE: {
        InX xs[3] = {};
        float* dxs[3] = {nullptr, nullptr, nullptr};
        bool acc[3] = {false, false, false};
        for (int k = 0; k < op.nin; ++k) {
          xs[k] = view(ctx, E, op.in[k], input);
          dxs[k] = E.gptr(op.in[k]);
          acc[k] = op.acc[k];
        }
        launch_fuse_bwd(xs, op.nin, op.wsm[0] >= 0 ? W + op.wsm[0] : nullptr,
                        op.wsm[1] >= 0 ? W + op.wsm[1] : nullptr,
                        op.wsm[2] >= 0 ? W + op.wsm[2] : nullptr, op.fuse_method, op.act, dy, dxs,
                        acc, (long)to.numel(), to.c, s);
        break;
      }
    }
    if (gsk.part && np != E.gstat_P[i - 1])
      throw std::logic_error("BN backward sums: planned and launched partial counts differ");
    if (gsk.part) E.gstat_region[i - 1] = 0;
    ck_bwd(E, i, s);
  }
}

// cand_mask: the keep bits whose anchors (above the NMS threshold) pre_nms appends to the
// soft-NMS candidate list (2: the first pass's person/valid/>=thresh, 1: the second pass's
// person/valid for the ASR metric, 0: no list); the run_nms that follows consumes it
// nms_t: the soft-NMS score threshold of the candidate list (< 0: the context's)
void run_pre_nms(phx_ctx* ctx, Exec& E, hipStream_t s, int cand_mask = 0, float nms_t = -1.f) {
  const Program& P = E.prog;
  Scope scope(ctx, "pre_nms", 0.0,
              (double)E.B * ctx->A * (ctx->mc.num_classes + 4 + 4 + 6) * 4.0, s);
  const float S = (float)ctx->mc.image_size;
  // every list starts empty: a step that failed between a pre_nms and its run_nms (which
  // normally resets the counts) must not leave stale candidates for the next soft-NMS
  if (cand_mask) PHX_HIP(hipMemsetAsync(E.cand_count, 0, (size_t)E.B * sizeof(int), s));
  launch_pre_nms(E.tptr(P.cls_out[0], nullptr), E.tptr(P.box_out[0], nullptr),
                 E.lev_dev, (int)E.lev.size(), reinterpret_cast<const float*>(ctx->d_anchors.get()),
                 ctx->A, E.B, ctx->mc.num_classes, ctx->mc.num_anchors(), S, S, ctx->filter_thresh,
                 E.scores, E.classes, E.boxes, E.keep, E.ntiles, s,
                 cand_mask ? NmsCand{E.cand_list, E.cand_count, cand_mask, nms_t < 0.f ? ctx->nms_thresh : nms_t}
                           : NmsCand{},
                 E.tbf(P.cls_out[0]) != 0);
}

// postprocess.nms with method 'gaussian': sigma 0.5 -> soft_nms_sigma 0.25
void run_nms(phx_ctx* ctx, Exec& E, int keep_mask, float* ob, float* os, int* oc, hipStream_t s,
             float nms_t = -1.f) {
  Scope scope(ctx, "soft_nms", 0.0, (double)E.B * ctx->A * 5.0, s);
  const float t = nms_t < 0.f ? ctx->nms_thresh : nms_t;
  launch_soft_nms(E.boxes, E.scores, E.keep, keep_mask, nullptr, E.B, ctx->A, t,
                  0.25f, PHX_MAX_OUT, (float)ctx->mc.image_size, ob, os, oc, E.nms_ws, s,
                  NmsCand{E.cand_list, E.cand_count, keep_mask, t});
}

// PHX_GUARD_BYTES: after a step, every executor allocation's guard band must still be 0xA5
void check_guards(phx_ctx* ctx, hipStream_t s) {
  PHX_HIP(hipStreamSynchronize(s));
  if (ctx->s1) PHX_HIP(hipStreamSynchronize(ctx->s1));
  const size_t gb = guard_bytes();
  std::vector<unsigned char> h(gb);
  for (auto& ep : ctx->execs) {
    for (size_t i = 0; i < ep->guards.size(); ++i) {
      const Guard& g = ep->guards[i];
      for (int side = 0; side < 2; ++side) {
        const char* band = side ? g.base + g.size : g.base - gb;
        PHX_HIP(hipMemcpy(h.data(), band, gb, hipMemcpyDeviceToHost));
        size_t first = gb, last = 0;
        for (size_t k = 0; k < gb; ++k)
          if (h[k] != 0xA5) {
            first = std::min(first, k);
            last = k;
          }
        if (first < gb) {
          if (side)
            fprintf(stderr, "phx guard: exec B=%d tag=%d allocation %zu (%zu bytes) overwritten at +%zu..+%zu past its end\n",
                    ep->B, ep->tag, i, g.size, first, last);
          else
            fprintf(stderr, "phx guard: exec B=%d tag=%d allocation %zu (%zu bytes) overwritten at -%zu..-%zu before its start\n",
                    ep->B, ep->tag, i, g.size, gb - last, gb - first);
          PHX_HIP(hipMemset(const_cast<char*>(band), 0xA5, gb));
        }
      }
    }
  }
}

}  // namespace

phx::ExtTiming*& phx::ext_timing() {
  static ExtTiming* t = nullptr;
  return t;
}

phx::ProfScope phx::prof_begin(phx_ctx* ctx, const char* kind, double flops, double bytes, hipStream_t s) {
  ProfScope r{nullptr, 0, s};
  if (!ctx || !ctx->prof.on) return r;
  Prof* p = &ctx->prof;
  Prof::Rec rec{kind, p->ev(), p->ev(), flops, bytes, 157.3};
  PHX_HIP(hipEventRecord(rec.a, s));
  p->recs.push_back(rec);
  r.p = p;
  r.idx = p->recs.size() - 1;
  return r;
}

void phx::prof_end(const ProfScope& r) {
  if (r.p) PHX_HIP(hipEventRecord(static_cast<Prof*>(r.p)->recs[r.idx].b, r.s));
}

int phx::ctx_image_size(const phx_ctx* ctx) { return ctx->mc.image_size; }
bool phx::ctx_profiling(const phx_ctx* ctx) { return ctx->prof.on; }
uint64_t phx::ctx_seed(const phx_ctx* ctx) { return ctx->seed; }
int phx::ctx_device(const phx_ctx* ctx) { return ctx->device; }
uint64_t phx::ctx_generation(const phx_ctx* ctx) {
  uint32_t f, n;
  std::memcpy(&f, &ctx->filter_thresh, 4);
  std::memcpy(&n, &ctx->nms_thresh, 4);
  return (ctx->w_ver * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)f << 32 | n);
}

void phx::def_first_pass(phx_ctx* ctx, const float* images, int B, int64_t step, int gimg0, float* boxes, int* count,
                    hipStream_t s, bool train, int pass, float score_thresh, float* scores) {
  if (!ctx->weights_loaded) throw std::logic_error("weights not loaded");
  if (B <= 0 || B > ctx->max_batch) throw std::out_of_range("batch exceeds max_batch");
  Exec& E = ctx->exec_for(B);
  // the protege's layers are frozen (inference BN); the call's training flag still reaches its
  // drop connect (attack_detection.py:46-47, 183)
  run_forward(ctx, E, images, s, pass, step, gimg0, train, true);
  // odet_model(images, score_thresh) (attack_detection.py:96-127): an explicit threshold replaces
  // the config's for the soft-NMS only ("score_thresh or 0.001", postprocess.py:186-188), while
  // filter_valid_boxes keeps reading self.config's (:79-94)
  const float nt = score_thresh < 0.f ? -1.f : (score_thresh != 0.f ? score_thresh : 0.001f);
  run_pre_nms(ctx, E, s, 4, nt);  // person anchors only (attack_detection.py:116-121)
  run_nms(ctx, E, 4, E.nms1_boxes, E.nms1_scores, E.nms1_count, s, nt);
  const float S = (float)ctx->mc.image_size;
  def_filter(E.nms1_boxes, E.nms1_scores, E.nms1_count, B, PHX_MAX_OUT, S, S, ctx->filter_thresh, boxes, count, s,
             scores);
}

namespace {
// run `fn(side)` on the executor's side stream after the work enqueued on `s` so far; join_side
// makes `s` wait for it
void check_ready(phx_ctx* ctx, int B) {
  if (!ctx->weights_loaded) throw std::logic_error("weights not loaded");
  if (B <= 0 || B > ctx->max_batch) throw std::out_of_range("batch exceeds max_batch");
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
#define PHX_TRY(ctx)                                                           \
  try {
#define PHX_CATCH(ctx)                                                         \
  }                                                                            \
  catch (const std::out_of_range& e) { return fail(ctx, PHX_ECAP, e.what()); } \
  catch (const std::invalid_argument& e) { return fail(ctx, PHX_EINVAL, e.what()); } \
  catch (const std::logic_error& e) { return fail(ctx, PHX_ESTATE, e.what()); } \
  catch (const HipError& e) { return fail(ctx, PHX_EHIP, e.what()); }          \
  catch (const std::exception& e) { return fail(ctx, PHX_EINVAL, e.what()); }

extern "C" {

int phx_abi_version(void) { return PHX_ABI_VERSION; }

int phx_create(const phx_config* cfg, int device, phx_ctx** out) {
  g_create_err.clear();
  if (!cfg || !out || !cfg->model_name) {
    g_create_err = "phx_create: null config, model name or output pointer";
    return PHX_EINVAL;
  }
  *out = nullptr;
  auto ctx = std::make_unique<phx_ctx>();
  try {
    if (!get_model_config(cfg->model_name, &ctx->mc)) {
      g_create_err = std::string("unknown model '") + cfg->model_name +
                     "' (efficientdet-d0..d7, efficientdet-lite0..lite4)";
      return PHX_EINVAL;
    }
    if (cfg->image_size < 0 || cfg->max_batch < 0) throw std::invalid_argument("negative image_size / max_batch");
    if (cfg->bn_mode != PHX_BN_LOCAL && cfg->bn_mode != PHX_BN_FROZEN && cfg->bn_mode != PHX_BN_SYNC)
      throw std::invalid_argument("unknown bn_mode");
    if (!(cfg->score_thresh >= 0.f && cfg->score_thresh <= 1.f)) throw std::invalid_argument("score_thresh outside [0, 1]");
    if (cfg->image_size > 0) ctx->mc.image_size = cfg->image_size;
    ctx->device = device;
    ctx->max_batch = cfg->max_batch > 0 ? cfg->max_batch : 1;
    ctx->bn_mode = cfg->bn_mode;
    if (cfg->compute_dtype != PHX_DTYPE_F32 && cfg->compute_dtype != PHX_DTYPE_BF16)
      throw std::invalid_argument("unknown compute_dtype");
    ctx->bf16 = cfg->compute_dtype == PHX_DTYPE_BF16;
    ctx->set_score_thresh(cfg->score_thresh);
    ctx->seed = cfg->seed;
    NetBuilder nb(ctx->mc, 0);
    nb.build();
    ctx->weights = nb.weights();
    ctx->wfloats = nb.weight_floats();
    std::ostringstream js;
    js << "[";
    for (size_t i = 0; i < ctx->weights.size(); ++i) {
      const WeightEntry& w = ctx->weights[i];
      js << (i ? "," : "") << "{\"name\":\"" << json_escape(w.name) << "\",\"shape\":[";
      for (size_t k = 0; k < w.shape.size(); ++k) js << (k ? "," : "") << w.shape[k];
      js << "],\"offset\":" << w.offset << ",\"kind\":\"" << w.kind << "\"}";
    }
    js << "]";
    ctx->manifest_json = js.str();
    // anchors
    int f = ctx->mc.image_size, a = 0;
    for (int l = 1; l <= ctx->mc.max_level; ++l) {
      f = (f - 1) / 2 + 1;
      if (l >= ctx->mc.min_level) a += f * f * ctx->mc.num_anchors();
    }
    ctx->A = a;
  } catch (const std::exception& e) {
    g_create_err = std::string("phx_create(") + cfg->model_name + "): " + e.what();
    return PHX_EINVAL;
  }
  *out = ctx.release();
  return PHX_OK;
}

int phx_set_allreduce(phx_ctx* ctx, phx_allreduce_fn fn, void* user) {
  if (!ctx) return PHX_EINVAL;
  ctx->ar_fn = fn;
  ctx->ar_user = user;
  return PHX_OK;
}

int phx_set_score_thresh(phx_ctx* ctx, float t) {
  if (!ctx) return PHX_EINVAL;
  if (!(t >= 0.f && t <= 1.f)) return fail(ctx, PHX_EINVAL, "score_thresh outside [0, 1]");
  PHX_TRY(ctx)
  ctx->pre_drop();
  ctx->set_score_thresh(t);
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_model_info(const phx_ctx* ctx, char* buf, size_t cap, size_t* needed) {
  if (!ctx) return PHX_EINVAL;
  const std::string js = ctx->model_info();
  if (needed) *needed = js.size() + 1;
  if (buf && cap > 0) {
    size_t c = std::min(cap - 1, js.size());
    memcpy(buf, js.data(), c);
    buf[c] = 0;
  }
  return PHX_OK;
}

void phx_destroy(phx_ctx* ctx) { delete ctx; }

const char* phx_last_error(const phx_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

int phx_weight_manifest(const phx_ctx* ctx, char* buf, size_t cap, size_t* needed) {
  if (!ctx) return PHX_EINVAL;
  size_t n = ctx->manifest_json.size() + 1;
  if (needed) *needed = n;
  if (buf && cap > 0) {
    size_t c = std::min(cap - 1, ctx->manifest_json.size());
    memcpy(buf, ctx->manifest_json.data(), c);
    buf[c] = 0;
  }
  return PHX_OK;
}

size_t phx_weight_count(const phx_ctx* ctx) { return ctx ? ctx->wfloats : 0; }
int phx_num_anchors(const phx_ctx* ctx) { return ctx ? ctx->A : 0; }
int phx_image_size(const phx_ctx* ctx) { return ctx ? ctx->mc.image_size : 0; }

int phx_workspace_bytes(phx_ctx* ctx, int B, size_t* bytes) {
  if (!ctx || !bytes || B <= 0) return PHX_EINVAL;
  if (B > ctx->max_batch) return fail(ctx, PHX_ECAP, "batch exceeds max_batch");
  PHX_TRY(ctx)
  PHX_HIP(hipSetDevice(ctx->device));
  size_t tot = ctx->exec_for(B).bytes;
  for (const auto& e : ctx->execs)  // + the concurrent first pass's executor, once a step made it
    if (e->B == B && e->tag != 0) tot += e->bytes;
  *bytes = tot;
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_load_weights(phx_ctx* ctx, const float* blob, size_t nfloats) {
  if (!ctx || !blob) return PHX_EINVAL;
  if (nfloats != ctx->wfloats) return fail(ctx, PHX_EINVAL, "weight blob size mismatch");
  PHX_TRY(ctx)
  PHX_HIP(hipSetDevice(ctx->device));
  ctx->pre_drop();
  if (!ctx->d_w) ctx->d_w.reset(dalloc<float>(ctx->wfloats));
  PHX_HIP(hipMemcpy(ctx->d_w.get(), blob, nfloats * sizeof(float), hipMemcpyHostToDevice));
  ++ctx->w_ver;
  // transposed copies of every 1x1 kernel: [Cout][Cin] for the forward GEMM
  std::vector<float> wt;
  ctx->wt_pairs.clear();
  for (const WeightEntry& w : ctx->weights) {
    if (w.kind != "kernel" || w.shape.size() != 4 || w.shape[0] != 1 || w.shape[1] != 1) continue;
    const int ci = w.shape[2], co = w.shape[3];
    ctx->wt_pairs.push_back({(long)w.offset, (long)wt.size()});
    size_t base = wt.size();
    wt.resize(base + (size_t)ci * co);
    for (int i = 0; i < ci; ++i)
      for (int o = 0; o < co; ++o) wt[base + (size_t)o * ci + i] = blob[w.offset + (size_t)i * co + o];
  }
  ctx->d_wt.reset(dalloc<float>(wt.size()));
  PHX_HIP(hipMemcpy(ctx->d_wt.get(), wt.data(), wt.size() * sizeof(float), hipMemcpyHostToDevice));
  if (!ctx->d_anchors) {
    std::vector<float> an = make_anchors(ctx->mc);
    if ((int)an.size() != ctx->A * 4) throw std::runtime_error("anchor generation mismatch");
    ctx->d_anchors.reset(dalloc<float>(an.size()));
    PHX_HIP(hipMemcpy(ctx->d_anchors.get(), an.data(), an.size() * sizeof(float),
                      hipMemcpyHostToDevice));
  }
  ctx->weights_loaded = true;
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_read_weights(phx_ctx* ctx, float* blob, size_t nfloats) {
  if (!ctx || !blob || nfloats != ctx->wfloats) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (!ctx->weights_loaded) throw std::logic_error("weights not loaded");
  PHX_HIP(hipDeviceSynchronize());
  PHX_HIP(hipMemcpy(blob, ctx->d_w.get(), nfloats * sizeof(float), hipMemcpyDeviceToHost));
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_detect(phx_ctx* ctx, const float* images, int B, float* scores, int32_t* classes,
               float* boxes, void* stream) {
  if (!ctx || !images) return PHX_EINVAL;
  PHX_TRY(ctx)
  check_ready(ctx, B);
  hipStream_t s = (hipStream_t)stream;
  Exec& E = ctx->exec_for(B);
  run_forward(ctx, E, images, s, 2, 0, 0);
  run_pre_nms(ctx, E, s);
  const long BA = (long)B * ctx->A;
  if (scores) PHX_HIP(hipMemcpyAsync(scores, E.scores, BA * 4, hipMemcpyDeviceToDevice, s));
  if (classes) PHX_HIP(hipMemcpyAsync(classes, E.classes, BA * 4, hipMemcpyDeviceToDevice, s));
  if (boxes) PHX_HIP(hipMemcpyAsync(boxes, E.boxes, BA * 16, hipMemcpyDeviceToDevice, s));
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_first_pass(phx_ctx* ctx, const float* images, int B, float* ob, float* os, int32_t* oc,
                   void* stream) {
  if (!ctx || !images || !ob || !os || !oc) return PHX_EINVAL;
  PHX_TRY(ctx)
  check_ready(ctx, B);
  hipStream_t s = (hipStream_t)stream;
  Exec& E = ctx->exec_for(B);
  run_forward(ctx, E, images, s, 0, 0, 0);
  run_pre_nms(ctx, E, s, 2);
  run_nms(ctx, E, 2, ob, os, oc, s);
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_soft_nms(phx_ctx* ctx, const float* boxes, const float* scores, const int32_t* count,
                 int B, int N, float* ob, float* os, int32_t* oc, void* stream) {
  if (!ctx || !boxes || !scores || B <= 0 || N <= 0) return PHX_EINVAL;
  PHX_TRY(ctx)
  hipStream_t s = (hipStream_t)stream;
  const size_t need = soft_nms_work_floats(B, N);
  if (need > ctx->sn_cap) {
    PHX_HIP(hipStreamSynchronize(s));
    ctx->sn_ws.reset(dalloc<float>(need));
    ctx->sn_cap = need;
  }
  launch_soft_nms(boxes, scores, nullptr, 0, count, B, N, ctx->nms_thresh, 0.25f, PHX_MAX_OUT,
                  (float)ctx->mc.image_size, ob, os, oc, (float*)ctx->sn_ws.get(), s);
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_brightness_match(phx_ctx* ctx, const float* src, int P, const float* tgt, int H, int W,
                         int B, float* out, void* stream) {
  if (!ctx || !src || !tgt || !out || B <= 0 || B > ctx->max_batch) return PHX_EINVAL;
  PHX_TRY(ctx)
  PHX_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  // its own small scratch (per-image Y partial sums + means), not an executor
  const size_t need = (size_t)B * 2 * 64 * sizeof(double) + (size_t)B * 2 * sizeof(float);
  if (need > ctx->bm_cap) {
    PHX_HIP(hipStreamSynchronize(s));
    ctx->bm_ws.reset(dalloc<char>(need));
    ctx->bm_cap = need;
  }
  double* ysum = reinterpret_cast<double*>(ctx->bm_ws.get());
  float* ymean = reinterpret_cast<float*>(ysum + (size_t)B * 2 * 64);
  EotDims d{};
  d.B = B;
  d.P = P;
  d.H = H;
  d.W = W;
  d.maxb = PHX_MAX_OUT;
  d.span_stride = std::max(H, W);
  launch_eot_match(d, src, nullptr, tgt, out, ysum, ymean, false, s);
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_letterbox(phx_ctx* ctx, const uint8_t* src, const int64_t* offsets, const int32_t* dims, int B,
                  const float* mean_rgb, const float* stddev_rgb, int out_h, int out_w, float* out,
                  void* stream) {
  if (!ctx) return PHX_EINVAL;
  if (!src || !offsets || !dims || !mean_rgb || !stddev_rgb || !out || B <= 0 || out_h <= 0 || out_w <= 0)
    return fail(ctx, PHX_EINVAL, "letterbox: null pointer or empty shape");
  PHX_TRY(ctx)
  PHX_HIP(hipSetDevice(ctx->device));
  launch_letterbox(src, offsets, dims, B, mean_rgb, stddev_rgb, out_h, out_w, out, (hipStream_t)stream);
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_augment(phx_ctx* ctx, const float* in, int B, int H, int W, int64_t step, int global_image_offset,
                float* out, void* stream) {
  if (!ctx) return PHX_EINVAL;
  if (!in || !out || B <= 0 || H <= 0 || W <= 0) return fail(ctx, PHX_EINVAL, "augment: null pointer or empty shape");
  if (in == out) return fail(ctx, PHX_EINVAL, "augment: in and out alias (the mirror reads other pixels)");
  PHX_TRY(ctx)
  PHX_HIP(hipSetDevice(ctx->device));
  const size_t need = augment_scratch_doubles(B) * sizeof(double);
  if (need > ctx->aug_cap) {  // first call for this batch size allocates (synchronous)
    ctx->aug_ws.reset(dalloc<char>(need));
    ctx->aug_cap = need;
  }
  launch_augment(in, out, B, H, W, ctx->seed, step, global_image_offset,
                 reinterpret_cast<double*>(ctx->aug_ws.get()), (hipStream_t)stream);
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_adv_patch(phx_ctx* ctx, uint8_t* images, int B, int H, int W, const float* boxes, const int32_t* count,
                  int max_boxes, const uint8_t* patch, int patch_size, double scale, int out_h, int out_w,
                  int64_t step, int global_image_offset, void* stream) {
  if (!ctx) return PHX_EINVAL;
  if (!images || !boxes || !count || !patch || B <= 0 || H <= 0 || W <= 0 || max_boxes < 0 || patch_size <= 0 ||
      out_h <= 0 || out_w <= 0)
    return fail(ctx, PHX_EINVAL, "adv_patch: null pointer or empty shape");
  PHX_TRY(ctx)
  PHX_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  const int P = patch_size;
  // placements (AdversarialPatch._create, adv_patch.py:60-91), in double as Python computes them
  int rounds = 0;
  std::vector<ApBox> tab;
  for (int b = 0; b < B; ++b) {
    if (count[b] < 0 || count[b] > max_boxes) throw std::invalid_argument("adv_patch: box count out of range");
    rounds = std::max(rounds, (int)count[b]);
  }
  tab.assign((size_t)std::max(rounds, 1) * B, ApBox{0, 0, 0, 0, 0});
  std::vector<int> round_pix(std::max(rounds, 1), 0);
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < count[b]; ++k) {
      const float* q = boxes + ((size_t)b * max_boxes + k) * 4;
      // float32 boxes (the detector's dtype) under numpy's promotion: h, w in float32, then float64
      const double ymin = q[0], xmin = q[1];
      const double h = (float)(q[2] - q[0]), w = (float)(q[3] - q[1]);
      const double long_side = std::max(h, w);
      const int pw = (int)(long_side * scale), ph = pw;
      if (ph < 1) throw std::invalid_argument("adv_patch: patch side below 1 pixel (cv2.resize to an empty size)");
      if (ph > H || pw > W) throw std::invalid_argument("adv_patch: patch larger than the image");
      double ymp = std::max((ymin + h / 2.0) - ph / 2.0, 0.0), xmp = std::max((xmin + w / 2.0) - pw / 2.0, 0.0);
      if (ymp + ph > H) ymp = H - ph;
      if (xmp + pw > W) xmp = W - pw;
      tab[(size_t)k * B + b] = ApBox{1, (int)ymp, (int)xmp, ph, pw};
      round_pix[k] = std::max(round_pix[k], ph * pw);
    }
  // the rescale of AdversarialPatch.rescale (adv_patch.py:93-108)
  const double sc = std::min((double)out_w / W, (double)out_h / H);
  const int sh = (int)(H * sc), sw = (int)(W * sc);
  if (sh < 1 || sw < 1) throw std::invalid_argument("adv_patch: the rescaled image is empty");
  const size_t need = (size_t)P * P * 3 + sizeof(unsigned long long) * (1 + (size_t)B) + sizeof(ApBox) * tab.size() + 64;
  if (need > ctx->ap_cap) {
    ctx->ap_ws.reset(dalloc<char>(need));
    ctx->ap_cap = need;
  }
  char* ws = static_cast<char*>(ctx->ap_ws.get());
  auto* ysum = reinterpret_cast<unsigned long long*>(ws);
  auto* ysrc = ysum + B;
  auto* dtab = reinterpret_cast<ApBox*>(ysrc + 1);
  uint8_t* printed = reinterpret_cast<uint8_t*>(dtab + tab.size());
  PHX_HIP(hipMemcpyAsync(dtab, tab.data(), sizeof(ApBox) * tab.size(), hipMemcpyHostToDevice, s));
  launch_ap_print(patch, printed, P, ysrc, s);
  for (int k = 0; k < rounds; ++k) {
    launch_ap_ysum(images, B, H, W, out_h, out_w, sh, sw, ysum, s);
    launch_ap_paste(images, B, H, W, printed, P, dtab + (size_t)k * B, round_pix[k], k, ysum, ysrc, out_h, out_w,
                    ctx->seed, step, global_image_offset, s);
  }
  // the host table must outlive its (pageable, staged) copy
  PHX_HIP(hipStreamSynchronize(s));
  return PHX_OK;
  PHX_CATCH(ctx)
}

namespace {
void eot_forward(phx_ctx* ctx, Exec& E, const float* images, int B, const float* boxes,
                 const int32_t* count, const float* params, int64_t step, int gimg0,
                 hipStream_t s) {
  EotDims d = E.ed;
  d.B = B;
  Scope scope(ctx, "eot_fwd", 0.0, (double)B * (2.0 * PHX_NPATCH + 3.0 * d.H * d.W * 3) * 4.0, s);
  launch_eot_place(d, boxes, count, params, ctx->seed, step, gimg0, E.img, E.place, E.spans, E.err,
                   s);
  launch_eot_match(d, params, E.img, images, E.matched, E.ysum, E.ymean, true, s);
  launch_eot_resize(d, E.matched, E.place, E.spans, ctx->seed, step, gimg0, E.rstore, s);
  launch_eot_composite(d, images, E.place, E.rstore, E.patched, E.owner, s);
}

// copy caller boxes [B,maxb,4] into the [B,100,4] slot layout of the injected-box buffers
void stage_boxes(Exec& E, const float* boxes, const int32_t* count, int B, int maxb,
                 hipStream_t s) {
  if (maxb > PHX_MAX_OUT) throw std::out_of_range("maxb > 100");
  if (maxb < PHX_MAX_OUT) PHX_HIP(hipMemsetAsync(E.inj_boxes, 0, (size_t)B * PHX_MAX_OUT * 16, s));
  PHX_HIP(hipMemcpy2DAsync(E.inj_boxes, PHX_MAX_OUT * 16, boxes, (size_t)maxb * 16,
                           (size_t)maxb * 16, B, hipMemcpyDeviceToDevice, s));
  PHX_HIP(hipMemcpyAsync(E.inj_count, count, B * sizeof(int), hipMemcpyDeviceToDevice, s));
}

}  // namespace

int phx_patch_images(phx_ctx* ctx, const float* images, int B, const float* boxes,
                     const int32_t* count, int maxb, const float* params, int64_t step,
                     int gimg0, float* out_images, float* placements, void* stream) {
  if (!ctx || !images || !boxes || !count || !params || !out_images) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (B <= 0 || B > ctx->max_batch) throw std::out_of_range("batch exceeds max_batch");
  hipStream_t s = (hipStream_t)stream;
  Exec& E = ctx->exec_for(B);
  ctx->last = &E;
  stage_boxes(E, boxes, count, B, maxb, s);
  eot_forward(ctx, E, images, B, E.inj_boxes, E.inj_count, params, step, gimg0, s);
  const int S = ctx->mc.image_size;
  PHX_HIP(hipMemcpyAsync(out_images, E.patched, (size_t)B * S * S * 12, hipMemcpyDeviceToDevice, s));
  if (placements) {
    std::vector<BoxPlace> hp((size_t)B * PHX_MAX_OUT);
    PHX_HIP(hipStreamSynchronize(s));
    PHX_HIP(hipMemcpy(hp.data(), E.place, hp.size() * sizeof(BoxPlace), hipMemcpyDeviceToHost));
    std::vector<float> pl((size_t)B * maxb * 8, 0.f);
    for (int b = 0; b < B; ++b)
      for (int k = 0; k < maxb; ++k) {
        const BoxPlace& P = hp[(size_t)b * PHX_MAX_OUT + k];
        float* o = &pl[((size_t)b * maxb + k) * 8];
        o[0] = (float)P.ymin; o[1] = (float)P.xmin; o[2] = (float)P.ps; o[3] = (float)P.diag;
        o[4] = P.angle; o[5] = P.delta; o[6] = (float)P.valid; o[7] = 0.f;
      }
    PHX_HIP(hipMemcpy(placements, pl.data(), pl.size() * 4, hipMemcpyHostToDevice));
  }
  return PHX_OK;
  PHX_CATCH(ctx)
}

// the concurrent first pass of phx_step_grad (on unless PHX_CONC=0; read per call so a test can
// compare both orders in one process)
static bool concurrent_first_pass() {
  const char* e = std::getenv("PHX_CONC");
  return !(e && e[0] == '0');
}

// the cross-step first-pass prefetch runs where a second stream is allowed: bn=local (bn=sync issues
// collectives that every rank must order alike; bn=frozen has no deferred statistics to carry), not
// in a profiled step (one stream), not under the checksum / guard diagnostics, not with PHX_CONC=0
static bool prefetch_ok(phx_ctx* ctx, const Exec& E) {
  return ctx->s2 && concurrent_first_pass() && ctx->bn_mode == PHX_BN_LOCAL && !ctx->prof.on && !E.ck_on &&
         !guard_bytes();
}

int phx_set_next(phx_ctx* ctx, const float* next_images, int B, int32_t global_image_offset) {
  if (!ctx) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (next_images) check_ready(ctx, B);
  PHX_HIP(hipSetDevice(ctx->device));
  if (next_images && !ctx->s2) {
    PHX_HIP(hipStreamCreateWithFlags(&ctx->s2, hipStreamNonBlocking));
    PHX_HIP(hipEventCreateWithFlags(&ctx->ev_pfork, hipEventDisableTiming));
    PHX_HIP(hipEventCreateWithFlags(&ctx->ev_pdone, hipEventDisableTiming));
  }
  ctx->next = next_images ? phx_ctx::Next{next_images, B, global_image_offset} : phx_ctx::Next{};
  // NULL also withdraws a first pass already prefetched for the next step (the caller refilled that
  // batch's buffer in place: the prefetch saw the old contents); the step then runs its own
  if (!next_images) ctx->pre_drop();
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_sync(phx_ctx* ctx, void* stream) {
  if (!ctx) return PHX_EINVAL;
  PHX_TRY(ctx)
  ctx->pre_join((hipStream_t)stream);
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_step_grad(phx_ctx* ctx, const float* images, int B, const float* boxes,
                  const int32_t* count, int maxb, const float* params, int64_t step, int gimg0,
                  int add_tv, float* grad, float* metrics, void* stream) {
  if (!ctx || !images || !params || !grad || !metrics) return PHX_EINVAL;
  PHX_TRY(ctx)
  check_ready(ctx, B);
  hipStream_t s = (hipStream_t)stream;
  Exec& E = ctx->exec_for(B);
  ctx->last = &E;
  const bool inject = boxes != nullptr;
  // a first pass the previous step prefetched for exactly this batch (phx_set_next)
  const bool use_pre = !inject && ctx->pre.pending && ctx->pre.images == images && ctx->pre.B == B &&
                       ctx->pre.step == step && ctx->pre.gimg0 == gimg0;
  ctx->pre_join(s);
  ctx->pre.pending = false;
  if (inject && !count) throw std::invalid_argument("boxes without count");
  if (inject && maxb > PHX_MAX_OUT) throw std::out_of_range("maxb > 100");
  // the metric row zeroed and the caller's boxes staged in one launch (16-B aligned boxes)
  const bool inject_k = inject && (reinterpret_cast<uintptr_t>(boxes) & 15) == 0;
  launch_step_prologue(metrics, PHX_NMETRIC, inject_k ? boxes : nullptr, count, B, maxb, E.inj_boxes,
                       E.inj_count, s);
  ck_begin(E, s);
  // Injected placement: the first pass only feeds the ASR denominator (and the moving statistics),
  // so it runs on a second stream beside the second pass and the backward, on its own executor
  // (its own activation arena).  Both passes defer their moving-statistics updates, applied in
  // pass order after the join, so every result equals the one-stream order bit for bit.  Not with
  // bn=sync: every rank must issue its collectives in one order.  PHX_CONC=0 turns it off.
  Exec* E1p = nullptr;
  if (concurrent_first_pass() && ctx->bn_mode != PHX_BN_SYNC && !ctx->s1) {
    PHX_HIP(hipStreamCreateWithFlags(&ctx->s1, hipStreamNonBlocking));
    PHX_HIP(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    PHX_HIP(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
  }
  // (a profiled step runs on one stream: its per-launch-group events time each kernel alone)
  if (inject && concurrent_first_pass() && ctx->bn_mode == PHX_BN_LOCAL && !ctx->prof.on) {
    E1p = &ctx->exec_for(B, 1);
    ctx->last = &E;
  }
  const bool fork = E1p != nullptr;
  // (an error part-way leaves neither executor deferring)
  struct DeferReset {
    phx_ctx* c;
    Exec *a, *b;
    ~DeferReset() {
      c->fwd_hook = nullptr;  // never left armed (it refers to this call's frame)
      a->defer_mov = false;
      if (b) b->defer_mov = false;
    }
  } defer_reset{ctx, &E, E1p};
  // Where the side stream starts: when the second pass's forward reaches the backbone's stage 6
  // (the first op at 1/32 of the image side), so the first pass's HBM-bound early layers run beside
  // the second pass's latency-bound deep layers, BiFPN and heads rather than beside its own early
  // layers (C2 12.06 -> 11.89 ms).  PHX_FORK_FRAC: 0 = at the step start, 0 < f < 1 = after that
  // fraction of the ops (experiments).
  static const double fork_frac = [] {
    const char* e = std::getenv("PHX_FORK_FRAC");
    return e ? atof(e) : -1.0;
  }();
  auto side = [&]() {
    Exec& E1 = *E1p;
    hipStream_t s1 = ctx->s1;
    E1.defer_mov = true;
    PHX_HIP(hipEventRecord(ctx->ev_fork, s));
    PHX_HIP(hipStreamWaitEvent(s1, ctx->ev_fork, 0));
    ck_begin(E1, s1);
    run_forward(ctx, E1, images, s1, 0, step, gimg0);
    E1.defer_mov = false;
    run_pre_nms(ctx, E1, s1, 2);
    ck_note(E1, "p0 scores", E1.scores, (size_t)B * ctx->A * 4, s1);
    run_nms(ctx, E1, 2, E1.nms1_boxes, E1.nms1_scores, E1.nms1_count, s1);
    launch_count_ge(E1.nms1_scores, E1.nms1_count, B, PHX_MAX_OUT, 0.5f, metrics + PHX_M_ASR_DEN, s1);
    PHX_HIP(hipEventRecord(ctx->ev_join, s1));
  };
  if (fork) {
    E.defer_mov = true;
    if (fork_frac == 0.0) {
      side();
    } else {
      ctx->fwd_hook = side;
      if (fork_frac > 0.0) {
        ctx->fwd_hook_at = (size_t)(fork_frac * (double)E.prog.ops.size());
      } else {
        // the first op at 1/32 of the image side (the backbone's stage 6)
        ctx->fwd_hook_at = E.prog.ops.size();
        for (size_t i = 0; i < E.prog.ops.size(); ++i)
          if (E.prog.tensors[E.prog.ops[i].out].h * 32 <= ctx->mc.image_size) {
            ctx->fwd_hook_at = i;
            break;
          }
      }
    }
  }
  Exec* Efp = &E;  // the executor whose first-pass detections place the patches
  if (!fork && use_pre) {
    // 1'. the prefetched first pass (side executor): its moving-statistics updates, deferred, go in
    // now — after the previous step's second pass, before this step's — and its ASR denominator
    Efp = &ctx->exec_for(B, 1);
    ctx->last = &E;
    launch_bn_moving_apply(E.mov_tab, E.n_mov, E.mov_cmax, ctx->w(), Efp->side, nullptr, s);
    launch_count_ge(Efp->nms1_scores, Efp->nms1_count, B, PHX_MAX_OUT, 0.5f, metrics + PHX_M_ASR_DEN, s);
  } else if (!fork) {
    // 1. first pass: clean forward, pre_nms, person/valid/threshold filter, soft-NMS
    run_forward(ctx, E, images, s, 0, step, gimg0);
    run_pre_nms(ctx, E, s, 2);
    run_nms(ctx, E, 2, E.nms1_boxes, E.nms1_scores, E.nms1_count, s);
    launch_count_ge(E.nms1_scores, E.nms1_count, B, PHX_MAX_OUT, 0.5f, metrics + PHX_M_ASR_DEN, s);
  }
  if (inject && !inject_k) stage_boxes(E, boxes, count, B, maxb, s);  // (unaligned caller boxes)
  // 2. EOT paste
  eot_forward(ctx, E, images, B, inject ? E.inj_boxes : Efp->nms1_boxes,
              inject ? E.inj_count : Efp->nms1_count, params, step, gimg0, s);
  launch_eot_count(E.ed, E.place, metrics, s);
  // the next batch's first pass (phx_set_next) on s2 beside this step's second pass and backward:
  // it starts once this step's own first pass and paste are done with the side executor's
  // detections, and defers its moving-statistics updates to the step that uses it
  // (consumed by this call either way: a step with caller boxes drops it)
  const phx_ctx::Next nx = ctx->next;
  ctx->next = phx_ctx::Next{};
  auto prefetch = [&]() {
      Exec& E1 = ctx->exec_for(B, 1);
      ctx->last = &E;
      PHX_HIP(hipEventRecord(ctx->ev_pfork, s));
      PHX_HIP(hipStreamWaitEvent(ctx->s2, ctx->ev_pfork, 0));
      struct Defer {
        Exec& e;
        ~Defer() { e.defer_mov = false; }
      } defer{E1};
      try {
        E1.defer_mov = true;
        run_forward(ctx, E1, nx.images, ctx->s2, 0, step + 1, nx.gimg0);
        E1.defer_mov = false;
        run_pre_nms(ctx, E1, ctx->s2, 2);
        run_nms(ctx, E1, 2, E1.nms1_boxes, E1.nms1_scores, E1.nms1_count, ctx->s2);
        PHX_HIP(hipEventRecord(ctx->ev_pdone, ctx->s2));
      } catch (...) {
        // a part-way enqueued prefetch: drain it (its side executor is shared with the injected flow's
        // concurrent pass on s1) and leave nothing pending
        (void)hipStreamSynchronize(ctx->s2);
        ctx->pre = phx_ctx::Pre{};
        throw;
      }
      ctx->pre = phx_ctx::Pre{nx.images, B, nx.gimg0, step + 1, true};
  };
  if (!inject && nx.images && nx.B == B && prefetch_ok(ctx, E)) {
    // forked, like the injected flow's concurrent pass, when the second pass reaches the backbone's
    // stage 6, so its HBM-bound early layers run beside the second pass's deep layers and the
    // backward rather than beside the second pass's own early layers (PHX_PF_FORK=0: right here)
    const char* pe = std::getenv("PHX_PF_FORK");
    if (pe && pe[0] == '0') {
      prefetch();
    } else {
      ctx->fwd_hook = prefetch;
      ctx->fwd_hook_at = E.prog.ops.size();
      for (size_t i = 0; i < E.prog.ops.size(); ++i)
        if (E.prog.tensors[E.prog.ops[i].out].h * 32 <= ctx->mc.image_size) {
          ctx->fwd_hook_at = i;
          break;
        }
    }
  }
  ck_note(E, "eot patched", E.patched, (size_t)B * ctx->mc.image_size * ctx->mc.image_size * 12, s);
  // 3. second pass + loss
  run_forward(ctx, E, E.patched, s, 1, step, gimg0);
  if (ctx->fwd_hook) {
    auto h = std::move(ctx->fwd_hook);
    ctx->fwd_hook = nullptr;
    h();
  }
  E.defer_mov = false;
  run_pre_nms(ctx, E, s, 1);
  ck_note(E, "p1 scores", E.scores, (size_t)B * ctx->A * 4, s);
  ck_note(E, "p1 keep", E.keep, (size_t)B * ctx->A, s);
  // 5. ASR metric: soft-NMS over second-pass person boxes (attacker.py:203-205).  It reads the
  // pre_nms outputs only (the backward reads them too, nothing writes them until the next step),
  // so it runs on the side stream beside the backward and joins at the end of the step
  const bool side_nms = ctx->s1 != nullptr && concurrent_first_pass() && ctx->bn_mode != PHX_BN_SYNC && !ctx->prof.on;
  if (side_nms) {
    PHX_HIP(hipEventRecord(ctx->ev_fork, s));
    PHX_HIP(hipStreamWaitEvent(ctx->s1, ctx->ev_fork, 0));
    run_nms(ctx, E, 1, E.nms2_boxes, E.nms2_scores, E.nms2_count, ctx->s1);
    launch_count_ge(E.nms2_scores, E.nms2_count, B, PHX_MAX_OUT, 0.5f, metrics + PHX_M_ASR_NUM, ctx->s1);
    PHX_HIP(hipEventRecord(ctx->ev_join, ctx->s1));
  }
  launch_image_max(E.scores, E.keep, B, ctx->A, E.mraw, E.argm, E.nties, E.imax_scratch, s);
  launch_loss(E.mraw, B, params, E.dm, grad + PHX_NPATCH, metrics, s);
  ck_note(E, "image max", E.mraw, (size_t)B * 4, s);
  // 4. victim data-gradient -> d(patched images)
  run_backward(ctx, E, E.patched, s);
  if (!side_nms) {
    run_nms(ctx, E, 1, E.nms2_boxes, E.nms2_scores, E.nms2_count, s);
    launch_count_ge(E.nms2_scores, E.nms2_count, B, PHX_MAX_OUT, 0.5f, metrics + PHX_M_ASR_NUM, s);
  }
  // 6. EOT backward -> d patch (+ TV)
  EotDims d = E.ed;
  d.B = B;
  const float* dimg = E.gptr(E.prog.input);
  Scope scope(ctx, "eot_bwd", 0.0, (double)B * (3.0 * PHX_NPATCH + 2.0 * d.H * d.W * 3) * 4.0, s);
  launch_eot_rot_bwd(d, dimg, E.owner, E.place, E.rstore, E.dstore, s);
  launch_eot_resize_bwd(d, E.place, E.spans, E.dstore, E.rstore, E.dmatched, s);
  launch_eot_patch_bwd(d, params, E.img, E.ymean, E.dmatched, E.dsum, grad, add_tv != 0, s);
  launch_tv(params, PHX_PATCH_SIZE, E.tvs, metrics, add_tv != 0, s);
  ck_note(E, "grad", grad, (size_t)(PHX_NPATCH + 1) * 4, s);
  if (fork || side_nms) PHX_HIP(hipStreamWaitEvent(s, ctx->ev_join, 0));
  if (fork) launch_bn_moving_apply(E.mov_tab, E.n_mov, E.mov_cmax, ctx->w(), E1p->side, E.side, s);
  if (E.ck_on) {
    // every forward tensor once more after the join: a tensor whose hash changed after its producer
    // was overwritten later in the step (PHX_CKSUM)
    ck_post(E, 1, s);
    if (fork) ck_post(*E1p, 0, s);
  }
  if (guard_bytes()) check_guards(ctx, s);
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_eval_step(phx_ctx* ctx, const float* images, int B, const float* boxes, const int32_t* count,
                  int maxb, const float* params, int64_t step, int gimg0, int add_tv, float* metrics,
                  float* out_boxes, float* out_scores, int32_t* out_count, void* stream) {
  if (!ctx || !images || !params || !metrics) return PHX_EINVAL;
  PHX_TRY(ctx)
  check_ready(ctx, B);
  hipStream_t s = (hipStream_t)stream;
  Exec& E = ctx->exec_for(B);
  ctx->last = &E;
  PHX_HIP(hipMemsetAsync(metrics, 0, PHX_NMETRIC * sizeof(float), s));
  run_forward(ctx, E, images, s, 0, step, gimg0, false);
  run_pre_nms(ctx, E, s, 2);
  run_nms(ctx, E, 2, E.nms1_boxes, E.nms1_scores, E.nms1_count, s);
  launch_count_ge(E.nms1_scores, E.nms1_count, B, PHX_MAX_OUT, 0.5f, metrics + PHX_M_ASR_DEN, s);
  const bool inject = boxes != nullptr;
  if (inject) {
    if (!count) throw std::invalid_argument("boxes without count");
    stage_boxes(E, boxes, count, B, maxb, s);
  }
  eot_forward(ctx, E, images, B, inject ? E.inj_boxes : E.nms1_boxes, inject ? E.inj_count : E.nms1_count,
              params, step, gimg0, s);
  launch_eot_count(E.ed, E.place, metrics, s);
  run_forward(ctx, E, E.patched, s, 1, step, gimg0, false);
  run_pre_nms(ctx, E, s, 1);
  launch_image_max(E.scores, E.keep, B, ctx->A, E.mraw, E.argm, E.nties, E.imax_scratch, s);
  launch_loss(E.mraw, B, params, E.dm, E.dscale_scratch, metrics, s);
  run_nms(ctx, E, 1, E.nms2_boxes, E.nms2_scores, E.nms2_count, s);
  launch_count_ge(E.nms2_scores, E.nms2_count, B, PHX_MAX_OUT, 0.5f, metrics + PHX_M_ASR_NUM, s);
  launch_tv(params, PHX_PATCH_SIZE, E.tvs, metrics, add_tv != 0, s);
  if (out_boxes) PHX_HIP(hipMemcpyAsync(out_boxes, E.nms2_boxes, (size_t)B * PHX_MAX_OUT * 16, hipMemcpyDeviceToDevice, s));
  if (out_scores) PHX_HIP(hipMemcpyAsync(out_scores, E.nms2_scores, (size_t)B * PHX_MAX_OUT * 4, hipMemcpyDeviceToDevice, s));
  if (out_count) PHX_HIP(hipMemcpyAsync(out_count, E.nms2_count, (size_t)B * 4, hipMemcpyDeviceToDevice, s));
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_profile(phx_ctx* ctx, int enable) {
  if (!ctx) return PHX_EINVAL;
  ctx->prof.on = enable != 0;
  ctx->prof.recs.clear();
  ctx->prof.used = 0;
  return PHX_OK;
}

int phx_profile_report(phx_ctx* ctx, char* buf, size_t cap, size_t* needed) {
  if (!ctx) return PHX_EINVAL;
  PHX_TRY(ctx)
  // the copy call after a size query returns the string that query measured (rebuilding it could
  // print a timing differently and no longer fit the caller's buffer)
  if (buf && cap && !ctx->prof.report.empty()) {
    const std::string out = std::move(ctx->prof.report);
    ctx->prof.report.clear();
    if (needed) *needed = out.size() + 1;
    const size_t c = std::min(cap - 1, out.size());
    memcpy(buf, out.data(), c);
    buf[c] = 0;
    return PHX_OK;
  }
  // per launch group: measured time and the roofline time of its algorithmic work at the MI355X
  // peaks (HBM 8 TB/s; fp32 MFMA 157.3 TFLOP/s, bf16 2.5 PFLOP/s for bf16 GEMMs); roof = sum over
  // launches of max(hbm, mfma)
  struct Agg { long n = 0; double ms = 0, flops = 0, bytes = 0, hbm_ms = 0, mfma_ms = 0, roof_ms = 0; };
  std::map<std::string, Agg> agg;
  for (auto& r : ctx->prof.recs) {
    PHX_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    PHX_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    Agg& a = agg[r.kind];
    a.n++;
    a.ms += ms;
    a.flops += r.flops;
    a.bytes += r.bytes;
    const double th = r.bytes / 8.0e12 * 1e3, tm = r.flops / (r.peak_tflops * 1e12) * 1e3;
    a.hbm_ms += th;
    a.mfma_ms += tm;
    a.roof_ms += std::max(th, tm);
  }
  std::ostringstream js;
  js << "{";
  bool first = true;
  for (auto& kv : agg) {
    js << (first ? "" : ",") << "\"" << kv.first << "\":{\"count\":" << kv.second.n
       << ",\"ms\":" << kv.second.ms << ",\"flops\":" << kv.second.flops
       << ",\"bytes\":" << kv.second.bytes << ",\"hbm_ms\":" << kv.second.hbm_ms
       << ",\"mfma_ms\":" << kv.second.mfma_ms << ",\"roof_ms\":" << kv.second.roof_ms << "}";
    first = false;
  }
  js << "}";
  std::string out = js.str();
  if (needed) *needed = out.size() + 1;
  if (!buf) ctx->prof.report = out;
  if (buf && cap) {
    size_t c = std::min(cap - 1, out.size());
    memcpy(buf, out.data(), c);
    buf[c] = 0;
  }
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_adam_clip(phx_ctx* ctx, float* params, const float* grad, float* m, float* v, float lr,
                  int64_t t, void* stream) {
  if (!params || !grad || !m || !v || t < 1) return PHX_EINVAL;
  PHX_TRY(ctx)
  launch_adam_clip(params, grad, m, v, PHX_NPARAM, lr, t, (hipStream_t)stream);
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_debug_last_patched(phx_ctx* ctx, float* out, void* stream) {
  if (!ctx || !out || ctx->execs.empty()) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (!ctx->last) throw std::logic_error("no step has run");
  Exec& E = *ctx->last;
  const int S = ctx->mc.image_size;
  PHX_HIP(hipMemcpyAsync(out, E.patched, (size_t)E.B * S * S * 12, hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_debug_last_image_grad(phx_ctx* ctx, float* out, void* stream) {
  if (!ctx || !out || ctx->execs.empty()) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (!ctx->last) throw std::logic_error("no step has run");
  Exec& E = *ctx->last;
  const int S = ctx->mc.image_size;
  PHX_HIP(hipMemcpyAsync(out, E.gptr(E.prog.input), (size_t)E.B * S * S * 12, hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_debug_tap(phx_ctx* ctx, const char* op_name, int which, float* out, size_t nfloats, void* stream) {
  if (!ctx || !op_name || !out || ctx->execs.empty()) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (!ctx->last) throw std::logic_error("no step has run");
  Exec& E = *ctx->last;
  for (size_t i = 0; i < E.prog.ops.size(); ++i) {
    const Op& op = E.prog.ops[i];
    if (op.name != op_name) continue;
    const int t = (op.t == OP_BN && which == 0) ? op.in[0] : op.out;
    if (nfloats != E.prog.tensors[t].numel())
      throw std::invalid_argument("tap: size mismatch (the tensor has " + std::to_string(E.prog.tensors[t].numel()) +
                                  " elements)");
    if (which == 0 && op.t == OP_FUSE && E.fuse_folded[i])
      throw std::invalid_argument("tap: this fuse is computed on load by its depthwise conv, never stored");
    if (which == 1 && op.t == OP_DW && E.sepb[i])
      throw std::invalid_argument("tap: this depthwise output's gradient is formed in LDS by the fused "
                                  "separable-conv backward, never stored (PHX_SEPB=0 keeps it)");
    if (which == 0 && op.t == OP_DW && E.sep[i])
      throw std::invalid_argument("tap: this depthwise output feeds the fused separable conv's registers only, "
                                  "never stored (PHX_SEP=0 at victim creation keeps it)");
    const float* src = which == 0 ? E.tptr(t, nullptr) : E.gptr(op.out);
    if (!src) throw std::invalid_argument("tap: no gradient for this tensor");
    if (which == 0 && E.tbf(t)) launch_bf16_to_f32(src, out, (long)nfloats, (hipStream_t)stream);
    else PHX_HIP(hipMemcpyAsync(out, src, nfloats * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return PHX_OK;
  }
  throw std::invalid_argument(std::string("tap: no op named ") + op_name);
  PHX_CATCH(ctx)
}

int phx_debug_tensor(phx_ctx* ctx, int tag, int op_index, int which, void* out, size_t nbytes, void* stream) {
  if (!ctx || !out || ctx->execs.empty()) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (!ctx->last) throw std::logic_error("no step has run");
  Exec* E = nullptr;
  for (auto& e : ctx->execs)
    if (e->B == ctx->last->B && e->tag == tag) E = e.get();
  if (!E) throw std::invalid_argument("tensor: no executor with this tag");
  if (op_index < 0 || op_index >= (int)E->prog.ops.size() || which < 0 || which > 2)
    throw std::invalid_argument("tensor: bad op index / which");
  const Op& op = E->prog.ops[op_index];
  const int t = which == 0 ? op.out : op.in[which - 1];
  if (t < 0 || t == E->prog.input) throw std::invalid_argument("tensor: no such arena tensor");
  const size_t nb = E->prog.tensors[t].numel() * (E->tbf(t) ? 2 : 4);
  if (nb != nbytes) throw std::invalid_argument("tensor: size mismatch (" + std::to_string(nb) + " bytes)");
  PHX_HIP(hipMemcpyAsync(out, E->tptr(t, nullptr), nb, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_debug_checksums(phx_ctx* ctx, int tag, char* buf, size_t cap, size_t* needed) {
  if (!ctx || ctx->execs.empty()) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (!ctx->last) throw std::logic_error("no step has run");
  Exec* E = nullptr;
  for (auto& e : ctx->execs)
    if (e->B == ctx->last->B && e->tag == tag) E = e.get();
  if (!E) throw std::invalid_argument("checksums: no executor with this tag");
  std::string out;
  if (E->ck && !E->ck_names.empty()) {
    PHX_HIP(hipDeviceSynchronize());
    std::vector<unsigned long long> h(E->ck_names.size());
    PHX_HIP(hipMemcpy(h.data(), E->ck, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    char v[32];
    for (size_t i = 0; i < h.size(); ++i) {
      snprintf(v, sizeof v, "%016llx", h[i]);
      out += E->ck_names[i] + "\t" + v + "\n";
    }
  }
  if (needed) *needed = out.size() + 1;
  if (buf && cap) {
    const size_t n = std::min(cap - 1, out.size());
    memcpy(buf, out.data(), n);
    buf[n] = 0;
  }
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_debug_last_detections(phx_ctx* ctx, float* scores, int32_t* classes, float* boxes, void* stream) {
  if (!ctx || ctx->execs.empty()) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (!ctx->last) throw std::logic_error("no step has run");
  Exec& E = *ctx->last;
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (size_t)E.B * ctx->A;
  if (scores) PHX_HIP(hipMemcpyAsync(scores, E.scores, n * 4, hipMemcpyDeviceToDevice, s));
  if (classes) PHX_HIP(hipMemcpyAsync(classes, E.classes, n * 4, hipMemcpyDeviceToDevice, s));
  if (boxes) PHX_HIP(hipMemcpyAsync(boxes, E.boxes, n * 16, hipMemcpyDeviceToDevice, s));
  return PHX_OK;
  PHX_CATCH(ctx)
}

int phx_debug_last_maxscores(phx_ctx* ctx, float* m, int32_t* anchor, void* stream) {
  if (!ctx || ctx->execs.empty()) return PHX_EINVAL;
  PHX_TRY(ctx)
  if (!ctx->last) throw std::logic_error("no step has run");
  Exec& E = *ctx->last;
  hipStream_t s = (hipStream_t)stream;
  if (m) PHX_HIP(hipMemcpyAsync(m, E.mraw, E.B * 4, hipMemcpyDeviceToDevice, s));
  if (anchor) PHX_HIP(hipMemcpyAsync(anchor, E.argm, E.B * 4, hipMemcpyDeviceToDevice, s));
  return PHX_OK;
  PHX_CATCH(ctx)
}

}  // extern "C"
