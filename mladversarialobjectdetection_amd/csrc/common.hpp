// common.hpp — shared device helpers for the phx HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace phx {

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define PHX_HIP(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      throw ::phx::HipError(std::string(#expr) + ": " + hipGetErrorString(e_) + " @" + \
                            __FILE__ + ":" + std::to_string(__LINE__));                \
  } while (0)

#define PHX_LAUNCH_CHECK() PHX_HIP(hipGetLastError())

constexpr int kWave = 64;

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ------------------------------------------------------------------------------------------
// activations (utils.py:36-53).  swish = x*sigmoid(x) (tf.nn.swish); relu6 grad passes on
// the open interval (0,6) (TF Relu6Grad).
// ------------------------------------------------------------------------------------------
// v_exp_f32 + v_rcp_f32 (1 ulp each): the IEEE divide sequence would cost ~10 instructions per
// element in every BN-view load
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}

__device__ __forceinline__ float act_fwd(float z, int act) {
  if (act == 1) return z * sigmoidf_(z);
  if (act == 2) return fminf(fmaxf(z, 0.0f), 6.0f);
  return z;
}
// d act / d z
__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == 1) {
    float s = sigmoidf_(z);
    return s * (1.0f + z * (1.0f - s));
  }
  if (act == 2) return (z > 0.0f && z < 6.0f) ? 1.0f : 0.0f;
  return 1.0f;
}

// ------------------------------------------------------------------------------------------
// bf16 (the C4 configuration's activation / matrix-core type): round-to-nearest-even packing by
// v_cvt_pk_bf16_f32, widening by a 16-bit shift.
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f4v_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint2 pack_bf16x4(float4 v) {
  const f4v_t w = {v.x, v.y, v.z, v.w};
  return __builtin_bit_cast(uint2, __builtin_convertvector(w, bf16x4_t));
}
__device__ __forceinline__ float4 unpack_bf16x4(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ float round_bf16(float f) {
  return __uint_as_float((uint32_t)__builtin_bit_cast(unsigned short, (__bf16)f) << 16);
}

// ------------------------------------------------------------------------------------------
// n / d for a drop-connect survival probability d in (2^-20, 1], correctly rounded as IEEE division
// (TF's `inputs / survival_prob`, utils.py:336-344), without v_div_scale / v_div_fmas.  hipcc lowers
// `/` to that sequence, whose v_div_fmas reads VCC; in the residual adds of a bf16 D4 step running
// beside the side stream's first pass it produced results scaled by 2^-64 for whole 16-lane groups
// (scripts/diag_add.py).  This is the same Newton sequence without the scaling and
// fix-up steps, which only act when |n| < 2^-103 or |n / d| nears the exponent limits: those (and
// 0, inf, nan) keep the plain division, so every result equals n / d bit for bit.
// PHX_DROP_HWDIV=1 (build flag) restores the plain division everywhere (A/B diagnostics).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float div_surv(float n, float d) {
#if defined(PHX_DROP_HWDIV) && PHX_DROP_HWDIV
  return n / d;
#else
  const float a = fabsf(n);
  if (!(a >= 0x1p-100f && a <= 0x1p100f)) return n == 0.f ? n : n / d;
  float r = __builtin_amdgcn_rcpf(d);
  r = fmaf(fmaf(-d, r, 1.f), r, r);
  float q = n * r;
  q = fmaf(fmaf(-d, q, n), r, q);
  return fmaf(fmaf(-d, q, n), r, q);
#endif
}

// ------------------------------------------------------------------------------------------
// Activation storage.  A PHX_DTYPE_BF16 context stores every activation (the arena tensors: conv /
// depthwise / fuse / resample / add outputs, i.e. the BN inputs) as bf16 — SURVEY.md 8a R4 "C4:
// bf16 act, fp32 acc" — while gradients, statistics, EOT and the images stay fp32.  Kernels take the
// storage type as a template flag (BF) and keep float* parameters as untyped base pointers; element
// e of a bf16 tensor is the 16-bit word e.  Loads widen to fp32 (exact), stores round to nearest even.
// ------------------------------------------------------------------------------------------
template <bool BF>
__device__ __forceinline__ float4 ald4(const float* p, long e) {
  if constexpr (BF) return unpack_bf16x4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(p) + e));
  else return *reinterpret_cast<const float4*>(p + e);
}
template <bool BF>
__device__ __forceinline__ float ald1(const float* p, long e) {
  if constexpr (BF) return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(p)[e] << 16);
  else return p[e];
}
template <bool BF>
__device__ __forceinline__ void ast4(float* p, long e, float4 v) {
  if constexpr (BF) *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p) + e) = pack_bf16x4(v);
  else *reinterpret_cast<float4*>(p + e) = v;
}
template <bool BF>
__device__ __forceinline__ void ast1(float* p, long e, float v) {
  if constexpr (BF) reinterpret_cast<uint16_t*>(p)[e] = __builtin_bit_cast(unsigned short, (__bf16)v);
  else p[e] = v;
}
// the value a store of v leaves in memory (BN statistics are taken over the stored values)
template <bool BF>
__device__ __forceinline__ float ast_val(float v) {
  if constexpr (BF) return round_bf16(v);
  else return v;
}

// ------------------------------------------------------------------------------------------
// InX: an input tensor as its consumers see it.  The output of a training-mode batch norm is
// never materialised: consumers read the BN input y and apply a = act((y - mu) * sc + be) on
// load (sc = gamma * rstd, be = beta), so every BN costs one statistics pass instead of a
// statistics pass plus a read-modify-write pass over HBM.  mu == nullptr means a raw tensor.
// ------------------------------------------------------------------------------------------
struct InX {
  const float* p;
  const float* mu;
  const float* sc;
  const float* be;
  int act;
  int bf = 0;  // p holds bf16 elements (a PHX_DTYPE_BF16 context's activation arena)
};

struct Chan4 {
  float mu[4], sc[4], be[4];
};

__device__ __forceinline__ Chan4 inx_chan4(const InX& v, int c) {
  Chan4 k;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    k.mu[j] = v.mu[c + j];
    k.sc[j] = v.sc[c + j];
    k.be[j] = v.be[c + j];
  }
  return k;
}

__device__ __forceinline__ float4 inx_apply4(const InX& v, const Chan4& k, float4 x) {
  x.x = act_fwd((x.x - k.mu[0]) * k.sc[0] + k.be[0], v.act);
  x.y = act_fwd((x.y - k.mu[1]) * k.sc[1] + k.be[1], v.act);
  x.z = act_fwd((x.z - k.mu[2]) * k.sc[2] + k.be[2], v.act);
  x.w = act_fwd((x.w - k.mu[3]) * k.sc[3] + k.be[3], v.act);
  return x;
}

// element e (flat index) of channel c (BF: bf16 storage)
template <bool BF = false>
__device__ __forceinline__ float inx_load1(const InX& v, long e, int c) {
  float x = ald1<BF>(v.p, e);
  if (v.mu) x = act_fwd((x - v.mu[c]) * v.sc[c] + v.be[c], v.act);
  return x;
}

// 4 consecutive channels c..c+3 at flat index e
template <bool BF = false>
__device__ __forceinline__ float4 inx_load4(const InX& v, long e, int c) {
  float4 x = ald4<BF>(v.p, e);
  if (v.mu) x = inx_apply4(v, inx_chan4(v, c), x);
  return x;
}

// ------------------------------------------------------------------------------------------
// GradX: the gradient w.r.t. a BN input y as its consumer (the producing conv's dgrad) sees
// it.  The BN backward only reduces sum(dz) and sum(dz*xhat); the consumer rebuilds
//   dy = sc * (dz - mdz - xhat * mdzx),  dz = da * act'(z),  z = (y-mu)*sc + be,
//   xhat = (y - mu) * rstd
// on load, so dy is never written to HBM.  y == nullptr means da is the gradient itself.
// ------------------------------------------------------------------------------------------
struct GradX {
  const float* da;
  const float* y;
  const float* mu;
  const float* rstd;
  const float* sc;
  const float* be;
  const float* mdz;
  const float* mdzx;
  int act;
  int ybf = 0;  // y holds bf16 elements (the gradient da stays fp32)
};

struct GChan4 {
  float4 mu, rs, sc, be, m1, m2;
};

__device__ __forceinline__ GChan4 gx_chan4(const GradX& g, int c) {
  GChan4 k;
  k.mu = *reinterpret_cast<const float4*>(g.mu + c);
  k.rs = *reinterpret_cast<const float4*>(g.rstd + c);
  k.sc = *reinterpret_cast<const float4*>(g.sc + c);
  k.be = *reinterpret_cast<const float4*>(g.be + c);
  k.m1 = *reinterpret_cast<const float4*>(g.mdz + c);
  k.m2 = *reinterpret_cast<const float4*>(g.mdzx + c);
  return k;
}

__device__ __forceinline__ float gx_one(float d, float y, float mu, float rs, float sc, float be,
                                        float m1, float m2, int act) {
  const float yc = y - mu;
  float dz = d;
  if (act) dz *= act_grad(yc * sc + be, act);
  return sc * (dz - m1 - (yc * rs) * m2);
}

__device__ __forceinline__ float4 gx_apply4(const GradX& g, const GChan4& k, float4 d, float4 y) {
  float4 o;
  o.x = gx_one(d.x, y.x, k.mu.x, k.rs.x, k.sc.x, k.be.x, k.m1.x, k.m2.x, g.act);
  o.y = gx_one(d.y, y.y, k.mu.y, k.rs.y, k.sc.y, k.be.y, k.m1.y, k.m2.y, g.act);
  o.z = gx_one(d.z, y.z, k.mu.z, k.rs.z, k.sc.z, k.be.z, k.m1.z, k.m2.z, g.act);
  o.w = gx_one(d.w, y.w, k.mu.w, k.rs.w, k.sc.w, k.be.w, k.m1.w, k.m2.w, g.act);
  return o;
}

// 4 consecutive channels c..c+3 at flat index e (BF: y in bf16 storage)
template <bool BF = false>
__device__ __forceinline__ float4 gx_load4(const GradX& g, long e, int c) {
  float4 d = *reinterpret_cast<const float4*>(g.da + e);
  if (!g.y) return d;
  float4 y = ald4<BF>(g.y, e);
  return gx_apply4(g, gx_chan4(g, c), d, y);
}

// ------------------------------------------------------------------------------------------
// StatSink: training-mode BN batch statistics computed by the kernel that PRODUCES the BN input
// (GEMM epilogue, depthwise conv, stem), so the statistics cost no extra pass over HBM.  Each
// producer workgroup reduces the rows it wrote to a per-channel (sum, M2) pair — M2 about the
// workgroup's own mean, so no cancellation — and stores it as partial p of channel c at
// part[c*P + p] (cnt[p] = rows covered).  Channel-major, so k_bn_finalize reads each channel's P
// partials contiguously (one workgroup per channel, fp64, fixed order: bit-reproducible), then
// writes mean / rstd / gamma*rstd and updates the moving statistics.
// ------------------------------------------------------------------------------------------
// BiFPN node fuse (efficientdet_keras.py:91-110): y = act(sum_i x_i * w_i / (sum_j w_j + 1e-4))
// with w = relu(wsm) (fastattn, method 0) or act(sum_i x_i) (method 1); inputs through InX views
struct FuseView {
  InX x[3];
  int nin;
  const float* w[3];
  int method, act;
};

__device__ __forceinline__ void fuse_weights(const float* w0, const float* w1, const float* w2,
                                             int nin, int method, float* wv, float* den) {
  if (method == 0) {
    wv[0] = fmaxf(w0[0], 0.f);
    wv[1] = fmaxf(w1[0], 0.f);
    wv[2] = nin > 2 ? fmaxf(w2[0], 0.f) : 0.f;
    float s = wv[0] + wv[1];
    if (nin > 2) s += wv[2];
    *den = s + 0.0001f;
  } else {
    wv[0] = wv[1] = wv[2] = 1.f;
    *den = 1.f;
  }
}

// one fused value from the three (already BN-applied) inputs, in k_fuse_fwd's operation order
__device__ __forceinline__ float fuse_combine(float x0, float x1, float x2, int nin, int method,
                                              const float* wv, float den, int act) {
  float v;
  if (method == 0) {
    v = x0 * wv[0] / den;
    v = v + x1 * wv[1] / den;
    if (nin > 2) v = v + x2 * wv[2] / den;
  } else {
    v = x0 + x1;
    if (nin > 2) v = v + x2;
  }
  return act_fwd(v, act);
}

// members of one grouped launch (the per-level convs of a class/box head)
constexpr int kMaxSeg = 5;

// member i of a grouped launch's by-value argument array, read at constant offsets only (a
// run-time index into kernel arguments turns every field access into a vector load)
template <class T, int NS>
__device__ __forceinline__ T pick_seg(const T (&arr)[NS], int i) {
  T v = arr[0];
#pragma unroll
  for (int k = 1; k < NS; ++k)
    if (i == k) v = arr[k];
  return v;
}

struct StatSink {
  float2* part;  // [C][P] (sum, M2); nullptr = no statistics wanted
  float* cnt;    // [P]
  int C;
  int P;         // partial rows (set by the producer's launcher)
};

__device__ __forceinline__ void sink_put(const StatSink& k, long p, int c, float n, float mean,
                                         float m2) {
  k.part[(long)c * k.P + p] = make_float2(n * mean, m2);
}
__device__ __forceinline__ void sink_cnt(const StatSink& k, long p, float n) { k.cnt[p] = n; }

// ------------------------------------------------------------------------------------------
// GradSink: the reduction half of a training-mode BN backward, computed by the kernel that
// finishes the gradient da of the BN OUTPUT (the last consumer's dgrad in the reverse sweep):
//   dz = da * act'(z), z = (y - mu) * sc + be, xhat = (y - mu) * rstd;  sums of dz and dz*xhat.
// Each workgroup stores its per-channel (sum dz, sum dz*xhat) as partial p at part[c*P + p];
// k_bn_finalize<true> adds them in fp64 and writes mean(dz), mean(dz*xhat) (GradX's mdz, mdzx).
// ------------------------------------------------------------------------------------------
struct GradSink {
  float2* part;  // [C][P]; nullptr = off
  int C, P;
  const float* y;     // BN input
  const float* mu;
  const float* rstd;
  const float* sc;
  const float* be;
  int act;
  int ybf = 0;  // y holds bf16 elements
};

struct GSChan4 {
  float4 mu, rs, sc, be;
};

__device__ __forceinline__ GSChan4 gs_chan4(const GradSink& g, int c) {
  GSChan4 k;
  k.mu = *reinterpret_cast<const float4*>(g.mu + c);
  k.rs = *reinterpret_cast<const float4*>(g.rstd + c);
  k.sc = *reinterpret_cast<const float4*>(g.sc + c);
  k.be = *reinterpret_cast<const float4*>(g.be + c);
  return k;
}

__device__ __forceinline__ void gs_one(float da, float y, float mu, float rs, float sc, float be,
                                       int act, float& s1, float& s2) {
  const float yc = y - mu;
  float dz = da;
  if (act) dz *= act_grad(yc * sc + be, act);
  s1 += dz;
  s2 = fmaf(dz, yc * rs, s2);
}

__device__ __forceinline__ void gs_acc4(const GradSink& g, const GSChan4& k, float4 da, float4 y,
                                        float4& s1, float4& s2) {
  gs_one(da.x, y.x, k.mu.x, k.rs.x, k.sc.x, k.be.x, g.act, s1.x, s2.x);
  gs_one(da.y, y.y, k.mu.y, k.rs.y, k.sc.y, k.be.y, g.act, s1.y, s2.y);
  gs_one(da.z, y.z, k.mu.z, k.rs.z, k.sc.z, k.be.z, g.act, s1.z, s2.z);
  gs_one(da.w, y.w, k.mu.w, k.rs.w, k.sc.w, k.be.w, g.act, s1.w, s2.w);
}

__device__ __forceinline__ void gsink_put(const GradSink& g, long p, int c, float s1, float s2) {
  g.part[(long)c * g.P + p] = make_float2(s1, s2);
}

// (n, mean, M2) += (nb, mb, m2b)
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float mb,
                                           float m2b) {
  const float nt = n + nb;
  if (nb <= 0.f) return;
  const float f = nb / nt;
  const float d = mb - mean;
  mean = fmaf(d, f, mean);
  m2 += m2b + d * d * n * f;
  n = nt;
}

// ------------------------------------------------------------------------------------------
// BN finalize epilogues (k_bn_finalize, k_colred_final).
// ------------------------------------------------------------------------------------------
// one moving-average step, m - (m - batch) * (1 - momentum) in fp64 rounded to float
__device__ __forceinline__ float moving_update(float m, double batch) { return (float)(m - (m - batch) * 0.01); }

struct StatsEpi {
  const float* y;  // for the shift (row 0)
  long M;
  float* mean;
  float* rstd;
  const float* gamma;
  float* sc;
  float* mmean;
  float* mvar;
  float eps;
  int ybf = 0;  // y in bf16 storage
  double* side = nullptr;  // deferred moving statistics: (mean, uvar) pairs, moving stats untouched
  int C = 0;               // channels
  // the per-channel inputs of the epilogue, loaded before the fold (k_bn_finalize issues them with
  // the partials, so the epilogue costs no second memory round trip)
  struct Pre {
    float ref, g, mm, mv;
  };
  __device__ Pre pre(int c) const {
    Pre r;
    r.ref = !y ? 0.f : ybf ? ald1<true>(y, c) : y[c];
    r.g = gamma[c];
    r.mm = (!side && mmean) ? mmean[c] : 0.f;
    r.mv = (!side && mmean) ? mvar[c] : 0.f;
    return r;
  }
  __device__ void operator()(int, int c, double s0, double s1) const { fin(pre(c), c, s0, s1); }
  __device__ void fin(const Pre& pr, int c, double s0, double s1) const {
    const double ref = (double)pr.ref;
    const double dm = s0 / (double)M;            // mean - ref
    double var = s1 / (double)M - dm * dm;
    if (var < 0.0) var = 0.0;
    const double mu = ref + dm;
    mean[c] = (float)mu;
    const double rs = 1.0 / sqrt(var + (double)eps);
    rstd[c] = (float)rs;
    sc[c] = (float)(rs * (double)pr.g);
    // Keras: moving -= (moving - batch) * (1 - momentum); the fused op reports the
    // Bessel-corrected variance for the moving average [TF-recall].
    const double uvar = M > 1 ? var * (double)M / (double)(M - 1) : var;
    if (side) {
      side[2 * c] = mu;
      side[2 * c + 1] = uvar;
    } else if (mmean) {
      mmean[c] = moving_update(pr.mm, mu);
      mvar[c] = moving_update(pr.mv, uvar);
    }
  }
};

struct BwdEpi2 {
  long M;
  float* mdz;
  float* mdzx;
  int C = 0;  // channels
  struct Pre {};
  __device__ Pre pre(int) const { return Pre{}; }
  __device__ void fin(const Pre&, int c, double s0, double s1) const { (*this)(0, c, s0, s1); }
  __device__ void operator()(int, int c, double s0, double s1) const {
    mdz[c] = (float)(s0 / (double)M);
    mdzx[c] = (float)(s1 / (double)M);
  }
};

// ------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11), counter-based: identical draws for a given
// (key, counter) on any device / GPU count.  Matches oracle/philox.py bit for bit.
// ------------------------------------------------------------------------------------------
struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)M0 * c.x;
    uint64_t p1 = (uint64_t)M1 * c.z;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// [0,1) with 24 random bits (exact in fp32)
__host__ __device__ inline float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }
// (0,1]
__host__ __device__ inline float u01_open0(uint32_t v) {
  return (float)((v >> 8) + 1u) * (1.0f / 16777216.0f);
}

// RNG streams (counter word w = step << 8 | stream)
enum RngStream : uint32_t {
  RNG_PRINT = 1,      // per image: print-variation w[3], b[3] (attacker.py:365-372)
  RNG_PLACE = 2,      // per box: centre jitter (attacker.py:474-475)
  RNG_BOX = 3,        // per box: brightness delta, angle (attacker.py:427, 436)
  RNG_NOISE = 4,      // per box element: U(-.01,.01) noise (attacker.py:426)
  RNG_DROP = 5,       // per (MBConv block, pass, image): drop-connect uniform (utils.py:336-339)
  RNG_AUG = 6,        // input pipeline: per image flips, per batch contrast / brightness
                      // (train_data_generator.py:201-204, 222-225)
  RNG_DSHUF = 7,      // defender Masker: per image shuffle key (attack_detection.py:487)
  RNG_DFLIP = 8,      // defender Masker: per image left-right / up-down flips (:488-489)
  RNG_DROPOUT = 9,    // defender U-Net: per (layer, image, element) Dropout(0.2) uniform
  RNG_APNOISE = 10,   // inference compositor: per (image, box slot, element pair) U(-.01, .01)
                      // (adv_patch.py:144-149)
};

}  // namespace phx
