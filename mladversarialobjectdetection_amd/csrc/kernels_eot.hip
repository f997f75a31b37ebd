// kernels_eot.hip — the expectation-over-transformation patch pipeline (Patcher,
// attacker.py:344-498; BrightnessMatcher, brightness_matcher.py:14-73) forward and backward,
// TV loss and the Adam update.
//
// Layout / parallelisation (MI355X-first, not the reference's map_fn x while_loop):
//   * placement of every (image, box) slot in one tiny kernel; a compact list of valid boxes and
//     a prefix of their pixel chunks lets the per-box kernels run as ONE launch whose workgroups
//     walk (box, chunk) work items — no per-box launches, no host round trip, graph-capturable.
//   * the sequential paste loop becomes a per-pixel fold: every output pixel walks the boxes of
//     its image in order (v <- clip(r_k < -1 ? v : r_k)), so overlapping pastes compose exactly
//     as the reference's tensor_scatter_nd_update chain, with full pixel parallelism.  The fold
//     records the owning box per pixel/channel, which is all the backward needs.
//   * the rotation gradient is TF's registered rule for ImageProjectiveTransformV3: an inverse
//     warp of the upstream gradient with fill 0 (not the exact adjoint) [TF-recall].
//   * resize is TF ScaleAndTranslate (triangle kernel, antialias, half-pixel centres, span
//     weights normalised) with its exact adjoint in the backward.
// Ops that decide discrete geometry follow TF's fp32 operation order with FMA contraction off.
#include "common.hpp"
#include "post.hpp"

#pragma clang fp contract(off)

namespace phx {

// ------------------------------------------------------------------------------------------
// RNG helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ u32x4 rng(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2,
                                     int64_t step, uint32_t stream) {
  return philox4x32_10(u32x4{c0, c1, c2, (uint32_t)((uint64_t)step << 8) | stream},
                       (uint32_t)seed, (uint32_t)(seed >> 32));
}
// tf.random.uniform(minval, maxval): u * (maxval - minval) + minval
__device__ __forceinline__ float runif(uint32_t v, float lo, float hi) {
  return u01(v) * (hi - lo) + lo;
}
// tf.random.normal(mean, stddev): z * stddev + mean, z by Box-Muller
__device__ __forceinline__ float rnorm(uint32_t a, uint32_t b, float mean, float sd) {
  float u1 = u01_open0(a), u2 = u01(b);
  float z = sqrtf(-2.0f * logf(u1)) * cosf(6.28318530717958647692f * u2);
  return z * sd + mean;
}

// ------------------------------------------------------------------------------------------
// placement (Patcher.create, attacker.py:448-488) + print params + span tables
// ------------------------------------------------------------------------------------------
// workspace layout for the compact lists lives right after `place` (see EotLists below)
struct EotLists {
  int nvalid;
  int total_chunks;
};

// output rows per separable-resize work item (k_eot_resize, k_eot_resize_bwd_rows)
constexpr int kResizeRT = 4;

// PHX_EOT_V1=1: the round-4 composite and resize-adjoint kernels (A/B and the bit-identity test;
// read per call)
static bool eot_v1() {
  const char* e = std::getenv("PHX_EOT_V1");
  return e && e[0] == '1';
}

__global__ __launch_bounds__(256) void k_eot_place(EotDims d, const float* __restrict__ boxes,
                                                   const int* __restrict__ count,
                                                   const float* __restrict__ params,
                                                   uint64_t seed, int64_t step, int gimg0,
                                                   ImgParams* __restrict__ img,
                                                   BoxPlace* __restrict__ place,
                                                   int* __restrict__ lists, int* __restrict__ err,
                                                   PlaceRule rule) {
  const int t = threadIdx.x;
  const float scale = params ? params[PHX_NPATCH_DEV] : 0.f;
  const float Hf = (float)d.H, Wf = (float)d.W;
  for (int b = t; b < d.B; b += blockDim.x) {
    u32x4 r = rng(seed, 0, 0, (uint32_t)(gimg0 + b), step, RNG_PRINT);
    u32x4 r2 = rng(seed, 1, 0, (uint32_t)(gimg0 + b), step, RNG_PRINT);
    u32x4 r3 = rng(seed, 2, 0, (uint32_t)(gimg0 + b), step, RNG_PRINT);
    ImgParams p;
    p.w[0] = rnorm(r.x, r.y, 0.5f, 0.1f);
    p.w[1] = rnorm(r.z, r.w, 0.5f, 0.1f);
    p.w[2] = rnorm(r2.x, r2.y, 0.5f, 0.1f);
    p.b[0] = rnorm(r2.z, r2.w, 0.0f, 0.01f);
    p.b[1] = rnorm(r3.x, r3.y, 0.0f, 0.01f);
    p.b[2] = rnorm(r3.z, r3.w, 0.0f, 0.01f);
    img[b] = p;
  }
  const int nslot = d.B * d.maxb;
  for (int sl = t; sl < nslot; sl += blockDim.x) {
    const int b = sl / d.maxb, k = sl % d.maxb;
    BoxPlace P{};
    P.valid = 0;
    if (k < count[b]) {
      const float* bx = boxes + (long)sl * 4;
      const float ymin = bx[0], xmin = bx[1], ymax = bx[2], xmax = bx[3];
      const float h = ymax - ymin, w = xmax - xmin;
      const float longer = fmaxf(h, w);
      u32x4 r = rng(seed, 0, (uint32_t)k, (uint32_t)(gimg0 + b), step, RNG_PLACE);
      const float bscale = rule.random_scale ? runif(r.z, rule.scale_lo, rule.scale_hi) : scale;
      const float psf = floorf(longer * bscale);
      const float diag = fminf(1.41421354f * psf, Wf);
      const float tol = rule.tol;
      const float oy = (ymin + h / 2.0f) + runif(r.x, (-tol * h) / 2.0f, (tol * h) / 2.0f);
      const float ox = (xmin + w / 2.0f) + runif(r.y, (-tol * w) / 2.0f, (tol * w) / 2.0f);
      float yp = fmaxf(oy - diag / 2.0f, 0.0f);
      float xp = fmaxf(ox - diag / 2.0f, 0.0f);
      if (yp + diag > Hf) yp = Hf - diag;
      if (xp + diag > Wf) xp = Wf - diag;
      P.ymin = (int)yp;
      P.xmin = (int)xp;
      P.ps = (int)psf;
      P.diag = (int)diag;
      P.valid = (psf * psf > 4.0f) && P.ps <= d.span_stride ? 1 : 0;
      // attacker.py:430-433: top = left = floor((diag - ps) / 2)
      P.pad = (P.diag - P.ps) >= 0 ? (P.diag - P.ps) / 2 : -(((P.ps - P.diag) + 1) / 2);
      u32x4 q = rng(seed, 1, (uint32_t)k, (uint32_t)(gimg0 + b), step, RNG_BOX);
      P.delta = runif(q.x, -0.3f, 0.3f);
      const float amax = 0.34906584f;  // float32(20 * pi / 180)
      P.angle = runif(q.y, -amax, amax);
      // tfa.image.angles_to_projective_transforms (fp32)
      const float side = (float)P.diag;
      const float c = cosf(P.angle), s = sinf(P.angle);
      const float xo = ((side - 1.0f) - (c * (side - 1.0f) - s * (side - 1.0f))) / 2.0f;
      const float yo = ((side - 1.0f) - (s * (side - 1.0f) + c * (side - 1.0f))) / 2.0f;
      P.fwd[0] = c; P.fwd[1] = -s; P.fwd[2] = xo;
      P.fwd[3] = s; P.fwd[4] = c;  P.fwd[5] = yo;
      // inverse (gradient transform, image_ops _image_projective_transform_v3_grad)
      double a = c, bb = -s, tx = xo, dd = s, e = c, ty = yo;
      double det = a * e - bb * dd;
      P.inv[0] = (float)(e / det);
      P.inv[1] = (float)(-bb / det);
      P.inv[2] = (float)((bb * ty - e * tx) / det);
      P.inv[3] = (float)(-dd / det);
      P.inv[4] = (float)(a / det);
      P.inv[5] = (float)((dd * tx - a * ty) / det);
    }
    place[sl] = P;
  }
  __syncthreads();
  // R offsets, compact valid list, per-image lists and chunk prefix: one workgroup scan per
  // 256 slots with running totals
  int* nvalid = lists;                 // [1]
  int* total_chunks = lists + 1;       // [1]
  int* img_n = lists + 2;              // [B]
  int* img_first = img_n + d.B;        // [B]  index into vlist of the image's first box
  int* vlist = img_first + d.B;        // [B*maxb] slot ids
  int* cprefix = vlist + nslot;        // [B*maxb+1] chunk prefix over vlist
  int* tprefix = cprefix + nslot + 1;  // [B*maxb+1] resize row-tile prefix over vlist
  __shared__ long s_need[256];
  __shared__ int s_ch[256], s_v[256], s_tl[256];
  __shared__ long run_off;
  __shared__ int run_ch, run_v, run_tl;
  if (t == 0) { run_off = 0; run_ch = 0; run_v = 0; run_tl = 0; }
  __syncthreads();
  for (int base = 0; base < nslot; base += 256) {
    const int sl = base + t;
    long need = 0;
    int ch = 0, v = 0, tl = 0;
    if (sl < nslot && place[sl].valid) {
      const int ps = place[sl].ps;
      need = (long)ps * ps * 3;
      ch = (ps * ps + 255) / 256;
      tl = (ps + kResizeRT - 1) / kResizeRT;
      v = 1;
    }
    s_need[t] = need; s_ch[t] = ch; s_v[t] = v; s_tl[t] = tl;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
      long a1 = t >= off ? s_need[t - off] : 0;
      int a2 = t >= off ? s_ch[t - off] : 0;
      int a3 = t >= off ? s_v[t - off] : 0;
      int a4 = t >= off ? s_tl[t - off] : 0;
      __syncthreads();
      s_need[t] += a1; s_ch[t] += a2; s_v[t] += a3; s_tl[t] += a4;
      __syncthreads();
    }
    if (sl < nslot) {
      const long ex_off = run_off + s_need[t] - need;
      const int ex_ch = run_ch + s_ch[t] - ch;
      const int ex_v = run_v + s_v[t] - v;
      const int ex_tl = run_tl + s_tl[t] - tl;
      if (sl % d.maxb == 0) img_first[sl / d.maxb] = ex_v;
      if (v) {
        place[sl].roff = ex_off;
        vlist[ex_v] = sl;
        cprefix[ex_v] = ex_ch;
        tprefix[ex_v] = ex_tl;
      }
    }
    __syncthreads();
    if (t == 255) {
      run_off += s_need[255]; run_ch += s_ch[255]; run_v += s_v[255]; run_tl += s_tl[255];
    }
    __syncthreads();
  }
  if (t == 0) {
    *nvalid = run_v;
    *total_chunks = run_ch;
    cprefix[run_v] = run_ch;
    tprefix[run_v] = run_tl;
    if (err) *err = 0;
  }
  __syncthreads();
  for (int b = t; b < d.B; b += blockDim.x)
    img_n[b] = (b + 1 < d.B ? img_first[b + 1] : run_v) - img_first[b];
}

// TF ScaleAndTranslate span computation (ComputeSpansCore, triangle kernel, antialias=True,
// translate=0) for output index i of a resize input_size -> ps.
__device__ __forceinline__ void tf_span(int i, int ps, int in_size, SpanEntry* out) {
  const float scale = (float)ps / (float)in_size;
  const float inv_scale = (float)(1.0 / (double)scale);
  const float kscale = fmaxf(inv_scale, 1.0f);
  const float one_over_k = 1.0f / kscale;
  const float radius = 1.0f;
  const float sample_f = ((float)i + 0.5f) * inv_scale + (-inv_scale * 0.0f);
  long start = (long)ceilf(sample_f - radius * kscale - 0.5f);
  long end = (long)floorf(sample_f + radius * kscale - 0.5f);
  start = start < 0 ? 0 : (start > in_size - 1 ? in_size - 1 : start);
  end = (end < 0 ? 0 : (end > in_size - 1 ? in_size - 1 : end)) + 1;
  float total = 0.0f;
  for (long src = start; src < end; ++src) {
    float pos = (float)src + 0.5f - sample_f;
    float x = fabsf(pos * one_over_k);
    total += x < 1.0f ? 1.0f - x : 0.0f;
  }
  out->start = (int)start;
  out->end = (int)end;
  out->inv_total = fabsf(total) >= 1000.0f * 1.17549435e-38f ? 1.0f / total : 0.0f;
  out->sample_f = sample_f;
}

__device__ __forceinline__ float span_weight(const SpanEntry& sp, int src, float one_over_k) {
  float pos = (float)src + 0.5f - sp.sample_f;
  float x = fabsf(pos * one_over_k);
  float w = x < 1.0f ? 1.0f - x : 0.0f;
  return w * sp.inv_total;
}

__global__ __launch_bounds__(256) void k_eot_spans(EotDims d, const BoxPlace* __restrict__ place,
                                                   SpanEntry* __restrict__ spans) {
  const int sl = blockIdx.y;
  const BoxPlace& P = place[sl];
  if (!P.valid) return;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < P.ps; i += gridDim.x * blockDim.x)
    tf_span(i, P.ps, d.P, &spans[(long)sl * d.span_stride + i]);
}

// XCD bands of the forward resize (k_eot_resize): band x holds row tiles x*nt/8 .. (x+1)*nt/8 - 1 of
// every valid box (nt its row tiles).  One workgroup per image: bvpre[x][v] = band-x tiles of the
// image's boxes before valid box v (eight exclusive scans in LDS), bcnt[x][b] = the image's total.
constexpr int kBandMaxBoxes = 128;
__global__ __launch_bounds__(kBandMaxBoxes) void k_eot_bands(EotDims d, const BoxPlace* __restrict__ place) {
  const int nslot = d.B * d.maxb;
  const int* lists = reinterpret_cast<const int*>(place + nslot);
  const int* img_n = lists + 2;
  const int* img_first = img_n + d.B;
  const int* vlist = img_first + d.B;
  int* bcnt = const_cast<int*>(vlist + 3 * nslot + 2);  // after tprefix: [8][B]
  int* bvpre = bcnt + 8 * d.B;                          // [8][B*maxb]
  __shared__ int sc[8][kBandMaxBoxes];
  const int b = blockIdx.x, j = threadIdx.x, n = img_n[b], v = img_first[b] + j;
  const int nt = j < n ? (place[vlist[v]].ps + kResizeRT - 1) / kResizeRT : 0;
  int c[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    c[x] = (x + 1) * nt / 8 - x * nt / 8;
    sc[x][j] = c[x];
  }
  __syncthreads();
  for (int off = 1; off < kBandMaxBoxes; off <<= 1) {
    int a[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) a[x] = j >= off ? sc[x][j - off] : 0;
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 8; ++x) sc[x][j] += a[x];
    __syncthreads();
  }
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    if (j < n) bvpre[x * nslot + v] = sc[x][j] - c[x];
    if (j == 0) bcnt[x * d.B + b] = n ? sc[x][n - 1] : 0;
  }
}

void launch_eot_place(const EotDims& d, const float* boxes, const int* count, const float* params,
                      uint64_t seed, int64_t step, int gimg0, ImgParams* img, BoxPlace* place,
                      SpanEntry* spans, int* err, hipStream_t s, PlaceRule rule) {
  int* lists = reinterpret_cast<int*>(place + (long)d.B * d.maxb);
  hipLaunchKernelGGL(k_eot_place, dim3(1), dim3(256), 0, s, d, boxes, count, params, seed, step,
                     gimg0, img, place, lists, err, rule);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_eot_spans, dim3(2, d.B * d.maxb), dim3(256), 0, s, d, place, spans);
  PHX_LAUNCH_CHECK();
  if (d.maxb > kBandMaxBoxes) throw std::invalid_argument("eot: more than 128 box slots per image");
  hipLaunchKernelGGL(k_eot_bands, dim3(d.B), dim3(kBandMaxBoxes), 0, s, d, place);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// brightness matcher (brightness_matcher.py:43-73), fused with the print variation
// ------------------------------------------------------------------------------------------
struct Yuv {
  float y, u, v;
};
__device__ __forceinline__ Yuv rgb2yuv(float r, float g, float b) {
  Yuv o;
  o.y = r * 0.299f + g * 0.587f + b * 0.114f;
  o.u = r * -0.14714119f + g * -0.28886916f + b * 0.43601035f;
  o.v = r * 0.61497538f + g * -0.51496512f + b * -0.10001026f;
  return o;
}
constexpr float kTo01 = 127.0f / 255.0f;   // _rescale_0_1 constant
constexpr float kBack = 255.0f / 127.0f;   // _rescale_back constant

__device__ __forceinline__ float print_px(const float* patch, const ImgParams& p, long e, int c,
                                          bool apply) {
  float x = patch[e];
  if (!apply) return x;
  float v = p.w[c] * x + p.b[c];
  return fminf(fmaxf(v, -1.0f), 1.0f);
}

// partial sums of Y: z = 0 source (printed patch), z = 1 target (image)
__global__ __launch_bounds__(256) void k_eot_ysum(EotDims d, const float* __restrict__ src,
                                                  long src_stride, const ImgParams* __restrict__ img,
                                                  const float* __restrict__ tgt, int apply,
                                                  double* __restrict__ ysum) {
  const int b = blockIdx.y, z = blockIdx.z;
  const long npx = z == 0 ? (long)d.P * d.P : (long)d.H * d.W;
  const ImgParams p = img ? img[b] : ImgParams{};
  const float* base = z == 0 ? src + (long)b * src_stride : tgt + (long)b * d.H * d.W * 3;
  double acc = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < npx;
       i += (long)gridDim.x * blockDim.x) {
    float r, g, bl;
    if (z == 0) {
      r = (print_px(base, p, i * 3 + 0, 0, apply) + 1.0f) * kTo01;
      g = (print_px(base, p, i * 3 + 1, 1, apply) + 1.0f) * kTo01;
      bl = (print_px(base, p, i * 3 + 2, 2, apply) + 1.0f) * kTo01;
    } else {
      r = (base[i * 3 + 0] + 1.0f) * kTo01;
      g = (base[i * 3 + 1] + 1.0f) * kTo01;
      bl = (base[i * 3 + 2] + 1.0f) * kTo01;
    }
    acc += rgb2yuv(r, g, bl).y;
  }
  __shared__ double sh[256];
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) ysum[((long)b * 2 + z) * gridDim.x + blockIdx.x] = sh[0];
}

__global__ void k_eot_ymean(EotDims d, const double* __restrict__ ysum, int chunks,
                            float* __restrict__ ymean) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.B * 2) return;
  double s = 0.0;
  for (int k0 = 0; k0 < chunks; k0 += 16) {  // 16 loads in flight per round, added in order
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = ysum[(long)i * chunks + min(k0 + u, chunks - 1)];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (k0 + u < chunks) s += v[u];
  }
  const long npx = (i % 2) == 0 ? (long)d.P * d.P : (long)d.H * d.W;
  ymean[i] = (float)(s / (double)npx);
}

__device__ __forceinline__ void match_px(float p0, float p1, float p2, float mus, float mut,
                                         float* o) {
  Yuv s = rgb2yuv((p0 + 1.0f) * kTo01, (p1 + 1.0f) * kTo01, (p2 + 1.0f) * kTo01);
  float yc = (s.y - mus) + mut;
  float yp = fminf(fmaxf(yc, 0.0f), 1.0f);
  float r = yp + 1.13988303f * s.v;
  float g = yp + -0.394642334f * s.u + -0.58062185f * s.v;
  float bl = yp + 2.03206185f * s.u;
  o[0] = fminf(fmaxf(r, 0.0f), 1.0f) * kBack - 1.0f;
  o[1] = fminf(fmaxf(g, 0.0f), 1.0f) * kBack - 1.0f;
  o[2] = fminf(fmaxf(bl, 0.0f), 1.0f) * kBack - 1.0f;
}

__global__ __launch_bounds__(256) void k_eot_match(EotDims d, const float* __restrict__ src,
                                                   long src_stride, const ImgParams* __restrict__ img,
                                                   const float* __restrict__ ymean, int apply,
                                                   float* __restrict__ out) {
  const int b = blockIdx.y;
  const long npx = (long)d.P * d.P;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npx) return;
  const ImgParams p = img ? img[b] : ImgParams{};
  const float* base = src + (long)b * src_stride;
  float o[3];
  match_px(print_px(base, p, i * 3, 0, apply), print_px(base, p, i * 3 + 1, 1, apply),
           print_px(base, p, i * 3 + 2, 2, apply), ymean[b * 2], ymean[b * 2 + 1], o);
  float* op = out + ((long)b * npx + i) * 3;
  op[0] = o[0]; op[1] = o[1]; op[2] = o[2];
}

static constexpr int kYChunks = 64;

void launch_eot_match(const EotDims& d, const float* patch, const ImgParams* img, const float* tgt,
                      float* matched, double* ysum, float* ymean, bool apply_print,
                      hipStream_t s) {
  // apply_print: one shared patch + per-image print params; otherwise `patch` holds one
  // source image per batch entry.
  long stride = apply_print ? 0 : (long)d.P * d.P * 3;
  hipLaunchKernelGGL(k_eot_ysum, dim3(kYChunks, d.B, 2), dim3(256), 0, s, d, patch, stride, img,
                     tgt, apply_print ? 1 : 0, ysum);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_eot_ymean, dim3(cdiv(d.B * 2, 64)), dim3(64), 0, s, d, ysum, kYChunks,
                     ymean);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_eot_match, dim3(cdiv((long)d.P * d.P, 256), d.B), dim3(256), 0, s, d, patch,
                     stride, img, ymean, apply_print ? 1 : 0, matched);
  PHX_LAUNCH_CHECK();
}

void launch_eot_match_batch(const EotDims& d, const float* src, const ImgParams* img, const float* tgt,
                            float* matched, double* ysum, float* ymean, hipStream_t s) {
  const long stride = (long)d.P * d.P * 3;
  hipLaunchKernelGGL(k_eot_ysum, dim3(kYChunks, d.B, 2), dim3(256), 0, s, d, src, stride, img, tgt, 1, ysum);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_eot_ymean, dim3(cdiv(d.B * 2, 64)), dim3(64), 0, s, d, ysum, kYChunks, ymean);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_eot_match, dim3(cdiv((long)d.P * d.P, 256), d.B), dim3(256), 0, s, d, src, stride, img,
                     ymean, 1, matched);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// per-box kernels walk (valid box, 256-pixel chunk) work items
// ------------------------------------------------------------------------------------------
struct ListView {
  const int* nvalid;
  const int* total_chunks;
  const int* img_n;
  const int* img_first;
  const int* vlist;
  const int* cprefix;
  const int* tprefix;  // resize row tiles (kResizeRT rows) per valid box, prefix over vlist
  const int* bcnt;     // [8][B] XCD-band row tiles of image b (k_eot_bands)
  const int* bvpre;    // [8][B*maxb] XCD-band row tiles before valid box v within its image
};

__device__ __forceinline__ ListView lists_of(const EotDims& d, const BoxPlace* place) {
  const int* l = reinterpret_cast<const int*>(place + (long)d.B * d.maxb);
  ListView v;
  v.nvalid = l;
  v.total_chunks = l + 1;
  v.img_n = l + 2;
  v.img_first = v.img_n + d.B;
  v.vlist = v.img_first + d.B;
  v.cprefix = v.vlist + d.B * d.maxb;
  v.tprefix = v.cprefix + d.B * d.maxb + 1;
  v.bcnt = v.tprefix + d.B * d.maxb + 1;
  v.bvpre = v.bcnt + 8 * d.B;
  return v;
}

// binary search: largest v with cprefix[v] <= item
__device__ __forceinline__ int find_box(const int* cprefix, int nv, int item) {
  int lo = 0, hi = nv - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (cprefix[mid] <= item) lo = mid; else hi = mid - 1;
  }
  return lo;
}

constexpr int kBoxGrid = 2048;

// resize (+noise +brightness): R_pre[i,j,c] = sum_x Wc[j,x] sum_y Wr[i,y] m[y,x,c] + n + delta.
// Separable, vertical pass first: a work item is (valid box, kResizeRT output rows).  Its lanes
// run along x, so the vertical taps read whole NHWC rows of `matched` (coalesced); the
// kResizeRT x nx x 3 intermediate stays in LDS for the horizontal pass.
constexpr int kResizeGrid = 1280;  // 5 workgroups per CU (31 KB of LDS each)

__global__ __launch_bounds__(256) void k_eot_resize(EotDims d, const float* __restrict__ matched,
                                                    const BoxPlace* __restrict__ place,
                                                    const SpanEntry* __restrict__ spans,
                                                    uint64_t seed, int64_t step, int gimg0,
                                                    float* __restrict__ rstore, float amp) {
  extern __shared__ float V[];  // [kResizeRT][nx][3], then the band prefix [B+1]
  const ListView L = lists_of(d, place);
  // XCD bands: workgroup j runs on XCD x = j % 8 and takes only band x's row tiles of every box —
  // the x-th eighth of each box's output rows, whose vertical spans read about the x-th eighth of the
  // source rows — so an XCD's L2 holds one band of an image's matched patch for all its boxes
  // instead of every XCD streaming whole images.  Each row tile's arithmetic is unchanged.
  const int xb = blockIdx.x & 7;
  int* const bx = reinterpret_cast<int*>(V + kResizeRT * d.P * 3);  // [B+1] band-x tiles before image b
  if (threadIdx.x == 0) bx[0] = 0;
  for (int b0 = 0; b0 < d.B; b0 += 256) {  // (chunks of 256 images, running total in bx[b0])
    __shared__ int sx[256];
    const int bb = b0 + (int)threadIdx.x;
    sx[threadIdx.x] = bb < d.B ? L.bcnt[xb * d.B + bb] : 0;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
      const int a = threadIdx.x >= (unsigned)off ? sx[threadIdx.x - off] : 0;
      __syncthreads();
      sx[threadIdx.x] += a;
      __syncthreads();
    }
    if (bb < d.B) bx[bb + 1] = bx[b0] + sx[threadIdx.x];
    __syncthreads();
  }
  const int* bv = L.bvpre + xb * d.B * d.maxb;
  const int total = bx[d.B];
  for (int item = blockIdx.x >> 3; item < total; item += gridDim.x >> 3) {
    int b = 0;
    {
      int lo = 0, hi = d.B - 1;  // largest image with bx[b] <= item
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (bx[mid] <= item) lo = mid; else hi = mid - 1;
      }
      b = lo;
    }
    const int local = item - bx[b];
    const int v = L.img_first[b] + find_box(bv + L.img_first[b], L.img_n[b], local);
    const int sl = L.vlist[v];
    const BoxPlace P = place[sl];
    const int k = sl % d.maxb;
    const int nt = (P.ps + kResizeRT - 1) / kResizeRT;
    const int i0 = (xb * nt / 8 + (local - bv[v])) * kResizeRT;
    const int ni = min(kResizeRT, P.ps - i0);
    const SpanEntry* sp = spans + (long)sl * d.span_stride;
    const float scale = (float)P.ps / (float)d.P;
    const float inv_scale = (float)(1.0 / (double)scale);
    const float one_over_k = 1.0f / fmaxf(inv_scale, 1.0f);
    const int xlo = sp[0].start, nx = sp[P.ps - 1].end - xlo;
    const float* m = matched + (long)b * d.P * d.P * 3;
    // two columns per lane (xa and xa + h2 of the same output row: one span, two independent
    // chains of loads), 8 source rows' loads in flight per chain before any is accumulated; the
    // accumulation order of each output value is unchanged
    const int h2 = (nx + 1) >> 1;
    for (int e2 = threadIdx.x; e2 < ni * h2; e2 += blockDim.x) {
      const int ii = e2 / h2, xa = e2 - ii * h2, xb = xa + h2;
      const bool okb = xb < nx;
      const SpanEntry si = sp[i0 + ii];
      const float* ca = m + (long)(xlo + xa) * 3;
      const float* cb = m + (long)(xlo + (okb ? xb : xa)) * 3;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f;
      int y = si.start;
      for (; y + 8 <= si.end; y += 8) {
        float qa[8][3], qb[8][3];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const long ro = (long)(y + u) * d.P * 3;
          qa[u][0] = ca[ro + 0];
          qa[u][1] = ca[ro + 1];
          qa[u][2] = ca[ro + 2];
          qb[u][0] = cb[ro + 0];
          qb[u][1] = cb[ro + 1];
          qb[u][2] = cb[ro + 2];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float wy = span_weight(si, y + u, one_over_k);
          a0 += wy * qa[u][0];
          a1 += wy * qa[u][1];
          a2 += wy * qa[u][2];
          b0 += wy * qb[u][0];
          b1 += wy * qb[u][1];
          b2 += wy * qb[u][2];
        }
      }
      for (; y < si.end; ++y) {
        const float wy = span_weight(si, y, one_over_k);
        const long ro = (long)y * d.P * 3;
        a0 += wy * ca[ro + 0];
        a1 += wy * ca[ro + 1];
        a2 += wy * ca[ro + 2];
        b0 += wy * cb[ro + 0];
        b1 += wy * cb[ro + 1];
        b2 += wy * cb[ro + 2];
      }
      float* o = V + (ii * nx + xa) * 3;
      o[0] = a0; o[1] = a1; o[2] = a2;
      if (okb) {
        float* ob = V + (ii * nx + xb) * 3;
        ob[0] = b0; ob[1] = b1; ob[2] = b2;
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < ni * P.ps; e += blockDim.x) {
      const int ii = e / P.ps, j = e - ii * P.ps;
      const SpanEntry sj = sp[j];
      const float* row = V + (ii * nx - xlo) * 3;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
      for (int x = sj.start; x < sj.end; ++x) {
        const float wx = span_weight(sj, x, one_over_k);
        a0 += wx * row[x * 3 + 0];
        a1 += wx * row[x * 3 + 1];
        a2 += wx * row[x * 3 + 2];
      }
      const int px = (i0 + ii) * P.ps + j;
      u32x4 r = rng(seed, (uint32_t)px, (uint32_t)k, (uint32_t)(gimg0 + b), step, RNG_NOISE);
      float* o = rstore + P.roff + (long)px * 3;
      o[0] = (a0 + runif(r.x, -amp, amp)) + P.delta;
      o[1] = (a1 + runif(r.y, -amp, amp)) + P.delta;
      o[2] = (a2 + runif(r.z, -amp, amp)) + P.delta;
    }
    __syncthreads();
  }
}

// (A v2 that walked the union of a tile's row spans once per column — one load of each source row
// for all kResizeRT output rows, weights tabulated in LDS — measured 2.42 ms against v1's 1.73 ms on
// the first-pass flow, and was dropped.)
static_assert(kResizeGrid % 8 == 0, "k_eot_resize: XCD bands need a multiple of 8 workgroups");
void launch_eot_resize(const EotDims& d, const float* matched, const BoxPlace* place,
                       const SpanEntry* spans, uint64_t seed, int64_t step, int gimg0,
                       float* rstore, hipStream_t s, float noise_amp) {
  const size_t shm = (size_t)kResizeRT * d.P * 3 * sizeof(float) + (size_t)(d.B + 1) * sizeof(int);
  hipLaunchKernelGGL(k_eot_resize, dim3(kResizeGrid), dim3(256), shm, s, d, matched, place, spans,
                     seed, step, gimg0, rstore, noise_amp);
  PHX_LAUNCH_CHECK();
}

// padded, clipped R sample: inside the ps x ps block -> clip(pre), pad / outside -> -2
__device__ __forceinline__ float rread(const float* R, const BoxPlace& P, int yy, int xx, int c) {
  int ry = yy - P.pad, rx = xx - P.pad;
  if (yy < 0 || yy >= P.diag || xx < 0 || xx >= P.diag) return -2.0f;
  if (ry < 0 || ry >= P.ps || rx < 0 || rx >= P.ps) return -2.0f;
  float v = R[((long)ry * P.ps + rx) * 3 + c];
  return fminf(fmaxf(v, -1.0f), 1.0f);
}

// TF ImageProjectiveTransform bilinear sample (fill_value for out-of-range taps)
template <typename Read>
__device__ __forceinline__ float tf_bilinear(float x, float y, Read rd) {
  const float y_floor = floorf(y), x_floor = floorf(x);
  const float y_ceil = y_floor + 1.0f, x_ceil = x_floor + 1.0f;
  const int yf = (int)y_floor, xf = (int)x_floor, yc = (int)y_ceil, xc = (int)x_ceil;
  const float v_yf = (x_ceil - x) * rd(yf, xf) + (x - x_floor) * rd(yf, xc);
  const float v_yc = (x_ceil - x) * rd(yc, xf) + (x - x_floor) * rd(yc, xc);
  return (y_ceil - y) * v_yf + (y - y_floor) * v_yc;
}

__global__ __launch_bounds__(256) void k_eot_composite(EotDims d, const float* __restrict__ img_in,
                                                       const BoxPlace* __restrict__ place,
                                                       const float* __restrict__ rstore,
                                                       float* __restrict__ img_out,
                                                       int16_t* __restrict__ owner,
                                                       float* __restrict__ mask) {
  const long npx = (long)d.H * d.W;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  // when a workgroup's pixels lie in one image (always for the image sizes the models use), its
  // boxes' extents are staged in LDS once (a pixel walking vlist -> place per box paid two
  // dependent global round trips per box); otherwise each lane reads them itself
  const ListView L = lists_of(d, place);
  const long first = (long)blockIdx.x * blockDim.x;
  const long last = min(first + (long)blockDim.x, (long)d.B * npx) - 1;
  const bool staged = first / npx == last / npx;
  __shared__ int s_sl[PHX_MAX_OUT], s_y0[PHX_MAX_OUT], s_x0[PHX_MAX_OUT], s_dg[PHX_MAX_OUT];
  if (staged) {
    const int b0 = (int)(first / npx);
    const int n0 = L.img_n[b0], f0 = L.img_first[b0];  // <= d.maxb <= PHX_MAX_OUT (launcher)
    for (int q = threadIdx.x; q < n0; q += blockDim.x) {
      const int sl = L.vlist[f0 + q];
      s_sl[q] = sl;
      s_y0[q] = place[sl].ymin;
      s_x0[q] = place[sl].xmin;
      s_dg[q] = place[sl].diag;
    }
    __syncthreads();
  }
  if (idx >= (long)d.B * npx) return;
  const int b = (int)(idx / npx);
  const int n = L.img_n[b], f = L.img_first[b];
  const int p = (int)(idx % npx);
  const int y = p / d.W, x = p % d.W;
  const float* ip = img_in + idx * 3;
  float v[3] = {ip[0], ip[1], ip[2]};
  int16_t own[3] = {-1, -1, -1};
  bool covered = false;
  for (int q = 0; q < n; ++q) {
    int sl, y0, x0, dg;
    if (staged) {
      sl = s_sl[q]; y0 = s_y0[q]; x0 = s_x0[q]; dg = s_dg[q];
    } else {
      sl = L.vlist[f + q]; y0 = place[sl].ymin; x0 = place[sl].xmin; dg = place[sl].diag;
    }
    const int qy = y - y0, qx = x - x0;
    if (qy < 0 || qy >= dg || qx < 0 || qx >= dg) continue;
    const BoxPlace& P = place[sl];
    covered = true;
    const float ox = (float)qx, oy = (float)qy;
    const float proj = 0.0f * ox + 0.0f * oy + 1.0f;
    const float inx = (P.fwd[0] * ox + P.fwd[1] * oy + P.fwd[2]) / proj;
    const float iny = (P.fwd[3] * ox + P.fwd[4] * oy + P.fwd[5]) / proj;
    const float* R = rstore + P.roff;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float r = tf_bilinear(inx, iny, [&](int yy, int xx) { return rread(R, P, yy, xx, c); });
      if (r < -1.0f) {
        v[c] = fminf(fmaxf(v[c], -1.0f), 1.0f);
      } else {
        v[c] = fminf(fmaxf(r, -1.0f), 1.0f);
        own[c] = (int16_t)(sl % d.maxb);
      }
    }
  }
  float* op = img_out + idx * 3;
  if (mask) {
    float* mp = mask + idx * 3;
    mp[0] = covered ? ip[0] - v[0] : 0.f;
    mp[1] = covered ? ip[1] - v[1] : 0.f;
    mp[2] = covered ? ip[2] - v[2] : 0.f;
  }
  op[0] = v[0]; op[1] = v[1]; op[2] = v[2];
  if (owner) {
    owner[idx * 3 + 0] = own[0];
    owner[idx * 3 + 1] = own[1];
    owner[idx * 3 + 2] = own[2];
  }
}

// v2: the workgroup first keeps only its image's boxes whose square meets the workgroup's pixel
// rectangle (wave 0, ballot compaction: the boxes stay in paste order), so a pixel walks the few
// boxes that can cover it instead of all of them (the first-pass flow pastes ~90 per image);
// a box that covers none of the workgroup's pixels changes none of them: bit-identical to v1
__global__ __launch_bounds__(256) void k_eot_composite2(EotDims d, const float* __restrict__ img_in,
                                                        const BoxPlace* __restrict__ place,
                                                        const float* __restrict__ rstore,
                                                        float* __restrict__ img_out,
                                                        int16_t* __restrict__ owner,
                                                        float* __restrict__ mask) {
  const long npx = (long)d.H * d.W;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const ListView L = lists_of(d, place);
  const long first = (long)blockIdx.x * blockDim.x;
  const long last = min(first + (long)blockDim.x, (long)d.B * npx) - 1;
  const bool staged = first / npx == last / npx;
  __shared__ int s_sl[PHX_MAX_OUT], s_y0[PHX_MAX_OUT], s_x0[PHX_MAX_OUT], s_dg[PHX_MAX_OUT];
  __shared__ int s_n;
  if (staged && threadIdx.x < 64) {
    const int b0 = (int)(first / npx);
    const int n0 = L.img_n[b0], f0 = L.img_first[b0];  // <= d.maxb <= PHX_MAX_OUT (launcher)
    const int p0 = (int)(first % npx), p1 = (int)(last % npx);
    const int ry0 = p0 / d.W, ry1 = p1 / d.W;
    const int cx0 = ry0 == ry1 ? p0 % d.W : 0, cx1 = ry0 == ry1 ? p1 % d.W : d.W - 1;
    const int lane = threadIdx.x;
    int cnt = 0;
    for (int q0 = 0; q0 < n0; q0 += 64) {
      const int q = q0 + lane;
      int sl = 0, y0 = 0, x0 = 0, dg = 0;
      bool hit = false;
      if (q < n0) {
        sl = L.vlist[f0 + q];
        y0 = place[sl].ymin;
        x0 = place[sl].xmin;
        dg = place[sl].diag;
        hit = y0 <= ry1 && y0 + dg > ry0 && x0 <= cx1 && x0 + dg > cx0;
      }
      const unsigned long long bal = __ballot(hit);
      const int pos = cnt + __popcll(bal & ((1ull << lane) - 1ull));
      if (hit) {
        s_sl[pos] = sl;
        s_y0[pos] = y0;
        s_x0[pos] = x0;
        s_dg[pos] = dg;
      }
      cnt += __popcll(bal);
    }
    if (lane == 0) s_n = cnt;
  }
  __syncthreads();
  if (idx >= (long)d.B * npx) return;
  const int b = (int)(idx / npx);
  const int n = staged ? s_n : L.img_n[b], f = L.img_first[b];
  const int p = (int)(idx % npx);
  const int y = p / d.W, x = p % d.W;
  const float* ip = img_in + idx * 3;
  float v[3] = {ip[0], ip[1], ip[2]};
  int16_t own[3] = {-1, -1, -1};
  bool covered = false;
  for (int q = 0; q < n; ++q) {
    int sl, y0, x0, dg;
    if (staged) {
      sl = s_sl[q]; y0 = s_y0[q]; x0 = s_x0[q]; dg = s_dg[q];
    } else {
      sl = L.vlist[f + q]; y0 = place[sl].ymin; x0 = place[sl].xmin; dg = place[sl].diag;
    }
    const int qy = y - y0, qx = x - x0;
    if (qy < 0 || qy >= dg || qx < 0 || qx >= dg) continue;
    const BoxPlace& P = place[sl];
    covered = true;
    const float ox = (float)qx, oy = (float)qy;
    const float proj = 0.0f * ox + 0.0f * oy + 1.0f;
    const float inx = (P.fwd[0] * ox + P.fwd[1] * oy + P.fwd[2]) / proj;
    const float iny = (P.fwd[3] * ox + P.fwd[4] * oy + P.fwd[5]) / proj;
    const float* R = rstore + P.roff;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float r = tf_bilinear(inx, iny, [&](int yy, int xx) { return rread(R, P, yy, xx, c); });
      if (r < -1.0f) {
        v[c] = fminf(fmaxf(v[c], -1.0f), 1.0f);
      } else {
        v[c] = fminf(fmaxf(r, -1.0f), 1.0f);
        own[c] = (int16_t)(sl % d.maxb);
      }
    }
  }
  float* op = img_out + idx * 3;
  if (mask) {
    float* mp = mask + idx * 3;
    mp[0] = covered ? ip[0] - v[0] : 0.f;
    mp[1] = covered ? ip[1] - v[1] : 0.f;
    mp[2] = covered ? ip[2] - v[2] : 0.f;
  }
  op[0] = v[0]; op[1] = v[1]; op[2] = v[2];
  if (owner) {
    owner[idx * 3 + 0] = own[0];
    owner[idx * 3 + 1] = own[1];
    owner[idx * 3 + 2] = own[2];
  }
}

void launch_eot_composite(const EotDims& d, const float* img_in, const BoxPlace* place,
                          const float* rstore, float* img_out, int16_t* owner, hipStream_t s,
                          float* mask) {
  long n = (long)d.B * d.H * d.W;
  if (d.maxb > PHX_MAX_OUT) throw std::runtime_error("eot composite: more box slots than PHX_MAX_OUT");
  if (eot_v1())
    hipLaunchKernelGGL(k_eot_composite, dim3(cdiv(n, 256)), dim3(256), 0, s, d, img_in, place, rstore,
                       img_out, owner, mask);
  else
    hipLaunchKernelGGL(k_eot_composite2, dim3(cdiv(n, 256)), dim3(256), 0, s, d, img_in, place, rstore,
                       img_out, owner, mask);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
// dR_pre[i,j,c] = [-1 <= pre <= 1] * bilinear(inverse transform, G_k, fill 0) at padded
// (i+pad, j+pad), where G_k = dimg restricted to pixels owned by box k.
__global__ __launch_bounds__(256) void k_eot_rot_bwd(EotDims d, const float* __restrict__ dimg,
                                                     const int16_t* __restrict__ owner,
                                                     const BoxPlace* __restrict__ place,
                                                     const float* __restrict__ rstore,
                                                     float* __restrict__ dstore) {
  const ListView L = lists_of(d, place);
  const int nv = *L.nvalid, total = *L.total_chunks;
  for (int item = blockIdx.x; item < total; item += gridDim.x) {
    const int v = find_box(L.cprefix, nv, item);
    const int sl = L.vlist[v];
    const BoxPlace P = place[sl];
    const int b = sl / d.maxb, k = sl % d.maxb;
    const int px = (item - L.cprefix[v]) * 256 + threadIdx.x;
    if (px >= P.ps * P.ps) continue;
    const int i = px / P.ps, j = px % P.ps;
    const float ox = (float)(j + P.pad), oy = (float)(i + P.pad);
    const float proj = 0.0f * ox + 0.0f * oy + 1.0f;
    const float inx = (P.inv[0] * ox + P.inv[1] * oy + P.inv[2]) / proj;
    const float iny = (P.inv[3] * ox + P.inv[4] * oy + P.inv[5]) / proj;
    const float* R = rstore + P.roff + (long)px * 3;
    float* o = dstore + P.roff + (long)px * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float g = tf_bilinear(inx, iny, [&](int yy, int xx) -> float {
        if (yy < 0 || yy >= P.diag || xx < 0 || xx >= P.diag) return 0.0f;
        long e = (((long)b * d.H + (P.ymin + yy)) * d.W + (P.xmin + xx)) * 3 + c;
        return owner[e] == k ? dimg[e] : 0.0f;
      });
      float pre = R[c];
      o[c] = (pre >= -1.0f && pre <= 1.0f) ? g : 0.0f;
    }
  }
}

void launch_eot_rot_bwd(const EotDims& d, const float* dimg, const int16_t* owner,
                        const BoxPlace* place, const float* rstore, float* dstore,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_eot_rot_bwd, dim3(kBoxGrid), dim3(256), 0, s, d, dimg, owner, place, rstore,
                     dstore);
  PHX_LAUNCH_CHECK();
}

// Exact adjoint of the antialiased resize, separable: per box U[i][x] = sum_j Wc[j,x] dR[i,j]
// (rows kernel, work items of kResizeRT rows, U rows of valid box v at tprefix[v]*kResizeRT*P*3 of
// the row buffer), then per source pixel dmatched[y,x] = sum over the image's boxes of
// sum_i Wr[i,y] U[i][x] (cols kernel, lanes along x: coalesced U rows).
// output indices whose span may contain source index `src` (conservative, clamped to [0, ps))
__device__ __forceinline__ void adj_range(int src, float inv_scale, float ks, int ps, int* lo, int* hi) {
  *lo = max((int)floorf(((float)src - ks - 0.5f) / inv_scale - 0.5f) - 1, 0);
  *hi = min((int)ceilf(((float)src + ks + 1.5f) / inv_scale - 0.5f) + 1, ps - 1);
}

__global__ __launch_bounds__(256) void k_eot_resize_bwd_rows(EotDims d, const BoxPlace* __restrict__ place,
                                                             const SpanEntry* __restrict__ spans,
                                                             const float* __restrict__ dstore,
                                                             float* __restrict__ tstore) {
  const ListView L = lists_of(d, place);
  const int nv = *L.nvalid, total = L.tprefix[nv];
  for (int item = blockIdx.x; item < total; item += gridDim.x) {
    const int v = find_box(L.tprefix, nv, item);
    const int sl = L.vlist[v];
    const BoxPlace P = place[sl];
    const int i0 = (item - L.tprefix[v]) * kResizeRT;
    const int ni = min(kResizeRT, P.ps - i0);
    const SpanEntry* sp = spans + (long)sl * d.span_stride;
    const float scale = (float)P.ps / (float)d.P;
    const float inv_scale = (float)(1.0 / (double)scale);
    const float ks = fmaxf(inv_scale, 1.0f);
    const float one_over_k = 1.0f / ks;
    const float* D = dstore + P.roff;
    float* U = tstore + (long)L.tprefix[v] * kResizeRT * d.P * 3;
    for (int e = threadIdx.x; e < ni * d.P; e += blockDim.x) {
      const int ii = e / d.P, x = e - ii * d.P;
      const int i = i0 + ii;
      int jlo, jhi;
      adj_range(x, inv_scale, ks, P.ps, &jlo, &jhi);
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
      for (int j = jlo; j <= jhi; ++j) {
        const SpanEntry sj = sp[j];
        if (x < sj.start || x >= sj.end) continue;
        const float w = span_weight(sj, x, one_over_k);
        const float* g = D + ((long)i * P.ps + j) * 3;
        a0 += w * g[0];
        a1 += w * g[1];
        a2 += w * g[2];
      }
      float* o = U + ((long)i * d.P + x) * 3;
      o[0] = a0; o[1] = a1; o[2] = a2;
    }
  }
}

// PX source pixels per lane, P/PX apart in one row: they share the row's boxes, spans and weights,
// and their U loads are independent (PX chains of loads in flight per lane instead of one)
template <int PX>
__global__ __launch_bounds__(256) void k_eot_resize_bwd_cols(EotDims d, const BoxPlace* __restrict__ place,
                                                             const SpanEntry* __restrict__ spans,
                                                             const float* __restrict__ tstore,
                                                             float* __restrict__ dmatched) {
  const int b = blockIdx.y;
  const long npx = (long)d.P * d.P;
  const int pw = d.P / PX;  // lanes per row
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const ListView L = lists_of(d, place);
  const int n = L.img_n[b], f = L.img_first[b];  // <= d.maxb <= PHX_MAX_OUT (launcher)
  // the image's boxes, resolved once per workgroup (a lane walking vlist -> place -> spans per box
  // paid two dependent global round trips per box before its own loads)
  __shared__ int s_ps[PHX_MAX_OUT];
  __shared__ long s_span[PHX_MAX_OUT], s_u[PHX_MAX_OUT];
  __shared__ float s_inv[PHX_MAX_OUT], s_ks[PHX_MAX_OUT], s_ok[PHX_MAX_OUT];
  for (int q = threadIdx.x; q < n; q += blockDim.x) {
    const int v = f + q;
    const int sl = L.vlist[v];
    const int ps = place[sl].ps;
    const float scale = (float)ps / (float)d.P;
    const float inv_scale = (float)(1.0 / (double)scale);
    const float ks = fmaxf(inv_scale, 1.0f);
    s_ps[q] = ps;
    s_span[q] = (long)sl * d.span_stride;
    s_u[q] = (long)L.tprefix[v] * kResizeRT * d.P * 3;
    s_inv[q] = inv_scale;
    s_ks[q] = ks;
    s_ok[q] = 1.0f / ks;
  }
  __syncthreads();
  if (p >= (long)d.P * pw) return;
  const int y = (int)(p / pw), x0 = (int)(p % pw);
  float a[PX][3];
#pragma unroll
  for (int k = 0; k < PX; ++k) a[k][0] = a[k][1] = a[k][2] = 0.f;
  for (int q = 0; q < n; ++q) {
    const SpanEntry* sp = spans + s_span[q];
    const float one_over_k = s_ok[q];
    int ilo, ihi;
    adj_range(y, s_inv[q], s_ks[q], s_ps[q], &ilo, &ihi);
    const float* U = tstore + s_u[q] + (long)x0 * 3;
    for (int i = ilo; i <= ihi; ++i) {
      const SpanEntry si = sp[i];
      if (y < si.start || y >= si.end) continue;
      const float wy = span_weight(si, y, one_over_k);
      const float* g = U + (long)i * d.P * 3;
      float v[PX][3];
#pragma unroll
      for (int k = 0; k < PX; ++k) {
        v[k][0] = g[(long)k * pw * 3 + 0];
        v[k][1] = g[(long)k * pw * 3 + 1];
        v[k][2] = g[(long)k * pw * 3 + 2];
      }
#pragma unroll
      for (int k = 0; k < PX; ++k) {
        a[k][0] += wy * v[k][0];
        a[k][1] += wy * v[k][1];
        a[k][2] += wy * v[k][2];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < PX; ++k) {
    float* o = dmatched + ((long)b * npx + (long)y * d.P + x0 + (long)k * pw) * 3;
    o[0] = a[k][0]; o[1] = a[k][1]; o[2] = a[k][2];
  }
}

// v2 rows: the work item's kResizeRT rows of dR and the box's spans staged in LDS first (v1 read
// every dR value from memory once per output column whose span holds it); same sums, same order
__global__ __launch_bounds__(256) void k_eot_resize_bwd_rows2(EotDims d, const BoxPlace* __restrict__ place,
                                                              const SpanEntry* __restrict__ spans,
                                                              const float* __restrict__ dstore,
                                                              float* __restrict__ tstore) {
  extern __shared__ float sh_rows[];  // [kResizeRT][ps][3] dR rows, then [ps] spans
  const ListView L = lists_of(d, place);
  const int nv = *L.nvalid, total = L.tprefix[nv];
  for (int item = blockIdx.x; item < total; item += gridDim.x) {
    const int v = find_box(L.tprefix, nv, item);
    const int sl = L.vlist[v];
    const BoxPlace P = place[sl];
    const int i0 = (item - L.tprefix[v]) * kResizeRT;
    const int ni = min(kResizeRT, P.ps - i0);
    const SpanEntry* sp = spans + (long)sl * d.span_stride;
    const float scale = (float)P.ps / (float)d.P;
    const float inv_scale = (float)(1.0 / (double)scale);
    const float ks = fmaxf(inv_scale, 1.0f);
    const float one_over_k = 1.0f / ks;
    const float* D = dstore + P.roff + (long)i0 * P.ps * 3;
    float* Dl = sh_rows;
    SpanEntry* Sl = reinterpret_cast<SpanEntry*>(sh_rows + (long)kResizeRT * d.span_stride * 3);
    for (int e = threadIdx.x; e < ni * P.ps * 3; e += blockDim.x) Dl[e] = D[e];
    for (int j = threadIdx.x; j < P.ps; j += blockDim.x) Sl[j] = sp[j];
    __syncthreads();
    float* U = tstore + (long)L.tprefix[v] * kResizeRT * d.P * 3;
    for (int e = threadIdx.x; e < ni * d.P; e += blockDim.x) {
      const int ii = e / d.P, x = e - ii * d.P;
      const int i = i0 + ii;
      int jlo, jhi;
      adj_range(x, inv_scale, ks, P.ps, &jlo, &jhi);
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
      for (int j = jlo; j <= jhi; ++j) {
        const SpanEntry sj = Sl[j];
        if (x < sj.start || x >= sj.end) continue;
        const float w = span_weight(sj, x, one_over_k);
        const float* g = Dl + ((long)ii * P.ps + j) * 3;
        a0 += w * g[0];
        a1 += w * g[1];
        a2 += w * g[2];
      }
      float* o = U + ((long)i * d.P + x) * 3;
      o[0] = a0; o[1] = a1; o[2] = a2;
    }
    __syncthreads();
  }
}

// v2 cols: a lane owns one source column and RB consecutive source rows; per box it walks the
// output rows whose spans meet its rows once, loading U[i][x] once and adding it to every row of
// the block inside span(i) — each dmatched value gets the same terms in the same order (boxes
// ascending, then i ascending) as v1 with about 2 * scale / (RB / scale + 2) times fewer U loads
template <int RB>
__global__ __launch_bounds__(256) void k_eot_resize_bwd_cols2(EotDims d, const BoxPlace* __restrict__ place,
                                                              const SpanEntry* __restrict__ spans,
                                                              const float* __restrict__ tstore,
                                                              float* __restrict__ dmatched) {
  const int b = blockIdx.z;
  const long npx = (long)d.P * d.P;
  const ListView L = lists_of(d, place);
  const int n = L.img_n[b], f = L.img_first[b];  // <= d.maxb <= PHX_MAX_OUT (launcher)
  __shared__ int s_ps[PHX_MAX_OUT];
  __shared__ long s_span[PHX_MAX_OUT], s_u[PHX_MAX_OUT];
  __shared__ float s_inv[PHX_MAX_OUT], s_ks[PHX_MAX_OUT], s_ok[PHX_MAX_OUT];
  for (int q = threadIdx.x; q < n; q += blockDim.x) {
    const int v = f + q;
    const int sl = L.vlist[v];
    const int ps = place[sl].ps;
    const float scale = (float)ps / (float)d.P;
    const float inv_scale = (float)(1.0 / (double)scale);
    const float ks = fmaxf(inv_scale, 1.0f);
    s_ps[q] = ps;
    s_span[q] = (long)sl * d.span_stride;
    s_u[q] = (long)L.tprefix[v] * kResizeRT * d.P * 3;
    s_inv[q] = inv_scale;
    s_ks[q] = ks;
    s_ok[q] = 1.0f / ks;
  }
  __syncthreads();
  const int x = (int)blockIdx.x * 64 + (int)(threadIdx.x & 63);
  const int y0 = ((int)blockIdx.y * 4 + (int)(threadIdx.x >> 6)) * RB;
  if (x >= d.P || y0 >= d.P) return;
  const int nr = min(RB, d.P - y0);
  float a[RB][3];
#pragma unroll
  for (int r = 0; r < RB; ++r) a[r][0] = a[r][1] = a[r][2] = 0.f;
  for (int q = 0; q < n; ++q) {
    const SpanEntry* sp = spans + s_span[q];
    const float one_over_k = s_ok[q];
    int ilo, ihi, t0, t1;
    adj_range(y0, s_inv[q], s_ks[q], s_ps[q], &ilo, &t0);
    adj_range(y0 + nr - 1, s_inv[q], s_ks[q], s_ps[q], &t1, &ihi);
    const float* U = tstore + s_u[q] + (long)x * 3;
    for (int i = ilo; i <= ihi; i += 4) {
      // four output rows' loads in flight (clamped to ihi: valid rows of the box), added in order
      SpanEntry si[4];
      float g[4][3];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int iu = min(i + u, ihi);
        si[u] = sp[iu];
        const float* gp = U + (long)iu * d.P * 3;
        g[u][0] = gp[0];
        g[u][1] = gp[1];
        g[u][2] = gp[2];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (i + u > ihi) break;
        if (si[u].end <= y0 || si[u].start >= y0 + nr) continue;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const int y = y0 + r;
          if (y < si[u].start || y >= si[u].end) continue;
          const float wy = span_weight(si[u], y, one_over_k);
          a[r][0] += wy * g[u][0];
          a[r][1] += wy * g[u][1];
          a[r][2] += wy * g[u][2];
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    if (r >= nr) continue;
    float* o = dmatched + ((long)b * npx + (long)(y0 + r) * d.P + x) * 3;
    o[0] = a[r][0]; o[1] = a[r][1]; o[2] = a[r][2];
  }
}

void launch_eot_resize_bwd(const EotDims& d, const BoxPlace* place, const SpanEntry* spans,
                           const float* dstore, float* tstore, float* dmatched, hipStream_t s) {
  if (d.maxb > PHX_MAX_OUT) throw std::runtime_error("eot resize backward: more box slots than PHX_MAX_OUT");
  if (!eot_v1()) {
    const size_t shm = (size_t)kResizeRT * d.span_stride * 3 * sizeof(float) + (size_t)d.span_stride * sizeof(SpanEntry);
    static const size_t cap = [] {  // the dynamic LDS limit raised to what 160 KB leaves (once)
      hipFuncAttributes fa{};
      if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_eot_resize_bwd_rows2)) != hipSuccess) return (size_t)0;
      const size_t c = 160 * 1024 - fa.sharedSizeBytes;
      return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_eot_resize_bwd_rows2),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)c) == hipSuccess ? c : (size_t)0;
    }();
    if (shm > cap) throw std::runtime_error("eot resize backward: span rows exceed the LDS");
    hipLaunchKernelGGL(k_eot_resize_bwd_rows2, dim3(kBoxGrid), dim3(256), shm, s, d, place, spans, dstore, tstore);
    PHX_LAUNCH_CHECK();
    constexpr int RB = 16;
    hipLaunchKernelGGL(k_eot_resize_bwd_cols2<RB>, dim3(cdiv(d.P, 64), cdiv(d.P, 4 * RB), d.B), dim3(256), 0, s, d,
                       place, spans, tstore, dmatched);
    PHX_LAUNCH_CHECK();
    return;
  }
  hipLaunchKernelGGL(k_eot_resize_bwd_rows, dim3(kBoxGrid), dim3(256), 0, s, d, place, spans, dstore,
                     tstore);
  PHX_LAUNCH_CHECK();
  if (d.P % 4 == 0)
    hipLaunchKernelGGL(k_eot_resize_bwd_cols<4>, dim3(cdiv((long)d.P * d.P / 4, 256), d.B), dim3(256), 0, s, d,
                       place, spans, tstore, dmatched);
  else
    hipLaunchKernelGGL(k_eot_resize_bwd_cols<1>, dim3(cdiv((long)d.P * d.P, 256), d.B), dim3(256), 0, s, d,
                       place, spans, tstore, dmatched);
  PHX_LAUNCH_CHECK();
}

long eot_resize_scratch_floats(const EotDims& d) {
  const long tiles = (d.span_stride + kResizeRT - 1) / kResizeRT;
  return (long)d.B * d.maxb * tiles * kResizeRT * d.P * 3;
}

// brightness-matcher backward per pixel: returns d(print output) for the 3 channels given
// dmatched and mean(dYc); also the pixel's dYc contribution.
struct MatchBwd {
  float dp[3];
  float dyc;
};
__device__ __forceinline__ MatchBwd match_bwd_px(const float* p, float mus, float mut,
                                                 const float* dm, float mean_dyc) {
  Yuv s = rgb2yuv((p[0] + 1.0f) * kTo01, (p[1] + 1.0f) * kTo01, (p[2] + 1.0f) * kTo01);
  float yc = (s.y - mus) + mut;
  float yp = fminf(fmaxf(yc, 0.0f), 1.0f);
  float rgb[3] = {yp + 1.13988303f * s.v, yp + -0.394642334f * s.u + -0.58062185f * s.v,
                  yp + 2.03206185f * s.u};
  float drgb[3];
#pragma unroll
  for (int c = 0; c < 3; ++c)
    drgb[c] = (rgb[c] >= 0.0f && rgb[c] <= 1.0f) ? dm[c] * kBack : 0.0f;
  float dyp = drgb[0] + drgb[1] + drgb[2];
  float du = -0.394642334f * drgb[1] + 2.03206185f * drgb[2];
  float dv = 1.13988303f * drgb[0] + -0.58062185f * drgb[1];
  float dyc = (yc >= 0.0f && yc <= 1.0f) ? dyp : 0.0f;
  float dy = dyc - mean_dyc;  // d/dY through Y - mean(Y)
  MatchBwd o;
  o.dyc = dyc;
  // d s_c = dY*ky_c + dU*ku_c + dV*kv_c ; dp = ds * 127/255
  o.dp[0] = (dy * 0.299f + du * -0.14714119f + dv * 0.61497538f) * kTo01;
  o.dp[1] = (dy * 0.587f + du * -0.28886916f + dv * -0.51496512f) * kTo01;
  o.dp[2] = (dy * 0.114f + du * 0.43601035f + dv * -0.10001026f) * kTo01;
  return o;
}

__global__ __launch_bounds__(256) void k_eot_dyc_sum(EotDims d, const float* __restrict__ patch,
                                                     const ImgParams* __restrict__ img,
                                                     const float* __restrict__ ymean,
                                                     const float* __restrict__ dmatched,
                                                     double* __restrict__ dsum) {
  const int b = blockIdx.y;
  const long npx = (long)d.P * d.P;
  const ImgParams ip = img[b];
  double acc = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < npx;
       i += (long)gridDim.x * blockDim.x) {
    float p[3];
    for (int c = 0; c < 3; ++c) p[c] = print_px(patch, ip, i * 3 + c, c, true);
    MatchBwd mb = match_bwd_px(p, ymean[b * 2], ymean[b * 2 + 1],
                               dmatched + ((long)b * npx + i) * 3, 0.0f);
    acc += mb.dyc;
  }
  __shared__ double sh[256];
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) dsum[(long)b * gridDim.x + blockIdx.x] = sh[0];
}

__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__global__ __launch_bounds__(256) void k_eot_patch_grad(EotDims d, const float* __restrict__ patch,
                                                        const ImgParams* __restrict__ img,
                                                        const float* __restrict__ ymean,
                                                        const float* __restrict__ dmatched,
                                                        const double* __restrict__ dsum, int chunks,
                                                        int add_tv, float* __restrict__ grad) {
  extern __shared__ float s_mdyc[];  // [B] mean dYc per image, folded once per workgroup
  const long npx = (long)d.P * d.P;
  for (int b = threadIdx.x; b < d.B; b += blockDim.x) {
    double s = 0.0;
    for (int k = 0; k < chunks; ++k) s += dsum[(long)b * chunks + k];
    s_mdyc[b] = (float)(s / (double)npx);
  }
  __syncthreads();
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npx) return;
  float g[3] = {0.f, 0.f, 0.f};
  for (int b = 0; b < d.B; ++b) {
    const float mean_dyc = s_mdyc[b];
    const ImgParams ip = img[b];
    float p[3], pre[3];
    for (int c = 0; c < 3; ++c) {
      pre[c] = ip.w[c] * patch[i * 3 + c] + ip.b[c];
      p[c] = fminf(fmaxf(pre[c], -1.0f), 1.0f);
    }
    MatchBwd mb = match_bwd_px(p, ymean[b * 2], ymean[b * 2 + 1],
                               dmatched + ((long)b * npx + i) * 3, mean_dyc);
    for (int c = 0; c < 3; ++c)
      if (pre[c] >= -1.0f && pre[c] <= 1.0f) g[c] += mb.dp[c] * ip.w[c];
  }
  if (add_tv) {
    // d/dp of 1e-5 * (sum |p[y+1]-p[y]| + sum |p[x+1]-p[x]|), abs grad = sign
    const int y = (int)(i / d.P), x = (int)(i % d.P);
    for (int c = 0; c < 3; ++c) {
      const float v = patch[i * 3 + c];
      float t = 0.f;
      if (y > 0) t += sgnf(v - patch[(i - d.P) * 3 + c]);
      if (y < d.P - 1) t -= sgnf(patch[(i + d.P) * 3 + c] - v);
      if (x > 0) t += sgnf(v - patch[(i - 1) * 3 + c]);
      if (x < d.P - 1) t -= sgnf(patch[(i + 1) * 3 + c] - v);
      g[c] += 1e-5f * t;
    }
  }
  grad[i * 3 + 0] = g[0];
  grad[i * 3 + 1] = g[1];
  grad[i * 3 + 2] = g[2];
}

void launch_eot_patch_bwd(const EotDims& d, const float* patch, const ImgParams* img,
                          const float* ymean, const float* dmatched, double* dsum, float* grad,
                          bool add_tv, hipStream_t s) {
  hipLaunchKernelGGL(k_eot_dyc_sum, dim3(kYChunks, d.B), dim3(256), 0, s, d, patch, img, ymean,
                     dmatched, dsum);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_eot_patch_grad, dim3(cdiv((long)d.P * d.P, 256)), dim3(256),
                     (size_t)d.B * sizeof(float), s, d, patch,
                     img, ymean, dmatched, dsum, kYChunks, add_tv ? 1 : 0, grad);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// total variation (tf.image.total_variation on a 3-D image, sum over everything)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tv_part(const float* __restrict__ p, int P,
                                                 double* __restrict__ part) {
  const long n = (long)P * P * 3;
  double acc = 0.0;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (long)gridDim.x * blockDim.x) {
    long px = e / 3;
    int y = (int)(px / P), x = (int)(px % P);
    float v = p[e];
    if (y + 1 < P) acc += fabsf(p[e + (long)P * 3] - v);
    if (x + 1 < P) acc += fabsf(p[e + 3] - v);
  }
  __shared__ double sh[256];
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

__global__ void k_tv_final(const double* __restrict__ part, int n, float* __restrict__ metrics,
                           int add) {
  __shared__ double sh[64];
  double a = 0.0;
  for (int i = threadIdx.x; i < n; i += 64) a += part[i];
  sh[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x) return;
  double s = 0.0;
  for (int i = 0; i < 64; ++i) s += sh[i];
  // TV is a global term: only the rank that adds it to the loss reports it, so the metric row
  // stays SUM-all-reducible over data-parallel ranks
  if (add) {
    metrics[PHX_M_TV] = (float)s;
    metrics[PHX_M_LOSS] += 1e-5f * (float)s;
  }
}

void launch_tv(const float* patch, int P, double* scratch, float* metrics, bool add_to_loss,
               hipStream_t s) {
  if (!add_to_loss) return;  // neither the loss term nor the metric on this rank
  const int nb = 256;
  hipLaunchKernelGGL(k_tv_part, dim3(nb), dim3(256), 0, s, patch, P, scratch);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_tv_final, dim3(1), dim3(64), 0, s, scratch, nb, metrics, add_to_loss ? 1 : 0);
  PHX_LAUNCH_CHECK();
}

__global__ void k_eot_count(EotDims d, const BoxPlace* __restrict__ place, float* metrics) {
  if (threadIdx.x) return;
  const ListView L = lists_of(d, place);
  metrics[PHX_M_NBOX] = (float)*L.nvalid;
}

void launch_eot_count(const EotDims& d, const BoxPlace* place, float* metrics, hipStream_t s) {
  hipLaunchKernelGGL(k_eot_count, dim3(1), dim3(64), 0, s, d, place, metrics);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// Keras Adam (ResourceApplyAdam) + constraints: params = [patch | scale]
//   alpha = lr * sqrt(1 - b2^t) / (1 - b1^t); m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2)
//   var -= m * alpha / (sqrt(v) + eps); var = clip(var)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ params,
                                              const float* __restrict__ grad,
                                              float* __restrict__ m, float* __restrict__ v, long n,
                                              float alpha, long npatch) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float b1 = 0.9f, b2 = 0.999f, eps = 1e-7f;
  float g = grad[i];
  float mi = m[i], vi = v[i];
  mi += (g - mi) * (1.0f - b1);
  vi += (g * g - vi) * (1.0f - b2);
  m[i] = mi;
  v[i] = vi;
  float x = params[i] - (mi * alpha) / (sqrtf(vi) + eps);
  if (npatch >= 0) {  // the attacker's constraints (npatch < 0: plain Adam, the defender's U-Net)
    if (i < npatch)
      x = fminf(fmaxf(x, -1.0f), 1.0f);
    else
      x = fminf(fmaxf(x, 0.0f), 1.0f);
  }
  params[i] = x;
}

void launch_adam_clip(float* params, const float* grad, float* m, float* v, long n, float lr,
                      int64_t t, hipStream_t s) {
  // beta powers as Keras: pow(beta, t) in fp32
  const float b1p = powf(0.9f, (float)t), b2p = powf(0.999f, (float)t);
  const float alpha = lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
  hipLaunchKernelGGL(k_adam, dim3(cdiv(n, 256)), dim3(256), 0, s, params, grad, m, v, n, alpha,
                     (long)PHX_NPATCH_DEV);
  PHX_LAUNCH_CHECK();
}

void launch_adam(float* params, const float* grad, float* m, float* v, long n, float lr, int64_t t, hipStream_t s) {
  const float b1p = powf(0.9f, (float)t), b2p = powf(0.999f, (float)t);
  const float alpha = lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
  hipLaunchKernelGGL(k_adam, dim3(cdiv(n, 256)), dim3(256), 0, s, params, grad, m, v, n, alpha, -1L);
  PHX_LAUNCH_CHECK();
}

}  // namespace phx
