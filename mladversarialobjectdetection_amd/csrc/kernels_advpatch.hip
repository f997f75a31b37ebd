// kernels_advpatch.hip — the reference's inference-time patch compositor (adv_patch.py:16-201,
// AdversarialPatch.add_adv_to_img) as a batch of uint8 images on the GPU.
//
// Per box, in order (each box's brightness match sees the image as patched so far):
//   1. target Y mean: rescale the current image into out_h x out_w (cv2 INTER_LINEAR, 127-grey
//      letterbox) and sum the Y of cv2's RGB2YUV — an exact integer (k_ap_ysum, 64-bit atomics);
//   2. the printed patch brightness-matched (RGB2YUV, Y' = trunc(clip(Y - mean_src + mean_tgt)),
//      YUV2RGB), resized to the box's ph x pw (cv2 INTER_AREA down / INTER_CUBIC up), the noise
//      U(-0.01, 0.01) in the normalised space, back to uint8, written into the image (k_ap_paste).
// Every OpenCV operation is restated in its own arithmetic (oracle/adv_patch.py): 11-bit fixed-point
// resize weights, 14-bit fixed-point colour conversion, INTER_AREA's float32 cell sums in OpenCV's
// order; the numpy float64 steps run in double.  Multiplies and adds that OpenCV / numpy round
// separately are issued as __fmul_rn / __dmul_rn etc. so no fused multiply-add changes a result.
// Bounds: HBM-trivial (an inference-time compositor); the per-pixel work is integer ALU.
#include <cstdint>

#include "common.hpp"
#include "kernels.hpp"

namespace phx {

namespace {

__device__ __forceinline__ int descale14(int x) { return (x + (1 << 13)) >> 14; }
__device__ __forceinline__ int sat_u8(int x) { return x < 0 ? 0 : (x > 255 ? 255 : x); }

__device__ __forceinline__ int y_of(int r, int g, int b) { return descale14(r * 4899 + g * 9617 + b * 1868); }

// cv2.cvtColor RGB2YUV -> Y' replaced -> YUV2RGB for one printed-patch pixel
struct Match {
  double sm, tm;  // source / target Y means
  __device__ __forceinline__ void px(const uint8_t* p, int* out) const {
    const int r = p[0], g = p[1], b = p[2];
    const int y = sat_u8(y_of(r, g, b));
    const int delta = 128 << 14;
    const int v = sat_u8(descale14((r - y) * 14369 + delta));
    const int u = sat_u8(descale14((b - y) * 8061 + delta));
    double t = __dadd_rn(__dadd_rn((double)y, -sm), tm);
    t = t < 0.0 ? 0.0 : (t > 255.0 ? 255.0 : t);
    const int y2 = (int)t;  // astype(uint8): truncation
    out[2] = sat_u8(y2 + descale14((u - 128) * 33292));
    out[1] = sat_u8(y2 + descale14((u - 128) * -6472 + (v - 128) * -9519));
    out[0] = sat_u8(y2 + descale14((v - 128) * 18678));
  }
};

// saturate_cast<short>(float): round half to even
__device__ __forceinline__ int round_short(float x) { return (int)rintf(x); }

// INTER_LINEAR tap of destination index d (resize(): fx in float32 from a double expression)
__device__ __forceinline__ void lin_tap(int d, double scale, int ssize, bool clamp, int* s, int* w0, int* w1) {
  const float f0 = (float)__dadd_rn(__dmul_rn(__dadd_rn((double)d, 0.5), scale), -0.5);
  int sx = (int)floorf(f0);
  float f = __fadd_rn(f0, -(float)sx);
  if (clamp) {
    if (sx < 0) { f = 0.f; sx = 0; }
    if (sx >= ssize - 1) { f = 0.f; sx = ssize - 1; }
  }
  *s = sx;
  *w0 = round_short(__fmul_rn(__fadd_rn(1.f, -f), 2048.f));
  *w1 = round_short(__fmul_rn(f, 2048.f));
}

// interpolateCubic (A = -0.75), float32 with every operation rounded
__device__ __forceinline__ void cubic_coeffs(float x, int* w) {
  const float A = -0.75f;
  const float x1 = __fadd_rn(x, 1.f);
  float c0 = __fadd_rn(__fmul_rn(A, x1), -__fmul_rn(5.f, A));
  c0 = __fadd_rn(__fmul_rn(c0, x1), __fmul_rn(8.f, A));
  c0 = __fadd_rn(__fmul_rn(c0, x1), -__fmul_rn(4.f, A));
  float c1 = __fadd_rn(__fmul_rn(__fadd_rn(A, 2.f), x), -__fadd_rn(A, 3.f));
  c1 = __fadd_rn(__fmul_rn(__fmul_rn(c1, x), x), 1.f);
  const float y = __fadd_rn(1.f, -x);
  float c2 = __fadd_rn(__fmul_rn(__fadd_rn(A, 2.f), y), -__fadd_rn(A, 3.f));
  c2 = __fadd_rn(__fmul_rn(__fmul_rn(c2, y), y), 1.f);
  const float c3 = __fadd_rn(__fadd_rn(__fadd_rn(1.f, -c0), -c1), -c2);
  w[0] = round_short(__fmul_rn(c0, 2048.f));
  w[1] = round_short(__fmul_rn(c1, 2048.f));
  w[2] = round_short(__fmul_rn(c2, 2048.f));
  w[3] = round_short(__fmul_rn(c3, 2048.f));
}

__device__ __forceinline__ void cubic_tap(int d, double scale, int* s, int* w) {
  const float f0 = (float)__dadd_rn(__dmul_rn(__dadd_rn((double)d, 0.5), scale), -0.5);
  const int sx = (int)floorf(f0);
  *s = sx;
  cubic_coeffs(__fadd_rn(f0, -(float)sx), w);
}

// one INTER_AREA table entry walk (computeResizeAreaTab) for destination index d: calls
// f(source index, float alpha) in OpenCV's order
template <class F>
__device__ __forceinline__ void area_entries(int d, double scale, int ssize, F f) {
  const double fs1 = __dmul_rn((double)d, scale);
  const double fs2 = __dadd_rn(fs1, scale);
  const double cell = fmin(scale, __dadd_rn((double)ssize, -fs1));
  int s1 = (int)ceil(fs1), s2 = (int)floor(fs2);
  s2 = min(s2, ssize - 1);
  s1 = min(s1, s2);
  if (__dadd_rn((double)s1, -fs1) > 1e-3) f(s1 - 1, (float)(__dadd_rn((double)s1, -fs1) / cell));
  for (int s = s1; s < s2; ++s) f(s, (float)(1.0 / cell));
  if (__dadd_rn(fs2, -(double)s2) > 1e-3) f(s2, (float)(fmin(fmin(__dadd_rn(fs2, -(double)s2), 1.0), cell) / cell));
}

}  // namespace

// printed patch (adv_patch.py:40-58: (p + 127) >> 1 exactly) and the sum of its Y
__global__ __launch_bounds__(256) void k_ap_print(const uint8_t* __restrict__ raw, uint8_t* __restrict__ printed, int n,
                                                  unsigned long long* __restrict__ ysum) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  int y = 0;
  if (i < n) {
    int c[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      c[k] = (raw[3 * i + k] + 127) >> 1;
      printed[3 * i + k] = (uint8_t)c[k];
    }
    y = sat_u8(y_of(c[0], c[1], c[2]));
  }
  for (int o = 32; o > 0; o >>= 1) y += __shfl_xor(y, o);
  if ((threadIdx.x & 63) == 0 && y) atomicAdd(ysum, (unsigned long long)y);
}

// sum over the out_h x out_w rescaled image (AdversarialPatch.rescale) of RGB2YUV's Y, per image;
// the grey letterbox (127, 127, 127) has Y = 127: `grey` = 127 * its pixel count
__global__ __launch_bounds__(256) void k_ap_ysum(const uint8_t* __restrict__ img, int H, int W, int sh, int sw,
                                                 int mode, double sy, double sx, unsigned long long grey,
                                                 unsigned long long* __restrict__ ysum) {
  const int b = blockIdx.y;
  if (blockIdx.x == 0 && threadIdx.x == 0 && grey) atomicAdd(ysum + b, grey);
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  const uint8_t* im = img + (long)b * H * W * 3;
  int yv = 0;
  if (p < (long)sh * sw) {
    const int oy = (int)(p / sw), ox = (int)(p - (long)oy * sw);
    int c[3];
    if (mode == 0) {  // identity
#pragma unroll
      for (int k = 0; k < 3; ++k) c[k] = im[((long)oy * W + ox) * 3 + k];
    } else if (mode == 1) {  // exact 2x decimation: resize() runs INTER_AREA, (sum + 2) >> 2
      const long r0 = ((long)(2 * oy) * W + 2 * ox) * 3, r1 = r0 + (long)W * 3;
#pragma unroll
      for (int k = 0; k < 3; ++k) c[k] = (im[r0 + k] + im[r0 + 3 + k] + im[r1 + k] + im[r1 + 3 + k] + 2) >> 2;
    } else {  // INTER_LINEAR, fixed point
      int xs, xw0, xw1, ys, yw0, yw1;
      lin_tap(ox, sx, W, true, &xs, &xw0, &xw1);
      lin_tap(oy, sy, H, false, &ys, &yw0, &yw1);
      const int xs1 = min(xs + 1, W - 1);
      const int y0 = min(max(ys, 0), H - 1), y1 = min(max(ys + 1, 0), H - 1);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int s0 = im[((long)y0 * W + xs) * 3 + k] * xw0 + im[((long)y0 * W + xs1) * 3 + k] * xw1;
        const int s1 = im[((long)y1 * W + xs) * 3 + k] * xw0 + im[((long)y1 * W + xs1) * 3 + k] * xw1;
        c[k] = (((yw0 * (s0 >> 4)) >> 16) + ((yw1 * (s1 >> 4)) >> 16) + 2) >> 2;
      }
    }
    yv = sat_u8(y_of(c[0], c[1], c[2]));
  }
  for (int o = 32; o > 0; o >>= 1) yv += __shfl_xor(yv, o);
  if ((threadIdx.x & 63) == 0 && yv) atomicAdd(ysum + b, (unsigned long long)yv);
}

// one box per image: brightness match, resize, noise, paste (adv_patch.py:166-201)
__global__ __launch_bounds__(256) void k_ap_paste(uint8_t* __restrict__ img, int H, int W,
                                                  const uint8_t* __restrict__ printed, int P,
                                                  const ApBox* __restrict__ boxes, int slot,
                                                  const unsigned long long* __restrict__ ysum,
                                                  const unsigned long long* __restrict__ ysrc, double npix_t,
                                                  uint64_t seed,
                                                  int64_t step, int gimg0) {
  const int b = blockIdx.y;
  const ApBox bx = boxes[b];
  if (!bx.valid) return;
  const int ph = bx.ph, pw = bx.pw;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)ph * pw) return;
  const int py = (int)(p / pw), px = (int)(p - (long)py * pw);
  Match m;
  m.sm = (double)*ysrc / ((double)P * (double)P);
  m.tm = (double)ysum[b] / npix_t;
  int v[3];
  if (ph == P) {  // no resize
    m.px(printed + ((long)py * P + px) * 3, v);
  } else if (ph > P) {  // INTER_CUBIC upscale
    const double scale = 1.0 / ((double)ph / (double)P);
    int xs, ys, xw[4], yw[4];
    cubic_tap(px, scale, &xs, xw);
    cubic_tap(py, scale, &ys, yw);
    long acc[3] = {0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sy = min(max(ys - 1 + r, 0), P - 1);
      int row[3] = {0, 0, 0};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int sxk = min(max(xs - 1 + k, 0), P - 1);
        int q[3];
        m.px(printed + ((long)sy * P + sxk) * 3, q);
#pragma unroll
        for (int c = 0; c < 3; ++c) row[c] += q[c] * xw[k];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] += (long)row[c] * yw[r];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = sat_u8((int)((acc[c] + (1L << 21)) >> 22));
  } else if (P % ph == 0) {  // INTER_AREA, integer factor
    const int f = P / ph;
    int s[3] = {0, 0, 0};
    for (int i = 0; i < f; ++i)
      for (int j = 0; j < f; ++j) {
        int q[3];
        m.px(printed + ((long)(py * f + i) * P + px * f + j) * 3, q);
        s[0] += q[0]; s[1] += q[1]; s[2] += q[2];
      }
    if (f == 2) {
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = (s[c] + 2) >> 2;
    } else {
      const float sc = 1.f / (float)(f * f);
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = sat_u8((int)rintf(__fmul_rn((float)s[c], sc)));
    }
  } else {  // INTER_AREA, fractional cells: rows of float32 cell sums in OpenCV's order
    const double scale = 1.0 / ((double)ph / (double)P);
    float sum[3] = {0.f, 0.f, 0.f};
    bool first = true;
    area_entries(py, scale, P, [&](int sy, float beta) {
      float buf[3] = {0.f, 0.f, 0.f};
      area_entries(px, scale, P, [&](int sxx, float alpha) {
        int q[3];
        m.px(printed + ((long)sy * P + sxx) * 3, q);
#pragma unroll
        for (int c = 0; c < 3; ++c) buf[c] = __fadd_rn(buf[c], __fmul_rn((float)q[c], alpha));
      });
#pragma unroll
      for (int c = 0; c < 3; ++c) sum[c] = first ? __fmul_rn(beta, buf[c]) : __fadd_rn(sum[c], __fmul_rn(beta, buf[c]));
      first = false;
    });
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = sat_u8((int)rintf(sum[c]));
  }
  // get_transformed_patch's float64 tail (adv_patch.py:177-187) with U(-0.01, 0.01) noise per
  // element: element e = 3 * p + c, pair e >> 1 (words x, y for the even element, z, w for the odd)
  uint8_t* dst = img + (((long)b * H + bx.y + py) * W + bx.x + px) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const long e = 3 * p + c;
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)(e >> 1), (uint32_t)slot, (uint32_t)(gimg0 + b),
                                        (uint32_t)((uint64_t)step << 8) | (uint32_t)RNG_APNOISE},
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint64_t bits = (e & 1) ? (((uint64_t)r.z << 32) | r.w) : (((uint64_t)r.x << 32) | r.y);
    const double u = (double)(bits >> 11) * (1.0 / 9007199254740992.0);
    const double nz = __dadd_rn(-0.01, __dmul_rn(u, 0.02));
    double t = __dadd_rn((double)v[c], -127.0) / 128.0;
    t = __dadd_rn(t, nz);
    t = t < -1.0 ? -1.0 : (t > 1.0 ? 1.0 : t);
    t = __dadd_rn(__dmul_rn(t, 128.0), 127.0);
    t = t < 0.0 ? 0.0 : (t > 255.0 ? 255.0 : t);
    dst[c] = (uint8_t)(int)t;
  }
}

void launch_ap_print(const uint8_t* raw, uint8_t* printed, int P, unsigned long long* ysum, hipStream_t s) {
  const int n = P * P;
  PHX_HIP(hipMemsetAsync(ysum, 0, sizeof(unsigned long long), s));
  hipLaunchKernelGGL(k_ap_print, dim3(cdiv(n, 256)), dim3(256), 0, s, raw, printed, n, ysum);
  PHX_LAUNCH_CHECK();
}

void launch_ap_ysum(const uint8_t* img, int B, int H, int W, int out_h, int out_w, int sh, int sw,
                    unsigned long long* ysum, hipStream_t s) {
  PHX_HIP(hipMemsetAsync(ysum, 0, (size_t)B * sizeof(unsigned long long), s));
  const int mode = (sh == H && sw == W) ? 0 : (H == 2 * sh && W == 2 * sw) ? 1 : 2;
  const double sy = 1.0 / ((double)sh / (double)H), sx = 1.0 / ((double)sw / (double)W);
  const unsigned long long grey = 127ull * (unsigned long long)((long)out_h * out_w - (long)sh * sw);
  hipLaunchKernelGGL(k_ap_ysum, dim3(cdiv((long)sh * sw, 256), B), dim3(256), 0, s, img, H, W, sh, sw, mode, sy,
                     sx, grey, ysum);
  PHX_LAUNCH_CHECK();
}

void launch_ap_paste(uint8_t* img, int B, int H, int W, const uint8_t* printed, int P, const ApBox* boxes,
                     int max_pix, int slot, const unsigned long long* ysum, const unsigned long long* ysrc, int out_h,
                     int out_w, uint64_t seed, int64_t step, int gimg0, hipStream_t s) {
  if (max_pix <= 0) return;
  hipLaunchKernelGGL(k_ap_paste, dim3(cdiv(max_pix, 256), B), dim3(256), 0, s, img, H, W, printed, P, boxes, slot,
                     ysum, ysrc, (double)out_h * (double)out_w, seed, step, gimg0);
  PHX_LAUNCH_CHECK();
}

}  // namespace phx
