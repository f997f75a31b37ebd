// kernels_data.hip — the training input pipeline on the GPU.
//
// Reference: train_data_generator.py
//   * DataSequence._map_fn (:55-77): (x - mean_rgb) / stddev_rgb in float64, scale =
//     min(S_h/h, S_w/w), cv2.resize(image, [int(w*scale), int(h*scale)]) with the default
//     INTER_LINEAR, pasted at the top-left of a zero [S_h, S_w, 3] canvas;
//   * the train-set map chain (:201-204, :222-225): tf.image.random_flip_left_right ->
//     RandomFlip('horizontal') -> RandomContrast(.2) -> tf.image.random_brightness(.2) ->
//     clip [-1, 1].
//
// Design.  Both stages are HBM-bound byte/float streams (a 512² canvas is 3 MB of fp32 out per
// image); the reference does the first on the CPU per image (PIL decode + cv2 in a Python
// generator) and the second as four tf.data maps.  Here:
//   * k_letterbox: one launch per batch, grid (canvas float4 groups, B).  A lane owns 4
//     consecutive floats of the flattened [S_h*S_w*3] canvas (one 16-B store), so the write
//     stream — the dominant traffic — is fully coalesced; its bilinear taps gather uint8 source
//     bytes (the source is 4x smaller than the output and neighbouring lanes share taps in L2).
//     cv2 INTER_LINEAR semantics for CV_64F: half-pixel centres, fx = (float)((dx+.5)*sx-.5),
//     float weights, x taps clamped with the weight forced to 0 at the borders, y rows clamped
//     (no weight change) — restated in oracle/data.py.
//   * augmentation: per-image channel sums first (k_aug_sums: a workgroup reduces a chunk of one
//     image into fp64 partials [B][chunk][3]), then one fused pass (k_aug_apply) that folds the
//     partials into the image means (fixed order), reads the (possibly mirrored) source pixel
//     and writes clip((x - mean)*f + mean + delta, -1, 1).  The two flips compose into one
//     mirror decision per image; flips commute with the per-image-channel contrast.
#include <stdexcept>

#include "kernels.hpp"

namespace phx {

struct LbArgs {
  const uint8_t* src;
  const int64_t* offsets;  // [B] byte offset of image b in src
  const int32_t* dims;     // [B,2] (h, w)
  float mean[3], inv_std[3], std[3];
  int oh, ow;
  float* out;
};

__device__ __forceinline__ float lb_pix(const uint8_t* s, int w, int y, int x, int c, const LbArgs& a) {
  // (x - mean) / std of the uint8 sample (the reference divides in float64; fp32 here)
  return ((float)s[((long)y * w + x) * 3 + c] - a.mean[c]) / a.std[c];
}

__global__ __launch_bounds__(256) void k_letterbox(LbArgs a) {
  const int b = blockIdx.y;
  const long n4 = (long)a.oh * a.ow * 3 / 4;
  const long i4 = (long)blockIdx.x * 256 + threadIdx.x;
  if (i4 >= n4) return;
  const int h = a.dims[2 * b], w = a.dims[2 * b + 1];
  const uint8_t* s = a.src + a.offsets[b];
  // train_data_generator.py:67-71 (python floats = double; int() truncates)
  const double sc = fmin((double)a.ow / w, (double)a.oh / h);
  const int sh = (int)(h * sc), sw = (int)(w * sc);
  // cv2 resize: inv_scale = dsize/ssize, scale = 1/inv_scale
  const double scx = 1.0 / ((double)sw / w), scy = 1.0 / ((double)sh / h);
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long e = i4 * 4 + j;
    const int c = (int)(e % 3);
    const long p = e / 3;
    const int oy = (int)(p / a.ow), ox = (int)(p - (long)oy * a.ow);
    if (oy >= sh || ox >= sw) {
      v[j] = 0.f;
      continue;
    }
    float fx = (float)((ox + 0.5) * scx - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { sx = 0; fx = 0.f; }
    if (sx >= w - 1) { sx = w - 1; fx = 0.f; }
    const int sx1 = min(sx + 1, w - 1);
    float fy = (float)((oy + 0.5) * scy - 0.5);
    int sy = (int)floorf(fy);
    fy -= (float)sy;
    const int y0 = min(max(sy, 0), h - 1), y1 = min(max(sy + 1, 0), h - 1);
    const float ax0 = 1.f - fx, ay0 = 1.f - fy;
    const float r0 = lb_pix(s, w, y0, sx, c, a) * ax0 + lb_pix(s, w, y0, sx1, c, a) * fx;
    const float r1 = lb_pix(s, w, y1, sx, c, a) * ax0 + lb_pix(s, w, y1, sx1, c, a) * fx;
    v[j] = r0 * ay0 + r1 * fy;
  }
  reinterpret_cast<float4*>(a.out + (long)b * a.oh * a.ow * 3)[i4] = make_float4(v[0], v[1], v[2], v[3]);
}

// ow % 4 == 0: a lane owns 4 consecutive canvas pixels of one row (12 floats, three 16-B stores),
// so the row's y taps / weights and the image constants are computed once per lane and the
// channel loop is static (no per-element divisions)
__global__ __launch_bounds__(256) void k_letterbox_px4(LbArgs a) {
  const int b = blockIdx.y;
  const long nq = (long)a.oh * a.ow / 4;
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const int h = a.dims[2 * b], w = a.dims[2 * b + 1];
  const uint8_t* s = a.src + a.offsets[b];
  const double sc = fmin((double)a.ow / w, (double)a.oh / h);
  const int sh = (int)(h * sc), sw = (int)(w * sc);
  const long p0 = q * 4;
  const int oy = (int)(p0 / a.ow), ox0 = (int)(p0 - (long)oy * a.ow);
  float v[12];
  if (oy >= sh || ox0 >= sw) {
#pragma unroll
    for (int j = 0; j < 12; ++j) v[j] = 0.f;
  } else {
    const double scx = 1.0 / ((double)sw / w), scy = 1.0 / ((double)sh / h);
    float fy = (float)((oy + 0.5) * scy - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const int y0 = min(max(sy, 0), h - 1), y1 = min(max(sy + 1, 0), h - 1);
    const float ay0 = 1.f - fy;
    const uint8_t* r0p = s + (long)y0 * w * 3;
    const uint8_t* r1p = s + (long)y1 * w * 3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ox = ox0 + j;
      if (ox >= sw) {
        v[3 * j] = v[3 * j + 1] = v[3 * j + 2] = 0.f;
        continue;
      }
      float fx = (float)((ox + 0.5) * scx - 0.5);
      int sx = (int)floorf(fx);
      fx -= (float)sx;
      if (sx < 0) { sx = 0; fx = 0.f; }
      if (sx >= w - 1) { sx = w - 1; fx = 0.f; }
      const int sx1 = min(sx + 1, w - 1);
      const float ax0 = 1.f - fx;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float m = a.mean[c], sd = a.std[c];
        const float t00 = ((float)r0p[sx * 3 + c] - m) / sd, t01 = ((float)r0p[sx1 * 3 + c] - m) / sd;
        const float t10 = ((float)r1p[sx * 3 + c] - m) / sd, t11 = ((float)r1p[sx1 * 3 + c] - m) / sd;
        const float r0 = t00 * ax0 + t01 * fx;
        const float r1 = t10 * ax0 + t11 * fx;
        v[3 * j + c] = r0 * ay0 + r1 * fy;
      }
    }
  }
  float4* o = reinterpret_cast<float4*>(a.out + ((long)b * a.oh * a.ow + p0) * 3);
  o[0] = make_float4(v[0], v[1], v[2], v[3]);
  o[1] = make_float4(v[4], v[5], v[6], v[7]);
  o[2] = make_float4(v[8], v[9], v[10], v[11]);
}

void launch_letterbox(const uint8_t* src, const int64_t* offsets, const int32_t* dims, int B,
                      const float* mean, const float* stdv, int oh, int ow, float* out, hipStream_t s) {
  if (((long)oh * ow * 3) % 4) throw std::invalid_argument("letterbox: out_h*out_w*3 % 4 != 0");
  LbArgs a{};
  a.src = src;
  a.offsets = offsets;
  a.dims = dims;
  for (int c = 0; c < 3; ++c) {
    a.mean[c] = mean[c];
    a.std[c] = stdv[c];
    a.inv_std[c] = 1.f / stdv[c];
  }
  a.oh = oh;
  a.ow = ow;
  a.out = out;
  if (ow % 4 == 0) {
    const long nq = (long)oh * ow / 4;
    hipLaunchKernelGGL(k_letterbox_px4, dim3((unsigned)cdiv(nq, 256), B), dim3(256), 0, s, a);
  } else {
    const long n4 = (long)oh * ow * 3 / 4;
    hipLaunchKernelGGL(k_letterbox, dim3((unsigned)cdiv(n4, 256), B), dim3(256), 0, s, a);
  }
  PHX_LAUNCH_CHECK();
}

// ---- augmentation ---------------------------------------------------------------------------
constexpr int kAugChunks = 64;  // workgroups per image for the channel sums

// partial channel sums of image b's pixel chunk: lanes walk pixels, fp32 runs folded into fp64
__global__ __launch_bounds__(256) void k_aug_sums(const float* __restrict__ in, long npix,
                                                  double* __restrict__ part) {
  const int b = blockIdx.y, k = blockIdx.x;
  const long per = (npix + kAugChunks - 1) / kAugChunks;
  const long p0 = (long)k * per, p1 = min(npix, p0 + per);
  const float* x = in + (long)b * npix * 3;
  double d[3] = {0.0, 0.0, 0.0};
  long p = p0 + threadIdx.x;
  while (p < p1) {
    float f[3] = {0.f, 0.f, 0.f};
    for (int it = 0; it < 64 && p < p1; ++it, p += 256) {
      f[0] += x[p * 3];
      f[1] += x[p * 3 + 1];
      f[2] += x[p * 3 + 2];
    }
    d[0] += f[0];
    d[1] += f[1];
    d[2] += f[2];
  }
  __shared__ double sh[3][256];
  for (int c = 0; c < 3; ++c) sh[c][threadIdx.x] = d[c];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int c = 0; c < 3; ++c) sh[c][threadIdx.x] += sh[c][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 3) part[((long)b * kAugChunks + k) * 3 + threadIdx.x] = sh[threadIdx.x][0];
}

struct AugArgs {
  const float* in;
  float* out;
  const double* part;
  int H, W;
  uint64_t seed;
  int64_t step;
  int gimg0;
};

__global__ __launch_bounds__(256) void k_aug_apply(AugArgs a) {
  const int b = blockIdx.y;
  __shared__ float mean_s[3];
  if (threadIdx.x < 3) {
    double s = 0.0;
    for (int k = 0; k < kAugChunks; ++k) s += a.part[((long)b * kAugChunks + k) * 3 + threadIdx.x];
    // tf.reduce_mean in fp32: the exact mean rounded once
    mean_s[threadIdx.x] = (float)(s / ((double)a.H * a.W));
  }
  __syncthreads();
  const long n4 = (long)a.H * a.W * 3 / 4;
  const long i4 = (long)blockIdx.x * 256 + threadIdx.x;
  if (i4 >= n4) return;
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
  const uint32_t ctr = (uint32_t)(((uint64_t)a.step << 8) | RNG_AUG);
  // per image: the two flips (tf.image.random_flip_left_right, RandomFlip): u < 0.5 each
  const u32x4 ri = philox4x32_10(u32x4{0u, 0u, (uint32_t)(a.gimg0 + b), ctr}, k0, k1);
  const bool mirror = (u01(ri.x) < 0.5f) != (u01(ri.y) < 0.5f);
  // per batch (one scalar each, as tf.image.random_contrast / random_brightness draw): keyed by
  // the step only, so every rank of a data-parallel job applies the global batch's factors
  const u32x4 rb = philox4x32_10(u32x4{1u, 0u, 0xFFFFFFFFu, ctr}, k0, k1);
  const float f = u01(rb.x) * (1.2f - 0.8f) + 0.8f;
  const float delta = u01(rb.y) * (0.2f - -0.2f) + -0.2f;
  const float* x = a.in + (long)b * a.H * a.W * 3;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long e = i4 * 4 + j;
    const int c = (int)(e % 3);
    const long p = e / 3;
    const int y = (int)(p / a.W), xx = (int)(p - (long)y * a.W);
    const int sx = mirror ? a.W - 1 - xx : xx;
    const float m = mean_s[c];
    float t = (x[((long)y * a.W + sx) * 3 + c] - m) * f + m;  // adjust_contrast
    t = t + delta;                                          // adjust_brightness
    v[j] = fminf(fmaxf(t, -1.f), 1.f);                      // clip_by_value
  }
  reinterpret_cast<float4*>(a.out + (long)b * a.H * a.W * 3)[i4] = make_float4(v[0], v[1], v[2], v[3]);
}

// W % 4 == 0 variants: a lane owns a quad of 4 pixels (three float4 = 12 floats, channel pattern
// 0,1,2,0 | 1,2,0,1 | 2,0,1,2), so loads and stores are 16 B and the mirror is a quad-reversal
__global__ __launch_bounds__(256) void k_aug_sums_q(const float4* __restrict__ in, long nq,
                                                    double* __restrict__ part) {
  const int b = blockIdx.y, k = blockIdx.x;
  const long per = (nq + kAugChunks - 1) / kAugChunks;
  const long q0 = (long)k * per, q1 = min(nq, q0 + per);
  const float4* x = in + (long)b * nq * 3;
  double d[3] = {0.0, 0.0, 0.0};
  long q = q0 + threadIdx.x;
  while (q < q1) {
    float f[3] = {0.f, 0.f, 0.f};
    for (int it = 0; it < 64 && q < q1; ++it, q += 256) {
      const float4 a = x[q * 3], bb = x[q * 3 + 1], c = x[q * 3 + 2];
      f[0] += (a.x + a.w) + (bb.z + c.y);
      f[1] += (a.y + bb.x) + (bb.w + c.z);
      f[2] += (a.z + bb.y) + (c.x + c.w);
    }
    d[0] += f[0];
    d[1] += f[1];
    d[2] += f[2];
  }
  __shared__ double sh[3][256];
  for (int c = 0; c < 3; ++c) sh[c][threadIdx.x] = d[c];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int c = 0; c < 3; ++c) sh[c][threadIdx.x] += sh[c][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 3) part[((long)b * kAugChunks + k) * 3 + threadIdx.x] = sh[threadIdx.x][0];
}

__global__ __launch_bounds__(256) void k_aug_apply_q(AugArgs a) {
  const int b = blockIdx.y;
  __shared__ float mean_s[3];
  if (threadIdx.x < 3) {
    double s = 0.0;
    for (int k = 0; k < kAugChunks; ++k) s += a.part[((long)b * kAugChunks + k) * 3 + threadIdx.x];
    mean_s[threadIdx.x] = (float)(s / ((double)a.H * a.W));
  }
  __syncthreads();
  const int wq = a.W / 4;
  const long nq = (long)a.H * wq;
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
  const uint32_t ctr = (uint32_t)(((uint64_t)a.step << 8) | RNG_AUG);
  const u32x4 ri = philox4x32_10(u32x4{0u, 0u, (uint32_t)(a.gimg0 + b), ctr}, k0, k1);
  const bool mirror = (u01(ri.x) < 0.5f) != (u01(ri.y) < 0.5f);
  const u32x4 rb = philox4x32_10(u32x4{1u, 0u, 0xFFFFFFFFu, ctr}, k0, k1);
  const float f = u01(rb.x) * (1.2f - 0.8f) + 0.8f;
  const float delta = u01(rb.y) * (0.2f - -0.2f) + -0.2f;
  const long y = q / wq, xq = q - y * wq;
  const long sq = mirror ? y * wq + (wq - 1 - xq) : q;
  const float4* x = reinterpret_cast<const float4*>(a.in) + (long)b * nq * 3 + sq * 3;
  const float4 l0 = x[0], l1 = x[1], l2 = x[2];
  float px[4][3] = {{l0.x, l0.y, l0.z}, {l0.w, l1.x, l1.y}, {l1.z, l1.w, l2.x}, {l2.y, l2.z, l2.w}};
  float v[12];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int sj = mirror ? 3 - j : j;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float m = mean_s[c];
      float t = (px[sj][c] - m) * f + m;
      t = t + delta;
      v[3 * j + c] = fminf(fmaxf(t, -1.f), 1.f);
    }
  }
  float4* o = reinterpret_cast<float4*>(a.out) + (long)b * nq * 3 + q * 3;
  o[0] = make_float4(v[0], v[1], v[2], v[3]);
  o[1] = make_float4(v[4], v[5], v[6], v[7]);
  o[2] = make_float4(v[8], v[9], v[10], v[11]);
}

size_t augment_scratch_doubles(int B) { return (size_t)B * kAugChunks * 3; }

void launch_augment(const float* in, float* out, int B, int H, int W, uint64_t seed, int64_t step,
                    int gimg0, double* scratch, hipStream_t s) {
  if (((long)H * W * 3) % 4) throw std::invalid_argument("augment: H*W*3 % 4 != 0");
  AugArgs a{in, out, scratch, H, W, seed, step, gimg0};
  if (W % 4 == 0) {
    const long nq = (long)H * W / 4;
    hipLaunchKernelGGL(k_aug_sums_q, dim3(kAugChunks, B), dim3(256), 0, s, reinterpret_cast<const float4*>(in),
                       nq, scratch);
    PHX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_aug_apply_q, dim3((unsigned)cdiv(nq, 256), B), dim3(256), 0, s, a);
    PHX_LAUNCH_CHECK();
    return;
  }
  hipLaunchKernelGGL(k_aug_sums, dim3(kAugChunks, B), dim3(256), 0, s, in, (long)H * W, scratch);
  PHX_LAUNCH_CHECK();
  const long n4 = (long)H * W * 3 / 4;
  hipLaunchKernelGGL(k_aug_apply, dim3((unsigned)cdiv(n4, 256), B), dim3(256), 0, s, a);
  PHX_LAUNCH_CHECK();
}

}  // namespace phx
