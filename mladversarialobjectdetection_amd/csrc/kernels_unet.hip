// kernels_unet.hip — the defender step's attention U-Net (generator.py:17-277) forward and weight
// gradient, its Masker extras (attack_detection.py:321-498) and its loss (attack_detection.py:194-198).
//
// Design (MI355X): every 3x3 convolution is a gather into a K-contiguous column matrix (im2col,
// K = 9*Cin padded to a multiple of 4) followed by the library's persistent MFMA GEMM
// (kernels_gemm.hip); the data gradient of a stride-1 conv is the same gather of dY against the
// flipped kernel, the transposed conv's forward is a parity gather (out[2i + k] += x[i] w[k]) and
// its data gradient a stride-2 gather.  Weight gradients reduce over the M = B*H*W rows: a
// workgroup owns a 64x64 (output channel, K) tile and a slice of rows, the slices' partials are
// folded in a fixed order (bit-reproducible).  BN statistics and BN-backward sums are fp64 column
// reductions over row blocks, folded in a fixed order.
#include <algorithm>

#include "common.hpp"
#include "kernels.hpp"
#include "post.hpp"
#include "unet.hpp"

namespace phx {

__device__ __forceinline__ float leaky(float x) { return x > 0.f ? x : 0.2f * x; }
__device__ __forceinline__ float leaky_grad(float z) { return z > 0.f ? 1.f : 0.2f; }

// ------------------------------------------------------------------------------------------
// gathers
// ------------------------------------------------------------------------------------------
// mode 0: conv, out (oy, ox) tap (ky, kx) reads x[oy*s + ky - pt, ox*s + kx - pl]
// mode 1: transposed conv (stride 2, TF 'same' = pads (0, 1) of the equivalent forward conv):
//         out (oy, ox) tap (ky, kx) reads x[(oy - ky) / 2, (ox - kx) / 2] when both are even
// col[m][k], k = (ky*3 + kx)*C + c, zero beyond 9C (K padded to Kp)
__global__ __launch_bounds__(256) void k_im2col(const float* __restrict__ x, float* __restrict__ col, int B,
                                                int H, int W, int C, int Ho, int Wo, int Kp, int mode,
                                                int s, int pt, int pl) {
  const long n = (long)B * Ho * Wo * Kp;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int k = (int)(i % Kp);
    const long m = i / Kp;
    float v = 0.f;
    if (k < 9 * C) {
      const int tap = k / C, c = k - tap * C;
      const int ky = tap / 3, kx = tap - ky * 3;
      const int ox = (int)(m % Wo);
      const long r = m / Wo;
      const int oy = (int)(r % Ho);
      const int b = (int)(r / Ho);
      int iy, ix;
      bool ok;
      if (mode == 0) {
        iy = oy * s + ky - pt;
        ix = ox * s + kx - pl;
        ok = true;
      } else {
        const int dy = oy - ky, dx = ox - kx;
        ok = dy >= 0 && dx >= 0 && !(dy & 1) && !(dx & 1);
        iy = dy >> 1;
        ix = dx >> 1;
      }
      if (ok && iy >= 0 && iy < H && ix >= 0 && ix < W) v = x[(((long)b * H + iy) * W + ix) * C + c];
    }
    col[i] = v;
  }
}

// derived weight matrices of the GEMMs (B operand [N][K]) from the Keras kernels
//  kind 0: conv fwd      Bt[co][(ky,kx,ci)] = W[ky][kx][ci][co]
//  kind 1: conv dgrad    Bt[ci][(ky,kx,co)] = W[2-ky][2-kx][ci][co]
//  kind 2: tconv fwd     Bt[co][(ky,kx,ci)] = Wt[ky][kx][co][ci]
//  kind 3: tconv dgrad   Bt[ci][(ky,kx,co)] = Wt[ky][kx][co][ci]
//  kind 4: 1x1 fwd       Bt[co][ci] = W[ci][co];  kind 5: 1x1 dgrad Bt[ci][co] = W[ci][co]
__global__ __launch_bounds__(256) void k_wprep(const float* __restrict__ w, float* __restrict__ bt, int kind,
                                               int ci, int co, int Kp) {
  const bool dg = kind == 1 || kind == 3 || kind == 5;
  const int N = dg ? ci : co;
  const int Kin = dg ? co : ci;  // channels along K
  const int taps = kind >= 4 ? 1 : 9;
  const long n = (long)N * Kp;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int nn = (int)(i / Kp), k = (int)(i % Kp);
    float v = 0.f;
    if (k < taps * Kin) {
      const int tap = k / Kin, c = k - tap * Kin;
      const int ky = tap / 3, kx = tap - ky * 3;
      long src;
      switch (kind) {
        case 0: src = (((long)ky * 3 + kx) * ci + c) * co + nn; break;
        case 1: src = (((long)(2 - ky) * 3 + (2 - kx)) * ci + nn) * co + c; break;
        case 2: src = (((long)ky * 3 + kx) * co + nn) * ci + c; break;
        case 3: src = (((long)ky * 3 + kx) * co + c) * ci + nn; break;
        case 4: src = (long)c * co + nn; break;
        default: src = (long)nn * co + c; break;
      }
      v = w[src];
    }
    bt[i] = v;
  }
}

// ------------------------------------------------------------------------------------------
// weight gradient on the fp32 matrix cores: part[z][co][k] = sum over the rows m of slice z of
// dy[m][co] * col[m][k], with col gathered on the fly (no column matrix in HBM):
//   SRC 0: col = a row-major matrix x[m * ldx + k] (1x1 convs: the layer input itself)
//   SRC 1: 3x3 conv, stride 1, pads (1, 1): col[m][(ky*3 + kx)*C + c] = x[b, oy+ky-1, ox+kx-1, c]
//   SRC 2: transposed conv (stride 2): col[m][(ky*3 + kx)*C + c] = x[b, (oy-ky)/2, (ox-kx)/2, c]
//          when both differences are even and >= 0 (x is H/2 x W/2; rows m are the H x W outputs)
// v_mfma_f32_16x16x4_f32: lane l feeds A[i = l&15][kk = l>>4] = dy[m0 + kk][co0 + i] and
// B[kk][j = l&15] of four accumulators t (a wave owns a 16 (co) x 64 (k) tile sharing the A
// operand).  VEC (channels a multiple of 4): the lane's four columns are k0 + 4j + t — one 16-B
// load feeds all four tiles (a 4-B load per tile made the kernel bound by address processing);
// otherwise k0 + 16t + j.  A wave takes every fourth 4-row step of the workgroup's slice, U steps'
// loads in flight; the four waves' tiles are summed through LDS in a fixed order
// (bit-reproducible).  A lane's columns never change, so their (tap, channel) decomposition is
// hoisted; its pixel advances by 16 rows per step.
// ------------------------------------------------------------------------------------------
typedef float floatx4 __attribute__((ext_vector_type(4)));

#ifndef PHX_WG_U
#define PHX_WG_U 4
#endif
#ifndef PHX_WG_SLICES
#define PHX_WG_SLICES 1024
#endif

template <int SRC, bool VEC>
__global__ __launch_bounds__(256) void k_wgrad_mfma(const float* __restrict__ dy, int ldy,
                                                    const float* __restrict__ x, int ldx, int H, int W, int C,
                                                    long M, int Co, int Kp, long rows_per_slice,
                                                    float* __restrict__ part) {
  __shared__ floatx4 red[4][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i16 = lane & 15, kk = lane >> 4;
  const int co = blockIdx.x * 16 + i16;
  const int k0 = blockIdx.y * 64;
  const long r0 = (long)blockIdx.z * rows_per_slice, r1 = min(M, r0 + rows_per_slice);
  const bool cok = co < Co;
  const int Kend = SRC == 0 ? Kp : 9 * C;
  // hoisted column decomposition of this lane's k columns (VEC: one quad, NQ = 1)
  constexpr int NQ = VEC ? 1 : 4;
  int koff[NQ], ky[NQ], kx[NQ];
  bool kok[NQ];
#pragma unroll
  for (int t = 0; t < NQ; ++t) {
    const int k = VEC ? k0 + 4 * i16 : k0 + 16 * t + i16;
    kok[t] = k < Kend;
    if (SRC == 0) {
      koff[t] = k;
      ky[t] = kx[t] = 0;
    } else {
      const int tap = kok[t] ? k / C : 0;
      koff[t] = kok[t] ? k - tap * C : 0;
      ky[t] = tap / 3;
      kx[t] = tap - ky[t] * 3;
    }
  }
  floatx4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  // this lane's first row and its pixel
  long m = r0 + 4 * wave + kk;
  int ox = 0, oy = 0, b = 0;
  if (SRC != 0) {
    const long mm = min(m, M - 1);
    ox = (int)(mm % W);
    const long q = mm / W;
    oy = (int)(q % H);
    b = (int)(q / H);
  }
  const int Hi = SRC == 2 ? H / 2 : H, Wi = SRC == 2 ? W / 2 : W;
  constexpr int U = PHX_WG_U;  // row steps whose loads are in flight together
  for (long m0 = r0 + 4 * wave; m0 < r1; m0 += 16 * U) {
    float av[U];
    floatx4 bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // loads from clamped (always valid) addresses, zeroed after they land
      const bool rok = m < r1;
      av[u] = dy[(rok && cok) ? m * ldy + co : 0];
      if (!(rok && cok)) av[u] = 0.f;
#pragma unroll
      for (int t = 0; t < NQ; ++t) {
        long addr = 0;
        bool ok = rok && kok[t];
        if (SRC == 0) {
          addr = m * ldx + koff[t];
        } else {
          int iy, ix;
          bool g;
          if (SRC == 1) {
            iy = oy + ky[t] - 1;
            ix = ox + kx[t] - 1;
            g = true;
          } else {
            const int dyy = oy - ky[t], dxx = ox - kx[t];
            g = dyy >= 0 && dxx >= 0 && !(dyy & 1) && !(dxx & 1);
            iy = dyy >> 1;
            ix = dxx >> 1;
          }
          ok = ok && g && iy >= 0 && iy < Hi && ix >= 0 && ix < Wi;
          addr = (((long)b * Hi + iy) * Wi + ix) * C + koff[t];
        }
        if constexpr (VEC) {
          const floatx4 v = *reinterpret_cast<const floatx4*>(x + (ok ? addr : 0));
          bv[u] = ok ? v : floatx4{0.f, 0.f, 0.f, 0.f};
        } else {
          const float v = x[ok ? addr : 0];
          bv[u][t] = ok ? v : 0.f;
        }
      }
      m += 16;
      if (SRC != 0) {
        ox += 16;
        while (ox >= W) {
          ox -= W;
          if (++oy == H) {
            oy = 0;
            ++b;
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u][t], acc[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) red[wave][t][lane] = acc[t];
  __syncthreads();
  // D layout: lane l holds column j = l&15, rows 4*(l>>4) + r
  float* out = part + (long)blockIdx.z * Co * Kp;
  for (int e = threadIdx.x; e < 4 * 64; e += 256) {
    const int t = e >> 6, l = e & 63;
    floatx4 s = red[0][t][l];
#pragma unroll
    for (int w = 1; w < 4; ++w) s += red[w][t][l];
    const int k = VEC ? k0 + 4 * (l & 15) + t : k0 + 16 * t + (l & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = blockIdx.x * 16 + 4 * (l >> 4) + r;
      if (c < Co && k < Kp) out[(long)c * Kp + k] = s[r];
    }
  }
}

// ------------------------------------------------------------------------------------------
// 3x3 convolutions with few channels (the U-Net's full-resolution levels): out[m][n] = bias[n] +
// sum_k col[m][k] * Bt[n][k] with the column matrix gathered on the fly (k_im2col's modes: 0 conv
// with stride s and pads (pt, pl), 1 stride-2 transposed conv) — the column matrix of these layers
// is 9x the layer input and would be written and read once more through HBM.
// v_mfma_f32_16x16x4_f32: lane l feeds A[i = l&15][kk = l>>4] = col[m0 + i][k0 + kk] (one gather)
// and B[kk][j = l&15] = Bt[16t + j][k0 + kk] from LDS; a wave owns 16 output rows x 16*NT
// columns and walks 16-row tiles (persistent).  The lane's (tap, channel) advances by 4 per step.
// ------------------------------------------------------------------------------------------
constexpr int kConvMaxKp = 288, kConvMaxN = 32;
#ifndef PHX_UN_XCD_TILES
#define PHX_UN_XCD_TILES 1
#endif

template <int NT, int MODE, bool VEC>
__global__ __launch_bounds__(256) void k_conv3_small(const float* __restrict__ x, const float* __restrict__ Bt,
                                                     const float* __restrict__ bias, float* __restrict__ out, int B,
                                                     int H, int W, int C, int Ho, int Wo, int N, int Kp, int s,
                                                     int pt, int pl) {
  constexpr int KB = 16;  // k steps (of 4) whose gathers are in flight together
  __shared__ float sb[(kConvMaxKp + 4 * KB - 1) / (4 * KB) * 4 * KB][16 * NT + 1];  // [k][n]
  const int KpR = (Kp + 4 * KB - 1) / (4 * KB) * (4 * KB);
  for (int e = threadIdx.x; e < KpR * 16 * NT; e += 256) {
    const int k = e / (16 * NT), n = e - k * 16 * NT;
    sb[k][n] = (n < N && k < Kp) ? Bt[(long)n * Kp + k] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i16 = lane & 15, kk = lane >> 4;
  const long M = (long)B * Ho * Wo;
  const long tiles = (M + 15) / 16;
  const int K9 = 9 * C;
  float bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bv[t] = (bias && 16 * t + i16 < N) ? bias[16 * t + i16] : 0.f;
  // XCD-aware tile ranges: workgroup j runs on XCD j % 8, and each XCD owns a contiguous range of the
  // 16-pixel tiles which its workgroups sweep together, so the input rows a 3x3 gather shares between
  // vertically neighbouring tiles are read through one L2 (round-robin tiles put the three rows of a
  // window on three XCDs).  Each tile's arithmetic is unchanged.  (Fewer than 8 workgroups: one range.)
  const int G = (int)gridDim.x;
  const bool xr = G >= 8 && PHX_UN_XCD_TILES;
  const int xcd = xr ? (int)(blockIdx.x & 7) : 0, wi = xr ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  const int gper = xr ? (G - xcd + 7) / 8 : G;
  const long tper = xr ? (tiles + 7) / 8 : tiles;
  const long tbeg = (long)xcd * tper, tend = min(tiles, tbeg + tper);
  for (long tile = tbeg + (long)wi * 4 + wave; tile < tend; tile += (long)gper * 4) {
    const long m = tile * 16 + i16;
    const bool rok = m < M;
    const long mm = rok ? m : M - 1;
    const int ox = (int)(mm % Wo);
    const long q = mm / Wo;
    const int oy = (int)(q % Ho);
    const int b = (int)(q / Ho);
    const float* xb = x + (long)b * H * W * C;
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    // this lane's column (VEC: its quad of columns 16 qs + 4 kk .. +3; else k0 + kk) as
    // (tap (ky, kx), channel c)
    int c = VEC ? 4 * kk : kk, ky = 0, kx = 0;
    while (c >= C) {
      c -= C;
      if (++kx == 3) {
        kx = 0;
        ++ky;
      }
    }
    auto gather_at = [&](bool& ok) -> long {
      int iy, ix;
      bool g;
      if (MODE == 0) {
        iy = oy * s + ky - pt;
        ix = ox * s + kx - pl;
        g = true;
      } else {
        const int dyy = oy - ky, dxx = ox - kx;
        g = dyy >= 0 && dxx >= 0 && !(dyy & 1) && !(dxx & 1);
        iy = dyy >> 1;
        ix = dxx >> 1;
      }
      ok = ok && g && iy >= 0 && iy < H && ix >= 0 && ix < W;
      return ok ? ((long)iy * W + ix) * C + c : 0;
    };
    auto advance = [&](int by) {
      c += by;
      while (c >= C) {
        c -= C;
        if (++kx == 3) {
          kx = 0;
          ++ky;
        }
      }
    };
    if constexpr (VEC) {
      // one 16-B gather per lane feeds 4 MFMA steps: step e of quad-step q uses column 16q + 4kk + e
      constexpr int QB = 4;
      for (int kb = 0; kb < Kp; kb += 16 * QB) {
        floatx4 a[QB];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          bool ok = rok && kb + 16 * u + 4 * kk < K9;
          const long off = gather_at(ok);
          const floatx4 v = *reinterpret_cast<const floatx4*>(xb + off);
          a[u] = ok ? v : floatx4{0.f, 0.f, 0.f, 0.f};
          advance(16);
        }
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int t = 0; t < NT; ++t)
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][e], sb[kb + 16 * u + 4 * kk + e][16 * t + i16],
                                                            acc[t], 0, 0, 0);
      }
    } else {
      for (int kb = 0; kb < Kp; kb += 4 * KB) {
        // gathers of KB steps from clamped (always valid) addresses, zeroed after the loads
        float a[KB];
#pragma unroll
        for (int u = 0; u < KB; ++u) {
          bool ok = rok && kb + 4 * u + kk < K9;
          const long off = gather_at(ok);
          const float v = xb[off];
          a[u] = ok ? v : 0.f;
          advance(4);
        }
#pragma unroll
        for (int u = 0; u < KB; ++u)
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], sb[kb + 4 * u + kk][16 * t + i16], acc[t], 0, 0, 0);
      }
    }
    // D layout: lane holds column j = l&15, rows 4*(l>>4) + r
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = 16 * t + i16;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long row = tile * 16 + 4 * kk + r;
        if (row < M) out[row * N + n] = acc[t][r] + bv[t];
      }
    }
  }
}

// fold the slices (fixed order) and scatter into the Keras kernel layout of the gradient
//  kind 0: conv  [ky][kx][ci][co] from (co, (ky,kx,ci));  kind 2: tconv [ky][kx][co][ci];
//  kind 4: 1x1 [ci][co]
// A workgroup folds 16 consecutive (co, k) outputs: 16 slice lanes per output each add every 16th
// slice (independent loads in flight), then lane 0 adds the 16 lane sums in order.
__global__ __launch_bounds__(256) void k_wgrad_fold(const float* __restrict__ part, int nslice, int Co, int Kp,
                                                    int Kin, int taps, int kind, float* __restrict__ g) {
  __shared__ float sh[16][17];
  const int j = threadIdx.x & 15, q = threadIdx.x >> 4;
  const long n = (long)Co * taps * Kin;
  const long i = (long)blockIdx.x * 16 + j;
  const int co = (int)(min(i, n - 1) / ((long)taps * Kin));
  const int k = (int)(min(i, n - 1) % ((long)taps * Kin));
  float s = 0.f;
  int z = q;
  // four slices' loads in flight, added in slice order
  for (; z + 48 < nslice; z += 64) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = part[((long)(z + 16 * u) * Co + co) * Kp + k];
#pragma unroll
    for (int u = 0; u < 4; ++u) s += v[u];
  }
  for (; z < nslice; z += 16) s += part[((long)z * Co + co) * Kp + k];
  sh[q][j] = s;
  __syncthreads();
  if (q == 0 && i < n) {
    float t = sh[0][j];
    for (int z = 1; z < 16; ++z) t += sh[z][j];
    const int tap = k / Kin, c = k - tap * Kin;
    long dst;
    if (kind == 2) dst = ((long)tap * Co + co) * Kin + c;
    else dst = ((long)tap * Kin + c) * Co + co;
    g[dst] = t;
  }
}

// ------------------------------------------------------------------------------------------
// fp64 column reductions over [M, C] (C <= 256): block z reduces its row range; thread t owns
// channel t % C (threads past the last whole group of C idle), then thread c folds its group.  Modes:
//   0 BN statistics: s0 = sum(y - y[0]), s1 = sum((y - y[0])^2)
//   1 BN backward:   dz = da * act'(z), z = (y - mu) * sc + be; s0 = sum dz, s1 = sum dz * xhat
//   2 column sums:   s0 = sum v
// ------------------------------------------------------------------------------------------
struct ColRed {
  const float* y;   // BN input (modes 0, 1) or values (mode 2)
  const float* da;  // mode 1: gradient of the activation output
  const float* mu;
  const float* rstd;
  const float* sc;
  const float* be;
  int act;          // 1 leaky, 0 identity
  int ld;           // row stride (floats)
};

__global__ __launch_bounds__(256) void k_colred64(ColRed r, long M, int C, long rows_per_block, int mode,
                                                  double* __restrict__ part) {
  __shared__ double s0s[256], s1s[256];
  const int t = threadIdx.x, lane_rows = 256 / C, c = t % C, r_off = t / C;
  const bool active = r_off < lane_rows;
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const double shift = mode == 0 ? (double)r.y[c] : 0.0;
  float mu = 0.f, rs = 0.f, scv = 0.f, be = 0.f;
  if (mode == 1) {
    mu = r.mu[c]; rs = r.rstd[c]; scv = r.sc[c]; be = r.be[c];
  }
  double a0 = 0.0, a1 = 0.0;
  long row = r0 + r_off;
  // 8 rows per lane in flight (a load-then-add loop waits one memory latency per row)
  if (active) {
    for (; row + 7 * (long)lane_rows < r1; row += 8 * (long)lane_rows) {
      float v[8], g[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = r.y[(row + u * (long)lane_rows) * r.ld + c];
        g[u] = mode == 1 ? r.da[(row + u * (long)lane_rows) * r.ld + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (mode == 0) {
          const double d = (double)v[u] - shift;
          a0 += d;
          a1 += d * d;
        } else if (mode == 1) {
          const float yc = v[u] - mu;
          float dz = g[u];
          if (r.act) dz *= leaky_grad(yc * scv + be);
          a0 += (double)dz;
          a1 += (double)dz * (double)(yc * rs);
        } else {
          a0 += (double)v[u];
        }
      }
    }
  }
  for (; active && row < r1; row += lane_rows) {
    const float v = r.y[row * r.ld + c];
    if (mode == 0) {
      const double d = (double)v - shift;
      a0 += d;
      a1 += d * d;
    } else if (mode == 1) {
      const float yc = v - mu;
      float dz = r.da[row * r.ld + c];
      if (r.act) dz *= leaky_grad(yc * scv + be);
      a0 += (double)dz;
      a1 += (double)dz * (double)(yc * rs);
    } else {
      a0 += (double)v;
    }
  }
  s0s[t] = a0;
  s1s[t] = a1;
  __syncthreads();
  if (t < C) {
    double b0 = 0.0, b1 = 0.0;
    for (int j = 0; j < lane_rows; ++j) {
      b0 += s0s[t + j * C];
      b1 += s1s[t + j * C];
    }
    part[((long)blockIdx.x * C + t) * 2 + 0] = b0;
    part[((long)blockIdx.x * C + t) * 2 + 1] = b1;
  }
}

// The finals fold the nblk row-block partials of a channel with one wave: lane l adds blocks
// l, l+64, ... (independent loads in flight), then a fixed xor tree (bit-reproducible).
__device__ __forceinline__ void wave_fold(const double* __restrict__ part, int nblk, int C, int c, double& s0,
                                          double& s1) {
  const int lane = threadIdx.x & 63;
  s0 = 0.0;
  s1 = 0.0;
  int z = lane;
  // four blocks' loads in flight, added in block order
  for (; z + 192 < nblk; z += 256) {
    double v0[4], v1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v0[u] = part[((long)(z + 64 * u) * C + c) * 2];
      v1[u] = part[((long)(z + 64 * u) * C + c) * 2 + 1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s0 += v0[u];
      s1 += v1[u];
    }
  }
  for (; z < nblk; z += 64) {
    s0 += part[((long)z * C + c) * 2];
    s1 += part[((long)z * C + c) * 2 + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o);
    s1 += __shfl_xor(s1, o);
  }
}

// BN statistics: mean / rstd / sc = gamma * rstd, moving statistics (momentum 0.99, Bessel)
__global__ __launch_bounds__(256) void k_un_bn_final(const double* __restrict__ part, int nblk, long M, int C,
                                                     const float* __restrict__ y0, const float* __restrict__ gamma,
                                                     float* __restrict__ mean, float* __restrict__ rstd,
                                                     float* __restrict__ sc, float* __restrict__ mmean,
                                                     float* __restrict__ mvar) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  double s0, s1;
  wave_fold(part, nblk, C, c, s0, s1);
  if ((threadIdx.x & 63) != 0) return;
  const double dm = s0 / (double)M;
  double var = s1 / (double)M - dm * dm;
  if (var < 0.0) var = 0.0;
  const double mu = (double)y0[c] + dm;
  const double rs = 1.0 / sqrt(var + 1e-3);
  mean[c] = (float)mu;
  rstd[c] = (float)rs;
  sc[c] = (float)(rs * (double)gamma[c]);
  if (mmean) {
    const double uvar = M > 1 ? var * (double)M / (double)(M - 1) : var;
    mmean[c] = (float)(mmean[c] - (mmean[c] - mu) * 0.01);
    mvar[c] = (float)(mvar[c] - (mvar[c] - uvar) * 0.01);
  }
}

// BN backward: mean(dz), mean(dz*xhat); d gamma = sum dz*xhat, d beta = sum dz
__global__ __launch_bounds__(256) void k_un_bnb_final(const double* __restrict__ part, int nblk, long M, int C,
                                                      float* __restrict__ mdz, float* __restrict__ mdzx,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  double s0, s1;
  wave_fold(part, nblk, C, c, s0, s1);
  if ((threadIdx.x & 63) != 0) return;
  mdz[c] = (float)(s0 / (double)M);
  mdzx[c] = (float)(s1 / (double)M);
  dgamma[c] = (float)s1;
  dbeta[c] = (float)s0;
}

// column sums (bias gradients)
__global__ __launch_bounds__(256) void k_un_colsum_final(const double* __restrict__ part, int nblk, int C,
                                                         float* __restrict__ out) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  double s0, s1;
  wave_fold(part, nblk, C, c, s0, s1);
  if ((threadIdx.x & 63) == 0) out[c] = (float)s0;
}

// ------------------------------------------------------------------------------------------
// elementwise
// ------------------------------------------------------------------------------------------
// a = act((y - mu) * sc + be), act 1 = leaky
__global__ __launch_bounds__(256) void k_un_bnact(const float* __restrict__ y, const float* __restrict__ mu,
                                                  const float* __restrict__ sc, const float* __restrict__ be,
                                                  float* __restrict__ a, long n, int C, int act) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float z = (y[i] - mu[c]) * sc[c] + be[c];
    a[i] = act ? leaky(z) : z;
  }
}

// dy = sc * (dz - mean dz - xhat * mean(dz xhat)), dz = da * act'(z)
__global__ __launch_bounds__(256) void k_un_bnb_apply(const float* __restrict__ da, const float* __restrict__ y,
                                                      const float* __restrict__ mu, const float* __restrict__ rstd,
                                                      const float* __restrict__ sc, const float* __restrict__ be,
                                                      const float* __restrict__ mdz, const float* __restrict__ mdzx,
                                                      float* __restrict__ dy, long n, int C, int act) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float yc = y[i] - mu[c];
    float dz = da[i];
    if (act) dz *= leaky_grad(yc * sc[c] + be[c]);
    dy[i] = sc[c] * (dz - mdz[c] - (yc * rstd[c]) * mdzx[c]);
  }
}

// 2x2 max-pool (valid) + the winning tap (first maximum in row-major window order), then Dropout
__global__ __launch_bounds__(256) void k_un_pool_drop(const float* __restrict__ x, float* __restrict__ out,
                                                      uint8_t* __restrict__ arg, int B, int H, int W, int C,
                                                      uint64_t seed, int64_t step, int gimg0, int layer) {
  const int Ho = H / 2, Wo = W / 2;
  const long n = (long)B * Ho * Wo * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long p = i / C;
    const int ox = (int)(p % Wo);
    const long r = p / Wo;
    const int oy = (int)(r % Ho);
    const int b = (int)(r / Ho);
    const float* base = x + (((long)b * H + 2 * oy) * W + 2 * ox) * C + c;
    float m = base[0];
    int am = 0;
    const float v1 = base[C], v2 = base[(long)W * C], v3 = base[(long)W * C + C];
    if (v1 > m) { m = v1; am = 1; }
    if (v2 > m) { m = v2; am = 2; }
    if (v3 > m) { m = v3; am = 3; }
    arg[i] = (uint8_t)am;
    if (layer < 0) {  // inference (training=False): Dropout is the identity
      out[i] = m;
      continue;
    }
    const long e = i - (long)b * Ho * Wo * C;  // element index within the image
    const u32x4 q = philox4x32_10(u32x4{(uint32_t)e, (uint32_t)layer, (uint32_t)(gimg0 + b),
                                        (uint32_t)((uint64_t)step << 8) | RNG_DROPOUT},
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
    out[i] = u01(q.x) >= 0.2f ? (m * 1.25f) : 0.f;
  }
}

// backward of pool + dropout: dx (the whole input, zeros off the winning taps) [+= when acc]
__global__ __launch_bounds__(256) void k_un_pool_drop_bwd(const float* __restrict__ dout,
                                                          const uint8_t* __restrict__ arg, float* __restrict__ dx,
                                                          int B, int H, int W, int C, uint64_t seed, int64_t step,
                                                          int gimg0, int layer, int acc) {
  const int Ho = H / 2, Wo = W / 2;
  const long n = (long)B * Ho * Wo * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long p = i / C;
    const int ox = (int)(p % Wo);
    const long r = p / Wo;
    const int oy = (int)(r % Ho);
    const int b = (int)(r / Ho);
    const long e = i - (long)b * Ho * Wo * C;
    const u32x4 q = philox4x32_10(u32x4{(uint32_t)e, (uint32_t)layer, (uint32_t)(gimg0 + b),
                                        (uint32_t)((uint64_t)step << 8) | RNG_DROPOUT},
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
    const float g = u01(q.x) >= 0.2f ? dout[i] * 1.25f : 0.f;
    const int am = arg[i];
    float* base = dx + (((long)b * H + 2 * oy) * W + 2 * ox) * C + c;
    const long off[4] = {0, C, (long)W * C, (long)W * C + C};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float v = k == am ? g : 0.f;
      if (acc) base[off[k]] += v;
      else base[off[k]] = v;
    }
  }
}

// attention, forward part 1: s = leaky(bn1(g) + bn2(x))  (the BN outputs are never stored)
__global__ __launch_bounds__(256) void k_att_s(const float* __restrict__ g, const float* __restrict__ x,
                                               const float* __restrict__ mu1, const float* __restrict__ sc1,
                                               const float* __restrict__ be1, const float* __restrict__ mu2,
                                               const float* __restrict__ sc2, const float* __restrict__ be2,
                                               float* __restrict__ s, long n, int C) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float zg = (g[i] - mu1[c]) * sc1[c] + be1[c];
    const float zx = (x[i] - mu2[c]) * sc2[c] + be2[c];
    s[i] = leaky(zg + zx);
  }
}

// t[m] = sum_c s[m][c] * w[c] + b  (the attention's 1-channel 1x1 conv)
__global__ __launch_bounds__(256) void k_att_t(const float* __restrict__ s, const float* __restrict__ w,
                                               const float* __restrict__ b, float* __restrict__ t, long M, int C) {
  for (long m = (long)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (long)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc = fmaf(s[m * C + c], w[c], acc);
    t[m] = acc + b[0];
  }
}

// attention, forward part 2 + concat + Dropout: a = sigmoid(bn3(t)); cat = [up, skip * a] (2C
// channels) times the Dropout mask of layer `layer`
__global__ __launch_bounds__(256) void k_att_cat(const float* __restrict__ up, const float* __restrict__ skip,
                                                 const float* __restrict__ t, const float* __restrict__ mu3,
                                                 const float* __restrict__ sc3, const float* __restrict__ be3,
                                                 float* __restrict__ cat, int B, long HW, int C, uint64_t seed,
                                                 int64_t step, int gimg0, int layer) {
  const long n = (long)B * HW * 2 * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c2 = (int)(i % (2 * C));
    const long m = i / (2 * C);
    float v;
    if (c2 < C) {
      v = up[m * C + c2];
    } else {
      const float z = (t[m] - mu3[0]) * sc3[0] + be3[0];
      const float a = 1.0f / (1.0f + expf(-z));
      v = skip[m * C + c2 - C] * a;
    }
    if (layer < 0) {  // inference: no Dropout
      cat[i] = v;
      continue;
    }
    const int b = (int)(m / HW);
    const long e = i - (long)b * HW * 2 * C;
    const u32x4 q = philox4x32_10(u32x4{(uint32_t)e, (uint32_t)layer, (uint32_t)(gimg0 + b),
                                        (uint32_t)((uint64_t)step << 8) | RNG_DROPOUT},
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
    cat[i] = u01(q.x) >= 0.2f ? v * 1.25f : 0.f;
  }
}

// backward of k_att_cat: dup = dcat[:, :C] (masked), dskip_direct = dcat[:, C:] * a, and per row
// dz3 = (sum_c dcat[:, C + c] * skip) * a (1 - a)  (the gradient of bn3's output)
__global__ __launch_bounds__(256) void k_att_cat_bwd(const float* __restrict__ dcat, const float* __restrict__ skip,
                                                     const float* __restrict__ t, const float* __restrict__ mu3,
                                                     const float* __restrict__ sc3, const float* __restrict__ be3,
                                                     float* __restrict__ dup, float* __restrict__ dskip,
                                                     float* __restrict__ dz3, int B, long HW, int C, uint64_t seed,
                                                     int64_t step, int gimg0, int layer) {
  // C lanes per pixel (C a power of two <= 64): lane c handles channels c (up) and C + c (skip);
  // the skip half's dot product with the gradient is reduced by a fixed xor tree
  const long M = (long)B * HW;
  const long gi = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long m = gi / C;
  const int c = (int)(gi - m * C);
  const bool ok = m < M;
  const long mc = ok ? m : M - 1;
  const int b = (int)(mc / HW);
  const float z = (t[mc] - mu3[0]) * sc3[0] + be3[0];
  const float a = 1.0f / (1.0f + expf(-z));
  auto keep = [&](int c2) {
    const long e = (mc - (long)b * HW) * 2 * C + c2;
    const u32x4 q = philox4x32_10(u32x4{(uint32_t)e, (uint32_t)layer, (uint32_t)(gimg0 + b),
                                        (uint32_t)((uint64_t)step << 8) | RNG_DROPOUT},
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
    return u01(q.x) >= 0.2f;
  };
  const float g0 = keep(c) ? dcat[mc * 2 * C + c] * 1.25f : 0.f;
  const float g1 = keep(C + c) ? dcat[mc * 2 * C + C + c] * 1.25f : 0.f;
  const float sk = skip[mc * C + c];
  if (ok) {
    dup[mc * C + c] = g0;
    dskip[mc * C + c] = g1 * a;
  }
  float da = g1 * sk;
  for (int o = 1; o < C; o <<= 1) da += __shfl_xor(da, o);
  if (ok && c == 0) dz3[mc] = da * (a * (1.0f - a));
}

// d(pre-leaky sum) of the attention: ds[m][c] = dt[m] * w3[c] * leaky'(bn1(g) + bn2(x))
__global__ __launch_bounds__(256) void k_att_s_bwd(const float* __restrict__ dt, const float* __restrict__ w3,
                                                   const float* __restrict__ g, const float* __restrict__ x,
                                                   const float* __restrict__ mu1, const float* __restrict__ sc1,
                                                   const float* __restrict__ be1, const float* __restrict__ mu2,
                                                   const float* __restrict__ sc2, const float* __restrict__ be2,
                                                   float* __restrict__ dsum, long n, int C) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long m = i / C;
    const float zg = (g[i] - mu1[c]) * sc1[c] + be1[c];
    const float zx = (x[i] - mu2[c]) * sc2[c] + be2[c];
    dsum[i] = dt[m] * w3[c] * leaky_grad(zg + zx);
  }
}

// output layer + loss: o = tanh(x W + b) (1x1, C -> 3), u = 2 o, per image mean((t - u)^2);
// dz = d loss / d(x W + b) = -2 (t - u) / (HW*3) * 2 * (1 - o^2); partial loss per block (fp64)
__global__ __launch_bounds__(256) void k_un_out_loss(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ bias, const float* __restrict__ tgt,
                                                     float* __restrict__ upd, float* __restrict__ dz,
                                                     double* __restrict__ lpart, long M, long HW, int C) {
  __shared__ double sh[256];
  double acc = 0.0;
  const float inv = 1.0f / (float)(HW * 3);
  for (long m = (long)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (long)gridDim.x * blockDim.x) {
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      float z = bias[o];
      for (int c = 0; c < C; ++c) z = fmaf(x[m * C + c], w[c * 3 + o], z);
      const float th = tanhf(z);
      const float u = 2.0f * th;
      const float d = tgt[m * 3 + o] - u;
      acc += (double)d * (double)d;
      upd[m * 3 + o] = u;
      dz[m * 3 + o] = (-2.0f * d * inv) * 2.0f * (1.0f - th * th);
    }
  }
  sh[threadIdx.x] = acc / (double)(HW * 3);
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) lpart[blockIdx.x] = sh[0];
}

__global__ void k_un_loss_final(const double* __restrict__ lpart, int n, float* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += lpart[i];
  out[0] = (float)s;
}

// dx[m][c] = sum_o dz[m][o] * w[c][o]  (+= when acc): the data gradient of a 1x1 conv with few outputs
__global__ __launch_bounds__(256) void k_un_small_dgrad(const float* __restrict__ dz, const float* __restrict__ w,
                                                        float* __restrict__ dx, long M, int C, int O, int acc) {
  const long n = M * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long m = i / C;
    float v = 0.f;
    for (int o = 0; o < O; ++o) v = fmaf(dz[m * O + o], w[c * O + o], v);
    if (acc) dx[i] += v;
    else dx[i] = v;
  }
}

__global__ __launch_bounds__(256) void k_un_add(float* __restrict__ a, const float* __restrict__ b, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) a[i] += b[i];
}

// ------------------------------------------------------------------------------------------
// Masker extras
// ------------------------------------------------------------------------------------------
// per target image b: source image perm[b] (tf.random.shuffle: ranks of one Philox key per image,
// ties by index) and its left-right / up-down flips (flip when u01 >= 0.5); one workgroup
__global__ void k_def_perm(int B, uint64_t seed, int64_t step, int gimg0, int* __restrict__ info) {
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    // the image whose key has rank b
    int src = 0;
    for (int j = 0; j < B; ++j) {
      const uint32_t kj = philox4x32_10(u32x4{0u, 0u, (uint32_t)(gimg0 + j), (uint32_t)((uint64_t)step << 8) | RNG_DSHUF},
                                        (uint32_t)seed, (uint32_t)(seed >> 32)).x;
      int rank = 0;
      for (int i = 0; i < B; ++i) {
        const uint32_t ki = philox4x32_10(u32x4{0u, 0u, (uint32_t)(gimg0 + i), (uint32_t)((uint64_t)step << 8) | RNG_DSHUF},
                                          (uint32_t)seed, (uint32_t)(seed >> 32)).x;
        rank += (ki < kj || (ki == kj && i < j)) ? 1 : 0;
      }
      if (rank == b) src = j;
    }
    const u32x4 f = philox4x32_10(u32x4{0u, 0u, (uint32_t)(gimg0 + b), (uint32_t)((uint64_t)step << 8) | RNG_DFLIP},
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
    info[b * 3 + 0] = src;
    info[b * 3 + 1] = u01(f.x) >= 0.5f ? 1 : 0;
    info[b * 3 + 2] = u01(f.y) >= 0.5f ? 1 : 0;
  }
}

// patches[b] = flips(images[perm[b], :P, :P])
__global__ __launch_bounds__(256) void k_def_crops(const float* __restrict__ images, const int* __restrict__ info,
                                                   float* __restrict__ out, int B, int H, int W, int P) {
  const long n = (long)B * P * P;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int x = (int)(i % P);
    const long r = i / P;
    const int y = (int)(r % P);
    const int b = (int)(r / P);
    const int src = info[b * 3], lr = info[b * 3 + 1], ud = info[b * 3 + 2];
    const int sy = ud ? P - 1 - y : y, sx = lr ? P - 1 - x : x;
    const float* s = images + (((long)src * H + sy) * W + sx) * 3;
    float* o = out + i * 3;
    o[0] = s[0];
    o[1] = s[1];
    o[2] = s[2];
  }
}

// odet_model's filter_valid_boxes after NMS (attack_detection.py:79-94, 121-125): keep boxes with
// w / W <= 1, h / H <= 1, area > 100 and score >= thresh, in order
__global__ void k_def_filter(const float* __restrict__ nb, const float* __restrict__ ns, const int* __restrict__ nc,
                             int B, int maxo, float Hf, float Wf, float thresh, float* __restrict__ ob,
                             int* __restrict__ oc, float* __restrict__ os) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int k = 0;
  for (int i = 0; i < nc[b]; ++i) {
    const float* bx = nb + ((long)b * maxo + i) * 4;
    const float h = bx[2] - bx[0], w = bx[3] - bx[1];
    const bool ok = (w / Wf <= 1.0f) && (h / Hf <= 1.0f) && (h * w > 100.0f) && ns[(long)b * maxo + i] >= thresh;
    if (ok) {
      float* o = ob + ((long)b * maxo + k) * 4;
      o[0] = bx[0]; o[1] = bx[1]; o[2] = bx[2]; o[3] = bx[3];
      if (os) os[(long)b * maxo + k] = ns[(long)b * maxo + i];
      ++k;
    }
  }
  oc[b] = k;
  // the rows past the kept boxes are zero (defined outputs: the caller's buffers are not cleared)
  for (int i = k; i < maxo; ++i) {
    float* o = ob + ((long)b * maxo + i) * 4;
    o[0] = o[1] = o[2] = o[3] = 0.f;
    if (os) os[(long)b * maxo + i] = 0.f;
  }
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
static dim3 grid_for(long n) { return dim3((unsigned)std::min<long>(std::max<long>(cdiv(n, 256), 1), 8192)); }

void un_im2col(const float* x, float* col, int B, int H, int W, int C, int Ho, int Wo, int Kp, int mode, int s,
               int pt, int pl, hipStream_t st) {
  hipLaunchKernelGGL(k_im2col, grid_for((long)B * Ho * Wo * Kp), dim3(256), 0, st, x, col, B, H, W, C, Ho, Wo, Kp,
                     mode, s, pt, pl);
  PHX_LAUNCH_CHECK();
}

void un_wprep(const float* w, float* bt, int kind, int ci, int co, int Kp, hipStream_t st) {
  const bool dg = kind == 1 || kind == 3 || kind == 5;
  hipLaunchKernelGGL(k_wprep, grid_for((long)(dg ? ci : co) * Kp), dim3(256), 0, st, w, bt, kind, ci, co, Kp);
  PHX_LAUNCH_CHECK();
}

bool un_conv3_small(const float* x, const float* Bt, const float* bias, float* out, int B, int H, int W, int C,
                    int Ho, int Wo, int N, int Kp, int mode, int s, int pt, int pl, hipStream_t st) {
  if (N > kConvMaxN || Kp > kConvMaxKp || Kp < 9 * C || (Kp & 3)) return false;
  const long tiles = cdiv((long)B * Ho * Wo, 16);
  const dim3 grid((unsigned)std::min<long>(std::max<long>(cdiv(tiles, 4), 1), 2048));
  const bool vec = C % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
#define PHX_CV(NT, MD, V) hipLaunchKernelGGL((k_conv3_small<NT, MD, V>), grid, dim3(256), 0, st, x, Bt, bias, out, B, H, W, C, Ho, Wo, N, Kp, s, pt, pl)
  switch ((N > 16 ? 4 : 0) + (mode ? 2 : 0) + (vec ? 1 : 0)) {
    case 0: PHX_CV(1, 0, false); break;
    case 1: PHX_CV(1, 0, true); break;
    case 2: PHX_CV(1, 1, false); break;
    case 3: PHX_CV(1, 1, true); break;
    case 4: PHX_CV(2, 0, false); break;
    case 5: PHX_CV(2, 0, true); break;
    case 6: PHX_CV(2, 1, false); break;
    default: PHX_CV(2, 1, true); break;
  }
#undef PHX_CV
  PHX_LAUNCH_CHECK();
  return true;
}

// row slices of a weight gradient: about 8 x PHX_WG_SLICES workgroups over the (co, k) tiles, at least 64 rows
// (and a multiple of 16) per slice, at most PHX_WG_SLICES slices (1024: C5 14.38 -> 14.00 ms against 256)
static long wgrad_rows_per_slice(long M, int Co, int Kp) {
  const long tiles = (long)cdiv(Co, 16) * cdiv(Kp, 64);
  long ns = std::min<long>(std::max<long>(cdiv(8 * PHX_WG_SLICES, tiles), 1), PHX_WG_SLICES);
  ns = std::max<long>(1, std::min<long>(ns, cdiv(M, 64)));
  return (cdiv(M, ns) + 15) / 16 * 16;
}

int un_wgrad_slices(long M, int Co, int Kp) { return (int)cdiv(M, wgrad_rows_per_slice(M, Co, Kp)); }

void un_wgrad(const float* dy, int ldy, const float* x, int ldx, int src, int B, int H, int W, int C, long M,
              int Co, int Kp, int Kin, int taps, int kind, float* part, float* g, hipStream_t st) {
  if (src != 0 && (M != (long)B * H * W || (src == 2 && ((H | W) & 1)) || Kp < 9 * C))
    throw std::runtime_error("un_wgrad: gather geometry does not match the rows");
  const long rps = wgrad_rows_per_slice(M, Co, Kp);
  const int ns = (int)cdiv(M, rps);
  const dim3 grid(cdiv(Co, 16), cdiv(Kp, 64), ns);
  // 16-B column loads when every quad of columns is one tap's channels and 16-B aligned
  const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                   (src == 0 ? (ldx % 4 == 0 && Kp % 4 == 0) : (C % 4 == 0));
#define PHX_WG(S, V) hipLaunchKernelGGL((k_wgrad_mfma<S, V>), grid, dim3(256), 0, st, dy, ldy, x, ldx, H, W, C, M, Co, Kp, rps, part)
  switch (src * 2 + (vec ? 1 : 0)) {
    case 0: PHX_WG(0, false); break;
    case 1: PHX_WG(0, true); break;
    case 2: PHX_WG(1, false); break;
    case 3: PHX_WG(1, true); break;
    case 4: PHX_WG(2, false); break;
    default: PHX_WG(2, true); break;
  }
#undef PHX_WG
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_wgrad_fold, dim3((unsigned)cdiv((long)Co * taps * Kin, 16)), dim3(256), 0, st, part, ns, Co,
                     Kp, Kin, taps, kind, g);
  PHX_LAUNCH_CHECK();
}

// row blocks of a column reduction: about 8192 elements per block (32 per lane), at most 1024
#ifndef PHX_UN_RED_ELEMS
#define PHX_UN_RED_ELEMS 8192
#endif
#ifndef PHX_UN_RED_MAXBLK
#define PHX_UN_RED_MAXBLK 1024
#endif
static int un_colred_blocks(long M, int C) {
  return (int)std::min<long>(std::max<long>(std::min<long>(cdiv(M * C, PHX_UN_RED_ELEMS), M), 1), PHX_UN_RED_MAXBLK);
}

static void colred(const ColRed& r, long M, int C, int mode, double* part, int* nblk, hipStream_t st) {
  if (C < 1 || C > 256) throw std::runtime_error("unet column reduction: C must be in [1, 256]");
  const int nb = un_colred_blocks(M, C);
  const long rpb = (M + nb - 1) / nb;
  hipLaunchKernelGGL(k_colred64, dim3(nb), dim3(256), 0, st, r, M, C, rpb, mode, part);
  PHX_LAUNCH_CHECK();
  *nblk = nb;
}

void un_bn_stats(const float* y, long M, int C, const float* gamma, float* mean, float* rstd, float* sc,
                 float* mmean, float* mvar, double* part, hipStream_t st) {
  ColRed r{y, nullptr, nullptr, nullptr, nullptr, nullptr, 0, C};
  int nb;
  colred(r, M, C, 0, part, &nb, st);
  hipLaunchKernelGGL(k_un_bn_final, dim3(cdiv(C, 4)), dim3(256), 0, st, part, nb, M, C, y, gamma, mean, rstd, sc,
                     mmean, mvar);
  PHX_LAUNCH_CHECK();
}

void un_bn_bwd(const float* da, const float* y, long M, int C, const float* mu, const float* rstd, const float* sc,
               const float* be, int act, float* mdz, float* mdzx, float* dgamma, float* dbeta, float* dy,
               double* part, hipStream_t st) {
  ColRed r{y, da, mu, rstd, sc, be, act, C};
  int nb;
  colred(r, M, C, 1, part, &nb, st);
  hipLaunchKernelGGL(k_un_bnb_final, dim3(cdiv(C, 4)), dim3(256), 0, st, part, nb, M, C, mdz, mdzx, dgamma, dbeta);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_un_bnb_apply, grid_for(M * C), dim3(256), 0, st, da, y, mu, rstd, sc, be, mdz, mdzx, dy, M * C,
                     C, act);
  PHX_LAUNCH_CHECK();
}

void un_colsum(const float* v, long M, int C, float* out, double* part, hipStream_t st) {
  ColRed r{v, nullptr, nullptr, nullptr, nullptr, nullptr, 0, C};
  int nb;
  colred(r, M, C, 2, part, &nb, st);
  hipLaunchKernelGGL(k_un_colsum_final, dim3(cdiv(C, 4)), dim3(256), 0, st, part, nb, C, out);
  PHX_LAUNCH_CHECK();
}

size_t un_colred_doubles(long M, int C) { return (size_t)un_colred_blocks(M, C) * C * 2; }

void un_bnact(const float* y, const float* mu, const float* sc, const float* be, float* a, long M, int C, int act,
              hipStream_t st) {
  hipLaunchKernelGGL(k_un_bnact, grid_for(M * C), dim3(256), 0, st, y, mu, sc, be, a, M * C, C, act);
  PHX_LAUNCH_CHECK();
}

void un_pool_drop(const float* x, float* out, uint8_t* arg, int B, int H, int W, int C, uint64_t seed, int64_t step,
                  int gimg0, int layer, hipStream_t st) {
  hipLaunchKernelGGL(k_un_pool_drop, grid_for((long)B * (H / 2) * (W / 2) * C), dim3(256), 0, st, x, out, arg, B, H, W,
                     C, seed, step, gimg0, layer);
  PHX_LAUNCH_CHECK();
}

void un_pool_drop_bwd(const float* dout, const uint8_t* arg, float* dx, int B, int H, int W, int C, uint64_t seed,
                      int64_t step, int gimg0, int layer, bool acc, hipStream_t st) {
  hipLaunchKernelGGL(k_un_pool_drop_bwd, grid_for((long)B * (H / 2) * (W / 2) * C), dim3(256), 0, st, dout, arg, dx, B,
                     H, W, C, seed, step, gimg0, layer, acc ? 1 : 0);
  PHX_LAUNCH_CHECK();
}

void un_att_s(const float* g, const float* x, const float* mu1, const float* sc1, const float* be1, const float* mu2,
              const float* sc2, const float* be2, float* s, long M, int C, hipStream_t st) {
  hipLaunchKernelGGL(k_att_s, grid_for(M * C), dim3(256), 0, st, g, x, mu1, sc1, be1, mu2, sc2, be2, s, M * C, C);
  PHX_LAUNCH_CHECK();
}

void un_att_t(const float* s, const float* w, const float* b, float* t, long M, int C, hipStream_t st) {
  hipLaunchKernelGGL(k_att_t, grid_for(M), dim3(256), 0, st, s, w, b, t, M, C);
  PHX_LAUNCH_CHECK();
}

void un_att_cat(const float* up, const float* skip, const float* t, const float* mu3, const float* sc3,
                const float* be3, float* cat, int B, long HW, int C, uint64_t seed, int64_t step, int gimg0, int layer,
                hipStream_t st) {
  hipLaunchKernelGGL(k_att_cat, grid_for((long)B * HW * 2 * C), dim3(256), 0, st, up, skip, t, mu3, sc3, be3, cat, B,
                     HW, C, seed, step, gimg0, layer);
  PHX_LAUNCH_CHECK();
}

void un_att_cat_bwd(const float* dcat, const float* skip, const float* t, const float* mu3, const float* sc3,
                    const float* be3, float* dup, float* dskip, float* dz3, int B, long HW, int C, uint64_t seed,
                    int64_t step, int gimg0, int layer, hipStream_t st) {
  if (C < 1 || C > 64 || (C & (C - 1))) throw std::runtime_error("att_cat_bwd: C must be a power of two <= 64");
  hipLaunchKernelGGL(k_att_cat_bwd, dim3((unsigned)cdiv((long)B * HW * C, 256)), dim3(256), 0, st, dcat, skip, t, mu3,
                     sc3, be3, dup, dskip, dz3, B, HW, C, seed, step, gimg0, layer);
  PHX_LAUNCH_CHECK();
}

void un_att_s_bwd(const float* dt, const float* w3, const float* g, const float* x, const float* mu1,
                  const float* sc1, const float* be1, const float* mu2, const float* sc2, const float* be2,
                  float* dsum, long M, int C, hipStream_t st) {
  hipLaunchKernelGGL(k_att_s_bwd, grid_for(M * C), dim3(256), 0, st, dt, w3, g, x, mu1, sc1, be1, mu2, sc2, be2, dsum,
                     M * C, C);
  PHX_LAUNCH_CHECK();
}

int un_loss_blocks(long M) { return (int)std::min<long>(cdiv(M, 256), 1024); }

void un_out_loss(const float* x, const float* w, const float* b, const float* tgt, float* upd, float* dz,
                 double* lpart, float* loss, long M, long HW, int C, hipStream_t st) {
  const int nb = un_loss_blocks(M);
  hipLaunchKernelGGL(k_un_out_loss, dim3(nb), dim3(256), 0, st, x, w, b, tgt, upd, dz, lpart, M, HW, C);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_un_loss_final, dim3(1), dim3(64), 0, st, lpart, nb, loss);
  PHX_LAUNCH_CHECK();
}

void un_small_dgrad(const float* dz, const float* w, float* dx, long M, int C, int O, bool acc, hipStream_t st) {
  hipLaunchKernelGGL(k_un_small_dgrad, grid_for(M * C), dim3(256), 0, st, dz, w, dx, M, C, O, acc ? 1 : 0);
  PHX_LAUNCH_CHECK();
}

void un_add(float* a, const float* b, long n, hipStream_t st) {
  hipLaunchKernelGGL(k_un_add, grid_for(n), dim3(256), 0, st, a, b, n);
  PHX_LAUNCH_CHECK();
}

void def_perm_crops(const float* images, int* info, float* crops, int B, int H, int W, int P, uint64_t seed,
                    int64_t step, int gimg0, hipStream_t st) {
  hipLaunchKernelGGL(k_def_perm, dim3(1), dim3(256), 0, st, B, seed, step, gimg0, info);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_def_crops, grid_for((long)B * P * P), dim3(256), 0, st, images, info, crops, B, H, W, P);
  PHX_LAUNCH_CHECK();
}

void def_filter(const float* nb, const float* ns, const int* nc, int B, int maxo, float H, float W, float thresh,
                float* ob, int* oc, hipStream_t st, float* os) {
  hipLaunchKernelGGL(k_def_filter, dim3(cdiv(B, 64)), dim3(64), 0, st, nb, ns, nc, B, maxo, H, W, thresh, ob, oc, os);
  PHX_LAUNCH_CHECK();
}

}  // namespace phx
