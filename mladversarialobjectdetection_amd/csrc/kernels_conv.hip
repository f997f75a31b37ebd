// kernels_conv.hip — convolution kernels of the victim forward and data-gradient (dgrad).
//
//  * 1x1 convolutions are GEMMs on the fp32 MFMA (v_mfma_f32_16x16x4_f32, exact f32, the
//    chip's full fp32 rate).  The MFMA's internal k index is permuted so that every lane
//    feeds four consecutive k from ONE 16-byte load (lane l: row l&15, k = 4*(l>>4)+t for
//    step t), for both operands, so A rows stream straight from HBM into registers.
//  * depthwise / stem convolutions are HBM-bound stencils: one lane per (pixel, 4 channels),
//    float4 NHWC accesses, neighbouring pixels served from L1/L2.
// Reference ops: Conv2D / DepthwiseConv2dNative with TF 'SAME' padding
// (efficientnet_model.py:305-359, 512-520; efficientdet_keras.py:196-207, 249-253, 387-411).
#include "common.hpp"
#include "kernels.hpp"

#include <algorithm>
#include <cstdlib>

namespace phx {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// stem: 3x3 stride 2, Cin = 3 (efficientnet_model.py:507-528).  Every EfficientDet image side is
// even, so TF SAME pads (0 top/left, 1 bottom/right) — the kernels rely on pt = pl = 0.  The
// filter index of every multiply is wave-uniform, so the 27*CO taps stream through scalar
// registers (s_load) and each lane keeps all CO output channels of its pixel in VGPRs.
// ------------------------------------------------------------------------------------------
template <int CO, bool STATS, bool BF>
__global__ __launch_bounds__(256) void k_stem_fwd(const float* __restrict__ x,
                                                  const float* __restrict__ w,
                                                  float* __restrict__ y, int B, int H, int W,
                                                  int Ho, int Wo, StatSink sink) {
  long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * Ho * Wo;
  if (STATS) {
    if (p >= total) p = total - 1;  // keep every lane for the block reduction (masked below)
  } else if (p >= total) {
    return;
  }
  const int ox = (int)(p % Wo);
  const long t = p / Wo;
  const int oy = (int)(t % Ho), b = (int)(t / Ho);
  float acc[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) acc[c] = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int iy = oy * 2 + i;
    if (iy >= H) continue;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int ix = ox * 2 + j;
      if (ix >= W) continue;
      const float* xp = x + (((long)b * H + iy) * W + ix) * 3;
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) {
        const float xv = xp[ci];
        const float* wp = w + ((i * 3 + j) * 3 + ci) * CO;
#pragma unroll
        for (int c = 0; c < CO; ++c) acc[c] = fmaf(xv, wp[c], acc[c]);
      }
    }
  }
  // fp32, training statistics: the block's 256 x CO outputs go through the LDS transpose the
  // statistics use anyway and leave as whole 16-B runs of the block's contiguous output (a lane's own
  // CO values were 8 stores of 16 B each at a 128-B lane stride)
  constexpr bool kStage = STATS && !BF && CO % 4 == 0;
  if constexpr (!kStage) {
#pragma unroll
    for (int c = 0; c < CO / 4; ++c)
      ast4<BF>(y, p * CO + 4 * c, make_float4(acc[4 * c], acc[4 * c + 1], acc[4 * c + 2], acc[4 * c + 3]));
  }
  if constexpr (STATS) {
    // statistics of the values as stored
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[c] = ast_val<BF>(acc[c]);
    // block statistics through an LDS transpose: G row groups x CO channels, two passes
    constexpr int G = 256 / CO, RG = (256 + G - 1) / G;
    __shared__ float tl[256][CO + 1];
    __shared__ float gm[G][CO], g2[G][CO], gn[G];
#pragma unroll
    for (int c = 0; c < CO; ++c) tl[threadIdx.x][c] = acc[c];
    __syncthreads();
    const int nval = (int)min<long>(256, total - (long)blockIdx.x * 256);
    if constexpr (kStage) {
      float4* yb = reinterpret_cast<float4*>(y + (long)blockIdx.x * 256 * CO);
      for (int e = threadIdx.x; e < nval * (CO / 4); e += 256) {
        const int px = e / (CO / 4), c4 = e - px * (CO / 4);
        yb[e] = make_float4(tl[px][4 * c4], tl[px][4 * c4 + 1], tl[px][4 * c4 + 2], tl[px][4 * c4 + 3]);
      }
    }
    const int t = threadIdx.x, c = t % CO, gi = t / CO;
    if (gi < G) {
      const int r0 = gi * RG, r1 = min(nval, r0 + RG);
      float sm = 0.f;
      for (int r = r0; r < r1; ++r) sm += tl[r][c];
      const float n = (float)max(0, r1 - r0);
      const float m = n > 0.f ? sm / n : 0.f;
      float q = 0.f;
      for (int r = r0; r < r1; ++r) {
        const float d = tl[r][c] - m;
        q = fmaf(d, d, q);
      }
      gm[gi][c] = m;
      g2[gi][c] = q;
      if (c == 0) gn[gi] = n;
    }
    __syncthreads();
    if (t < CO) {
      float tn = 0.f, tm = 0.f, t2 = 0.f;
      for (int k = 0; k < G; ++k) chan_merge(tn, tm, t2, gn[k], gm[k][t], g2[k][t]);
      sink_put(sink, blockIdx.x, t, tn, tm, t2);
      if (t == 0) sink_cnt(sink, blockIdx.x, tn);
    }
  }
}

// dgrad per 2x2 input quad (2Y+a, 2X+c): with pt = pl = 0, input row 2Y takes filter row 0 from
// output row Y and row 2 from Y-1, row 2Y+1 takes filter row 1 from Y (same for columns), so
// every (dy pixel, tap) pairing is fixed at compile time and the taps stay wave-uniform.
template <int CO>
__global__ __launch_bounds__(256) void k_stem_bwd(const float* __restrict__ dy,
                                                  const float* __restrict__ w,
                                                  float* __restrict__ dx, int B, int H, int W,
                                                  int Ho, int Wo, int acc_flag) {
  const int Hq = H >> 1, Wq = W >> 1;
  long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)B * Hq * Wq) return;
  const int X = (int)(q % Wq);
  const long t = q / Wq;
  const int Y = (int)(t % Hq), b = (int)(t / Hq);
  float o[2][2][3];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) o[a][c][ci] = 0.f;
  // the four dy pixels (Y - dyo, X - dxo)
#pragma unroll
  for (int dyo = 0; dyo < 2; ++dyo) {
#pragma unroll
    for (int dxo = 0; dxo < 2; ++dxo) {
      const int oy = Y - dyo, ox = X - dxo;
      if (oy < 0 || ox < 0 || oy >= Ho || ox >= Wo) continue;
      float g[CO];
      const float4* gp = reinterpret_cast<const float4*>(dy + (((long)b * Ho + oy) * Wo + ox) * CO);
#pragma unroll
      for (int c = 0; c < CO / 4; ++c) {
        const float4 v = gp[c];
        g[4 * c] = v.x; g[4 * c + 1] = v.y; g[4 * c + 2] = v.z; g[4 * c + 3] = v.w;
      }
      // rows: dyo = 0 -> (a=0,i=0), (a=1,i=1); dyo = 1 -> (a=0,i=2).  Columns alike.
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int i = dyo ? 2 : a;
        if (dyo && a) continue;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int j = dxo ? 2 : c;
          if (dxo && c) continue;
#pragma unroll
          for (int ci = 0; ci < 3; ++ci) {
            const float* wp = w + ((i * 3 + j) * 3 + ci) * CO;
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int k = 0; k < CO; k += 2) {
              s0 = fmaf(g[k], wp[k], s0);
              s1 = fmaf(g[k + 1], wp[k + 1], s1);
            }
            o[a][c][ci] += s0 + s1;
          }
        }
      }
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    float2* op = reinterpret_cast<float2*>(dx + (((long)b * H + 2 * Y + a) * W + 2 * X) * 3);
    float2 v0 = make_float2(o[a][0][0], o[a][0][1]);
    float2 v1 = make_float2(o[a][0][2], o[a][1][0]);
    float2 v2 = make_float2(o[a][1][1], o[a][1][2]);
    if (acc_flag) {
      const float2 p0 = op[0], p1 = op[1], p2 = op[2];
      v0.x += p0.x; v0.y += p0.y; v1.x += p1.x; v1.y += p1.y; v2.x += p2.x; v2.y += p2.y;
    }
    op[0] = v0;
    op[1] = v1;
    op[2] = v2;
  }
}

// Stem dgrad fused with the stem BN's backward (GradX view) and restricted to the pixels that
// are read: the image gradient's only consumer is the EOT rotation backward, which reads it where
// a pasted patch owns the pixel (k_eot_rot_bwd), so a 32x32-pixel tile without an owned pixel
// writes zeros and skips its dy reads.  A live tile stages its 17x17 dy window into LDS with the
// BN backward applied once per element (neighbouring quads re-read each dy pixel from LDS), then
// each lane computes one 2x2 input quad as k_stem_bwd does.
constexpr int kStemTQ = 16;  // quads per tile side

template <int CO, bool BF>
__global__ __launch_bounds__(256) void k_stem_bwd_gx(GradX g, const float* __restrict__ w,
                                                     const int16_t* __restrict__ owner,
                                                     float* __restrict__ dx, int B, int H, int W,
                                                     int Ho, int Wo, int tiles_x) {
  constexpr int WIN = kStemTQ + 1, C4 = CO / 4;
  __shared__ float4 sdy[WIN * WIN * C4];
  __shared__ int s_live;
  const int b = blockIdx.y;
  const int ty = blockIdx.x / tiles_x, tx = blockIdx.x - ty * tiles_x;
  const int Y0 = ty * kStemTQ, X0 = tx * kStemTQ;
  const int qy = threadIdx.x / kStemTQ, qx = threadIdx.x % kStemTQ;
  const int Y = Y0 + qy, X = X0 + qx;
  const int Hq = H >> 1, Wq = W >> 1;
  const bool inq = Y < Hq && X < Wq;
  bool own = inq;
  if (inq && owner) {
    own = false;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int16_t* op = owner + (((long)b * H + 2 * Y + a) * W + 2 * X) * 3;
#pragma unroll
      for (int e = 0; e < 6; ++e) own |= op[e] >= 0;
    }
  }
  if (threadIdx.x == 0) s_live = 0;
  __syncthreads();
  if (own) s_live = 1;
  __syncthreads();
  if (!s_live) {
    if (inq) {
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        float2* op = reinterpret_cast<float2*>(dx + (((long)b * H + 2 * Y + a) * W + 2 * X) * 3);
        op[0] = op[1] = op[2] = make_float2(0.f, 0.f);
      }
    }
    return;
  }
  // dy window rows Y0-1 .. Y0+15, cols X0-1 .. X0+15 (input row 2Y uses dy rows Y and Y-1)
  for (int e = threadIdx.x; e < WIN * WIN * C4; e += 256) {
    const int p = e / C4, c4 = e - p * C4;
    const int wy = p / WIN, wx = p - wy * WIN;
    const int oy = Y0 - 1 + wy, ox = X0 - 1 + wx;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (oy >= 0 && oy < Ho && ox >= 0 && ox < Wo) {
      const long i = (((long)b * Ho + oy) * Wo + ox) * CO + c4 * 4;
      v = *reinterpret_cast<const float4*>(g.da + i);
      if (g.y) v = gx_apply4(g, gx_chan4(g, c4 * 4), v, ald4<BF>(g.y, i));
    }
    sdy[e] = v;
  }
  __syncthreads();
  if (!inq) return;
  float o[2][2][3];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) o[a][c][ci] = 0.f;
#pragma unroll
  for (int dyo = 0; dyo < 2; ++dyo) {
#pragma unroll
    for (int dxo = 0; dxo < 2; ++dxo) {
      const int oy = Y - dyo, ox = X - dxo;
      if (oy < 0 || ox < 0 || oy >= Ho || ox >= Wo) continue;
      float gg[CO];
      const float4* gp = sdy + ((qy - dyo + 1) * WIN + (qx - dxo + 1)) * C4;
#pragma unroll
      for (int c = 0; c < C4; ++c) {
        const float4 v = gp[c];
        gg[4 * c] = v.x; gg[4 * c + 1] = v.y; gg[4 * c + 2] = v.z; gg[4 * c + 3] = v.w;
      }
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int i = dyo ? 2 : a;
        if (dyo && a) continue;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int j = dxo ? 2 : c;
          if (dxo && c) continue;
#pragma unroll
          for (int ci = 0; ci < 3; ++ci) {
            const float* wp = w + ((i * 3 + j) * 3 + ci) * CO;
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int k = 0; k < CO; k += 2) {
              s0 = fmaf(gg[k], wp[k], s0);
              s1 = fmaf(gg[k + 1], wp[k + 1], s1);
            }
            o[a][c][ci] += s0 + s1;
          }
        }
      }
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    float2* op = reinterpret_cast<float2*>(dx + (((long)b * H + 2 * Y + a) * W + 2 * X) * 3);
    op[0] = make_float2(o[a][0][0], o[a][0][1]);
    op[1] = make_float2(o[a][0][2], o[a][1][0]);
    op[2] = make_float2(o[a][1][1], o[a][1][2]);
  }
}

template <template <int> class Launch, class... Args>
static void stem_dispatch(int Co, Args... args) {
  switch (Co) {
    case 32: Launch<32>::go(args...); break;
    case 40: Launch<40>::go(args...); break;
    case 48: Launch<48>::go(args...); break;
    case 56: Launch<56>::go(args...); break;
    case 64: Launch<64>::go(args...); break;
    default: throw std::invalid_argument("stem: unsupported output channels");
  }
}

template <int CO>
struct StemFwd {
  static void go(const float* x, const float* w, float* y, int B, int H, int W, int Ho, int Wo,
                 StatSink sink, bool ybf, hipStream_t s) {
    long total = (long)B * Ho * Wo;
    sink.P = cdiv(total, 256);
    const dim3 g(cdiv(total, 256));
    if (sink.part && ybf)
      hipLaunchKernelGGL((k_stem_fwd<CO, true, true>), g, dim3(256), 0, s, x, w, y, B, H, W, Ho, Wo, sink);
    else if (sink.part)
      hipLaunchKernelGGL((k_stem_fwd<CO, true, false>), g, dim3(256), 0, s, x, w, y, B, H, W, Ho, Wo, sink);
    else if (ybf)
      hipLaunchKernelGGL((k_stem_fwd<CO, false, true>), g, dim3(256), 0, s, x, w, y, B, H, W, Ho, Wo, sink);
    else
      hipLaunchKernelGGL((k_stem_fwd<CO, false, false>), g, dim3(256), 0, s, x, w, y, B, H, W, Ho, Wo, sink);
  }
};
template <int CO>
struct StemBwd {
  static void go(const float* dy, const float* w, float* dx, int B, int H, int W, int Ho, int Wo,
                 int acc, hipStream_t s) {
    long total = (long)B * (H / 2) * (W / 2);
    hipLaunchKernelGGL((k_stem_bwd<CO>), dim3(cdiv(total, 256)), dim3(256), 0, s, dy, w, dx, B, H, W, Ho,
                       Wo, acc);
  }
};

template <int CO>
struct StemBwdGx {
  static void go(GradX g, const float* w, const int16_t* owner, float* dx, int B, int H, int W,
                 int Ho, int Wo, hipStream_t s) {
    const int tx = cdiv(W / 2, kStemTQ), ty = cdiv(H / 2, kStemTQ);
    if (g.ybf)
      hipLaunchKernelGGL((k_stem_bwd_gx<CO, true>), dim3(tx * ty, B), dim3(256), 0, s, g, w, owner, dx, B, H, W,
                         Ho, Wo, tx);
    else
      hipLaunchKernelGGL((k_stem_bwd_gx<CO, false>), dim3(tx * ty, B), dim3(256), 0, s, g, w, owner, dx, B, H, W,
                         Ho, Wo, tx);
  }
};

bool stem_bwd_gx_supported(int Co) { return Co == 32 || Co == 40 || Co == 48; }

void launch_stem_bwd_gx(GradX g, const float* w, const int16_t* owner, float* dx, int B, int H, int W,
                        int Ho, int Wo, int Co, int pt, int pl, hipStream_t s) {
  if (pt != 0 || pl != 0 || (H & 1) || (W & 1)) throw std::invalid_argument("stem: odd image side");
  switch (Co) {
    case 32: StemBwdGx<32>::go(g, w, owner, dx, B, H, W, Ho, Wo, s); break;
    case 40: StemBwdGx<40>::go(g, w, owner, dx, B, H, W, Ho, Wo, s); break;
    case 48: StemBwdGx<48>::go(g, w, owner, dx, B, H, W, Ho, Wo, s); break;
    default: throw std::invalid_argument("stem_bwd_gx: unsupported output channels");
  }
  PHX_LAUNCH_CHECK();
}

int launch_stem_fwd(const float* x, const float* w, float* y, int B, int H, int W, int Ho, int Wo,
                    int Co, int pt, int pl, hipStream_t s, StatSink sink, bool ybf) {
  if (pt != 0 || pl != 0 || (H & 1) || (W & 1)) throw std::invalid_argument("stem: odd image side");
  stem_dispatch<StemFwd>(Co, x, w, y, B, H, W, Ho, Wo, sink, ybf, s);
  PHX_LAUNCH_CHECK();
  return cdiv((long)B * Ho * Wo, 256);
}

void launch_stem_bwd(const float* dy, const float* w, float* dx, int B, int H, int W, int Ho,
                     int Wo, int Co, int pt, int pl, bool acc, hipStream_t s) {
  if (pt != 0 || pl != 0 || (H & 1) || (W & 1)) throw std::invalid_argument("stem: odd image side");
  stem_dispatch<StemBwd>(Co, dy, w, dx, B, H, W, Ho, Wo, acc ? 1 : 0, s);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// fp32 MFMA GEMM: C[M,N] (+)= A'[M,K] * Bt[N,K]^T + bias, A' = A as seen through an InX view
// (BN + activation applied on load) optionally scaled per (image, k) (SE excitation).
//
//  * block = 4 waves in a WM x WN grid (WM*WN = 4); a wave owns 32 rows x 16*NT columns, i.e.
//    2 x NT accumulator tiles of v_mfma_f32_16x16x4_f32.  Small-M shapes use WM = 1/2 and a
//    K split (blockIdx.z) with an fp32 partial slab reduced by a second kernel, so the late
//    backbone layers (M = 4096 rows, K = 1152) still fill the 256 CUs.
//  * K loop is register double-buffered: chunk k+1's loads are in flight during chunk k's MFMAs.
//  * epilogue transposes through LDS so every store instruction writes whole 16-B-per-lane
//    row segments (the 64-B-row-fragment layout of the accumulators would otherwise dominate
//    the HBM write traffic of the wide, shallow layers).
// ------------------------------------------------------------------------------------------
template <int NT>
struct GemmFrag {
  float4 a[2];
  float4 b[NT];
};

// MODE 0: raw A, 1: BN view (InX), 2: BN view x SE rowscale, 3: gradient view (GradX)
template <int NT, int MODE, int ST>
__device__ __forceinline__ void gemm_load(GemmFrag<NT>& f, const InX& Ax, const GradX& Gx,
                                          const float* __restrict__ Bt, int K, int klim, int kk,
                                          const int* rows, const bool* rok, const int* cols,
                                          const bool* cok, const float* __restrict__ rowscale,
                                          int rows_per_img) {
  const bool kok = kk < klim;  // klim: end of this workgroup's K slice (row stride stays K)
  Chan4 ck;
  GChan4 gk;
  if (MODE == 1 || MODE == 2) {
    if (kok) ck = inx_chan4(Ax, kk);
  }
  if (MODE == 3) {
    if (kok) gk = gx_chan4(Gx, kk);
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    if (rok[mt] && kok) {
      const long e = (long)rows[mt] * K + kk;
      float4 v;
      if (MODE == 3) {
        v = *reinterpret_cast<const float4*>(Gx.da + e);
        float4 yv = ald4<ST == 2>(Gx.y, e);
        v = gx_apply4(Gx, gk, v, yv);
      } else {
        v = ald4<ST == 1>(Ax.p, e);
        if (MODE == 1 || MODE == 2) v = inx_apply4(Ax, ck, v);
        if (MODE == 2) {
          float4 sc = *reinterpret_cast<const float4*>(rowscale + (long)(rows[mt] / rows_per_img) * K + kk);
          v.x *= sc.x; v.y *= sc.y; v.z *= sc.z; v.w *= sc.w;
        }
      }
      f.a[mt] = v;
    } else {
      f.a[mt] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    f.b[nt] = (cok[nt] && kok) ? *reinterpret_cast<const float4*>(Bt + (long)cols[nt] * K + kk)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
}

// The 16-wide (NT = 1) path's loads run PHX_GEMM_PD chunks ahead: the raw loads (A or da / y, B)
// land in a ring of registers and the view is applied just before the chunk's MFMAs, so a wave
// keeps PD chunks of HBM reads in flight instead of one.  The view's per-channel parameters of the
// workgroup's K slice sit in an LDS table (filled once per workgroup) rather than in the ring.
// Same arithmetic in the same order as gemm_load: bit-identical.
#ifndef PHX_GEMM_PD
#define PHX_GEMM_PD 2
#endif
constexpr int kGemmTab = 256;  // K-slice length the channel table holds (longer slices: PD = 1)

template <int MODE>
struct GemmRaw1 {
  float4 a[2];
  float4 y[2];   // MODE 3: the BN input y
  float4 rs[2];  // MODE 2: the SE row scale
  float4 b;
};

template <int MODE, int ST>
__device__ __forceinline__ void gemm_raw1(GemmRaw1<MODE>& f, const InX& Ax, const GradX& Gx,
                                          const float* __restrict__ Bt, int K, int klim, int kk,
                                          const int* rows, const bool* rok, int col, bool cok,
                                          const float* __restrict__ rowscale, int rows_per_img) {
  const bool kok = kk < klim;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    if (rok[mt] && kok) {
      const long e = (long)rows[mt] * K + kk;
      if (MODE == 3) {
        f.a[mt] = *reinterpret_cast<const float4*>(Gx.da + e);
        f.y[mt] = ald4<ST == 2>(Gx.y, e);
      } else {
        f.a[mt] = ald4<ST == 1>(Ax.p, e);
        if (MODE == 2)
          f.rs[mt] = *reinterpret_cast<const float4*>(rowscale + (long)(rows[mt] / rows_per_img) * K + kk);
      }
    }
  }
  f.b = (cok && kok) ? *reinterpret_cast<const float4*>(Bt + (long)col * K + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// tab: parameter p of slice channel kl at tab[p * kGemmTab + kl] (MODE 1/2: mu, sc, be; MODE 3:
// mu, rstd, sc, be, mdz, mdzx)
template <int MODE>
__device__ __forceinline__ void gemm_apply1(GemmFrag<1>& f, const GemmRaw1<MODE>& r, const InX& Ax,
                                            const GradX& Gx, const float* tab, int kl, bool kok,
                                            const bool* rok) {
  Chan4 ck;
  GChan4 gk;
  if (kok) {
    if (MODE == 1 || MODE == 2) {
      const float4 m = *reinterpret_cast<const float4*>(tab + kl);
      const float4 s = *reinterpret_cast<const float4*>(tab + kGemmTab + kl);
      const float4 b = *reinterpret_cast<const float4*>(tab + 2 * kGemmTab + kl);
      ck.mu[0] = m.x; ck.mu[1] = m.y; ck.mu[2] = m.z; ck.mu[3] = m.w;
      ck.sc[0] = s.x; ck.sc[1] = s.y; ck.sc[2] = s.z; ck.sc[3] = s.w;
      ck.be[0] = b.x; ck.be[1] = b.y; ck.be[2] = b.z; ck.be[3] = b.w;
    }
    if (MODE == 3) {
      gk.mu = *reinterpret_cast<const float4*>(tab + kl);
      gk.rs = *reinterpret_cast<const float4*>(tab + kGemmTab + kl);
      gk.sc = *reinterpret_cast<const float4*>(tab + 2 * kGemmTab + kl);
      gk.be = *reinterpret_cast<const float4*>(tab + 3 * kGemmTab + kl);
      gk.m1 = *reinterpret_cast<const float4*>(tab + 4 * kGemmTab + kl);
      gk.m2 = *reinterpret_cast<const float4*>(tab + 5 * kGemmTab + kl);
    }
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    if (rok[mt] && kok) {
      float4 v = r.a[mt];
      if (MODE == 3) {
        v = gx_apply4(Gx, gk, v, r.y[mt]);
      } else {
        if (MODE == 1 || MODE == 2) v = inx_apply4(Ax, ck, v);
        if (MODE == 2) {
          v.x *= r.rs[mt].x; v.y *= r.rs[mt].y; v.z *= r.rs[mt].z; v.w *= r.rs[mt].w;
        }
      }
      f.a[mt] = v;
    } else {
      f.a[mt] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  f.b[0] = r.b;
}

// Column statistics of a block's C tile for the BN that consumes it (StatSink).  Lane (q, r) of a
// wave holds rows 4q+j (j < 4) of column r in each of its 2 x NT accumulator tiles: a column's 32
// wave rows sit in 8 registers of 4 lanes (r, r+16, r+32, r+48).  Two passes over the registers
// (mean, then M2 about it) plus xor-shuffles give each wave (n, mean, M2) per column; the WM
// waves that share columns are merged through LDS (Chan) and written as partial row blockIdx.x.
template <int NT, int WM, bool BF>
__device__ __forceinline__ void gemm_stats(const floatx4 (&acc)[2][NT], const float* __restrict__ bias,
                                           int M, int N, int m_base, int n_base, int wave, int wm,
                                           int wn, int lane, const StatSink& sink) {
  __shared__ float2 wstat[4][16 * NT];
  __shared__ float wcnt[4];
  const int q = lane >> 4, r = lane & 15;
  const float n = (float)max(0, min(32, M - m_base));
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = n_base + nt * 16 + r;
    const float b = (bias && col < N) ? bias[col] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (m_base + mt * 16 + 4 * q + j < M) s += ast_val<BF>(acc[mt][nt][j] + b);
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    const float mean = n > 0.f ? s / n : 0.f;
    float m2 = 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (m_base + mt * 16 + 4 * q + j < M) {
          const float d = ast_val<BF>(acc[mt][nt][j] + b) - mean;
          m2 = fmaf(d, d, m2);
        }
    m2 += __shfl_xor(m2, 16);
    m2 += __shfl_xor(m2, 32);
    if (q == 0) wstat[wave][nt * 16 + r] = make_float2(mean, m2);
  }
  if (lane == 0) wcnt[wave] = n;
  __syncthreads();
  if (wm == 0) {
    for (int cl = lane; cl < 16 * NT; cl += 64) {
      const int col = n_base + cl;
      if (col >= N) continue;
      float tn = 0.f, tm = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        const int wv = wn * WM + w;
        const float2 v = wstat[wv][cl];
        chan_merge(tn, tm, t2, wcnt[wv], v.x, v.y);
      }
      sink_put(sink, blockIdx.x, col, tn, tm, t2);
    }
    if (wn == 0 && lane == 0) {
      float tn = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) tn += wcnt[w];
      sink_cnt(sink, blockIdx.x, tn);
    }
  }
}

// BN-backward sums (GradSink) of a dgrad block's output tile: value v (+ the accumulated C when
// acc_flag) at rows 4q+j of column r per accumulator tile, the BN input y loaded at the same
// element; xor-shuffles over q, then the WM waves sharing the columns meet in LDS.
template <int NT, int WM, bool YBF>
__device__ __forceinline__ void gemm_gsums(const floatx4 (&acc)[2][NT], const float* __restrict__ C,
                                           int acc_flag, int M, int N, int m_base, int n_base, int wave,
                                           int wm, int wn, int lane, const GradSink& g) {
  __shared__ float2 wsum[4][16 * NT];
  const int q = lane >> 4, r = lane & 15;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = n_base + nt * 16 + r;
    float s1 = 0.f, s2 = 0.f;
    if (col < N) {
      const float mu = g.mu[col], rs = g.rstd[col], sc = g.sc[col], be = g.be[col];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = m_base + mt * 16 + 4 * q + j;
          if (row < M) {
            const long e = (long)row * N + col;
            float v = acc[mt][nt][j];
            if (acc_flag) v += C[e];
            gs_one(v, ald1<YBF>(g.y, e), mu, rs, sc, be, g.act, s1, s2);
          }
        }
    }
    s1 += __shfl_xor(s1, 16);
    s1 += __shfl_xor(s1, 32);
    s2 += __shfl_xor(s2, 16);
    s2 += __shfl_xor(s2, 32);
    if (q == 0) wsum[wave][nt * 16 + r] = make_float2(s1, s2);
  }
  __syncthreads();
  if (wm == 0) {
    for (int cl = lane; cl < 16 * NT; cl += 64) {
      const int col = n_base + cl;
      if (col >= N) continue;
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        const float2 v = wsum[wn * WM + w][cl];
        t1 += v.x;
        t2 += v.y;
      }
      gsink_put(g, blockIdx.x, col, t1, t2);
    }
  }
}

// STATS: the BN batch statistics of C (bias included) are reduced in the epilogue into partial
// row blockIdx.x of the StatSink (one (sum, M2) per column over the block's 32*WM rows).
// SK: 0 plain, 1 StatSink (forward BN statistics), 2 GradSink (BN-backward sums of a dgrad)
// ST: activation storage (as k_gemm2): 0 fp32; 1 forward with bf16 A and C; 2 dgrad with a bf16 y
template <int NT, int WM, int MODE, int SK, int ST>
__global__ __launch_bounds__(256) void k_gemm(InX Ax, GradX Gx, const float* __restrict__ Bt,
                                              const float* __restrict__ bias,
                                              float* __restrict__ C, int M, int N, int K,
                                              int acc_flag, const float* __restrict__ rowscale,
                                              int rows_per_img, int kslice,
                                              float* __restrict__ partial, StatSink sink,
                                              GradSink gsk) {
  constexpr int WN = 4 / WM;
  constexpr int LDW = 16 * NT + 4;  // LDS row pitch (floats) of a wave's staging tile
  __shared__ float stage[4][16 * LDW];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int q = lane >> 4, r = lane & 15;
  const int m_base = blockIdx.x * (32 * WM) + wm * 32;
  const int n_base = blockIdx.y * (16 * NT * WN) + wn * (16 * NT);
  const int kbeg = blockIdx.z * kslice;
  const int kend = min(K, kbeg + kslice);

  floatx4 acc[2][NT];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

  int rows[2];
  bool rok[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    rows[mt] = m_base + mt * 16 + r;
    rok[mt] = rows[mt] < M;
  }
  int cols[NT];
  bool cok[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    cols[nt] = n_base + nt * 16 + r;
    cok[nt] = cols[nt] < N;
  }

  constexpr int PD = NT == 1 ? PHX_GEMM_PD : 1;
  bool done = false;
  if constexpr (PD > 1) {
    constexpr int NP = MODE == 3 ? 6 : (MODE == 1 || MODE == 2) ? 3 : 0;
    __shared__ __attribute__((aligned(16))) float ctab[NP > 0 ? NP * kGemmTab : 1];
    const int klen = kend - kbeg;  // uniform over the workgroup
    if (NP == 0 || klen <= kGemmTab) {
      done = true;
      if constexpr (NP > 0) {
        for (int i = threadIdx.x; i < NP * klen; i += 256) {
          const int pp = i / klen, kl = i - pp * klen;
          const float* src;
          if constexpr (MODE == 3) {
            src = pp == 0 ? Gx.mu : pp == 1 ? Gx.rstd : pp == 2 ? Gx.sc : pp == 3 ? Gx.be : pp == 4 ? Gx.mdz : Gx.mdzx;
          } else {
            src = pp == 0 ? Ax.mu : pp == 1 ? Ax.sc : Ax.be;
          }
          ctab[pp * kGemmTab + kl] = src[kbeg + kl];
        }
      }
      GemmRaw1<MODE> rr[PD];
#pragma unroll
      for (int i = 0; i < PD; ++i) {
        const int kc = kbeg + 16 * i;
        if (kc < kend)
          gemm_raw1<MODE, ST>(rr[i], Ax, Gx, Bt, K, kend, kc + 4 * q, rows, rok, cols[0], cok[0], rowscale,
                              rows_per_img);
      }
      if constexpr (NP > 0) __syncthreads();
      for (int k0 = kbeg; k0 < kend; k0 += 16 * PD) {
#pragma unroll
        for (int i = 0; i < PD; ++i) {
          const int kc = k0 + 16 * i;
          if (kc < kend) {
            GemmFrag<1> f;
            gemm_apply1<MODE>(f, rr[i], Ax, Gx, ctab, kc - kbeg + 4 * q, kc + 4 * q < kend, rok);
            const int kn = kc + 16 * PD;
            if (kn < kend)
              gemm_raw1<MODE, ST>(rr[i], Ax, Gx, Bt, K, kend, kn + 4 * q, rows, rok, cols[0], cok[0], rowscale,
                                  rows_per_img);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
              acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[mt].x, f.b[0].x, acc[mt][0], 0, 0, 0);
              acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[mt].y, f.b[0].y, acc[mt][0], 0, 0, 0);
              acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[mt].z, f.b[0].z, acc[mt][0], 0, 0, 0);
              acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[mt].w, f.b[0].w, acc[mt][0], 0, 0, 0);
            }
          }
        }
      }
    }
  }
  if (!done) {
  GemmFrag<NT> cur, nxt;
  if (kbeg < kend)
    gemm_load<NT, MODE, ST>(cur, Ax, Gx, Bt, K, kend, kbeg + 4 * q, rows, rok, cols, cok, rowscale,
                        rows_per_img);
  for (int k0 = kbeg; k0 < kend; k0 += 16) {
    const bool more = k0 + 16 < kend;
    if (more)
      gemm_load<NT, MODE, ST>(nxt, Ax, Gx, Bt, K, kend, k0 + 16 + 4 * q, rows, rok, cols, cok, rowscale,
                          rows_per_img);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.a[mt].x, cur.b[nt].x, acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.a[mt].y, cur.b[nt].y, acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.a[mt].z, cur.b[nt].z, acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.a[mt].w, cur.b[nt].w, acc[mt][nt], 0, 0, 0);
      }
    }
    if (more) cur = nxt;
  }
  }

  constexpr bool CBF = ST == 1;
  if constexpr (SK == 1) gemm_stats<NT, WM, CBF>(acc, bias, M, N, m_base, n_base, wave, wm, wn, lane, sink);
  if constexpr (SK == 2) gemm_gsums<NT, WM, ST == 2>(acc, C, acc_flag, M, N, m_base, n_base, wave, wm, wn, lane, gsk);

  // epilogue: accumulator element j of tile (mt,nt) is row 4q+j, col r.  Stage 16 rows at a
  // time through LDS and store row segments with 16-B lanes.
  float* st = stage[wave];
  const bool split = partial != nullptr;
  const bool cbf = CBF && !split;  // split-K partial slabs stay fp32
  float* out = split ? partial + (long)blockIdx.z * M * N : C;
  const int ncols = min(16 * NT, N - n_base);  // valid columns of this wave
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[(4 * q + j) * LDW + nt * 16 + r] = acc[mt][nt][j];
    // the staging tile is private to this wave: program order orders its LDS write/read
    if (ncols > 0) {
      const int row0 = m_base + mt * 16;
      if ((ncols & 3) == 0 && (N & 3) == 0 && (n_base & 3) == 0) {
        const int c4n = ncols >> 2;  // float4 per row
        for (int e = lane; e < 16 * c4n; e += 64) {
          const int rr = e / c4n, c4 = e % c4n;
          const int row = row0 + rr;
          if (row >= M) continue;
          const int col = n_base + c4 * 4;
          float4 v = *reinterpret_cast<const float4*>(st + rr * LDW + c4 * 4);
          if (!split) {
            if (bias) {
              v.x += bias[col]; v.y += bias[col + 1]; v.z += bias[col + 2]; v.w += bias[col + 3];
            }
            const long ce = (long)row * N + col;
            if (acc_flag) {
              const float4 o = cbf ? ald4<true>(out, ce) : *reinterpret_cast<const float4*>(out + ce);
              v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
            }
            if (cbf) ast4<true>(out, ce, v);
            else *reinterpret_cast<float4*>(out + ce) = v;
          } else {
            *reinterpret_cast<float4*>(out + (long)row * N + col) = v;
          }
        }
      } else {
        for (int e = lane; e < 16 * ncols; e += 64) {
          const int rr = e / ncols, cc = e % ncols;
          const int row = row0 + rr;
          if (row >= M) continue;
          const int col = n_base + cc;
          float v = st[rr * LDW + cc];
          const long ce = (long)row * N + col;
          if (!split) {
            if (bias) v += bias[col];
            if (acc_flag) v += cbf ? ald1<true>(out, ce) : out[ce];
          }
          if (cbf) ast1<true>(out, ce, v);
          else out[ce] = v;
        }
      }
    }
  }
}

// slabs whose loads a split-K reduce issues together (more are added one by one)
constexpr int kSkMax = 8;

// split-K reduction: C (+)= sum_s partial[s] + bias (BF: C holds bf16 activations)
template <bool BF>
__global__ __launch_bounds__(256) void k_gemm_splitk_reduce(const float* __restrict__ partial,
                                                            int S, long MN, int N,
                                                            const float* __restrict__ bias,
                                                            float* __restrict__ C, int acc_flag) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= MN) return;
  // every slab's load in flight at once (clamped to the last slab past S), added in slab order
  float p[kSkMax];
#pragma unroll
  for (int s = 0; s < kSkMax; ++s) p[s] = partial[(long)min(s, S - 1) * MN + i];
  float v = 0.f;
#pragma unroll
  for (int s = 0; s < kSkMax; ++s)
    if (s < S) v += p[s];
  for (int s = kSkMax; s < S; ++s) v += partial[(long)s * MN + i];
  if (bias) v += bias[i % N];
  if (acc_flag) v += ald1<BF>(C, i);
  ast1<BF>(C, i, v);
}

// split-K reduction with the BN column statistics of the result (forward GEMMs feeding a BN):
// block b owns rows [b*RB, (b+1)*RB); lane t owns column quad t % N4 of every (256/N4)-th row,
// keeps shifted sums (shift = its first value) and the block merges its lanes (Chan) into
// partial row b of the StatSink.  N4 = N/4 <= 256.  BF: C holds bf16 activations (statistics of
// the stored values).
template <bool BF>
__global__ __launch_bounds__(256) void k_gemm_splitk_reduce_stats(const float* __restrict__ partial,
                                                                  int S, int M, int N, int RB,
                                                                  const float* __restrict__ bias,
                                                                  float* __restrict__ C,
                                                                  StatSink sink) {
  __shared__ float4 sm[256], s2[256];
  __shared__ float sn[256];
  const int N4 = N >> 2, rpi = 256 / N4;
  const int t = threadIdx.x, c4 = t % N4, rs = t / N4;
  const int r0 = blockIdx.x * RB, r1 = min(M, r0 + RB);
  const long MN = (long)M * N;
  float n = 0.f;
  float4 sh = make_float4(0.f, 0.f, 0.f, 0.f), a = sh, q = sh;
  if (rs < rpi) {
    const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + c4 * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = r0 + rs; r < r1; r += rpi) {
      const long e = (long)r * N + c4 * 4;
      // every slab's load in flight at once (clamped to the last slab past S), added in slab order
      float4 p[kSkMax];
#pragma unroll
      for (int k = 0; k < kSkMax; ++k) p[k] = *reinterpret_cast<const float4*>(partial + min(k, S - 1) * MN + e);
      float4 v = bv;
#pragma unroll
      for (int k = 0; k < kSkMax; ++k)
        if (k < S) {
          v.x += p[k].x; v.y += p[k].y; v.z += p[k].z; v.w += p[k].w;
        }
      for (int k = kSkMax; k < S; ++k) {
        const float4 q = *reinterpret_cast<const float4*>(partial + k * MN + e);
        v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
      }
      ast4<BF>(C, e, v);
      if constexpr (BF) v = make_float4(round_bf16(v.x), round_bf16(v.y), round_bf16(v.z), round_bf16(v.w));
      if (n == 0.f) sh = v;
      const float4 d = make_float4(v.x - sh.x, v.y - sh.y, v.z - sh.z, v.w - sh.w);
      a.x += d.x; a.y += d.y; a.z += d.z; a.w += d.w;
      q.x = fmaf(d.x, d.x, q.x); q.y = fmaf(d.y, d.y, q.y); q.z = fmaf(d.z, d.z, q.z); q.w = fmaf(d.w, d.w, q.w);
      n += 1.f;
    }
  }
  // (n, mean, M2) of this lane
  const float inv = n > 0.f ? 1.f / n : 0.f;
  sm[t] = make_float4(sh.x + a.x * inv, sh.y + a.y * inv, sh.z + a.z * inv, sh.w + a.w * inv);
  s2[t] = make_float4(q.x - a.x * a.x * inv, q.y - a.y * a.y * inv, q.z - a.z * a.z * inv, q.w - a.w * a.w * inv);
  sn[t] = n;
  __syncthreads();
  if (rs == 0) {
    float tn[4] = {0.f, 0.f, 0.f, 0.f}, tm[4] = {0.f, 0.f, 0.f, 0.f}, t2[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < rpi; ++k) {
      const int u = k * N4 + c4;
      const float4 m = sm[u], v = s2[u];
      chan_merge(tn[0], tm[0], t2[0], sn[u], m.x, fmaxf(v.x, 0.f));
      chan_merge(tn[1], tm[1], t2[1], sn[u], m.y, fmaxf(v.y, 0.f));
      chan_merge(tn[2], tm[2], t2[2], sn[u], m.z, fmaxf(v.z, 0.f));
      chan_merge(tn[3], tm[3], t2[3], sn[u], m.w, fmaxf(v.w, 0.f));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) sink_put(sink, blockIdx.x, c4 * 4 + j, tn[j], tm[j], t2[j]);
    if (c4 == 0) sink_cnt(sink, blockIdx.x, tn[0]);
  }
}

struct GemmCall {
  InX A;
  GradX G;
  const float* Bt;
  const float* bias;
  float* C;
  int M, N, K, accf;
  const float* rs;
  int rpi, kslice;
  float* part;
  StatSink sink;
  GradSink gsk;
};

// st: activation storage (ST of k_gemm).  bf16 storage variants exist for NT = 1 only: a bf16
// context runs this kernel for its N <= 16 convs (gemm_impl_for), which plan NT = 1.
template <int WM, int MODE, int SK>
static void gemm_dispatch_nt(int nt, dim3 g, hipStream_t s, const GemmCall& a, int st) {
#define PHX_G(NT_, ST_)                                                                                \
    PHX_TLAUNCH((k_gemm<NT_, WM, MODE, SK, ST_>), g, dim3(256), 0, s, a.A, a.G, a.Bt, a.bias,   \
                       a.C, a.M, a.N, a.K, a.accf, a.rs, a.rpi, a.kslice, a.part, a.sink, a.gsk);
  if (st) {
    constexpr bool fwd = MODE == 1 || MODE == 2 || SK == 1, dgrad = MODE == 3 || SK == 2;
    if (nt != 1) throw std::runtime_error("gemm: bf16 storage needs NT = 1");
    if (st == 1 && !dgrad) {
      PHX_G(1, 1)
    } else if (st == 2 && !fwd) {
      PHX_G(1, 2)
    } else {
      throw std::logic_error("gemm: storage variant does not match the mode");
    }
    return;
  }
  switch (nt) {
    case 1: PHX_G(1, 0) break;
    case 2: PHX_G(2, 0) break;
    case 3: PHX_G(3, 0) break;
    case 4: PHX_G(4, 0) break;
    case 5: PHX_G(5, 0) break;
    case 6: PHX_G(6, 0) break;
    case 7: PHX_G(7, 0) break;
    case 8: PHX_G(8, 0) break;
    default: throw std::runtime_error("gemm: bad NT");
  }
#undef PHX_G
}

template <int MODE, int SK>
static void gemm_dispatch(int wm, int nt, dim3 g, hipStream_t s, const GemmCall& a, int st) {
  if (wm == 4) gemm_dispatch_nt<4, MODE, SK>(nt, g, s, a, st);
  else if (wm == 2) gemm_dispatch_nt<2, MODE, SK>(nt, g, s, a, st);
  else gemm_dispatch_nt<1, MODE, SK>(nt, g, s, a, st);
}

GemmPlan plan_gemm(int M, int N, int K) {
  GemmPlan p;
  p.nt = N <= 128 ? (N + 15) / 16 : 8;
  const long target = 512;  // ~2 workgroups per CU
  p.wm = 1;
  for (int wm : {4, 2, 1}) {
    const int wn = 4 / wm;
    long wgs = (long)cdiv(M, 32 * wm) * cdiv(N, 16 * p.nt * wn);
    // wide waves along N only help when N spans them
    if (wn > 1 && 16 * p.nt * (wn - 1) >= N) continue;
    p.wm = wm;
    if (wgs >= target) break;
  }
  const int wn = 4 / p.wm;
  p.gx = cdiv(M, 32 * p.wm);
  p.gy = cdiv(N, 16 * p.nt * wn);
  long wgs = (long)p.gx * p.gy;
  p.splits = 1;
  if (wgs < 256 && K >= 256) {
    int s = (int)((target + wgs - 1) / wgs);
    s = std::min(s, K / 128);
    p.splits = std::max(1, s);
  }
  p.kslice = ((K + p.splits - 1) / p.splits + 15) / 16 * 16;
  p.splits = (K + p.kslice - 1) / p.kslice;
  return p;
}

size_t gemm_partial_floats(int M, int N, int K, bool bf16) {
  GemmPlan p = plan_gemm(M, N, K);
  Gemm2Plan q = plan_gemm2(M, N, K, gemm2_target_wgs(), bf16);
  // the implicit-im2col launches plan without the A-resident and wave-split-K kernels: they may
  // split K across workgroups where a 1x1 conv of the same shape does not
  Gemm2Plan g = plan_gemm2(M, N, K, gemm2_target_wgs(), bf16, false);
  const size_t a = p.splits > 1 ? (size_t)p.splits * M * N : 0;
  const size_t b = q.splits > 1 ? (size_t)q.splits * M * N : 0;
  const size_t c = g.splits > 1 ? (size_t)g.splits * M * N : 0;
  return std::max(a, std::max(b, c));
}

// which GEMM implementation launch_gemm / launch_gemm_dgrad use: PHX_GEMM=1 (16x16x4 register
// kernel) or 2 (LDS-tiled persistent 32x32x2 kernel, default); PHX_GEMM_WGS: persistent width
static int gemm_impl_env() {
  static int v = [] {
    const char* e = getenv("PHX_GEMM");
    return e ? atoi(e) : 0;
  }();
  return v;
}
// default (0): the 32x32 LDS-tiled kernel except for 16-wide outputs, where its 32-column tile
// would idle half the matrix core and the 16x16 register kernel streams faster (tools/gemm_bench)
int gemm_impl_for(int N, bool) {
  const int e = gemm_impl_env();
  if (e) return e;
  return N <= 16 ? 1 : 2;
}
int gemm_impl() { return gemm_impl_env() ? gemm_impl_env() : 2; }
int gemm2_target_wgs() {
  static int v = [] {
    const char* e = getenv("PHX_GEMM_WGS");
    return e ? atoi(e) : 1024;
  }();
  return v;
}

// rows per block of the split-K reduce-with-statistics kernel: about PHX_SKR_BLOCKS blocks
// (default 512: a lane walks half as many rows, -0.06 ms/step against 256)
static int splitk_stats_rb(int M, int N) {
  static const long blocks = [] {
    const char* e = getenv("PHX_SKR_BLOCKS");
    return e ? std::max(1L, atol(e)) : 512L;
  }();
  const int rpi = 256 / (N / 4);
  return rpi * std::max(1, cdiv(M, (long)rpi * blocks));
}

int gemm_splitk_stats_partials(int M, int N) { return cdiv(M, splitk_stats_rb(M, N)); }

// 0: the statistics cannot be fused into this GEMM (split-K with N > 1024)
int gemm_stat_partials(int M, int N, int K, bool bf16) {
  if (gemm_impl_for(N, bf16) == 2) {
    Gemm2Plan q = plan_gemm2(M, N, K, gemm2_target_wgs(), bf16);
    if (q.splits > 1) return N <= 1024 ? gemm_splitk_stats_partials(M, N) : 0;
    return q.P;
  }
  GemmPlan p = plan_gemm(M, N, K);
  if (p.splits > 1) return N <= 1024 ? gemm_splitk_stats_partials(M, N) : 0;
  return p.gx;
}

// reduce the split-K partial slabs into C (+ bias, + C when acc); with a StatSink the BN column
// statistics of the result come out of the same pass.  Returns the StatSink partial rows.
int gemm_splitk_finish(const float* partial, int splits, int M, int N, const float* bias, float* C,
                       bool acc, StatSink sink, hipStream_t s, bool cbf) {
  if (sink.part) {
    const int rb = splitk_stats_rb(M, N);
    sink.P = cdiv(M, rb);
    if (cbf)
      PHX_TLAUNCH(k_gemm_splitk_reduce_stats<true>, dim3(cdiv(M, rb)), dim3(256), 0, s, partial, splits,
                         M, N, rb, bias, C, sink);
    else
      PHX_TLAUNCH(k_gemm_splitk_reduce_stats<false>, dim3(cdiv(M, rb)), dim3(256), 0, s, partial, splits,
                         M, N, rb, bias, C, sink);
    PHX_LAUNCH_CHECK();
    return sink.P;
  }
  long mn = (long)M * N;
  if (cbf)
    PHX_TLAUNCH(k_gemm_splitk_reduce<true>, dim3(cdiv(mn, 256)), dim3(256), 0, s, partial, splits, mn, N,
                       bias, C, acc ? 1 : 0);
  else
    PHX_TLAUNCH(k_gemm_splitk_reduce<false>, dim3(cdiv(mn, 256)), dim3(256), 0, s, partial, splits, mn, N,
                       bias, C, acc ? 1 : 0);
  PHX_LAUNCH_CHECK();
  return 0;
}

int gemm1_run(int mode, InX A, GradX G, const float* Bt, const float* bias, float* C, int M, int N,
              int K, bool acc, const float* rowscale, int rows_per_img, hipStream_t s, float* partial,
              StatSink sink, GradSink gsk) {
  if (K % 4 != 0) throw std::runtime_error("gemm: K must be a multiple of 4");
  GemmPlan p = plan_gemm(M, N, K);
  float* part = p.splits > 1 ? partial : nullptr;
  if (p.splits > 1 && !partial) throw std::runtime_error("gemm: split-K needs a partial buffer");
  const bool stats = sink.part != nullptr;
  if (stats && (acc || mode == 3 || (N & 3) || (p.splits > 1 && N > 1024)))
    throw std::runtime_error("gemm: unsupported statistics epilogue");
  const bool kstats = stats && p.splits == 1;
  if (stats) sink.P = p.splits > 1 ? cdiv(M, splitk_stats_rb(M, N)) : p.gx;
  const bool gs = gsk.part != nullptr;
  if (gs && p.splits > 1) throw std::runtime_error("gemm: GradSink with split-K");
  gsk.P = p.gx;
  dim3 g(p.gx, p.gy, p.splits);
  GemmCall a{A, G, Bt, bias, C, M, N, K, acc ? 1 : 0, rowscale, mode == 2 ? rows_per_img : 1,
             p.kslice, part, sink, gsk};
  const int st = A.bf ? 1 : ((G.y && G.ybf) || (gs && gsk.ybf)) ? 2 : 0;
  switch (mode) {
    case 0:
      if (kstats) gemm_dispatch<0, 1>(p.wm, p.nt, g, s, a, st);
      else if (gs) gemm_dispatch<0, 2>(p.wm, p.nt, g, s, a, st);
      else gemm_dispatch<0, 0>(p.wm, p.nt, g, s, a, st);
      break;
    case 1: kstats ? gemm_dispatch<1, 1>(p.wm, p.nt, g, s, a, st) : gemm_dispatch<1, 0>(p.wm, p.nt, g, s, a, st); break;
    case 2: kstats ? gemm_dispatch<2, 1>(p.wm, p.nt, g, s, a, st) : gemm_dispatch<2, 0>(p.wm, p.nt, g, s, a, st); break;
    default: gs ? gemm_dispatch<3, 2>(p.wm, p.nt, g, s, a, st) : gemm_dispatch<3, 0>(p.wm, p.nt, g, s, a, st); break;
  }
  if (gs) {
    PHX_LAUNCH_CHECK();
    return p.gx;
  }
  PHX_LAUNCH_CHECK();
  if (p.splits > 1) {
    const int np = gemm_splitk_finish(partial, p.splits, M, N, bias, C, acc, sink, s, st == 1);
    if (stats) return np;
  }
  return p.gx;
}

int launch_gemm(InX A, const float* Bt, const float* bias, float* C, int M, int N, int K,
                bool acc, const float* rowscale, int rows_per_img, hipStream_t s,
                float* partial, StatSink sink, bool bf16) {
  if (rowscale && !A.mu) throw std::runtime_error("gemm: rowscale requires a BN view");
  const int mode = rowscale ? 2 : (A.mu ? 1 : 0);
  if (gemm_impl_for(N, bf16) == 2)
    return gemm2_run(mode, A, GradX{}, Bt, bias, C, M, N, K, acc, rowscale, rows_per_img, s, partial, sink,
                     gemm2_target_wgs(), GradSink{}, bf16);
  return gemm1_run(mode, A, GradX{}, Bt, bias, C, M, N, K, acc, rowscale, rows_per_img, s, partial, sink,
                   GradSink{});
}

// A 3x3 convolution as one GEMM whose A operand is the column matrix gathered on the fly (k_gemm2
// MODE 4): out[m][n] = bias[n] + sum_k col[m][k] Bt[n][k], k = (ky*3 + kx)*C + c, for the gathers of
// k_im2col (mode 0: stride s, pads (pt, pl); mode 1: the stride-2 transposed conv's parity gather).
// Needs power-of-2 C >= 4 and spatial sizes (shifts and masks in the kernel) and K = 9C; returns
// false (nothing launched) otherwise.
static int ilog2_exact(long v) {
  int l = 0;
  while ((1L << l) < v) ++l;
  return (1L << l) == v ? l : -1;
}

bool gemm_gather_ok(int B, int H, int W, int C, int Ho, int Wo, int K, int mode, int s, int pt, int pl) {
  const int lC = ilog2_exact(C), lW = ilog2_exact(W), lH = ilog2_exact(H), lWo = ilog2_exact(Wo),
            lHo = ilog2_exact(Ho);
  return C >= 4 && K == 9 * C && lC >= 0 && lC <= 15 && lW >= 0 && lW <= 15 &&
         lH >= 0 && lH <= 15 && lWo >= 0 && lWo <= 15 && lHo >= 0 && lHo <= 15 && (s == 1 || s == 2) && pt >= 0 &&
         pt <= 3 && pl >= 0 && pl <= 3 && (mode == 0 || (mode == 1 && s == 2)) &&
         (long)B * Ho * Wo < (1L << 31) && ((long)B << (lH + lW + lC)) < (1L << 40);
}

int launch_gemm_gather(const float* x, int B, int H, int W, int C, int Ho, int Wo, int mode, int s, int pt, int pl,
                       const float* Bt, const float* bias, float* out, int N, int K, hipStream_t st, float* partial) {
  if (!gemm_gather_ok(B, H, W, C, Ho, Wo, K, mode, s, pt, pl))
    throw std::runtime_error("gemm gather: unsupported geometry");
  if (reinterpret_cast<uintptr_t>(x) & 15) throw std::runtime_error("gemm gather: input not 16-B aligned");
  const uint32_t geo = (uint32_t)ilog2_exact(C) | (uint32_t)ilog2_exact(Wo) << 4 | (uint32_t)ilog2_exact(Ho) << 8 |
                       (uint32_t)ilog2_exact(W) << 12 | (uint32_t)ilog2_exact(H) << 16 | (uint32_t)(s - 1) << 20 |
                       (uint32_t)pt << 21 | (uint32_t)pl << 23 | (uint32_t)mode << 25;
  return gemm2_run(4, InX{x, nullptr, nullptr, nullptr, 0}, GradX{}, Bt, bias, out, B * Ho * Wo, N, K, false,
                   nullptr, (int)geo, st, partial, StatSink{}, gemm2_target_wgs(), GradSink{}, false);
}

bool gemm_fold_ok(int M, int N, int K, bool bf16) {
  return gemm_impl_for(N, bf16) == 2 && plan_gemm2(M, N, K, gemm2_target_wgs(), bf16).splits == 1;
}

// GradSink partial rows a dgrad GEMM of this shape writes (0: the sums cannot be fused: split-K)
int gemm_dgrad_gsink_partials(int M, int N, int K, bool bf16) {
  if (gemm_impl_for(N, bf16) == 2) {
    Gemm2Plan q = plan_gemm2(M, N, K, gemm2_target_wgs(), bf16);
    return q.splits > 1 ? 0 : q.P;
  }
  GemmPlan p = plan_gemm(M, N, K);
  return p.splits > 1 ? 0 : p.gx;
}

int launch_gemm_dgrad(GradX A, const float* Bt, float* C, int M, int N, int K, bool acc,
                      hipStream_t s, float* partial, GradSink gs, bool bf16) {
  InX raw{A.da, nullptr, nullptr, nullptr, 0};
  if (gemm_impl_for(N, bf16) == 2)
    return gemm2_run(A.y ? 3 : 0, raw, A, Bt, nullptr, C, M, N, K, acc, nullptr, 1, s, partial, StatSink{},
                     gemm2_target_wgs(), gs, bf16);
  return gemm1_run(A.y ? 3 : 0, raw, A, Bt, nullptr, C, M, N, K, acc, nullptr, 1, s, partial, StatSink{}, gs);
}

__global__ void k_transpose(const float* __restrict__ in, float* __restrict__ out, int rows,
                            int cols) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)rows * cols) return;
  int r = (int)(idx / cols), c = (int)(idx % cols);
  out[(long)c * rows + r] = in[idx];
}

void launch_transpose(const float* in, float* out, int rows, int cols, hipStream_t s) {
  long n = (long)rows * cols;
  hipLaunchKernelGGL(k_transpose, dim3(cdiv(n, 256)), dim3(256), 0, s, in, out, rows, cols);
  PHX_LAUNCH_CHECK();
}

}  // namespace phx
