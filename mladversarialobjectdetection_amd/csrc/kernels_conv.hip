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

namespace phx {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// stem: 3x3 stride 2, Cin = 3
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_stem_fwd(const float* __restrict__ x,
                                                  const float* __restrict__ w,
                                                  float* __restrict__ y, int B, int H, int W,
                                                  int Ho, int Wo, int Co, int pt, int pl) {
  const int C4 = Co >> 2;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * Ho * Wo * C4;
  if (idx >= total) return;
  int c4 = (int)(idx % C4);
  long p = idx / C4;
  int ox = (int)(p % Wo);
  long t = p / Wo;
  int oy = (int)(t % Ho);
  int b = (int)(t / Ho);
  const int co = c4 * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = 0; i < 3; ++i) {
    int iy = oy * 2 - pt + i;
    if (iy < 0 || iy >= H) continue;
    for (int j = 0; j < 3; ++j) {
      int ix = ox * 2 - pl + j;
      if (ix < 0 || ix >= W) continue;
      const float* xp = x + (((long)b * H + iy) * W + ix) * 3;
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) {
        float xv = xp[ci];
        float4 wv = *reinterpret_cast<const float4*>(w + ((i * 3 + j) * 3 + ci) * Co + co);
        acc.x += xv * wv.x;
        acc.y += xv * wv.y;
        acc.z += xv * wv.z;
        acc.w += xv * wv.w;
      }
    }
  }
  *reinterpret_cast<float4*>(y + p * Co + co) = acc;
}

__global__ __launch_bounds__(256) void k_stem_bwd(GradX dy,
                                                  const float* __restrict__ w,
                                                  float* __restrict__ dx, int B, int H, int W,
                                                  int Ho, int Wo, int Co, int pt, int pl,
                                                  int acc_flag) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * H * W;
  if (idx >= total) return;
  int ix = (int)(idx % W);
  long t = idx / W;
  int iy = (int)(t % H);
  int b = (int)(t / H);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  for (int i = 0; i < 3; ++i) {
    int ty = iy + pt - i;
    if (ty < 0 || (ty & 1)) continue;
    int oy = ty >> 1;
    if (oy >= Ho) continue;
    for (int j = 0; j < 3; ++j) {
      int tx = ix + pl - j;
      if (tx < 0 || (tx & 1)) continue;
      int ox = tx >> 1;
      if (ox >= Wo) continue;
      const long gbase = (((long)b * Ho + oy) * Wo + ox) * Co;
      const float* wp = w + (i * 3 + j) * 3 * Co;
      for (int co = 0; co < Co; co += 4) {
        float4 gv = gx_load4(dy, gbase + co, co);
        float4 w0 = *reinterpret_cast<const float4*>(wp + co);
        float4 w1 = *reinterpret_cast<const float4*>(wp + Co + co);
        float4 w2 = *reinterpret_cast<const float4*>(wp + 2 * Co + co);
        a0 += gv.x * w0.x + gv.y * w0.y + gv.z * w0.z + gv.w * w0.w;
        a1 += gv.x * w1.x + gv.y * w1.y + gv.z * w1.z + gv.w * w1.w;
        a2 += gv.x * w2.x + gv.y * w2.y + gv.z * w2.z + gv.w * w2.w;
      }
    }
  }
  float* o = dx + idx * 3;
  if (acc_flag) {
    o[0] += a0; o[1] += a1; o[2] += a2;
  } else {
    o[0] = a0; o[1] = a1; o[2] = a2;
  }
}

void launch_stem_fwd(const float* x, const float* w, float* y, int B, int H, int W, int Ho, int Wo,
                     int Co, int pt, int pl, hipStream_t s) {
  long total = (long)B * Ho * Wo * (Co / 4);
  hipLaunchKernelGGL(k_stem_fwd, dim3(cdiv(total, 256)), dim3(256), 0, s, x, w, y, B, H, W, Ho, Wo,
                     Co, pt, pl);
  PHX_LAUNCH_CHECK();
}

void launch_stem_bwd(GradX dy, const float* w, float* dx, int B, int H, int W, int Ho,
                     int Wo, int Co, int pt, int pl, bool acc, hipStream_t s) {
  long total = (long)B * H * W;
  hipLaunchKernelGGL(k_stem_bwd, dim3(cdiv(total, 256)), dim3(256), 0, s, dy, w, dx, B, H, W, Ho,
                     Wo, Co, pt, pl, acc ? 1 : 0);
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
template <int NT, int MODE>
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
        float4 yv = *reinterpret_cast<const float4*>(Gx.y + e);
        v = gx_apply4(Gx, gk, v, yv);
      } else {
        v = *reinterpret_cast<const float4*>(Ax.p + e);
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

template <int NT, int WM, int MODE>
__global__ __launch_bounds__(256) void k_gemm(InX Ax, GradX Gx, const float* __restrict__ Bt,
                                              const float* __restrict__ bias,
                                              float* __restrict__ C, int M, int N, int K,
                                              int acc_flag, const float* __restrict__ rowscale,
                                              int rows_per_img, int kslice,
                                              float* __restrict__ partial) {
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

  GemmFrag<NT> cur, nxt;
  if (kbeg < kend)
    gemm_load<NT, MODE>(cur, Ax, Gx, Bt, K, kend, kbeg + 4 * q, rows, rok, cols, cok, rowscale,
                        rows_per_img);
  for (int k0 = kbeg; k0 < kend; k0 += 16) {
    const bool more = k0 + 16 < kend;
    if (more)
      gemm_load<NT, MODE>(nxt, Ax, Gx, Bt, K, kend, k0 + 16 + 4 * q, rows, rok, cols, cok, rowscale,
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

  // epilogue: accumulator element j of tile (mt,nt) is row 4q+j, col r.  Stage 16 rows at a
  // time through LDS and store row segments with 16-B lanes.
  float* st = stage[wave];
  const bool split = partial != nullptr;
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
            float4* cp = reinterpret_cast<float4*>(out + (long)row * N + col);
            if (acc_flag) {
              float4 o = *cp;
              v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
            }
            *cp = v;
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
          float* cp = out + (long)row * N + col;
          if (!split) {
            if (bias) v += bias[col];
            if (acc_flag) v += *cp;
          }
          *cp = v;
        }
      }
    }
  }
}

// split-K reduction: C (+)= sum_s partial[s] + bias
__global__ __launch_bounds__(256) void k_gemm_splitk_reduce(const float* __restrict__ partial,
                                                            int S, long MN, int N,
                                                            const float* __restrict__ bias,
                                                            float* __restrict__ C, int acc_flag) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= MN) return;
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += partial[(long)s * MN + i];
  if (bias) v += bias[i % N];
  if (acc_flag) v += C[i];
  C[i] = v;
}

template <int WM, int MODE>
static void gemm_dispatch_nt(int nt, dim3 g, hipStream_t s, InX A, GradX G, const float* Bt,
                             const float* bias, float* C, int M, int N, int K, int accf,
                             const float* rs, int rpi, int kslice, float* part) {
#define PHX_G(NT_)                                                                          \
  case NT_:                                                                                 \
    hipLaunchKernelGGL((k_gemm<NT_, WM, MODE>), g, dim3(256), 0, s, A, G, Bt, bias, C, M, N, K, \
                       accf, rs, rpi, kslice, part);                                        \
    break;
  switch (nt) {
    PHX_G(1) PHX_G(2) PHX_G(3) PHX_G(4) PHX_G(5) PHX_G(6) PHX_G(7) PHX_G(8)
    default: throw std::runtime_error("gemm: bad NT");
  }
#undef PHX_G
}

template <int MODE>
static void gemm_dispatch(int wm, int nt, dim3 g, hipStream_t s, InX A, GradX G, const float* Bt,
                          const float* bias, float* C, int M, int N, int K, int accf,
                          const float* rs, int rpi, int kslice, float* part) {
  if (wm == 4) gemm_dispatch_nt<4, MODE>(nt, g, s, A, G, Bt, bias, C, M, N, K, accf, rs, rpi, kslice, part);
  else if (wm == 2) gemm_dispatch_nt<2, MODE>(nt, g, s, A, G, Bt, bias, C, M, N, K, accf, rs, rpi, kslice, part);
  else gemm_dispatch_nt<1, MODE>(nt, g, s, A, G, Bt, bias, C, M, N, K, accf, rs, rpi, kslice, part);
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

size_t gemm_partial_floats(int M, int N, int K) {
  GemmPlan p = plan_gemm(M, N, K);
  return p.splits > 1 ? (size_t)p.splits * M * N : 0;
}

static void gemm_run(int mode, InX A, GradX G, const float* Bt, const float* bias, float* C, int M,
                     int N, int K, bool acc, const float* rowscale, int rows_per_img, hipStream_t s,
                     float* partial) {
  if (K % 4 != 0) throw std::runtime_error("gemm: K must be a multiple of 4");
  GemmPlan p = plan_gemm(M, N, K);
  float* part = p.splits > 1 ? partial : nullptr;
  if (p.splits > 1 && !partial) throw std::runtime_error("gemm: split-K needs a partial buffer");
  dim3 g(p.gx, p.gy, p.splits);
  const int af = acc ? 1 : 0;
  switch (mode) {
    case 0: gemm_dispatch<0>(p.wm, p.nt, g, s, A, G, Bt, bias, C, M, N, K, af, nullptr, 1, p.kslice, part); break;
    case 1: gemm_dispatch<1>(p.wm, p.nt, g, s, A, G, Bt, bias, C, M, N, K, af, nullptr, 1, p.kslice, part); break;
    case 2: gemm_dispatch<2>(p.wm, p.nt, g, s, A, G, Bt, bias, C, M, N, K, af, rowscale, rows_per_img, p.kslice, part); break;
    default: gemm_dispatch<3>(p.wm, p.nt, g, s, A, G, Bt, bias, C, M, N, K, af, nullptr, 1, p.kslice, part); break;
  }
  PHX_LAUNCH_CHECK();
  if (p.splits > 1) {
    long mn = (long)M * N;
    hipLaunchKernelGGL(k_gemm_splitk_reduce, dim3(cdiv(mn, 256)), dim3(256), 0, s, partial, p.splits, mn,
                       N, bias, C, af);
    PHX_LAUNCH_CHECK();
  }
}

void launch_gemm(InX A, const float* Bt, const float* bias, float* C, int M, int N, int K,
                 bool acc, const float* rowscale, int rows_per_img, hipStream_t s,
                 float* partial) {
  if (rowscale && !A.mu) throw std::runtime_error("gemm: rowscale requires a BN view");
  const int mode = rowscale ? 2 : (A.mu ? 1 : 0);
  gemm_run(mode, A, GradX{}, Bt, bias, C, M, N, K, acc, rowscale, rows_per_img, s, partial);
}

void launch_gemm_dgrad(GradX A, const float* Bt, float* C, int M, int N, int K, bool acc,
                       hipStream_t s, float* partial) {
  InX raw{A.da, nullptr, nullptr, nullptr, 0};
  if (A.y)
    gemm_run(3, raw, A, Bt, nullptr, C, M, N, K, acc, nullptr, 1, s, partial);
  else
    gemm_run(0, raw, A, Bt, nullptr, C, M, N, K, acc, nullptr, 1, s, partial);
}

// ------------------------------------------------------------------------------------------
// depthwise conv (TF SAME), one lane per (output pixel, 4 channels)
// ------------------------------------------------------------------------------------------


// ------------------------------------------------------------------------------------------
// LDS-tiled depthwise conv.  A workgroup owns OTH x OTW output pixels x (4*CG) channels: it
// stages the input tile (+halo) once into LDS with the consumer-side BN + activation applied
// once per element (not once per tap), then every lane produces OTH outputs of one column for
// 4 channels.  LDS image [row][col][cg] of float4: a wave's reads are contiguous 16-B slots.
// ------------------------------------------------------------------------------------------
struct DwTile {
  int cg, px, oth, otw, rin, cin;
};

static DwTile dw_tile(int C, int k, int stride) {
  DwTile t;
  const int c4 = C / 4;
  t.cg = (c4 % 8 == 0) ? 8 : (c4 % 4 == 0) ? 4 : (c4 % 2 == 0) ? 2 : 1;
  t.px = 256 / t.cg;
  t.otw = t.px;
  t.oth = stride == 1 ? 4 : 2;
  t.rin = (t.oth - 1) * stride + k;
  t.cin = (t.otw - 1) * stride + k;
  return t;
}

// XCD-aware block order: the NCG channel-group blocks of one pixel tile get linear ids
// L, L+8, L+16, ... (the same XCD under round-robin dispatch, back to back), so the NHWC lines
// each of them reads 16*CG bytes of are served from that XCD's L2 for the others.
__device__ __forceinline__ void dw_block_map(int L, int ncg, int* tile, int* cg) {
  const int grp = L / (8 * ncg), rem = L % (8 * ncg);
  *cg = rem / 8;
  *tile = grp * 8 + rem % 8;
}

__global__ __launch_bounds__(256) void k_dw_fwd_tiled(InX xv, const float* __restrict__ w,
                                                      float* __restrict__ y, int H, int W, int C,
                                                      int Ho, int Wo, int k, int stride, int pt,
                                                      int pl, DwTile T, int tiles_x, int ntiles,
                                                      int ncg) {
  extern __shared__ float4 tile[];
  const int b = blockIdx.z;
  int tl, cgi;
  dw_block_map(blockIdx.x, ncg, &tl, &cgi);
  if (tl >= ntiles) return;
  const int ty = tl / tiles_x, tx = tl % tiles_x;
  const int oy0 = ty * T.oth, ox0 = tx * T.otw;
  const int iy0 = oy0 * stride - pt, ix0 = ox0 * stride - pl;
  const bool xf = xv.mu != nullptr;
  const int n = T.rin * T.cin * T.cg;
  const int cg = threadIdx.x % T.cg, px = threadIdx.x / T.cg;
  const int ox = ox0 + px;
  {
    const int c0 = cgi * T.cg * 4;
    for (int e = threadIdx.x; e < n; e += 256) {
      const int ecg = e % T.cg;
      const int pcol = (e / T.cg) % T.cin;
      const int prow = e / (T.cg * T.cin);
      const int iy = iy0 + prow, ix = ix0 + pcol;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
        const int c = c0 + ecg * 4;
        v = *reinterpret_cast<const float4*>(xv.p + (((long)b * H + iy) * W + ix) * C + c);
        if (xf) v = inx_apply4(xv, inx_chan4(xv, c), v);
      }
      tile[e] = v;
    }
    __syncthreads();
    if (ox < Wo) {
      const int c = c0 + cg * 4;
      float4 acc[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int i = 0; i < k; ++i) {
        for (int j = 0; j < k; ++j) {
          const float4 wv = *reinterpret_cast<const float4*>(w + (i * k + j) * C + c);
          const int pcol = px * stride + j;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (r < T.oth) {
              const float4 xv4 = tile[((r * stride + i) * T.cin + pcol) * T.cg + cg];
              acc[r].x += xv4.x * wv.x;
              acc[r].y += xv4.y * wv.y;
              acc[r].z += xv4.z * wv.z;
              acc[r].w += xv4.w * wv.w;
            }
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int oy = oy0 + r;
        if (r < T.oth && oy < Ho)
          *reinterpret_cast<float4*>(y + (((long)b * Ho + oy) * Wo + ox) * C + c) = acc[r];
      }
    }
    __syncthreads();
  }
}

void launch_dw_fwd(InX x, const float* w, float* y, int B, int H, int W, int C, int Ho, int Wo,
                   int k, int stride, int pt, int pl, hipStream_t s) {
  if (C % 4) throw std::runtime_error("dw: C % 4 != 0");
  DwTile T = dw_tile(C, k, stride);
  const int tiles_x = cdiv(Wo, T.otw), tiles_y = cdiv(Ho, T.oth);
  const int ntiles = tiles_x * tiles_y, ncg = C / (4 * T.cg);
  size_t shm = (size_t)T.rin * T.cin * T.cg * sizeof(float4);
  dim3 g(cdiv(ntiles, 8) * 8 * ncg, 1, B);
  hipLaunchKernelGGL(k_dw_fwd_tiled, g, dim3(256), shm, s, x, w, y, H, W, C, Ho, Wo, k, stride, pt, pl,
                     T, tiles_x, ntiles, ncg);
  PHX_LAUNCH_CHECK();
}

// dgrad of the depthwise conv, gathered per input pixel: the workgroup stages the dy window its
// OTH x OTW input pixels need (gradient view applied once per element) and sums the taps.
static inline int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
__device__ __forceinline__ int floor_div_d(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

__global__ __launch_bounds__(256) void k_dw_bwd_tiled(GradX g, const float* __restrict__ w,
                                                      float* __restrict__ dx, int H, int W, int C,
                                                      int Ho, int Wo, int k, int stride, int pt,
                                                      int pl, DwTile T, int rin, int cin,
                                                      int tiles_x, int ntiles, int ncg,
                                                      int acc_flag) {
  extern __shared__ float4 tile[];
  const int b = blockIdx.z;
  int tl, cgi;
  dw_block_map(blockIdx.x, ncg, &tl, &cgi);
  if (tl >= ntiles) return;
  const int ty = tl / tiles_x, tx = tl % tiles_x;
  const int iy0 = ty * T.oth, ix0 = tx * T.otw;  // this tile's input-space pixels
  const int oy_lo = floor_div_d(iy0 + pt - (k - 1), stride);
  const int ox_lo = floor_div_d(ix0 + pl - (k - 1), stride);
  const int n = rin * cin * T.cg;
  const int cg = threadIdx.x % T.cg, px = threadIdx.x / T.cg;
  const int ix = ix0 + px;
  {
    const int c0 = cgi * T.cg * 4;
    for (int e = threadIdx.x; e < n; e += 256) {
      const int ecg = e % T.cg;
      const int pcol = (e / T.cg) % cin;
      const int prow = e / (T.cg * cin);
      const int oy = oy_lo + prow, ox = ox_lo + pcol;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (oy >= 0 && oy < Ho && ox >= 0 && ox < Wo)
        v = gx_load4(g, (((long)b * Ho + oy) * Wo + ox) * C + c0 + ecg * 4, c0 + ecg * 4);
      tile[e] = v;
    }
    __syncthreads();
    if (ix < W) {
      const int c = c0 + cg * 4;
      for (int r = 0; r < T.oth; ++r) {
        const int iy = iy0 + r;
        if (iy >= H) break;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int i = 0; i < k; ++i) {
          const int tyy = iy + pt - i;
          if (tyy < 0) break;
          if (tyy % stride) continue;
          const int oy = tyy / stride;
          if (oy >= Ho) continue;
          for (int j = 0; j < k; ++j) {
            const int txx = ix + pl - j;
            if (txx < 0) break;
            if (txx % stride) continue;
            const int ox = txx / stride;
            if (ox >= Wo) continue;
            const float4 gv = tile[((oy - oy_lo) * cin + (ox - ox_lo)) * T.cg + cg];
            const float4 wv = *reinterpret_cast<const float4*>(w + (i * k + j) * C + c);
            acc.x += gv.x * wv.x;
            acc.y += gv.y * wv.y;
            acc.z += gv.z * wv.z;
            acc.w += gv.w * wv.w;
          }
        }
        float4* o = reinterpret_cast<float4*>(dx + (((long)b * H + iy) * W + ix) * C + c);
        if (acc_flag) {
          float4 pv = *o;
          acc.x += pv.x; acc.y += pv.y; acc.z += pv.z; acc.w += pv.w;
        }
        *o = acc;
      }
    }
    __syncthreads();
  }
}

void launch_dw_bwd(GradX dy, const float* w, float* dx, int B, int H, int W, int C, int Ho,
                   int Wo, int k, int stride, int pt, int pl, bool acc, hipStream_t s) {
  if (C % 4) throw std::runtime_error("dw: C % 4 != 0");
  DwTile T = dw_tile(C, k, stride);
  T.oth = 4;
  const int rin = (T.oth - 1 + k - 1) / stride + 2;
  const int cin = (T.otw - 1 + k - 1) / stride + 2;
  const int tiles_x = cdiv(W, T.otw), tiles_y = cdiv(H, T.oth);
  const int ntiles = tiles_x * tiles_y, ncg = C / (4 * T.cg);
  size_t shm = (size_t)rin * cin * T.cg * sizeof(float4);
  dim3 g(cdiv(ntiles, 8) * 8 * ncg, 1, B);
  hipLaunchKernelGGL(k_dw_bwd_tiled, g, dim3(256), shm, s, dy, w, dx, H, W, C, Ho, Wo, k, stride, pt, pl,
                     T, rin, cin, tiles_x, ntiles, ncg, acc ? 1 : 0);
  PHX_LAUNCH_CHECK();
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
