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

__global__ __launch_bounds__(256) void k_stem_bwd(const float* __restrict__ dy,
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
      const float* g = dy + (((long)b * Ho + oy) * Wo + ox) * Co;
      const float* wp = w + (i * 3 + j) * 3 * Co;
      for (int co = 0; co < Co; co += 4) {
        float4 gv = *reinterpret_cast<const float4*>(g + co);
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

void launch_stem_bwd(const float* dy, const float* w, float* dx, int B, int H, int W, int Ho,
                     int Wo, int Co, int pt, int pl, bool acc, hipStream_t s) {
  long total = (long)B * H * W;
  hipLaunchKernelGGL(k_stem_bwd, dim3(cdiv(total, 256)), dim3(256), 0, s, dy, w, dx, B, H, W, Ho,
                     Wo, Co, pt, pl, acc ? 1 : 0);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// fp32 MFMA GEMM: C[M,N] (+)= A[M,K] * Bt[N,K]^T + bias.  Block = 4 waves along M, each wave
// owns 32 rows x (16*NT) columns = 2 x NT accumulator tiles of 16x16.  K % 4 == 0.
// ------------------------------------------------------------------------------------------
template <int NT, bool ROWSCALE>
__global__ __launch_bounds__(256) void k_gemm(const float* __restrict__ A,
                                              const float* __restrict__ Bt,
                                              const float* __restrict__ bias,
                                              float* __restrict__ C, int M, int N, int K,
                                              int acc_flag, const float* __restrict__ rowscale,
                                              int rows_per_img) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4, r = lane & 15;
  const int m_base = blockIdx.x * 128 + wave * 32;
  const int n_base = blockIdx.y * (16 * NT);

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

  for (int k0 = 0; k0 < K; k0 += 16) {
    const int kk = k0 + 4 * q;
    const bool kok = kk < K;
    float4 a[2];
    float4 b[NT];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      if (rok[mt] && kok) {
        a[mt] = *reinterpret_cast<const float4*>(A + (long)rows[mt] * K + kk);
        if (ROWSCALE) {
          float4 sc = *reinterpret_cast<const float4*>(rowscale + (long)(rows[mt] / rows_per_img) * K + kk);
          a[mt].x *= sc.x; a[mt].y *= sc.y; a[mt].z *= sc.z; a[mt].w *= sc.w;
        }
      } else {
        a[mt] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      b[nt] = (cok[nt] && kok) ? *reinterpret_cast<const float4*>(Bt + (long)cols[nt] * K + kk)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].x, b[nt].x, acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].y, b[nt].y, acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].z, b[nt].z, acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].w, b[nt].w, acc[mt][nt], 0, 0, 0);
      }
    }
  }
  // epilogue: accumulator element j of tile (mt,nt) is C[row = 4q+j][col = r]
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    if (!cok[nt]) continue;
    const float bv = bias ? bias[cols[nt]] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m_base + mt * 16 + 4 * q + j;
        if (row < M) {
          float v = acc[mt][nt][j] + bv;
          float* cp = C + (long)row * N + cols[nt];
          if (acc_flag) v += *cp;
          *cp = v;
        }
      }
    }
  }
}

template <bool RS>
static void gemm_dispatch(int nt, dim3 g, hipStream_t s, const float* A, const float* Bt,
                          const float* bias, float* C, int M, int N, int K, int accf,
                          const float* rs, int rpi) {
#define PHX_G(NT_)                                                                          \
  case NT_:                                                                                 \
    hipLaunchKernelGGL((k_gemm<NT_, RS>), g, dim3(256), 0, s, A, Bt, bias, C, M, N, K, accf, \
                       rs, rpi);                                                            \
    break;
  switch (nt) {
    PHX_G(1) PHX_G(2) PHX_G(3) PHX_G(4) PHX_G(5) PHX_G(6) PHX_G(7) PHX_G(8)
    default: throw std::runtime_error("gemm: bad NT");
  }
#undef PHX_G
}

void launch_gemm(const float* A, const float* Bt, const float* bias, float* C, int M, int N, int K,
                 bool acc, const float* rowscale, int rows_per_img, hipStream_t s) {
  if (K % 4 != 0) throw std::runtime_error("gemm: K must be a multiple of 4");
  int nt = N <= 128 ? (N + 15) / 16 : 8;
  dim3 g(cdiv(M, 128), cdiv(N, 16 * nt));
  if (rowscale)
    gemm_dispatch<true>(nt, g, s, A, Bt, bias, C, M, N, K, acc ? 1 : 0, rowscale, rows_per_img);
  else
    gemm_dispatch<false>(nt, g, s, A, Bt, bias, C, M, N, K, acc ? 1 : 0, nullptr, 1);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// depthwise conv (TF SAME), one lane per (output pixel, 4 channels)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dw_fwd(const float* __restrict__ x,
                                                const float* __restrict__ w,
                                                float* __restrict__ y, int B, int H, int W, int C,
                                                int Ho, int Wo, int k, int stride, int pt,
                                                int pl) {
  const int C4 = C >> 2;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * Ho * Wo * C4;
  if (idx >= total) return;
  int c = (int)(idx % C4) * 4;
  long p = idx / C4;
  int ox = (int)(p % Wo);
  long t = p / Wo;
  int oy = (int)(t % Ho);
  int b = (int)(t / Ho);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = 0; i < k; ++i) {
    int iy = oy * stride - pt + i;
    if (iy < 0 || iy >= H) continue;
    const float* xr = x + ((long)b * H + iy) * W * C + c;
    for (int j = 0; j < k; ++j) {
      int ix = ox * stride - pl + j;
      if (ix < 0 || ix >= W) continue;
      float4 xv = *reinterpret_cast<const float4*>(xr + (long)ix * C);
      float4 wv = *reinterpret_cast<const float4*>(w + (i * k + j) * C + c);
      acc.x += xv.x * wv.x;
      acc.y += xv.y * wv.y;
      acc.z += xv.z * wv.z;
      acc.w += xv.w * wv.w;
    }
  }
  *reinterpret_cast<float4*>(y + p * C + c) = acc;
}

__global__ __launch_bounds__(256) void k_dw_bwd(const float* __restrict__ dy,
                                                const float* __restrict__ w,
                                                float* __restrict__ dx, int B, int H, int W, int C,
                                                int Ho, int Wo, int k, int stride, int pt, int pl,
                                                int acc_flag) {
  const int C4 = C >> 2;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * H * W * C4;
  if (idx >= total) return;
  int c = (int)(idx % C4) * 4;
  long p = idx / C4;
  int ix = (int)(p % W);
  long t = p / W;
  int iy = (int)(t % H);
  int b = (int)(t / H);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = 0; i < k; ++i) {
    int ty = iy + pt - i;
    if (ty < 0) break;
    if (ty % stride) continue;
    int oy = ty / stride;
    if (oy >= Ho) continue;
    for (int j = 0; j < k; ++j) {
      int tx = ix + pl - j;
      if (tx < 0) break;
      if (tx % stride) continue;
      int ox = tx / stride;
      if (ox >= Wo) continue;
      float4 g = *reinterpret_cast<const float4*>(dy + (((long)b * Ho + oy) * Wo + ox) * C + c);
      float4 wv = *reinterpret_cast<const float4*>(w + (i * k + j) * C + c);
      acc.x += g.x * wv.x;
      acc.y += g.y * wv.y;
      acc.z += g.z * wv.z;
      acc.w += g.w * wv.w;
    }
  }
  float4* o = reinterpret_cast<float4*>(dx + p * C + c);
  if (acc_flag) {
    float4 v = *o;
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  *o = acc;
}

void launch_dw_fwd(const float* x, const float* w, float* y, int B, int H, int W, int C, int Ho,
                   int Wo, int k, int stride, int pt, int pl, hipStream_t s) {
  if (C % 4) throw std::runtime_error("dw: C % 4 != 0");
  long total = (long)B * Ho * Wo * (C / 4);
  hipLaunchKernelGGL(k_dw_fwd, dim3(cdiv(total, 256)), dim3(256), 0, s, x, w, y, B, H, W, C, Ho, Wo,
                     k, stride, pt, pl);
  PHX_LAUNCH_CHECK();
}

void launch_dw_bwd(const float* dy, const float* w, float* dx, int B, int H, int W, int C, int Ho,
                   int Wo, int k, int stride, int pt, int pl, bool acc, hipStream_t s) {
  if (C % 4) throw std::runtime_error("dw: C % 4 != 0");
  long total = (long)B * H * W * (C / 4);
  hipLaunchKernelGGL(k_dw_bwd, dim3(cdiv(total, 256)), dim3(256), 0, s, dy, w, dx, B, H, W, C, Ho,
                     Wo, k, stride, pt, pl, acc ? 1 : 0);
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
