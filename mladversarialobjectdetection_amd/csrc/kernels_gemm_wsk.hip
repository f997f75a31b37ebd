// kernels_gemm_wsk.hip — the deep-K 1x1-convolution GEMM: K split across the four waves of a
// workgroup instead of across workgroups (fp32 matrix cores, v_mfma_f32_32x32x2_f32).
//
//   C[M,N] (+)= A'[M,K] * Bt[N,K]^T (+ bias)      A' as in k_gemm2 (raw, BN view, x SE rowscale,
//                                                 gradient view, implicit im2col of a 3x3 conv)
//
// Why: the stage 5-7 convs (M = 4096-16384 rows, K = 320-1152) have fewer than 256 output tiles of
// the k_gemm2 sizes, so k_gemm2 split K across workgroups: fp32 partial slabs in HBM, a second
// launch to reduce them (with the BN statistics), and 16-deep K chunks per barrier whose fixed cost
// (load wait, view, LDS store, barrier, two LDS read latencies) dwarfed the 8-24 MFMAs a wave ran per
// chunk.  Here a workgroup owns one BM x BN output tile (TM x TN MFMA tiles of 32x32) and every wave
// computes the whole tile over its own 16-deep slice of each 64-deep K chunk:
//  * each barrier now covers TM*TN*8 MFMAs per wave on a 4x larger chunk, and the grid is one
//    workgroup per output tile (no partial slabs, no reduce launch);
//  * the four per-wave accumulators are summed through LDS in wave order 0, 1, 2, 3 (fixed order:
//    bit-reproducible run to run), each wave finishing TM*TN/4 of the tiles;
//  * epilogue as k_gemm2 (bias, accumulate, C store), and the consumer BN's batch statistics
//    (StatSink) or the BN-backward sums of a dgrad (GradSink) per 32-row tile: partial row
//    blockIdx.x * TM + i, so these shapes fuse their sinks like the unsplit ones (the split-K reduce
//    and the separate BN-backward reduction launches go away).
// LDS: two 64-deep chunks of A (BM rows) and B (BN rows), rows of 16 XOR-swizzled 16-B units
// (g2_off: a 16-lane ds_read_b128 group covers 16 distinct units, conflict-free); the cross-wave
// sum reuses the same array.
// BF (the C4 configuration's bf16 matrix cores, v_mfma_f32_32x32x16_bf16): 128-deep chunks, 32 k per
// wave (two MFMAs per tile), the A view applied in fp32 and rounded to bf16 in LDS as k_gemm2 does;
// ST as k_gemm2 (1: bf16 activations A and C, 2: a bf16 BN input y behind a gradient view).
#include "gemm2_kernel.hpp"

namespace phx {

template <int TM, int TN, bool BF>
struct G2K {
  static constexpr int BM = 32 * TM, BN = 32 * TN, BK = BF ? 128 : 64, LD = BK;
  static constexpr int WK = BK / 4;                  // k of a chunk per wave
  static constexpr int KQ = BK / 4, RPP = 256 / KQ;  // quads per row, rows per pass of 256 lanes
  static constexpr int NA = BM / RPP, NB = BN / RPP; // quads per thread per chunk
  static constexpr int ESZ = BF ? 2 : 4;
  static constexpr int IMG = 2 * (BM + BN) * LD * ESZ / 4;  // double-buffered chunk image (floats)
  static constexpr int RED = 4 * TM * TN * 1024;    // per-wave accumulators (floats)
  static constexpr int LDS_FLOATS = IMG > RED ? IMG : RED;
};

template <class P, int MODE>
struct G2KRegs {
  float4 a[P::NA];
  bool gok[MODE == 4 ? P::NA : 1];
  float4 y[MODE == 3 ? P::NA : 1];
  float4 rs[MODE == 2 ? P::NA : 1];
  float4 b[P::NB];
  Chan4 ck;
  GChan4 gk;
};

// the chunk at k0: thread t loads quad t % KQ of rows t / KQ + RPP*u (clamped addresses; g2k_store
// zeroes what lies outside the matrices)
template <class P, int MODE, int ST>
__device__ __forceinline__ void g2k_load(G2KRegs<P, MODE>& r, const Gemm2Args& a, int m0, int n0, int k0) {
  const int t = threadIdx.x;
  const int kk = k0 + 4 * (t % P::KQ);
  const int kc = kk < a.K ? kk : a.K - 4;
  if (MODE == 1 || MODE == 2) r.ck = inx_chan4(a.A, kc);
  if (MODE == 3) r.gk = gx_chan4(a.G, kc);
  if constexpr (MODE == 4) {
    // implicit im2col (k_gemm2 MODE 4): row -> (image, oy, ox), quad kc -> (tap, channel), zero taps
    // outside the input (the same gather as g2_load, so a column matrix in HBM gives the same values)
    const G2Geo g = g2_geo((uint32_t)a.rpi);
    const int tap = kc >> g.lC, c = kc & ((1 << g.lC) - 1);
    const int ky = (tap * 11) >> 5, kx = tap - 3 * ky;  // tap / 3 for tap < 9
#pragma unroll
    for (int u = 0; u < P::NA; ++u) {
      const int row = min(m0 + t / P::KQ + P::RPP * u, a.M - 1);
      const int ox = row & ((1 << g.lWo) - 1), oy = (row >> g.lWo) & ((1 << g.lHo) - 1);
      const int b = row >> (g.lWo + g.lHo);
      int iy, ix;
      bool ok = kk < a.K && tap < 9;
      if (g.mode == 0) {
        iy = oy * g.s + ky - g.pt;
        ix = ox * g.s + kx - g.pl;
      } else {
        const int dy = oy - ky, dx = ox - kx;
        ok = ok && dy >= 0 && dx >= 0 && !(dy & 1) && !(dx & 1);
        iy = dy >> 1;
        ix = dx >> 1;
      }
      ok = ok && iy >= 0 && iy < (1 << g.lH) && ix >= 0 && ix < (1 << g.lW);
      const long e = ok ? ((((long)b << g.lH) + iy) << g.lW | ix) << g.lC | c : 0;
      r.a[u] = *reinterpret_cast<const float4*>(a.A.p + e);
      r.gok[u] = ok;
    }
  }
  if constexpr (MODE != 4) {
#pragma unroll
    for (int u = 0; u < P::NA; ++u) {
      const int row = min(m0 + t / P::KQ + P::RPP * u, a.M - 1);
      const long e = (long)row * a.K + kc;
      if (MODE == 3) {
        r.a[u] = *reinterpret_cast<const float4*>(a.G.da + e);
        r.y[u] = ald4<ST == 2>(a.G.y, e);
      } else {
        r.a[u] = ald4<ST == 1>(a.A.p, e);
        if (MODE == 2) r.rs[u] = *reinterpret_cast<const float4*>(a.rowscale + (long)(row / a.rpi) * a.K + kc);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < P::NB; ++u) {
    const int col = min(n0 + t / P::KQ + P::RPP * u, a.N - 1);
    r.b[u] = *reinterpret_cast<const float4*>(a.Bt + (long)col * a.K + kc);
  }
}

template <class P>
__device__ __forceinline__ void g2k_put(float* img, int row, int k, float4 v) {
  char* p = reinterpret_cast<char*>(img) + (size_t)g2_off<P>(row, k) * P::ESZ;
  if constexpr (P::ESZ == 2) *reinterpret_cast<uint2*>(p) = pack_bf16x4(v);
  else *reinterpret_cast<float4*>(p) = v;
}

template <class P, int MODE, int ACT>
__device__ __forceinline__ void g2k_store_act(const G2KRegs<P, MODE>& r, const Gemm2Args& a, float* img, int m0,
                                              int n0, int k0) {
  const int t = threadIdx.x;
  const int q = t % P::KQ;
  const bool kok = k0 + 4 * q < a.K;
  InX ax = a.A;
  ax.act = ACT;
  GradX gx = a.G;
  gx.act = ACT;
#pragma unroll
  for (int u = 0; u < P::NA; ++u) {
    const int rl = t / P::KQ + P::RPP * u;
    float4 v = r.a[u];
    if (MODE == 4) {
      if (!(r.gok[u] && m0 + rl < a.M)) v = make_float4(0.f, 0.f, 0.f, 0.f);
    } else if (kok && m0 + rl < a.M) {
      if (MODE == 1 || MODE == 2) v = inx_apply4(ax, r.ck, v);
      if (MODE == 2) {
        v.x *= r.rs[u].x; v.y *= r.rs[u].y; v.z *= r.rs[u].z; v.w *= r.rs[u].w;
      }
      if (MODE == 3) v = gx_apply4(gx, r.gk, v, r.y[u]);
    } else {
      v = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    g2k_put<P>(img, rl, 4 * q, v);
  }
  char* bimg = reinterpret_cast<char*>(img) + (size_t)P::BM * P::LD * P::ESZ;
#pragma unroll
  for (int u = 0; u < P::NB; ++u) {
    const int cl = t / P::KQ + P::RPP * u;
    const bool ok = kok && n0 + cl < a.N;
    g2k_put<P>(reinterpret_cast<float*>(bimg), cl, 4 * q, ok ? r.b[u] : make_float4(0.f, 0.f, 0.f, 0.f));
  }
}

template <class P, int MODE>
__device__ __forceinline__ void g2k_store(const G2KRegs<P, MODE>& r, const Gemm2Args& a, float* img, int m0, int n0,
                                          int k0) {
  const int act = MODE == 0 ? 0 : MODE == 3 ? a.G.act : a.A.act;
  if (act == 1) g2k_store_act<P, MODE, 1>(r, a, img, m0, n0, k0);
  else if (act == 2) g2k_store_act<P, MODE, 2>(r, a, img, m0, n0, k0);
  else g2k_store_act<P, MODE, 0>(r, a, img, m0, n0, k0);
}

// SK: 0 plain, 1 StatSink, 2 GradSink (as k_gemm2).  Grid (cdiv(M, BM), cdiv(N, BN)).
template <int TM, int TN, int MODE, int SK, bool BF, int ST>
__global__ __launch_bounds__(256, 2) void k_gemm2k(Gemm2Args a) {
  using P = G2K<TM, TN, BF>;
  constexpr bool CBF = ST == 1;  // C holds bf16 activations
  constexpr int BM = P::BM, BN = P::BN, NT = TM * TN;
  __shared__ __attribute__((aligned(16))) float sm[P::LDS_FLOATS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int nch = (a.K + P::BK - 1) / P::BK;
  G2KRegs<P, MODE> rg;
  g2k_load<P, MODE, ST>(rg, a, m0, n0, 0);
  g2k_store<P, MODE>(rg, a, sm, m0, n0, 0);
  __syncthreads();
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  for (int c = 0; c < nch; ++c) {
    float* const img = sm + (c & 1) * (P::IMG / 2);
    // the next chunk's loads first (past the end: the last chunk again, unused), unconditionally so
    // the MFMAs below do not wait for them
    g2k_load<P, MODE, ST>(rg, a, m0, n0, min(c + 1, nch - 1) * P::BK);
    __builtin_amdgcn_sched_barrier(0);
    const int kvalid = a.K - (c * P::BK + P::WK * w);  // this wave's k of the chunk that exist
    if (kvalid > 0) {                                    // wave-uniform
      const char* As = reinterpret_cast<const char*>(img);
      const char* Bs = As + (size_t)BM * P::LD * P::ESZ;
      if constexpr (BF) {
        // lane (r32, h) feeds row / column r32 with k = 16*kk + 8*h .. +7 of the wave's slice
        bf16x8_t fa[2][TM], fb[2][TN];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            fa[kk][i] = *reinterpret_cast<const bf16x8_t*>(As + (size_t)g2_off<P>(i * 32 + r32, P::WK * w + 16 * kk + 8 * h) * 2);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            fb[kk][j] = *reinterpret_cast<const bf16x8_t*>(Bs + (size_t)g2_off<P>(j * 32 + r32, P::WK * w + 16 * kk + 8 * h) * 2);
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          if (kk > 0 && kvalid <= 16) break;  // wave-uniform
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[kk][i], fb[kk][j], acc[i][j], 0, 0, 0);
        }
      } else {
        const float* Af = reinterpret_cast<const float*>(As);
        const float* Bf = reinterpret_cast<const float*>(Bs);
        float4 fa[2][TM], fb[2][TN];
#pragma unroll
        for (int s8 = 0; s8 < 2; ++s8) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            fa[s8][i] = *reinterpret_cast<const float4*>(Af + g2_off<P>(i * 32 + r32, P::WK * w + 8 * s8 + 4 * h));
#pragma unroll
          for (int j = 0; j < TN; ++j)
            fb[s8][j] = *reinterpret_cast<const float4*>(Bf + g2_off<P>(j * 32 + r32, P::WK * w + 8 * s8 + 4 * h));
        }
#pragma unroll
        for (int s8 = 0; s8 < 2; ++s8) {
          if (s8 > 0 && kvalid <= 8) break;  // wave-uniform
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s8][i].x, fb[s8][j].x, acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s8][i].y, fb[s8][j].y, acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s8][i].z, fb[s8][j].z, acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s8][i].w, fb[s8][j].w, acc[i][j], 0, 0, 0);
            }
        }
      }
    }
    if (c + 1 < nch) g2k_store<P, MODE>(rg, a, sm + ((c + 1) & 1) * (P::IMG / 2), m0, n0, (c + 1) * P::BK);
    __syncthreads();
  }
  // ---- cross-wave sum: wave w stores its tiles as [w][tile][e/4][lane] float4 (1 KB per
  // instruction, contiguous), then wave v sums tiles v, v + 4, ... over the waves in order ----
  float4* red = reinterpret_cast<float4*>(sm);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4)
        red[((w * NT + i * TN + j) * 4 + e4) * 64 + lane] =
            make_float4(acc[i][j][4 * e4], acc[i][j][4 * e4 + 1], acc[i][j][4 * e4 + 2], acc[i][j][4 * e4 + 3]);
  __syncthreads();
  for (int qt = w; qt < NT; qt += 4) {  // wave-uniform
    const int i = qt / TN, j = qt % TN;
    float v[16];
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) {
      float4 s = red[(qt * 4 + e4) * 64 + lane];
#pragma unroll
      for (int ww = 1; ww < 4; ++ww) {
        const float4 o = red[((ww * NT + qt) * 4 + e4) * 64 + lane];
        s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
      }
      v[4 * e4] = s.x; v[4 * e4 + 1] = s.y; v[4 * e4 + 2] = s.z; v[4 * e4 + 3] = s.w;
    }
    // ---- epilogue of tile (i, j): lane (r32, h) holds column r32, rows (e&3) + 8*(e>>2) + 4*h ----
    const int row0 = m0 + i * 32;
    const int col = n0 + j * 32 + r32;
    const bool cok = col < a.N;
    const bool full = row0 + 32 <= a.M && n0 + j * 32 + 32 <= a.N;
    const float bv = a.bias ? a.bias[min(col, a.N - 1)] : 0.f;
    if (full) {
      const long cbase = (long)(row0 + 4 * h) * a.N + col;
      float old[16];
      if (a.acc) {
#pragma unroll
        for (int e = 0; e < 16; ++e) old[e] = ald1<CBF>(a.C, cbase + (long)((e & 3) + 8 * (e >> 2)) * a.N);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float x = v[e] + bv;
        v[e] = x;
        if (a.acc) x += old[e];
        ast1<CBF>(a.C, cbase + (long)((e & 3) + 8 * (e >> 2)) * a.N, x);
        if (SK == 2) v[e] = x;
        if (CBF && SK == 1) v[e] = round_bf16(x);  // statistics of the stored values
      }
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        float x = v[e] + bv;
        v[e] = x;
        if (cok && row < a.M) {
          const long ce = (long)row * a.N + col;
          if (a.acc) x += ald1<CBF>(a.C, ce);
          ast1<CBF>(a.C, ce, x);
          if (SK == 2) v[e] = x;
        }
        if (CBF && SK == 1) v[e] = round_bf16(x);
      }
    }
    const long prow = (long)blockIdx.x * TM + i;  // this tile's partial row of the sink
    if constexpr (SK == 1) {
      const float nw = (float)max(0, min(32, a.M - row0));
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (full || row0 + (e & 3) + 8 * (e >> 2) + 4 * h < a.M) s += v[e];
      s += __shfl_xor(s, 32);
      const float mean = nw > 0.f ? s / nw : 0.f;
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (full || row0 + (e & 3) + 8 * (e >> 2) + 4 * h < a.M) {
          const float d = v[e] - mean;
          q = fmaf(d, d, q);
        }
      q += __shfl_xor(q, 32);
      if (h == 0 && cok) sink_put(a.sink, prow, col, nw, mean, q);
      if (j == 0 && blockIdx.y == 0 && lane == 0) sink_cnt(a.sink, prow, nw);
    }
    if constexpr (SK == 2) {
      const int cc = min(col, a.N - 1);
      const float mu = a.gsk.mu[cc], rs = a.gsk.rstd[cc], sc = a.gsk.sc[cc], be = a.gsk.be[cc];
      float yv[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = min(row0 + (e & 3) + 8 * (e >> 2) + 4 * h, a.M - 1);
        yv[e] = ald1<ST == 2>(a.gsk.y, (long)row * a.N + cc);
      }
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (cok && row < a.M) gs_one(v[e], yv[e], mu, rs, sc, be, a.gsk.act, s1, s2);
      }
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 32);
      if (h == 0 && cok) gsink_put(a.gsk, prow, col, s1, s2);
    }
  }
}

// storage variants as g2_go: fp32 compute stores fp32 (ST 0); bf16 compute runs its forward modes on
// bf16 activations (ST 1) and its gradient views on a bf16 y (ST 2)
template <int TM, int TN, int MODE, int SK>
static void g2k_st(dim3 g, hipStream_t s, const Gemm2Args& a, bool bf, int st) {
  if (!bf) {
    if (st) throw std::logic_error("gemm2k: bf16 storage needs the bf16 compute type");
    PHX_TLAUNCH((k_gemm2k<TM, TN, MODE, SK, false, 0>), g, dim3(256), 0, s, a);
    return;
  }
  constexpr bool fwd_only = MODE == 1 || MODE == 2 || SK == 1;
  constexpr bool dgrad_only = MODE == 3 || SK == 2;
  if constexpr (fwd_only) {
    if (st != 1) throw std::logic_error("gemm2k: bf16 forward without bf16 activations");
    PHX_TLAUNCH((k_gemm2k<TM, TN, MODE, SK, true, 1>), g, dim3(256), 0, s, a);
  } else if constexpr (dgrad_only) {
    if (st != 2) throw std::logic_error("gemm2k: bf16 gradient view without bf16 activations");
    PHX_TLAUNCH((k_gemm2k<TM, TN, MODE, SK, true, 2>), g, dim3(256), 0, s, a);
  } else {
    if (st == 1) PHX_TLAUNCH((k_gemm2k<TM, TN, MODE, SK, true, 1>), g, dim3(256), 0, s, a);
    else if (st == 0) PHX_TLAUNCH((k_gemm2k<TM, TN, MODE, SK, true, 0>), g, dim3(256), 0, s, a);
    else throw std::logic_error("gemm2k: raw dgrad with a bf16 y");
  }
}

template <int TM, int TN>
static void g2k_go(int mode, int sk, dim3 g, hipStream_t s, const Gemm2Args& a, bool bf, int st) {
  switch (mode) {
    case 0:
      if (sk == 1) g2k_st<TM, TN, 0, 1>(g, s, a, bf, st);
      else if (sk == 2) g2k_st<TM, TN, 0, 2>(g, s, a, bf, st);
      else g2k_st<TM, TN, 0, 0>(g, s, a, bf, st);
      break;
    case 1:
      if (sk == 1) g2k_st<TM, TN, 1, 1>(g, s, a, bf, st);
      else g2k_st<TM, TN, 1, 0>(g, s, a, bf, st);
      break;
    case 2:
      if (sk == 1) g2k_st<TM, TN, 2, 1>(g, s, a, bf, st);
      else g2k_st<TM, TN, 2, 0>(g, s, a, bf, st);
      break;
    case 3:
      if (sk == 2) g2k_st<TM, TN, 3, 2>(g, s, a, bf, st);
      else g2k_st<TM, TN, 3, 0>(g, s, a, bf, st);
      break;
    case 4:  // the implicit im2col: fp32, no sinks (as k_gemm2)
      if (sk || bf || st) throw std::logic_error("gemm2k: the implicit im2col runs in fp32 without sinks");
      PHX_TLAUNCH((k_gemm2k<TM, TN, 4, 0, false, 0>), g, dim3(256), 0, s, a);
      break;
    default:
      throw std::logic_error("gemm2k: unknown mode");
  }
}

void g2k_launch(int tm, int tn, int mode, int sk, dim3 g, hipStream_t s, const Gemm2Args& a, bool bf, int st) {
  if ((mode == 1 || mode == 2) && sk == 2) throw std::logic_error("gemm2k: GradSink on a forward view");
  if (mode == 3 && sk == 1) throw std::logic_error("gemm2k: StatSink on a gradient view");
  switch (tm * 10 + tn) {
    case 11: g2k_go<1, 1>(mode, sk, g, s, a, bf, st); break;
    case 12: g2k_go<1, 2>(mode, sk, g, s, a, bf, st); break;
    case 13: g2k_go<1, 3>(mode, sk, g, s, a, bf, st); break;
    case 21: g2k_go<2, 1>(mode, sk, g, s, a, bf, st); break;
    case 22: g2k_go<2, 2>(mode, sk, g, s, a, bf, st); break;
    default: throw std::logic_error("gemm2k: no kernel for this tile");
  }
}

}  // namespace phx
