// kernels_sep.hip — the fused separable convolution of the BiFPN nodes and the class / box heads for
// gfx950: keras SeparableConv2D(3x3, SAME, depth_multiplier 1, bias) = depthwise 3x3 -> pointwise 1x1
// -> + bias, in one launch whose depthwise output never reaches HBM.
//
// Reference: OpAfterCombine's separable conv (efficientdet_keras.py:195-207, 214-221), ClassNet's
// conv_ops / classes (:447-455, 414-446) and BoxNet's (:535-547, 609-620); SURVEY.md 2.3 "depthwise
// fused with the following pointwise".
//
// Design (MI355X).  A 256-thread workgroup owns an 8 x 16 output tile of one image and all C input
// channels; wave w owns tile pixels 32w .. 32w + 31, one per MFMA row (lane r32).
//   1. The input window (10 x 18 pixels, 64 channels per pass) is staged into LDS once through the
//      input view — the producer BN + activation (InX) or the BiFPN node fuse (FuseView: the node's
//      weighted sum of up to three BN views + activation, so the fuse is never stored either) — with
//      padding zeros outside the image and a 68-float pixel pitch (consecutive pixels 4 banks apart:
//      the per-pixel reads below are conflict-free).
//   2. Each lane computes the depthwise outputs of its pixel for the channels it feeds the matrix core
//      — lane (r32, h) supplies channels 8s + 4h .. 8s + 4h + 3 of MFMA k-step s — straight into the
//      registers of the pointwise GEMM's A fragments: the depthwise result is never written anywhere
//      (not even LDS).  The taps are applied in the depthwise kernel's order (k_dw_fwd: rows, then
//      columns, fmaf from zero), so the A operand equals the unfused path's stored tensor bit for bit.
//   3. The pointwise GEMM runs on v_mfma_f32_32x32x2_f32 (exact fp32) over 64-column chunks of the
//      transposed kernel [N][C] staged in LDS (aliasing the dead window), in k_gemm2's k order, then
//      the epilogue adds the bias, stores the 32-column row segments and (STATS) reduces the consumer
//      BN's batch statistics of the stored values: per wave two-pass (sum, M2) over its valid rows,
//      merged over the four waves in a fixed order, one StatSink partial row per workgroup.
// Grouped launch: up to kMaxSeg members with the same taps, kernel, C and N (the per-level copies of
// a head conv) share one flat grid of (member, image, tile) work items, cut into 8 contiguous ranges
// (one per XCD: neighbouring tiles share halo lines in the XCD's L2).
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "dw_stage.hpp"
#include "kernels.hpp"

namespace phx {

typedef float sep_f16v __attribute__((ext_vector_type(16)));

// timing diagnostics only (wrong results; a separate build, make EXTRA=-DPHX_SEP_SKIP=mask): 1 window
// loads, 2 depthwise taps, 4 MFMAs, 8 output stores
#ifndef PHX_SEP_SKIP
#define PHX_SEP_SKIP 0
#endif
// timing diagnostics only (tools/sep_probe builds this file with -DPHX_SEP_STAMPS=1): wave 0 of the
// launch's first workgroup records the shader clock at each phase boundary
#if defined(PHX_SEP_STAMPS) && PHX_SEP_STAMPS
__device__ unsigned long long sep_stamps[16];
#define SEP_STAMP(k)                                                                   \
  do {                                                                                 \
    if (blockIdx.x == 0 && threadIdx.x < 64) {                                         \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                      \
      if (threadIdx.x == 0) sep_stamps[k] = t_;                                        \
    }                                                                                  \
  } while (0)
#else
#define SEP_STAMP(k) \
  do {               \
  } while (0)
#endif

namespace {

constexpr int kSepCC = 64;           // channels per staged window pass
constexpr int kSepWP = kSepCC + 4;   // LDS floats per window pixel
// tiles of 128 pixels: 16 x 8, or 8 x 16 / 4 x 16 for levels narrower than 16 (a 4 x 4 level in a
// 16 x 8 tile would stage a window of 180 pixels for 16 outputs); the window is the tile's rows that
// exist plus the halo, at most 180 pixels (10 x 18, 18 x 10, 18 x 6)
constexpr int kSepNPX = 180;
constexpr int kSepNC = 64;           // output columns per pointwise chunk
static_assert(18 * 10 <= kSepNPX && 10 * 18 <= kSepNPX && 6 * 18 <= kSepNPX, "window sizes");

struct SepGeom {
  int H, W;              // spatial size (stride 1, SAME: output = input)
  int ltw, th;           // tile: 1 << ltw columns, th rows
  int tiles_x, ntiles;   // tiles per image
  int w0;                // first flat work item of this member
};

template <class XV>
struct SepSeg {
  XV x;
  float* y;
  SepGeom g;
  StatSink sink;
};

template <int NS, class XV>
struct SepGroup {
  SepSeg<XV> s[NS];
  const float* wd;    // depthwise taps [3][3][C] (HWC)
  const float* bt;    // pointwise kernel transposed [N][C]
  const float* bias;  // [N] or nullptr
  int N, n, total, per, B;
  int np;  // column parts per tile
};

template <int C, int PT>
struct SepLds {
  static constexpr int BP = C + 4;                                    // kernel row pitch (floats)
  static constexpr int WIN = kSepNPX * kSepWP;                        // window floats
  static constexpr int BCH = 32 * PT * BP;                            // the part's kernel rows
  static constexpr int MAIN = WIN > BCH ? WIN : BCH;                  // window / kernel rows (aliased)
  static constexpr int NB = 32 * PT * (C / 4) / 256;                  // kernel-row float4 per thread
  static_assert(32 * PT * (C / 4) % 256 == 0, "k_sep_fwd: kernel rows split");
  static constexpr int TAPS = 9 * kSepCC;
  static constexpr int STAT = 4 * kSepNC * 2 + 4;                     // (mean, M2) per wave, counts
  static constexpr int FLOATS = MAIN + TAPS + STAT;
};

// stage window pass j (channels c0 .. c0 + 4*cq) through the view; ACT: the InX view's activation
// U loads in flight per lane (a fuse view's loads are up to three each); the window is rw columns by
// as many rows as npx / rw; padding (outside the image) is zero after the view
template <int ACT, class Stage, int U, class XV>
__device__ __forceinline__ void sep_stage(float* win, const XV& xv, int b, int H, int W, int C, int oy0, int ox0,
                                          int c0, int cq, int rw, int npx) {
  const int q = threadIdx.x & 15;
  if (q >= cq) return;  // (no barrier inside)
  Stage src;
  src.init(xv, c0 + 4 * q);
  for (int p0 = threadIdx.x >> 4; p0 < npx; p0 += 16 * U) {
    typename Stage::Raw v[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + 16 * u;
      const int wy = p / rw, wx = p - wy * rw;
      const int iy = oy0 - 1 + wy, ix = ox0 - 1 + wx;
      ok[u] = p < npx && iy >= 0 && iy < H && ix >= 0 && ix < W;
      const int iyc = min(max(iy, 0), H - 1), ixc = min(max(ix, 0), W - 1);
      if constexpr (PHX_SEP_SKIP & 1) v[u] = src.zero();
      else v[u] = src.load((((long)b * H + iyc) * W + ixc) * C + c0 + 4 * q);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + 16 * u;
      if (p < npx) {
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok[u]) o = src.template finish_t<ACT>(v[u]);
        *reinterpret_cast<float4*>(win + p * kSepWP + 4 * q) = o;
      }
    }
  }
}

// PT: 32-column tiles of the pointwise output per workgroup (a "part"; N > 32 PT splits into parts,
// each its own workgroup over the same tile, the depthwise pass repeated): the part's kernel rows are
// staged into LDS once, so the MFMA / store loop waits on no memory (its stores drain behind it)
template <int C, int NS, class XV, bool STATS, int PT>
__global__ __launch_bounds__(256, 2) void k_sep_fwd(SepGroup<NS, XV> grp) {
  using Stage = std::conditional_t<std::is_same<XV, InX>::value, StageInX<false>, StageFuse<false>>;
  using L = SepLds<C, PT>;
  static_assert(C == kSepCC, "k_sep_fwd: one window pass (C = 64)");
  constexpr int KS = C / 8;  // MFMA k steps (8 channels each)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* const win = sm;
  float* const bl = sm;  // the part's kernel rows [32 PT][BP], aliasing the window after the depthwise pass
  float* const taps = sm + L::MAIN;
  float2* const wst = reinterpret_cast<float2*>(taps + L::TAPS);
  float* const wcn = reinterpret_cast<float*>(wst + 4 * kSepNC);

  const int Lb = blockIdx.x;
  const int wj = (Lb & 7) * grp.per + (Lb >> 3);
  if ((Lb >> 3) >= grp.per || wj >= grp.total) return;  // workgroup-uniform, before any barrier
  SEP_STAMP(0);
  const int part = wj % grp.np, wi = wj / grp.np;  // (the parts of a tile are neighbours: one XCD's L2)
  int m = 0;
#pragma unroll
  for (int k = 1; k < NS; ++k)
    if (k < grp.n && wi >= grp.s[k].g.w0) m = k;
  const SepSeg<XV> sg = pick_seg(grp.s, m);
  const SepGeom& g = sg.g;
  const int local = wi - g.w0;
  const int b = local / g.ntiles, tile = local - b * g.ntiles;
  const int ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
  const int tw = 1 << g.ltw;
  const int oy0 = ty * g.th, ox0 = tx * tw;
  const int rw = tw + 2;                                   // window columns
  const int npx = rw * (min(g.th, g.H - oy0) + 2);         // window pixels (the tile's rows that exist)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  // this lane's pixel: MFMA row r32 of the wave's 32-pixel M tile
  const int pp = wave * 32 + r32;
  const int py = pp >> g.ltw, px = pp & (tw - 1);
  const bool pin = py < g.th && oy0 + py < g.H && ox0 + px < g.W;
  const int N = grp.N;
  const int n0 = part * 32 * PT;                 // the part's first column
  const int nc = min(32 * PT, N - n0);           // its columns

  // ---- prologue: the part's kernel rows and the taps go into registers; their loads fly with the
  // window's (one memory round trip) ----
  const float4* const bt4 = reinterpret_cast<const float4*>(grp.bt);
  float4 breg[L::NB];
#pragma unroll
  for (int u = 0; u < L::NB; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int r = e / (C / 4), qq = e - r * (C / 4);
    breg[u] = bt4[(long)(n0 + min(r, nc - 1)) * (C / 4) + qq];  // (rows past the part are zeroed when stored)
  }
  const int tq = threadIdx.x < 9 * (C / 4) ? (int)threadIdx.x : 0;
  const int tt = tq / (C / 4), tqq = tq - tt * (C / 4);
  const float4 tp = *reinterpret_cast<const float4*>(grp.wd + tt * C + 4 * tqq);

  // ---- 1: the window through the view; 2: depthwise outputs into the A fragments ----
  constexpr int SU = std::is_same<XV, InX>::value ? 12 : 6;
  if constexpr (Stage::kActT) {
    const int act = sg.x.act;
    if (act == 1) sep_stage<1, Stage, SU>(win, sg.x, b, g.H, g.W, C, oy0, ox0, 0, C / 4, rw, npx);
    else if (act == 2) sep_stage<2, Stage, SU>(win, sg.x, b, g.H, g.W, C, oy0, ox0, 0, C / 4, rw, npx);
    else sep_stage<0, Stage, SU>(win, sg.x, b, g.H, g.W, C, oy0, ox0, 0, C / 4, rw, npx);
  } else {
    sep_stage<0, Stage, SU>(win, sg.x, b, g.H, g.W, C, oy0, ox0, 0, C / 4, rw, npx);
  }
  if (threadIdx.x < 9 * (C / 4)) *reinterpret_cast<float4*>(taps + tt * kSepCC + 4 * tqq) = tp;
  SEP_STAMP(1);
  __syncthreads();
  SEP_STAMP(2);
  float4 a[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int c = 8 * s + 4 * h;  // this lane's channel quad at k step s
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (PHX_SEP_SKIP & 2) {
      acc = *reinterpret_cast<const float4*>(win + (py * rw + px) * kSepWP + c);
    } else if (pin) {
      const float* wp = win + (py * rw + px) * kSepWP + c;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float4 v = *reinterpret_cast<const float4*>(wp + (ky * rw + kx) * kSepWP);
          const float4 w = *reinterpret_cast<const float4*>(taps + (ky * 3 + kx) * kSepCC + c);
          acc.x = fmaf(v.x, w.x, acc.x);
          acc.y = fmaf(v.y, w.y, acc.y);
          acc.z = fmaf(v.z, w.z, acc.z);
          acc.w = fmaf(v.w, w.w, acc.w);
        }
    }
    a[s] = acc;
  }
  SEP_STAMP(3);
  __syncthreads();  // the window is dead: its space takes the part's kernel rows
#pragma unroll
  for (int u = 0; u < L::NB; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int r = e / (C / 4), qq = e - r * (C / 4);
    *reinterpret_cast<float4*>(bl + r * L::BP + 4 * qq) = r < nc ? breg[u] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  SEP_STAMP(4);

  // ---- 3: pointwise GEMM + bias (+ statistics), two 32-column tiles at a time ----
  const unsigned long long vb = __ballot(pin);
  const float nw = (float)__popcll(vb & 0xffffffffull);
  int roff[16];
  unsigned rmask = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int qe = wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    const int qy = oy0 + (qe >> g.ltw), qx = ox0 + (qe & (tw - 1));
    const bool ok = (qe >> g.ltw) < g.th && qy < g.H && qx < g.W;
    rmask |= ok ? 1u << e : 0u;
    roff[e] = (b * g.H + min(qy, g.H - 1)) * g.W + min(qx, g.W - 1);
  }
  const long bgidx = (long)b * g.ntiles + tile;  // partial row of this workgroup
#pragma unroll
  for (int tp0 = 0; tp0 < PT; tp0 += 2) {
    if (32 * tp0 >= nc) break;  // workgroup-uniform
    const int nt = min(2, min(PT - tp0, (nc - 32 * tp0 + 31) / 32));
    sep_f16v acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float4 fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
        fb[t] = *reinterpret_cast<const float4*>(bl + (32 * min(tp0 + t, PT - 1) + r32) * L::BP + 8 * s + 4 * h);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (t >= nt) break;
        if constexpr (PHX_SEP_SKIP & 4) {
          acc[t][s] += a[s].x * fb[t].y;
          continue;
        }
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s].x, fb[t].x, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s].y, fb[t].y, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s].z, fb[t].z, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s].w, fb[t].w, acc[t], 0, 0, 0);
      }
    }
    SEP_STAMP(5);
    // epilogue: lane (r32, h) holds column 32t + r32 of rows (e&3) + 8(e>>2) + 4h
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (t >= nt) break;
      const int cl = 32 * (tp0 + t) + r32;  // column within the part
      const int col = n0 + cl;
      const bool cok = cl < nc;
      const float bv = (grp.bias && cok) ? grp.bias[col] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float v = acc[t][e] + bv;
        acc[t][e] = v;
        if (cok && (rmask >> e & 1) && !(PHX_SEP_SKIP & 8)) sg.y[(long)roff[e] * N + col] = v;
      }
      if constexpr (STATS) {
        float sum = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e)
          if (rmask >> e & 1) sum += acc[t][e];
        sum += __shfl_xor(sum, 32);
        const float mean = nw > 0.f ? sum / nw : 0.f;
        float q2 = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e)
          if (rmask >> e & 1) {
            const float d = acc[t][e] - mean;
            q2 = fmaf(d, d, q2);
          }
        q2 += __shfl_xor(q2, 32);
        if (h == 0) wst[wave * kSepNC + cl] = make_float2(mean, q2);
      }
    }
    SEP_STAMP(6);
  }
  if constexpr (STATS) {  // (each part its own columns of the partial row)
    if (lane == 0) wcn[wave] = nw;
    __syncthreads();
    SEP_STAMP(7);
    if ((int)threadIdx.x < nc) {
      float tn = 0.f, tm = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float2 v = wst[w * kSepNC + threadIdx.x];
        chan_merge(tn, tm, t2, wcn[w], v.x, v.y);
      }
      sink_put(sg.sink, bgidx, n0 + threadIdx.x, tn, tm, t2);
      if (threadIdx.x == 0 && part == 0) sink_cnt(sg.sink, bgidx, tn);
    }
  }
  SEP_STAMP(8);
}

template <int C, int NS, class XV, int PT>
void sep_go(const SepGroup<NS, XV>& grp, bool stats, hipStream_t s) {
  using L = SepLds<C, PT>;
  const size_t lds = (size_t)L::FLOATS * sizeof(float);
  static_assert((size_t)L::FLOATS * sizeof(float) <= 160 * 1024, "k_sep_fwd: LDS");
  static const bool attr = [] {
    bool ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sep_fwd<C, NS, XV, true, PT>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    return ok && hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sep_fwd<C, NS, XV, false, PT>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  }();
  (void)attr;
  const dim3 grid(8 * grp.per), block(256);
  if (stats) hipLaunchKernelGGL((k_sep_fwd<C, NS, XV, true, PT>), grid, block, lds, s, grp);
  else hipLaunchKernelGGL((k_sep_fwd<C, NS, XV, false, PT>), grid, block, lds, s, grp);
  PHX_LAUNCH_CHECK();
}

SepGeom sep_geom(int H, int W, int w0) {
  SepGeom g{};
  g.H = H;
  g.W = W;
  g.ltw = W > 8 ? 4 : W > 4 ? 3 : 2;
  g.th = g.ltw == 4 ? 8 : 16;  // (window <= 180 pixels)
  g.tiles_x = cdiv(W, 1 << g.ltw);
  g.ntiles = g.tiles_x * cdiv(H, g.th);
  g.w0 = w0;
  return g;
}

// ---- backward: the pointwise data gradient and the depthwise transpose in one launch -------------
// For an 8 x 16 (or 16 x 8 / 16 x 4) tile of the depthwise input's gradient dx, the workgroup
//   1. stages the gradient of the pointwise output over the tile's window (tile + 1-pixel halo) through
//      the consumer BN's backward view (GradX: dy = sc (dz - mean dz - xhat mean dz xhat)), zero outside
//      the image;
//   2. multiplies it by the pointwise kernel on the fp32 matrix cores — dd = dy W^T for every window
//      pixel, the halo recomputed instead of stored (k_gemm2's k order: the dd of a pixel equals the
//      unfused dgrad's) — and writes dd over the staged window in LDS;
//   3. gathers dx from dd with the flipped taps in k_dw_bwd's order (accumulating into dx when the
//      depthwise input has several consumers), and with a GradSink the BN-backward sums of the BN whose
//      output the depthwise conv read, one partial row per tile.
// dd never reaches HBM.
template <int NS>
struct SepBwdGroup {
  struct Seg {
    GradX gv;     // the pointwise output's gradient view
    float* dx;    // [B,H,W,C]
    SepGeom g;
    int acc;
    GradSink gs;  // the depthwise input's BN (part == nullptr: none)
  } s[NS];
  const float* wd;  // depthwise taps [3][3][C]
  const float* wp;  // pointwise kernel HWIO [C][N]
  int n, total, per, B;
};

template <int C>
struct SepBwdLds {
  static constexpr int WIN = kSepNPX * kSepWP;    // g, then dd
  static constexpr int WPL = C * (kSepNC + 4);    // pointwise kernel [C][N + 4]
  static constexpr int TAPS = 9 * kSepCC;
  static constexpr int GS = 4 * 16 * 8;           // per wave, per quad: (s1, s2) float4 each
  static constexpr int FLOATS = WIN + WPL + TAPS + GS;
};

template <int C, int NS, bool GS, bool YBF>
__global__ __launch_bounds__(256, 2) void k_sep_bwd(SepBwdGroup<NS> grp) {
  static_assert(C == kSepCC, "k_sep_bwd: C = N = 64");
  constexpr int N = kSepNC, KS = N / 8, WPP = N + 4;
  using L = SepBwdLds<C>;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* const win = sm;
  float* const wpl = sm + L::WIN;
  float* const taps = wpl + L::WPL;
  float4* const gsl = reinterpret_cast<float4*>(taps + L::TAPS);

  const int Lb = blockIdx.x;
  const int wi = (Lb & 7) * grp.per + (Lb >> 3);
  if ((Lb >> 3) >= grp.per || wi >= grp.total) return;  // workgroup-uniform, before any barrier
  int m = 0;
#pragma unroll
  for (int k = 1; k < NS; ++k)
    if (k < grp.n && wi >= grp.s[k].g.w0) m = k;
  const auto sg = pick_seg(grp.s, m);
  const SepGeom& g = sg.g;
  const int local = wi - g.w0;
  const int b = local / g.ntiles, tile = local - b * g.ntiles;
  const int ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
  const int tw = 1 << g.ltw;
  const int iy0 = ty * g.th, ix0 = tx * tw;
  const int rw = tw + 2;
  const int npx = rw * (min(g.th, g.H - iy0) + 2);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int q = threadIdx.x & 15;

  // ---- 1: pointwise kernel, taps, the gradient window through the GradX view ----
  {
    const float4* w4 = reinterpret_cast<const float4*>(grp.wp);
#pragma unroll
    for (int u = 0; u < C * (N / 4) / 256; ++u) {
      const int e = threadIdx.x + 256 * u;
      const int r = e / (N / 4), qq = e - r * (N / 4);
      *reinterpret_cast<float4*>(wpl + r * WPP + 4 * qq) = w4[e];
    }
    if (threadIdx.x < 9 * (C / 4)) {
      const int t = threadIdx.x / (C / 4), qq = threadIdx.x - t * (C / 4);
      *reinterpret_cast<float4*>(taps + t * kSepCC + 4 * qq) = *reinterpret_cast<const float4*>(grp.wd + t * C + 4 * qq);
    }
  }
  {
    StageGradX<YBF> src;
    src.init(sg.gv, 4 * q);
    constexpr int U = 6;
    for (int p0 = threadIdx.x >> 4; p0 < npx; p0 += 16 * U) {
      typename StageGradX<YBF>::Raw v[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + 16 * u;
        const int wy = p / rw, wx = p - wy * rw;
        const int iy = iy0 - 1 + wy, ix = ix0 - 1 + wx;
        ok[u] = p < npx && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
        const int iyc = min(max(iy, 0), g.H - 1), ixc = min(max(ix, 0), g.W - 1);
        v[u] = src.load((((long)b * g.H + iyc) * g.W + ixc) * N + 4 * q);
      }
      const int act = src.act();
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + 16 * u;
        if (p < npx) {
          float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
          if (ok[u]) {
            if (act == 1) o = src.template finish_t<1>(v[u]);
            else if (act == 2) o = src.template finish_t<2>(v[u]);
            else o = src.template finish_t<0>(v[u]);
          }
          *reinterpret_cast<float4*>(win + p * kSepWP + 4 * q) = o;
        }
      }
    }
  }
  __syncthreads();

  // ---- 2: dd = g W^T over the window on the matrix cores (jobs: 32-pixel M tile x 32-channel half) ----
  const int mtl = (npx + 31) / 32;
  sep_f16v acc[3];
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) {
    const int job = wave + 4 * jj;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[jj][e] = 0.f;
    if (job >= 2 * mtl) continue;  // wave-uniform
    const int mt = job >> 1, nt = job & 1;
    const int pr = min(32 * mt + r32, kSepNPX - 1);  // (rows past the window read a valid pixel; not stored)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float4 fa = *reinterpret_cast<const float4*>(win + pr * kSepWP + 8 * s + 4 * h);
      const float4 fb = *reinterpret_cast<const float4*>(wpl + (32 * nt + r32) * WPP + 8 * s + 4 * h);
      acc[jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.x, fb.x, acc[jj], 0, 0, 0);
      acc[jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.y, fb.y, acc[jj], 0, 0, 0);
      acc[jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.z, fb.z, acc[jj], 0, 0, 0);
      acc[jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.w, fb.w, acc[jj], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave has read its g rows: the window now takes dd
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) {
    const int job = wave + 4 * jj;
    if (job >= 2 * mtl) continue;
    const int mt = job >> 1, nt = job & 1;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int p = 32 * mt + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (p < npx) win[p * kSepWP + 32 * nt + r32] = acc[jj][e];
    }
  }
  __syncthreads();

  // ---- 3: dx = the depthwise transpose of dd (k_dw_bwd's order), + GradSink sums ----
  constexpr int RPT = 8;
  const int col = (threadIdx.x >> 4) & (tw - 1);
  const int rg = threadIdx.x >> (4 + g.ltw);
  const int row0 = rg * RPT;
  const int ix = ix0 + col;
  const bool active = row0 < g.th && iy0 + row0 < g.H && ix < g.W;
  const int c = 4 * q;
  float4 a[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) a[r] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (active) {
    const float* base = win + (row0 * rw + col) * kSepWP + c;
#pragma unroll
    for (int ir = 0; ir < RPT + 2; ++ir) {
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) {
        const float4 v = *reinterpret_cast<const float4*>(base + (ir * rw + jj) * kSepWP);
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
          const int ii = ir - r;
          if (ii >= 0 && ii < 3) {
            const float4 w = *reinterpret_cast<const float4*>(taps + ((2 - ii) * 3 + (2 - jj)) * kSepCC + c);
            a[r].x = fmaf(v.x, w.x, a[r].x);
            a[r].y = fmaf(v.y, w.y, a[r].y);
            a[r].z = fmaf(v.z, w.z, a[r].z);
            a[r].w = fmaf(v.w, w.w, a[r].w);
          }
        }
      }
    }
  }
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  GSChan4 kk;
  if (GS && active) kk = gs_chan4(sg.gs, c);
  float4 old[RPT], yv[RPT];
  const int ixc = min(ix, g.W - 1);
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const long e = (((long)b * g.H + min(iy0 + row0 + r, g.H - 1)) * g.W + ixc) * C + c;
    if (sg.acc) old[r] = *reinterpret_cast<const float4*>(sg.dx + e);
    if constexpr (GS) yv[r] = ald4<YBF>(sg.gs.y, e);
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int iy = iy0 + row0 + r;
    if (!active || row0 + r >= g.th || iy >= g.H) continue;
    const long e = (((long)b * g.H + iy) * g.W + ix) * C + c;
    float4 v = a[r];
    if (sg.acc) {
      v.x += old[r].x; v.y += old[r].y; v.z += old[r].z; v.w += old[r].w;
    }
    *reinterpret_cast<float4*>(sg.dx + e) = v;
    if constexpr (GS) gs_acc4(sg.gs, kk, v, yv[r], s1, s2);
  }
  if constexpr (GS) {
    // lanes of one channel quad: 4 per wave (offsets 16, 32), then the 4 waves in order
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      s1.x += __shfl_xor(s1.x, o); s1.y += __shfl_xor(s1.y, o); s1.z += __shfl_xor(s1.z, o); s1.w += __shfl_xor(s1.w, o);
      s2.x += __shfl_xor(s2.x, o); s2.y += __shfl_xor(s2.y, o); s2.z += __shfl_xor(s2.z, o); s2.w += __shfl_xor(s2.w, o);
    }
    if (lane < 16) {
      gsl[(wave * 16 + q) * 2] = s1;
      gsl[(wave * 16 + q) * 2 + 1] = s2;
    }
    __syncthreads();
    if (threadIdx.x < 16) {
      float4 t1 = gsl[q * 2], t2 = gsl[q * 2 + 1];
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const float4 u = gsl[(w * 16 + q) * 2], v = gsl[(w * 16 + q) * 2 + 1];
        t1.x += u.x; t1.y += u.y; t1.z += u.z; t1.w += u.w;
        t2.x += v.x; t2.y += v.y; t2.z += v.z; t2.w += v.w;
      }
      const long p = (long)b * g.ntiles + tile;
      gsink_put(sg.gs, p, c + 0, t1.x, t2.x);
      gsink_put(sg.gs, p, c + 1, t1.y, t2.y);
      gsink_put(sg.gs, p, c + 2, t1.z, t2.z);
      gsink_put(sg.gs, p, c + 3, t1.w, t2.w);
    }
  }
}

template <int NS>
void sep_bwd_go(const SepBwdGroup<NS>& grp, bool gs, bool ybf, hipStream_t s) {
  const size_t lds = (size_t)SepBwdLds<64>::FLOATS * sizeof(float);
  static_assert((size_t)SepBwdLds<64>::FLOATS * sizeof(float) <= 160 * 1024, "k_sep_bwd: LDS");
  static const bool attr = [] {
    const void* ks[] = {reinterpret_cast<const void*>(&k_sep_bwd<64, NS, true, false>),
                        reinterpret_cast<const void*>(&k_sep_bwd<64, NS, false, false>),
                        reinterpret_cast<const void*>(&k_sep_bwd<64, NS, true, true>),
                        reinterpret_cast<const void*>(&k_sep_bwd<64, NS, false, true>)};
    bool ok = true;
    for (const void* k : ks)
      ok = ok && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    return ok;
  }();
  (void)attr;
  const dim3 grid(8 * grp.per), block(256);
  if (gs && ybf) hipLaunchKernelGGL((k_sep_bwd<64, NS, true, true>), grid, block, lds, s, grp);
  else if (gs) hipLaunchKernelGGL((k_sep_bwd<64, NS, true, false>), grid, block, lds, s, grp);
  else if (ybf) hipLaunchKernelGGL((k_sep_bwd<64, NS, false, true>), grid, block, lds, s, grp);
  else hipLaunchKernelGGL((k_sep_bwd<64, NS, false, false>), grid, block, lds, s, grp);
  PHX_LAUNCH_CHECK();
}

// N <= 64: one part of two 32-column tiles (each part writes its own columns of the statistics
// partial row; wider outputs are not planned, see sep_supported)
template <int NS, class XV>
int sep_dispatch(SepGroup<NS, XV>& grp, int C, bool stats, hipStream_t s) {
  if (C != 64 || grp.N > 64) throw std::invalid_argument("sep: unsupported shape");
  // (one 32-column part per workgroup — twice the workgroups, the depthwise pass repeated — measured
  // slower: P3 19.3 -> 25.7 us, C2 +0.15 ms; scripts/gpu_r06_seppt.sh)
  constexpr int pt = 2;
  grp.np = cdiv(grp.N, 32 * pt);
  const int total = grp.total;
  grp.total = total * grp.np;
  grp.per = cdiv(grp.total, 8);
  sep_go<64, NS, XV, pt>(grp, stats, s);
  grp.total = total;
  return 0;
}

}  // namespace

// N <= 64 (the BiFPN nodes, the head repeats, the box head's predict conv): the class head's predict
// conv (N = 810) measured slower fused — 146 us per group with its 64-column kernel chunks streamed
// through LDS, 206 us split into 224-column parts (the depthwise pass repeated per part) — than its
// two launches (the pointwise GEMM alone 105 us at P3)
bool sep_supported(int C, int N, bool bf16) { return !bf16 && C == 64 && N >= 1 && N <= 64; }

int sep_stat_partials(int B, int H, int W) { return B * sep_geom(H, W, 0).ntiles; }

void launch_sep_fwd(const SepMember* mem, int n, int B, int C, int N, const float* wd, const float* bt,
                    const float* bias, hipStream_t s, int* nps) {
  if (n < 1 || n > kMaxSeg) throw std::invalid_argument("sep: bad member count");
  if (!sep_supported(C, N, false)) throw std::invalid_argument("sep: unsupported shape");
  const bool stats = mem[0].sink.part != nullptr;
  for (int i = 0; i < n; ++i) {
    if ((mem[i].sink.part != nullptr) != stats) throw std::invalid_argument("sep: members differ in sinks");
    if (mem[i].fuse != mem[0].fuse) throw std::invalid_argument("sep: members differ in input views");
    if (mem[i].H <= 0 || mem[i].W <= 0) throw std::invalid_argument("sep: empty member");
  }
  if (mem[0].fuse && n != 1) throw std::invalid_argument("sep: a fused input view is not grouped");
  auto fill = [&](auto& grp) {
    grp.wd = wd;
    grp.bt = bt;
    grp.bias = bias;
    grp.N = N;
    grp.n = n;
    grp.B = B;
    int w0 = 0;
    for (int i = 0; i < n; ++i) {
      auto& sg = grp.s[i];
      sg.y = mem[i].y;
      sg.g = sep_geom(mem[i].H, mem[i].W, w0);
      sg.sink = mem[i].sink;
      sg.sink.C = N;
      sg.sink.P = B * sg.g.ntiles;
      if (nps) nps[i] = sg.sink.P;
      w0 += B * sg.g.ntiles;
    }
    grp.total = w0;
  };
  if (mem[0].fuse) {
    SepGroup<1, FuseView> grp{};
    grp.s[0].x = mem[0].f;
    fill(grp);
    sep_dispatch(grp, C, stats, s);
  } else if (n == 1) {
    SepGroup<1, InX> grp{};
    grp.s[0].x = mem[0].x;
    fill(grp);
    sep_dispatch(grp, C, stats, s);
  } else {
    SepGroup<kMaxSeg, InX> grp{};
    for (int i = 0; i < n; ++i) grp.s[i].x = mem[i].x;
    fill(grp);
    sep_dispatch(grp, C, stats, s);
  }
}

bool sep_bwd_supported(int C, int N, bool bf16) { return !bf16 && C == 64 && N == 64; }

void launch_sep_bwd(const SepBwdMember* mem, int n, int B, int C, int N, const float* wd, const float* wp,
                    hipStream_t s, int* nps) {
  if (n < 1 || n > kMaxSeg) throw std::invalid_argument("sep bwd: bad member count");
  if (!sep_bwd_supported(C, N, false)) throw std::invalid_argument("sep bwd: unsupported shape");
  const bool gs = mem[0].gs.part != nullptr;
  const bool ybf = (mem[0].gv.y && mem[0].gv.ybf) || (gs && mem[0].gs.ybf);
  for (int i = 0; i < n; ++i) {
    if ((mem[i].gs.part != nullptr) != gs) throw std::invalid_argument("sep bwd: members differ in sinks");
    if (mem[i].H <= 0 || mem[i].W <= 0) throw std::invalid_argument("sep bwd: empty member");
  }
  auto fill = [&](auto& grp) {
    grp.wd = wd;
    grp.wp = wp;
    grp.n = n;
    grp.B = B;
    int w0 = 0;
    for (int i = 0; i < n; ++i) {
      auto& sg = grp.s[i];
      sg.gv = mem[i].gv;
      sg.dx = mem[i].dx;
      sg.g = sep_geom(mem[i].H, mem[i].W, w0);
      sg.acc = mem[i].acc ? 1 : 0;
      sg.gs = mem[i].gs;
      sg.gs.C = C;
      sg.gs.P = B * sg.g.ntiles;
      if (nps) nps[i] = sg.gs.P;
      w0 += B * sg.g.ntiles;
    }
    grp.total = w0;
    grp.per = cdiv(w0, 8);
  };
  if (n == 1) {
    SepBwdGroup<1> grp{};
    fill(grp);
    sep_bwd_go(grp, gs, ybf, s);
  } else {
    SepBwdGroup<kMaxSeg> grp{};
    fill(grp);
    sep_bwd_go(grp, gs, ybf, s);
  }
}

}  // namespace phx
