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
};

template <int C>
struct SepLds {
  static constexpr int BP = C + 4;                                    // B row pitch (floats)
  static constexpr int WIN = kSepNPX * kSepWP;                        // window floats
  static constexpr int BCH = kSepNC * BP;                             // B chunk floats
  static constexpr int MAIN = WIN > 2 * BCH ? WIN : 2 * BCH;          // window / two B chunks (aliased)
  static constexpr int NB = kSepNC * (C / 4) / 256;                   // B-chunk float4 per thread
  static_assert(kSepNC * (C / 4) % 256 == 0, "k_sep_fwd: B chunk split");
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

template <int C, int NS, class XV, bool STATS>
__global__ __launch_bounds__(256, 2) void k_sep_fwd(SepGroup<NS, XV> grp) {
  using Stage = std::conditional_t<std::is_same<XV, InX>::value, StageInX<false>, StageFuse<false>>;
  using L = SepLds<C>;
  constexpr int NCH = (C + kSepCC - 1) / kSepCC;  // window passes
  constexpr int KS = C / 8;                        // MFMA k steps (8 channels each)
  static_assert(C % 8 == 0, "k_sep_fwd: C % 8");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* const win = sm;
  float* const taps = sm + L::MAIN;
  float2* const wst = reinterpret_cast<float2*>(taps + L::TAPS);
  float* const wcn = reinterpret_cast<float*>(wst + 4 * kSepNC);

  const int Lb = blockIdx.x;
  const int wi = (Lb & 7) * grp.per + (Lb >> 3);
  if ((Lb >> 3) >= grp.per || wi >= grp.total) return;  // workgroup-uniform, before any barrier
  SEP_STAMP(0);
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

  // ---- prologue: the taps of pass 0 and pointwise chunk 0 go into registers; their loads fly with
  // the window's (one memory round trip for all three) ----
  const float4* const bt4 = reinterpret_cast<const float4*>(grp.bt);
  const int N = grp.N;
  float4 breg[L::NB];
  auto load_b = [&](int n0) {
#pragma unroll
    for (int u = 0; u < L::NB; ++u) {
      const int e = threadIdx.x + 256 * u;
      const int r = e / (C / 4), q = e - r * (C / 4);
      const int n = min(n0 + r, N - 1);
      breg[u] = bt4[(long)n * (C / 4) + q];  // (rows past N are zeroed when stored)
    }
  };
  auto store_b = [&](float* bl, int n0) {
#pragma unroll
    for (int u = 0; u < L::NB; ++u) {
      const int e = threadIdx.x + 256 * u;
      const int r = e / (C / 4), q = e - r * (C / 4);
      *reinterpret_cast<float4*>(bl + r * L::BP + 4 * q) = n0 + r < N ? breg[u] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  load_b(0);

  // ---- 1-2: window passes, depthwise outputs into the A fragments ----
  constexpr int SU = std::is_same<XV, InX>::value ? 12 : 6;
  float4 a[KS];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c0 = j * kSepCC;
    constexpr int CQF = kSepCC / 4;
    const int cq = min(CQF, (C - c0) / 4);
    const int tq = threadIdx.x < 9 * cq ? (int)threadIdx.x : 0;
    const int tt = tq / cq, tqq = tq - tt * cq;
    const float4 tp = *reinterpret_cast<const float4*>(grp.wd + tt * C + c0 + 4 * tqq);
    if constexpr (Stage::kActT) {
      const int act = sg.x.act;
      if (act == 1) sep_stage<1, Stage, SU>(win, sg.x, b, g.H, g.W, C, oy0, ox0, c0, cq, rw, npx);
      else if (act == 2) sep_stage<2, Stage, SU>(win, sg.x, b, g.H, g.W, C, oy0, ox0, c0, cq, rw, npx);
      else sep_stage<0, Stage, SU>(win, sg.x, b, g.H, g.W, C, oy0, ox0, c0, cq, rw, npx);
    } else {
      sep_stage<0, Stage, SU>(win, sg.x, b, g.H, g.W, C, oy0, ox0, c0, cq, rw, npx);
    }
    if (threadIdx.x < 9 * cq) *reinterpret_cast<float4*>(taps + tt * kSepCC + 4 * tqq) = tp;
    SEP_STAMP(1);
    __syncthreads();
    SEP_STAMP(2);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (8 * j + s >= KS) break;
      const int c = 8 * s + 4 * h;  // pass-local channel of this lane's quad
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
      a[8 * j + s] = acc;
    }
    SEP_STAMP(3);
    __syncthreads();  // the window and taps are rewritten by the next pass (or the B chunks)
  }

  // ---- 3: pointwise GEMM + bias (+ statistics) over 64-column chunks, double-buffered: chunk k + 1
  // is written to the other buffer (its loads issued a chunk earlier) while chunk k multiplies ----
  float* const blb = sm;  // two B chunks [kSepNC][BP], aliasing the window
  store_b(blb, 0);
  if (N > kSepNC) load_b(kSepNC);
  __syncthreads();
  SEP_STAMP(4);
  // the wave's valid rows (pixels) for the statistics
  const unsigned long long vb = __ballot(pin);
  const float nw = (float)__popcll(vb & 0xffffffffull);
  // output offsets (pixels) of the 16 rows this lane holds in the C/D layout: rows (e&3) + 8(e>>2) + 4h
  int roff[16];
  unsigned rmask = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int q = wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    const int qy = oy0 + (q >> g.ltw), qx = ox0 + (q & (tw - 1));
    const bool ok = (q >> g.ltw) < g.th && qy < g.H && qx < g.W;
    rmask |= ok ? 1u << e : 0u;
    roff[e] = (b * g.H + min(qy, g.H - 1)) * g.W + min(qx, g.W - 1);
  }
  const long bgidx = (long)b * g.ntiles + tile;  // partial row of this workgroup
  for (int n0 = 0, k = 0; n0 < N; n0 += kSepNC, ++k) {
    const float* bl = blb + (k & 1) * L::BCH;
    sep_f16v acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
    const int nt = min(2, (N - n0 + 31) / 32);  // 32-column tiles of this chunk (wave-uniform)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float4 fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) fb[t] = *reinterpret_cast<const float4*>(bl + (32 * t + r32) * L::BP + 8 * s + 4 * h);
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
    // the next chunk into the other buffer (read by nobody since the previous chunk's barrier), and the
    // loads of the one after it
    if (n0 + kSepNC < N) {
      store_b(blb + ((k + 1) & 1) * L::BCH, n0 + kSepNC);
      if (n0 + 2 * kSepNC < N) load_b(n0 + 2 * kSepNC);
    }
    // epilogue: lane (r32, h) holds column 32t + r32 of rows (e&3) + 8(e>>2) + 4h
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (t >= nt) break;
      const int col = n0 + 32 * t + r32;
      const bool cok = col < N;
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
        if (h == 0) wst[wave * kSepNC + 32 * t + r32] = make_float2(mean, q2);
      }
    }
    SEP_STAMP(6);
    if constexpr (STATS) {
      if (lane == 0) wcn[wave] = nw;
      __syncthreads();
      SEP_STAMP(7);
      if (threadIdx.x < kSepNC && n0 + (int)threadIdx.x < N) {
        float tn = 0.f, tm = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float2 v = wst[w * kSepNC + threadIdx.x];
          chan_merge(tn, tm, t2, wcn[w], v.x, v.y);
        }
        sink_put(sg.sink, bgidx, n0 + threadIdx.x, tn, tm, t2);
        if (n0 == 0 && threadIdx.x == 0) sink_cnt(sg.sink, bgidx, tn);
      }
    }
    __syncthreads();  // (the next chunk's buffer is complete; the statistics scratch is free again)
  }
  SEP_STAMP(8);
}

template <int C, int NS, class XV>
void sep_go(const SepGroup<NS, XV>& grp, bool stats, hipStream_t s) {
  const size_t lds = (size_t)SepLds<C>::FLOATS * sizeof(float);
  static_assert((size_t)SepLds<C>::FLOATS * sizeof(float) <= 160 * 1024, "k_sep_fwd: LDS");
  const dim3 grid(8 * grp.per), block(256);
  if (stats) {
    static const bool attr = [] {
      return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sep_fwd<C, NS, XV, true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    }();
    (void)attr;
    hipLaunchKernelGGL((k_sep_fwd<C, NS, XV, true>), grid, block, lds, s, grp);
  } else {
    static const bool attr = [] {
      return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sep_fwd<C, NS, XV, false>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    }();
    (void)attr;
    hipLaunchKernelGGL((k_sep_fwd<C, NS, XV, false>), grid, block, lds, s, grp);
  }
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

template <int NS, class XV>
int sep_dispatch(SepGroup<NS, XV>& grp, int C, bool stats, hipStream_t s) {
  grp.per = cdiv(grp.total, 8);
  if (C == 64) sep_go<64, NS, XV>(grp, stats, s);
  else throw std::invalid_argument("sep: unsupported channel count");
  return 0;
}

}  // namespace

bool sep_supported(int C, int N, bool bf16) { return !bf16 && C == 64 && N >= 1; }

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

}  // namespace phx
