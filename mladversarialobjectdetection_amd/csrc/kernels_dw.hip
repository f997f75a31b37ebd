// kernels_dw.hip — depthwise k x k convolution (TF SAME) forward and data-gradient for gfx950.
//
// Reference: DepthwiseConv2D in MBConvBlock (efficientnet_model.py:224-417), the separable convs of
// BiFPN (efficientdet_keras.py:201-221) and of the class/box heads (efficientdet_keras.py:414-471);
// TF SAME padding.
//
// Design.  Depthwise conv is HBM-bound (k*k MACs per 8 bytes moved), so each workgroup owns one
// spatial tile x one slice of 4*CG channels and:
//   * stages the input window (tile + halo) into LDS exactly once, applying the producer BN +
//     activation (InX) or the consumer-side BN backward (GradX) once per element, with the
//     per-channel parameters hoisted into registers (a lane's channel group never changes);
//   * issues the staging loads four at a time before any use, so one block keeps 4 x 256
//     16-byte loads in flight instead of a dependent chain;
//   * keeps the k*k filter taps of its 4 channels in registers and walks RPT output rows per
//     lane with a sliding window over the staged rows (each LDS float4 is read once per lane
//     and feeds every output row that uses it);
//   * sizes the tile to the image: OTW = min(256/CG, Wout) columns and the remaining lanes take
//     further row groups, so the 4x4..16x16 BiFPN / head levels do not idle 3/4 of the block.
// Block order is XCD-aware: the NCG channel slices of one spatial tile are dispatched
// back-to-back on the same XCD, so the NHWC lines they each read a 16*CG-byte piece of are L2 hits
// for the others.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "dw_stage.hpp"
#include "kernels.hpp"

namespace phx {

struct DwGeom {
  int H, W, C;      // conv input  (fwd: x; bwd: dx)
  int Ho, Wo;       // conv output (fwd: y; bwd: dy)
  int pt, pl;
  int lcg;          // log2(CG)
  int otw, oth;     // tile (in the space of the tensor this launch writes)
  int nrg;          // row groups per block
  int rin, cin;     // staged window
  int tiles_x, ntiles, ncg;
  int per;          // work items per XCD
};

// Grouped launch: up to kMaxSeg convolutions with the same taps, kernel size, stride and channel
// count (the per-level members of a class/box-head conv) run as one grid, blockIdx.y = member.
// XV: the input view — InX (BN view) or FuseView (a BiFPN node's fuse computed on load, so the
// node's fused tensor is never written)
template <class XV>
struct DwFwdSegT {
  XV x;
  float* y;
  DwGeom g;
  StatSink sink;
};
using DwFwdSeg = DwFwdSegT<InX>;
template <int NS, class XV = InX>  // argument slots: 1 (ordinary launch, small kernarg) or kMaxSeg
struct DwFwdGroup {
  DwFwdSegT<XV> s[NS];
  const float* w;
};
struct DwBwdSeg {
  GradX gv;
  float* dx;
  DwGeom g;
  int acc;
  GradSink gs;
};
template <int NS>
struct DwBwdGroup {
  DwBwdSeg s[NS];
  const float* w;
};

// filter taps: read from LDS (all lanes of one channel group hit the same address, so the read is
// a broadcast).  25 float4 taps of a 5x5 kernel held in registers cost 100 VGPRs and halved
// occupancy (measured: the 5x5 forwards and data gradients 25 % faster from LDS, -2 % per step on
// D0 and D4); for 3x3 the LDS form is equal or slightly faster.
#ifndef PHX_DW_LDS_TAPS
#define PHX_DW_LDS_TAPS 2
#endif
template <int K>
struct Taps {
  // 1: 5x5 taps in LDS (25 float4 in registers halved occupancy), 2: every kernel size
  static constexpr bool kLds = PHX_DW_LDS_TAPS == 2 || (PHX_DW_LDS_TAPS == 1 && K > 3);
  float4 r[kLds ? 1 : K * K];
  const float4* l;
  int cg, CG;
  __device__ __forceinline__ void stage(float4* wt, const float* w, int C, int cgi, int lcg) {
    if constexpr (kLds) {
      const int n = (K * K) << lcg;
      for (int e = threadIdx.x; e < n; e += 256) {
        const int t = e >> lcg, k = e & ((1 << lcg) - 1);
        wt[e] = *reinterpret_cast<const float4*>(w + (long)t * C + (((cgi << lcg) + k) << 2));
      }
    }
  }
  __device__ __forceinline__ void init(const float4* wt, const float* w, int C, int c, int cg_,
                                       int lcg) {
    cg = cg_;
    CG = 1 << lcg;
    l = wt;
    if constexpr (!kLds) {
#pragma unroll
      for (int t = 0; t < K * K; ++t) r[t] = *reinterpret_cast<const float4*>(w + (long)t * C + c);
    }
  }
  __device__ __forceinline__ float4 operator()(int t) const {
    if constexpr (kLds) return l[t * CG + cg];
    else return r[t];
  }
};

// stage rows [r0, r0+rin) x cols [c0, c0+cin) of the NHWC source (sh x sw) into LDS.
// Loads inside the window are unconditional from clamped (valid) addresses, the padding zeros are
// selected when the values are written (slots of a batch past the window load nothing), and the source view's activation is a compile-time constant of the pass (a
// per-element switch on it was a third of the instructions of the staging loop).
template <int ACT, class Src, int U>
__device__ __forceinline__ void dw_stage_t(float4* tile, const Src& src, int b, int sh, int sw, int C,
                                           int r0, int c0, int chan, const DwGeom& g) {
  const int CG = 1 << g.lcg;
  const int npx = g.rin * g.cin;
  const int pstep = 256 >> g.lcg;
  const int ecg = threadIdx.x & (CG - 1);
  int p = threadIdx.x >> g.lcg;
  for (; p < npx; p += U * pstep) {
    typename Src::Raw v[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int pp = p + u * pstep;
      const int prow = pp / g.cin, pcol = pp - prow * g.cin;
      const int iy = r0 + prow, ix = c0 + pcol;
      ok[u] = pp < npx && iy >= 0 && iy < sh && ix >= 0 && ix < sw;
      const int iyc = min(max(iy, 0), sh - 1), ixc = min(max(ix, 0), sw - 1);
      if (pp < npx) v[u] = src.load((((long)b * sh + iyc) * sw + ixc) * C + chan);
      else v[u] = src.zero();  // past the window (the batch's tail): no load
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int pp = p + u * pstep;
      if (pp < npx)
        tile[(pp << g.lcg) + ecg] = ok[u] ? src.template finish_t<ACT>(v[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

template <class Src, int U = 4>
__device__ __forceinline__ void dw_stage(float4* tile, const Src& src, int b, int sh, int sw, int C,
                                         int r0, int c0, int chan, const DwGeom& g) {
  if constexpr (Src::kActT) {
    const int act = src.act();
    if (act == 1) dw_stage_t<1, Src, U>(tile, src, b, sh, sw, C, r0, c0, chan, g);
    else if (act == 2) dw_stage_t<2, Src, U>(tile, src, b, sh, sw, C, r0, c0, chan, g);
    else dw_stage_t<0, Src, U>(tile, src, b, sh, sw, C, r0, c0, chan, g);
  } else {
    dw_stage_t<0, Src, U>(tile, src, b, sh, sw, C, r0, c0, chan, g);
  }
}

// Per-channel (sum, M2) of the RPT x 4 outputs a lane holds, reduced over the block's lanes of the
// same channel group (xor-shuffles inside a wave, then the 4 waves through LDS) and written as
// partial row p of the StatSink.  Two register passes (mean, then M2 about it).
__device__ __forceinline__ float4 dw_xor_sum(float4 v, int lcg) {
  for (int o = 1 << lcg; o < 64; o <<= 1) {
    v.x += __shfl_xor(v.x, o);
    v.y += __shfl_xor(v.y, o);
    v.z += __shfl_xor(v.z, o);
    v.w += __shfl_xor(v.w, o);
  }
  return v;
}

template <int RPT>
__device__ __forceinline__ void dw_stats(const float4 (&acc)[RPT], unsigned vmask, int lcg, int c,
                                         long p, const StatSink& sink) {
  __shared__ float4 wm_[4][8], w2_[4][8];
  __shared__ float wn_[4][8];
  const int CG = 1 << lcg, cg = threadIdx.x & (CG - 1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float n = (float)__popc(vmask);
  for (int o = CG; o < 64; o <<= 1) n += __shfl_xor(n, o);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int r = 0; r < RPT; ++r)
    if (vmask >> r & 1) { s.x += acc[r].x; s.y += acc[r].y; s.z += acc[r].z; s.w += acc[r].w; }
  s = dw_xor_sum(s, lcg);
  const float inv = n > 0.f ? 1.f / n : 0.f;
  const float4 m = make_float4(s.x * inv, s.y * inv, s.z * inv, s.w * inv);
  float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int r = 0; r < RPT; ++r)
    if (vmask >> r & 1) {
      const float dx = acc[r].x - m.x, dy = acc[r].y - m.y, dz = acc[r].z - m.z, dw = acc[r].w - m.w;
      q.x = fmaf(dx, dx, q.x); q.y = fmaf(dy, dy, q.y); q.z = fmaf(dz, dz, q.z); q.w = fmaf(dw, dw, q.w);
    }
  q = dw_xor_sum(q, lcg);
  if (lane < CG) {
    wm_[wave][cg] = m;
    w2_[wave][cg] = q;
    wn_[wave][cg] = n;
  }
  __syncthreads();
  if (threadIdx.x < CG) {
    float tn[4] = {0.f, 0.f, 0.f, 0.f}, tm[4] = {0.f, 0.f, 0.f, 0.f}, t2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float4 a = wm_[w][cg], b = w2_[w][cg];
      const float nn = wn_[w][cg];
      chan_merge(tn[0], tm[0], t2[0], nn, a.x, b.x);
      chan_merge(tn[1], tm[1], t2[1], nn, a.y, b.y);
      chan_merge(tn[2], tm[2], t2[2], nn, a.z, b.z);
      chan_merge(tn[3], tm[3], t2[3], nn, a.w, b.w);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) sink_put(sink, p, c + j, tn[j], tm[j], t2[j]);
    if (threadIdx.x == 0) sink_cnt(sink, p, tn[0]);
  }
}

// ---- forward: y[oy][ox] = sum_ij a[oy*S - pt + i][ox*S - pl + j] * w[i][j] ----------------
// BF: input and output activations in bf16 storage (statistics of the stored values)
template <int K, int S, int RPT, bool STATS, int NS, class XV, int SU = 4, bool BF = false>
__global__ __launch_bounds__(256) void k_dw_fwd(DwFwdGroup<NS, XV> grp) {
  using Stage = std::conditional_t<std::is_same<XV, InX>::value, StageInX<BF>, StageFuse<BF>>;
  const DwFwdSegT<XV> sg = pick_seg(grp.s, NS == 1 ? 0 : (int)blockIdx.y);
  const XV& xv = sg.x;
  const DwGeom& g = sg.g;
  const StatSink& sink = sg.sink;
  const float* __restrict__ w = grp.w;
  float* __restrict__ y = sg.y;
  extern __shared__ float4 tile[];
  const int b = blockIdx.z;
  int tl, cgi;
  if (!dw_block_map(blockIdx.x, g.per, g.ncg, g.ntiles * g.ncg, &tl, &cgi)) return;
  const int CG = 1 << g.lcg;
  const int ty = tl / g.tiles_x, tx = tl - ty * g.tiles_x;
  const int oy0 = ty * g.oth, ox0 = tx * g.otw;
  const int cg = threadIdx.x & (CG - 1), q = threadIdx.x >> g.lcg;
  const int col = q % g.otw, rg = q / g.otw;
  const int c = (cgi * CG + cg) * 4;

  Stage src;
  src.init(xv, c);
  float4* wt = tile + g.rin * g.cin * CG;
  Taps<K> wr;
  wr.stage(wt, w, g.C, cgi, g.lcg);
  dw_stage<Stage, SU>(tile, src, b, g.H, g.W, g.C, oy0 * S - g.pt, ox0 * S - g.pl, c, g);
  __syncthreads();

  const int ox = ox0 + col;
  const int row0 = rg * RPT;  // first local output row of this lane
  const bool active = rg < g.nrg && ox < g.Wo && oy0 + row0 < g.Ho;
  if (!STATS && !active) return;
  float4 acc[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (active) {
    wr.init(wt, w, g.C, c, cg, g.lcg);
    constexpr int NR = (RPT - 1) * S + K;
    const float4* base = tile + ((row0 * S) * g.cin + col * S) * CG + cg;
#pragma unroll
    for (int ir = 0; ir < NR; ++ir) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const float4 v = base[(ir * g.cin + j) * CG];
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
          const int i = ir - r * S;
          if (i >= 0 && i < K) fma4(acc[r], v, wr(i * K + j));
        }
      }
      if constexpr (K > 3) __builtin_amdgcn_sched_barrier(0);  // stream rows: bound live VGPRs
    }
  }
  unsigned vmask = 0;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int oy = oy0 + row0 + r;
    if (active && oy < g.Ho) {
      vmask |= 1u << r;
      ast4<BF>(y, (((long)b * g.Ho + oy) * g.Wo + ox) * g.C + c, acc[r]);
    }
    if constexpr (BF && STATS)
      acc[r] = make_float4(round_bf16(acc[r].x), round_bf16(acc[r].y), round_bf16(acc[r].z), round_bf16(acc[r].w));
  }
  if constexpr (STATS) {
    dw_stats<RPT>(acc, vmask, g.lcg, c, (long)b * g.ntiles + tl, sink);
  }
}

// ---- data gradient: dx[iy][ix] = sum over (i,j) with (iy+pt-i) and (ix+pl-j) divisible by S of
//      dy[(iy+pt-i)/S][(ix+pl-j)/S] * w[i][j]  (the adjoint of the forward above) ---------------
// BN-backward sums (GradSink) of the RPT x 4 gradient values a lane wrote: plain sums, reduced
// over the lanes of the channel group and the 4 waves like dw_stats.
__device__ __forceinline__ void dw_gsums(float4 s1, float4 s2, int lcg, int c, long p, const GradSink& g) {
  __shared__ float4 a_[4][8], b_[4][8];
  const int CG = 1 << lcg, cg = threadIdx.x & (CG - 1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  s1 = dw_xor_sum(s1, lcg);
  s2 = dw_xor_sum(s2, lcg);
  if (lane < CG) {
    a_[wave][cg] = s1;
    b_[wave][cg] = s2;
  }
  __syncthreads();
  if (threadIdx.x < CG) {
    float4 t1 = a_[0][cg], t2 = b_[0][cg];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 u = a_[w][cg], v = b_[w][cg];
      t1.x += u.x; t1.y += u.y; t1.z += u.z; t1.w += u.w;
      t2.x += v.x; t2.y += v.y; t2.z += v.z; t2.w += v.w;
    }
    gsink_put(g, p, c + 0, t1.x, t2.x);
    gsink_put(g, p, c + 1, t1.y, t2.y);
    gsink_put(g, p, c + 2, t1.z, t2.z);
    gsink_put(g, p, c + 3, t1.w, t2.w);
  }
}

// YBF: the BN input y (gradient view, GradSink) in bf16 storage; dy and dx stay fp32
template <int K, int S, int RPT, bool GS, int NS, int SU = 4, bool YBF = false>
__global__ __launch_bounds__(256) void k_dw_bwd(DwBwdGroup<NS> grp) {
  const DwBwdSeg sg = pick_seg(grp.s, NS == 1 ? 0 : (int)blockIdx.y);
  const GradX& gv = sg.gv;
  const DwGeom& g = sg.g;
  const GradSink& gsk = sg.gs;
  const int acc_flag = sg.acc;
  const float* __restrict__ w = grp.w;
  float* __restrict__ dx = sg.dx;
  extern __shared__ float4 tile[];
  const int b = blockIdx.z;
  int tl, cgi;
  if (!dw_block_map(blockIdx.x, g.per, g.ncg, g.ntiles * g.ncg, &tl, &cgi)) return;
  const int CG = 1 << g.lcg;
  const int ty = tl / g.tiles_x, tx = tl - ty * g.tiles_x;
  const int iy0 = ty * g.oth, ix0 = tx * g.otw;  // input-space tile origin
  const int cg = threadIdx.x & (CG - 1), q = threadIdx.x >> g.lcg;
  const int col = q % g.otw, rg = q / g.otw;
  const int c = (cgi * CG + cg) * 4;
  // dy window origin: floor((iy0 + pt - (K-1)) / S)
  const int ay = iy0 + g.pt - (K - 1), ax = ix0 + g.pl - (K - 1);
  const int oy_lo = S == 1 ? ay : (ay >= 0 ? ay / S : -((-ay + S - 1) / S));
  const int ox_lo = S == 1 ? ax : (ax >= 0 ? ax / S : -((-ax + S - 1) / S));

  StageGradX<YBF> src;
  src.init(gv, c);
  float4* wt = tile + g.rin * g.cin * CG;
  Taps<K> wr;
  wr.stage(wt, w, g.C, cgi, g.lcg);
  dw_stage<StageGradX<YBF>, SU>(tile, src, b, g.Ho, g.Wo, g.C, oy_lo, ox_lo, c, g);
  __syncthreads();

  const int ix = ix0 + col;
  const int row0 = rg * RPT;
  const bool active = rg < g.nrg && ix < g.W && iy0 + row0 < g.H;
  if (!GS && !active) return;
  float4 acc[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (active) {
    wr.init(wt, w, g.C, c, cg, g.lcg);
    if constexpr (S == 1) {
      // local dy row of (output row r, tap i) = row0 + r + (K-1-i): a sliding window as forward
      constexpr int NR = RPT + K - 1;
      const float4* base = tile + (row0 * g.cin + col) * CG + cg;
#pragma unroll
      for (int ir = 0; ir < NR; ++ir) {
#pragma unroll
        for (int jj = 0; jj < K; ++jj) {
          const float4 v = base[(ir * g.cin + jj) * CG];
#pragma unroll
          for (int r = 0; r < RPT; ++r) {
            const int ii = ir - r;  // = K-1-i
            if (ii >= 0 && ii < K) fma4(acc[r], v, wr((K - 1 - ii) * K + (K - 1 - jj)));
          }
        }
        if constexpr (K > 3) __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      const int u0 = ix + g.pl;  // column parity decides which taps land on a dy sample
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const int t0 = iy0 + row0 + r + g.pt;
#pragma unroll
        for (int i = 0; i < K; ++i) {
          const int t = t0 - i;
          if (t & 1) continue;
          const int lr = (t >> 1) - oy_lo;
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const int u = u0 - j;
            if (u & 1) continue;
            const int lc = (u >> 1) - ox_lo;
            fma4(acc[r], tile[(lr * g.cin + lc) * CG + cg], wr(i * K + j));
          }
        }
      }
    }
  }
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  GSChan4 kk;
  if (GS && active) kk = gs_chan4(gsk, c);
  // the rows' old values (acc) and BN inputs (GradSink) are read before any is used, from clamped
  // addresses (a conditional load per row waited for each one in turn)
  float4 old[RPT], yv[RPT];
  const int ixc = min(ix, g.W - 1);
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const long e = (((long)b * g.H + min(iy0 + row0 + r, g.H - 1)) * g.W + ixc) * g.C + c;
    if (acc_flag) old[r] = *reinterpret_cast<const float4*>(dx + e);
    if constexpr (GS) yv[r] = ald4<YBF>(gsk.y, e);
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int iy = iy0 + row0 + r;
    if (!active || iy >= g.H) continue;
    const long e = (((long)b * g.H + iy) * g.W + ix) * g.C + c;
    float4* o = reinterpret_cast<float4*>(dx + e);
    float4 a = acc[r];
    if (acc_flag) {
      a.x += old[r].x; a.y += old[r].y; a.z += old[r].z; a.w += old[r].w;
    }
    *o = a;
    if constexpr (GS) gs_acc4(gsk, kk, a, yv[r], s1, s2);
  }
  if constexpr (GS) {
    dw_gsums(s1, s2, g.lcg, c, (long)b * g.ntiles + tl, gsk);
  }
}

// ---- host planning -------------------------------------------------------------------------
// output rows per lane of a forward launch: 4 at stride 1, 2 at stride 2 (4 rows at stride 2 — a
// larger window, half the occupancy — and 1 row measured slower: DESIGN.md section 5).  Staging keeps
// 8 loads in flight per lane for the stride-2 and stride-1 InX forwards (-0.035 ms/step and -4 % on
// the stride-2 launches against 4; 4 and 16 measured neutral after the tail-load fix), 4 for the
// fuse views (up to three loads each) and the data gradients (a GradX load is two float4; 8 deep
// measured 0.1 ms/step slower).
static int dw_rpt_fwd(int stride) { return stride == 1 ? 4 : 2; }

// log2 of the float4 channel groups a workgroup owns: up to 8 (32 channels), capped at 4 (16
// channels, twice as wide spatial tiles) for the stride-1 forwards and the 5x5 data gradients,
// where the narrower slices measured faster (-0.1 ms/step; the stride-2 and 3x3 stride-1 data
// gradients are faster at 8).  PHX_DW_MAXLCG overrides the cap for every launch.
static int dw_lcg(int C, int k, int s, bool bwd) {
  static int env_cap = [] {
    const char* e = std::getenv("PHX_DW_MAXLCG");
    return e ? std::min(3, std::max(0, atoi(e))) : -1;
  }();
  const int cap = env_cap >= 0 ? env_cap : ((!bwd && s == 1) || (bwd && k == 5)) ? 2 : 3;
  const int c4 = C / 4;
  const int l = (c4 % 8 == 0) ? 3 : (c4 % 4 == 0) ? 2 : (c4 % 2 == 0) ? 1 : 0;
  return std::min(l, cap);
}

// tile over an output space of (oh x ow) written by this launch
static DwGeom dw_plan(int H, int W, int C, int Ho, int Wo, int pt, int pl, int k, int s, int rpt,
                      bool bwd, int lcg = -1) {
  DwGeom g{};
  g.H = H; g.W = W; g.C = C; g.Ho = Ho; g.Wo = Wo; g.pt = pt; g.pl = pl;
  g.lcg = lcg >= 0 ? lcg : dw_lcg(C, k, s, bwd);
  const int px = 256 >> g.lcg;
  const int oh = bwd ? H : Ho, ow = bwd ? W : Wo;
  g.otw = ow < px ? ow : px;
  g.nrg = px / g.otw;
  const int need = (oh + rpt - 1) / rpt;  // row groups that cover the whole image
  if (g.nrg > need) g.nrg = need;
  g.oth = g.nrg * rpt;
  if (!bwd) {
    g.rin = (g.oth - 1) * s + k;
    g.cin = (g.otw - 1) * s + k;
  } else {
    g.rin = (g.oth - 1 + k - 1) / s + 2;
    g.cin = (g.otw - 1 + k - 1) / s + 2;
    if (s == 1) {
      g.rin = g.oth + k - 1;
      g.cin = g.otw + k - 1;
    }
  }
  g.tiles_x = cdiv(ow, g.otw);
  g.ntiles = g.tiles_x * cdiv(oh, g.oth);
  g.ncg = C / (4 << g.lcg);
  g.per = cdiv((long)g.ntiles * g.ncg, 8);
  return g;
}

static size_t dw_lds(const DwGeom& g, int k) {
  const bool lds_taps = PHX_DW_LDS_TAPS == 2 || (PHX_DW_LDS_TAPS == 1 && k > 3);
  return ((size_t)g.rin * g.cin + (lds_taps ? k * k : 0)) * (1 << g.lcg) * sizeof(float4);
}

static bool xv_bf(const InX& x) { return x.bf != 0; }
static bool xv_bf(const FuseView& f) { return f.x[0].bf != 0; }

template <int K, int S, int RPT, int NS, class XV, int SU, bool BF>
static void dw_fwd_launch(dim3 grid, size_t lds, const DwFwdGroup<NS, XV>& grp, bool stats, hipStream_t s) {
  if (stats) hipLaunchKernelGGL((k_dw_fwd<K, S, RPT, true, NS, XV, SU, BF>), grid, dim3(256), lds, s, grp);
  else hipLaunchKernelGGL((k_dw_fwd<K, S, RPT, false, NS, XV, SU, BF>), grid, dim3(256), lds, s, grp);
}

template <int K, int S, int RPT, int NS, class XV>
static void dw_fwd_go(const DwFwdGroup<NS, XV>& grp, int n, int B, bool stats, hipStream_t s) {
  const bool bf = xv_bf(grp.s[0].x);
  int gx = 1;
  size_t lds = 0;
  for (int i = 0; i < n; ++i) {
    gx = std::max(gx, 8 * grp.s[i].g.per);
    lds = std::max(lds, dw_lds(grp.s[i].g, K));
  }
  dim3 grid(gx, n, B);
  if constexpr (S == 2 || std::is_same<XV, InX>::value) {
    if (bf) dw_fwd_launch<K, S, RPT, NS, XV, 8, true>(grid, lds, grp, stats, s);
    else dw_fwd_launch<K, S, RPT, NS, XV, 8, false>(grid, lds, grp, stats, s);
  } else {
    if (bf) dw_fwd_launch<K, S, RPT, NS, XV, 4, true>(grid, lds, grp, stats, s);
    else dw_fwd_launch<K, S, RPT, NS, XV, 4, false>(grid, lds, grp, stats, s);
  }
}

template <int NS, class XV>
static void dw_fwd_dispatch(const DwFwdGroup<NS, XV>& grp, int n, int B, bool stats, int k, int stride,
                            hipStream_t s) {
  for (int i = 0; i < n; ++i)
    if (dw_lds(grp.s[i].g, k) > 160 * 1024) throw std::runtime_error("dw: LDS window too large");
  if (k == 3 && stride == 1) dw_fwd_go<3, 1, 4, NS, XV>(grp, n, B, stats, s);
  else if (k == 3 && stride == 2) dw_fwd_go<3, 2, 2, NS, XV>(grp, n, B, stats, s);
  else if (k == 5 && stride == 1) dw_fwd_go<5, 1, 4, NS, XV>(grp, n, B, stats, s);
  else if (k == 5 && stride == 2) dw_fwd_go<5, 2, 2, NS, XV>(grp, n, B, stats, s);
  else throw std::invalid_argument("dw: unsupported kernel/stride");
  PHX_LAUNCH_CHECK();
}

int dw_stat_partials(int B, int H, int W, int C, int Ho, int Wo, int k, int stride, int pt, int pl) {
  const int rpt = dw_rpt_fwd(stride);
  DwGeom g = dw_plan(H, W, C, Ho, Wo, pt, pl, k, stride, rpt, false);
  return B * g.ntiles;
}

int launch_dw_fwd(InX x, const float* w, float* y, int B, int H, int W, int C, int Ho, int Wo,
                  int k, int stride, int pt, int pl, hipStream_t s, StatSink sink) {
  if (C % 4) throw std::runtime_error("dw: C % 4 != 0");
  const int rpt = dw_rpt_fwd(stride);
  DwFwdGroup<1> grp{};
  grp.w = w;
  grp.s[0] = DwFwdSeg{x, y, dw_plan(H, W, C, Ho, Wo, pt, pl, k, stride, rpt, false), sink};
  grp.s[0].sink.P = B * grp.s[0].g.ntiles;
  dw_fwd_dispatch(grp, 1, B, sink.part != nullptr, k, stride, s);
  return B * grp.s[0].g.ntiles;
}

// BiFPN node: depthwise conv of the node's fuse, computed on load (3x3 stride 1 only)
void launch_dw_fwd_fused(const FuseView& fv, const float* w, float* y, int B, int H, int W, int C, int Ho,
                         int Wo, int k, int stride, int pt, int pl, hipStream_t s) {
  if (C % 4) throw std::runtime_error("dw: C % 4 != 0");
  if (k != 3 || stride != 1) throw std::invalid_argument("dw fused: 3x3 stride 1 only");
  DwFwdGroup<1, FuseView> grp{};
  grp.w = w;
  grp.s[0] = DwFwdSegT<FuseView>{fv, y, dw_plan(H, W, C, Ho, Wo, pt, pl, k, stride, 4, false), StatSink{}};
  // The small BiFPN levels (8x8 .. 32x32) give a few hundred workgroups or less, each walking its
  // staging batches and four output rows in turn: there one channel quad and one output row per lane
  // spread the same work over up to 16x the workgroups.  Each output keeps its tap order (rows, then
  // columns), and this launch has no statistics, so the outputs are bit-identical.
  static const long small_below = [] {
    const char* e = std::getenv("PHX_DW_FUSE_SMALL");  // workgroup count below which (0: off)
    return e ? std::atol(e) : 512L;
  }();
  const long wgs = (long)B * grp.s[0].g.ntiles * grp.s[0].g.ncg;
  if (wgs < small_below) {
    grp.s[0].g = dw_plan(H, W, C, Ho, Wo, pt, pl, k, stride, 1, false, 0);
    if (dw_lds(grp.s[0].g, k) > 160 * 1024) throw std::runtime_error("dw: LDS window too large");
    dw_fwd_go<3, 1, 1, 1, FuseView>(grp, 1, B, false, s);
    PHX_LAUNCH_CHECK();
    return;
  }
  if (dw_lds(grp.s[0].g, k) > 160 * 1024) throw std::runtime_error("dw: LDS window too large");
  dw_fwd_go<3, 1, 4, 1, FuseView>(grp, 1, B, false, s);
  PHX_LAUNCH_CHECK();
}

void launch_dw_fwd_group(const DwSeg* segs, int n, int B, int C, const float* w, int k, int stride,
                         hipStream_t s, int* nps) {
  if (C % 4) throw std::runtime_error("dw: C % 4 != 0");
  if (n < 1 || n > kMaxSeg) throw std::runtime_error("dw group: bad member count");
  const int rpt = dw_rpt_fwd(stride);
  DwFwdGroup<kMaxSeg> grp{};
  grp.w = w;
  const bool stats = segs[0].sink.part != nullptr;
  for (int i = 0; i < n; ++i) {
    const DwSeg& d = segs[i];
    if ((d.sink.part != nullptr) != stats) throw std::runtime_error("dw group: members differ in sinks");
    grp.s[i] = DwFwdSeg{d.x, d.out, dw_plan(d.H, d.W, C, d.Ho, d.Wo, d.pt, d.pl, k, stride, rpt, false), d.sink};
    grp.s[i].sink.P = B * grp.s[i].g.ntiles;
    nps[i] = grp.s[i].sink.P;
  }
  dw_fwd_dispatch(grp, n, B, stats, k, stride, s);
}

template <int K, int S, int NS>
static void dw_bwd_go(const DwBwdGroup<NS>& grp, int n, int B, bool gsums, hipStream_t s) {
  int gx = 1;
  size_t lds = 0;
  for (int i = 0; i < n; ++i) {
    gx = std::max(gx, 8 * grp.s[i].g.per);
    lds = std::max(lds, dw_lds(grp.s[i].g, K));
  }
  dim3 grid(gx, n, B);
  // the BN input y of every member shares the context's storage type
  const bool ybf = (grp.s[0].gv.y && grp.s[0].gv.ybf) || (gsums && grp.s[0].gs.ybf);
  if (ybf) {
    if (gsums)
      hipLaunchKernelGGL((k_dw_bwd<K, S, 4, true, NS, 4, true>), grid, dim3(256), lds, s, grp);
    else
      hipLaunchKernelGGL((k_dw_bwd<K, S, 4, false, NS, 4, true>), grid, dim3(256), lds, s, grp);
    return;
  }
  if (gsums)
    hipLaunchKernelGGL((k_dw_bwd<K, S, 4, true, NS>), grid, dim3(256), lds, s, grp);
  else
    hipLaunchKernelGGL((k_dw_bwd<K, S, 4, false, NS>), grid, dim3(256), lds, s, grp);
}

template <int NS>
static void dw_bwd_dispatch(const DwBwdGroup<NS>& grp, int n, int B, bool gsums, int k, int stride,
                            hipStream_t s) {
  for (int i = 0; i < n; ++i)
    if (dw_lds(grp.s[i].g, k) > 160 * 1024) throw std::runtime_error("dw: LDS window too large");
  if (k == 3 && stride == 1) dw_bwd_go<3, 1, NS>(grp, n, B, gsums, s);
  else if (k == 3 && stride == 2) dw_bwd_go<3, 2, NS>(grp, n, B, gsums, s);
  else if (k == 5 && stride == 1) dw_bwd_go<5, 1, NS>(grp, n, B, gsums, s);
  else if (k == 5 && stride == 2) dw_bwd_go<5, 2, NS>(grp, n, B, gsums, s);
  else throw std::invalid_argument("dw: unsupported kernel/stride");
  PHX_LAUNCH_CHECK();
}

int dw_bwd_partials(int B, int H, int W, int C, int Ho, int Wo, int k, int stride, int pt, int pl) {
  DwGeom g = dw_plan(H, W, C, Ho, Wo, pt, pl, k, stride, 4, true);
  return B * g.ntiles;
}

int launch_dw_bwd(GradX dy, const float* w, float* dx, int B, int H, int W, int C, int Ho,
                  int Wo, int k, int stride, int pt, int pl, bool acc, hipStream_t s, GradSink gs) {
  if (C % 4) throw std::runtime_error("dw: C % 4 != 0");
  DwBwdGroup<1> grp{};
  grp.w = w;
  grp.s[0] = DwBwdSeg{dy, dx, dw_plan(H, W, C, Ho, Wo, pt, pl, k, stride, 4, true), acc ? 1 : 0, gs};
  grp.s[0].gs.P = B * grp.s[0].g.ntiles;
  dw_bwd_dispatch(grp, 1, B, gs.part != nullptr, k, stride, s);
  return B * grp.s[0].g.ntiles;
}

void launch_dw_bwd_group(const DwSeg* segs, int n, int B, int C, const float* w, int k, int stride,
                         hipStream_t s, int* nps) {
  if (C % 4) throw std::runtime_error("dw: C % 4 != 0");
  if (n < 1 || n > kMaxSeg) throw std::runtime_error("dw group: bad member count");
  DwBwdGroup<kMaxSeg> grp{};
  grp.w = w;
  const bool gsums = segs[0].gs.part != nullptr;
  for (int i = 0; i < n; ++i) {
    const DwSeg& d = segs[i];
    if ((d.gs.part != nullptr) != gsums) throw std::runtime_error("dw group: members differ in sinks");
    grp.s[i] = DwBwdSeg{d.gv, d.out, dw_plan(d.H, d.W, C, d.Ho, d.Wo, d.pt, d.pl, k, stride, 4, true),
                        d.acc ? 1 : 0, d.gs};
    grp.s[i].gs.P = B * grp.s[i].g.ntiles;
    nps[i] = grp.s[i].gs.P;
  }
  dw_bwd_dispatch(grp, n, B, gsums, k, stride, s);
}

}  // namespace phx
