// kernels_norm.hip — batch norm (training-mode batch statistics), squeeze-excite, BiFPN fuse,
// pooling/resampling and elementwise kernels, forward and data-gradient.
//
// BN follows Keras BatchNormalization with training=True (utils.py:244-266 via
// util_keras.py:29-66, eps 1e-3, momentum 0.99): y_hat = (y - mu_B) * rsqrt(var_B + eps), biased
// batch variance over (N,H,W).  Reductions accumulate in fp64 so the statistics carry no
// cancellation error at M ~ 1e6 rows.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"

namespace phx {

// ------------------------------------------------------------------------------------------
// Column reduction over [nseg][seg_rows][C] (C % 4 == 0): every lane owns 4 consecutive channels
// (float4 loads, 256-B+ coalesced rows), accumulates 64-row runs in fp32 then folds them into
// fp64; workgroups reduce their rows in LDS and write fp64 partials [seg][chunk][C][2]; a second
// kernel sums the chunks per (seg, channel) with coalesced channel-major reads and hands the two
// sums to an epilogue functor.  BN statistics use a per-channel shift (the segment's first row) so
// E[y^2]-E[y]^2 carries no cancellation.
// ------------------------------------------------------------------------------------------
struct RedPlan {
  int tpr;       // threads per row (= C/4, capped at 256 per workgroup)
  int cgroups;   // channel groups (grid.y)
  int chunks;    // row chunks per segment (grid.x)
  long rpc;      // rows per chunk
};

// PHX_RED_BLOCKS: workgroups a column reduction aims for (default 1024); PHX_RED_DEPTH: rows a lane
// of a column reduction loads before consuming any (8 default, 4); the 2-D elementwise producers keep
// 4 (measured: 8 helps the BN-backward reductions by 14 %, is neutral for the SE pools and slows
// the SE backward apply)
static long red_target_blocks() {
  static long v = [] {
    const char* e = std::getenv("PHX_RED_BLOCKS");
    return e ? atol(e) : 1024L;
  }();
  return v;
}
static int red_depth() {
  static int v = [] {
    const char* e = std::getenv("PHX_RED_DEPTH");
    return (e && atoi(e) == 4) ? 4 : 8;
  }();
  return v;
}

// PHX_RED_MINROWS: minimum rows per lane of a chunk of a per-image reduction (nseg > 1: SE pools
// and SE backward; default 16: the deep layers get twice the workgroups, measured -0.17 ms/step
// against 32, while their SE MLPs fold more partials); PHX_RED_MINROWS1: the same for whole-tensor
// reductions (nseg == 1: BN statistics and BN-backward sums, default 8: -0.02 ms/step against 16)
static long red_min_rows(int nseg) {
  static long v = [] {
    const char* e = std::getenv("PHX_RED_MINROWS");
    return e ? std::max(1L, atol(e)) : 16L;
  }();
  static long v1 = [] {
    const char* e = std::getenv("PHX_RED_MINROWS1");
    return e ? std::max(1L, atol(e)) : 8L;
  }();
  return nseg > 1 ? v : v1;
}

static RedPlan red_plan(long seg_rows, int C, int nseg) {
  RedPlan p;
  int tpr_total = C / 4;
  p.cgroups = (tpr_total + 255) / 256;
  p.tpr = tpr_total < 256 ? tpr_total : 256;
  int rpi = 256 / p.tpr;
  long target_blocks = red_target_blocks();
  long per_seg = target_blocks / (nseg * p.cgroups);
  if (per_seg < 1) per_seg = 1;
  long rpc = (seg_rows + per_seg - 1) / per_seg;
  long minrows = (long)rpi * red_min_rows(nseg);
  if (rpc < minrows) rpc = minrows;
  rpc = (rpc + rpi - 1) / rpi * rpi;
  p.rpc = rpc;
  p.chunks = (int)((seg_rows + rpc - 1) / rpc);
  return p;
}

size_t colred_scratch_doubles(long seg_rows, int C, int nseg) {
  RedPlan p = red_plan(seg_rows, C, nseg);
  return (size_t)nseg * p.chunks * C * 2 + (size_t)nseg * C * 2;
}
size_t bn_stats_scratch_doubles(long M, int C) { return colred_scratch_doubles(M, C, 1); }

template <class F, int D>
__global__ __launch_bounds__(256) void k_colred_part(F f, long seg_rows, int C, long rpc,
                                                     double* __restrict__ part) {
  const int tpr_total = C >> 2;
  const int g0 = blockIdx.y * 256;
  const int tpr = min(tpr_total - g0, 256);
  const int rpi = 256 / tpr;
  const int t = threadIdx.x;
  const int rr = t / tpr, cc = t % tpr;
  const bool active = rr < rpi;
  const int c4 = g0 + cc;
  const int seg = blockIdx.z;
  const long m0 = (long)blockIdx.x * rpc;
  const long m1 = min(seg_rows, m0 + rpc);
  const long base = (long)seg * seg_rows;
  double d0[4] = {0, 0, 0, 0}, d1[4] = {0, 0, 0, 0};
  if (active) {
    f.init(seg, c4, base);
    long m = m0 + rr;
    while (m < m1) {
      float a0[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f};
      // 64-row fp32 runs; rows are loaded 4 at a time before any is consumed so every lane keeps
      // four 16-B loads (eight for two-operand functors) in flight
      int it = 0;
      for (; it + D <= 64 && m + (D - 1) * rpi < m1; it += D, m += D * rpi) {
        typename F::Raw v[D];
#pragma unroll
        for (int u = 0; u < D; ++u) v[u] = f.load(base + m + u * rpi, c4);
#pragma unroll
        for (int u = 0; u < D; ++u) f.add(v[u], a0, a1);
      }
      for (; it < 64 && m < m1; ++it, m += rpi) f.add(f.load(base + m, c4), a0, a1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        d0[j] += a0[j];
        d1[j] += a1[j];
      }
    }
  }
  // [value][lane]: a wave's 64 lanes store / load 64 consecutive doubles per value (lane-major
  // [lane][value] put lanes 4 apart on one bank: 313 k conflict cycles per launch, round 3)
  __shared__ double sh[8][256];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sh[j][t] = d0[j];
    sh[4 + j][t] = d1[j];
  }
  __syncthreads();
  if (rr == 0) {
    for (int r = 1; r < rpi; ++r) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        d0[j] += sh[j][r * tpr + cc];
        d1[j] += sh[4 + j][r * tpr + cc];
      }
    }
    double* out = part + (((long)seg * gridDim.x + blockIdx.x) * C + c4 * 4) * 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      out[j * 2 + 0] = d0[j];
      out[j * 2 + 1] = d1[j];
    }
  }
}

// sums over chunks: grid (ceil(C/16), nseg), 256 lanes = 16 channels x 16 chunk lanes
template <class E>
__global__ __launch_bounds__(256) void k_colred_final(E e, const double* __restrict__ part,
                                                      int chunks, int C) {
  const int seg = blockIdx.y;
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double s0 = 0.0, s1 = 0.0;
  if (c < C) {
    int k = g;
    // four chunks' loads in flight, added in chunk order
    for (; k + 48 < chunks; k += 64) {
      double2 p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        p[u] = *reinterpret_cast<const double2*>(part + (((long)seg * chunks + k + 16 * u) * C + c) * 2);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s0 += p[u].x;
        s1 += p[u].y;
      }
    }
    for (; k < chunks; k += 16) {
      const double2 p = *reinterpret_cast<const double2*>(part + (((long)seg * chunks + k) * C + c) * 2);
      s0 += p.x;
      s1 += p.y;
    }
  }
  __shared__ double sh[2][256];
  sh[0][threadIdx.x] = s0;
  sh[1][threadIdx.x] = s1;
  __syncthreads();
  if (g == 0 && c < C) {
    for (int k = 1; k < 16; ++k) {
      s0 += sh[0][k * 16 + cl];
      s1 += sh[1][k * 16 + cl];
    }
    e(seg, c, s0, s1);
  }
}

// first half only: chunk partials [nseg][chunks][C][2] in scratch; returns chunks
template <class F>
static int colred_parts(F f, long seg_rows, int C, int nseg, double* scratch, hipStream_t s) {
  if (C % 4) throw std::runtime_error("colred: C % 4 != 0");
  RedPlan p = red_plan(seg_rows, C, nseg);
  if (red_depth() == 8)
    hipLaunchKernelGGL((k_colred_part<F, 8>), dim3(p.chunks, p.cgroups, nseg), dim3(256), 0, s, f, seg_rows,
                       C, p.rpc, scratch);
  else
    hipLaunchKernelGGL((k_colred_part<F, 4>), dim3(p.chunks, p.cgroups, nseg), dim3(256), 0, s, f, seg_rows,
                       C, p.rpc, scratch);
  PHX_LAUNCH_CHECK();
  return p.chunks;
}

template <class F, class E>
static void colred(F f, E e, long seg_rows, int C, int nseg, double* scratch, hipStream_t s) {
  const int chunks = colred_parts(f, seg_rows, C, nseg, scratch, s);
  hipLaunchKernelGGL((k_colred_final<E>), dim3(cdiv(C, 16), nseg), dim3(256), 0, s, e, scratch,
                     chunks, C);
  PHX_LAUNCH_CHECK();
}

// ---- 2-D elementwise producers of a BN-output gradient, with the GradSink reduction ---------
// Same [nseg][seg_rows][C] lane layout as the column reduction: a lane owns 4 channels of every
// rpi-th row of its chunk, computes and stores the float4 result (functor F::out), and folds it
// into the BN-backward sums of its channels; the rpi lanes of a channel quad meet in LDS and the
// block writes partial (seg * chunks + chunk) of the GradSink.
// YBF: the GradSink's BN input y in bf16 storage
template <class F, int D, bool YBF>
__global__ __launch_bounds__(256) void k_ew_gstats(F f, long seg_rows, int C, long rpc,
                                                   GradSink g) {
  const int tpr_total = C >> 2;
  const int g0 = blockIdx.y * 256;
  const int tpr = min(tpr_total - g0, 256);
  const int rpi = 256 / tpr;
  const int t = threadIdx.x;
  const int rr = t / tpr, cc = t % tpr;
  const bool active = rr < rpi;
  const int c4 = g0 + cc;
  const int seg = blockIdx.z;
  const long m0 = (long)blockIdx.x * rpc;
  const long m1 = min(seg_rows, m0 + rpc);
  const long base = (long)seg * seg_rows;
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  if (active) {
    f.init(seg, c4);
    GSChan4 k;
    if (g.part) k = gs_chan4(g, c4 * 4);
    long m = m0 + rr;
    for (; m + (D - 1) * rpi < m1; m += D * rpi) {
      typename F::Raw v[D];
      float4 yv[D];
#pragma unroll
      for (int u = 0; u < D; ++u) {
        v[u] = f.load(base + m + u * rpi, c4);
        if (g.part) yv[u] = ald4<YBF>(g.y, (base + m + u * rpi) * C + c4 * 4);
      }
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const float4 o = f.out(v[u], base + m + u * rpi, c4);
        if (g.part) gs_acc4(g, k, o, yv[u], s1, s2);
      }
    }
    for (; m < m1; m += rpi) {
      const float4 o = f.out(f.load(base + m, c4), base + m, c4);
      if (g.part) gs_acc4(g, k, o, ald4<YBF>(g.y, (base + m) * C + c4 * 4), s1, s2);
    }
  }
  if (!g.part) return;
  __shared__ float4 sh1[256], sh2[256];
  sh1[t] = s1;
  sh2[t] = s2;
  __syncthreads();
  if (rr == 0) {
    for (int r = 1; r < rpi; ++r) {
      const float4 a = sh1[r * tpr + cc], b = sh2[r * tpr + cc];
      s1.x += a.x; s1.y += a.y; s1.z += a.z; s1.w += a.w;
      s2.x += b.x; s2.y += b.y; s2.z += b.z; s2.w += b.w;
    }
    const long p = (long)seg * gridDim.x + blockIdx.x;
    gsink_put(g, p, c4 * 4 + 0, s1.x, s2.x);
    gsink_put(g, p, c4 * 4 + 1, s1.y, s2.y);
    gsink_put(g, p, c4 * 4 + 2, s1.z, s2.z);
    gsink_put(g, p, c4 * 4 + 3, s1.w, s2.w);
  }
}

// rows per lane whose loads are in flight together (fp32 / bf16 BN input of the GradSink)
#ifndef PHX_EW_D
#define PHX_EW_D 4
#endif
#ifndef PHX_EW_DBF
#define PHX_EW_DBF 4
#endif
template <class F>
static int ew_gstats(F f, long seg_rows, int C, int nseg, GradSink g, hipStream_t s) {
  if (C % 4) throw std::runtime_error("ew_gstats: C % 4 != 0");
  RedPlan p = red_plan(seg_rows, C, nseg);
  g.P = nseg * p.chunks;
  if (g.part && g.ybf)
    hipLaunchKernelGGL((k_ew_gstats<F, PHX_EW_DBF, true>), dim3(p.chunks, p.cgroups, nseg), dim3(256), 0, s, f, seg_rows,
                       C, p.rpc, g);
  else
    hipLaunchKernelGGL((k_ew_gstats<F, PHX_EW_D, false>), dim3(p.chunks, p.cgroups, nseg), dim3(256), 0, s, f, seg_rows,
                       C, p.rpc, g);
  PHX_LAUNCH_CHECK();
  return g.P;
}

int ew_gstats_partials(long seg_rows, int C, int nseg) { return nseg * red_plan(seg_rows, C, nseg).chunks; }

// ---- BN forward statistics ------------------------------------------------------------------
template <bool BF>
struct StatsAcc {
  const float* y;
  int C;
  float ref[4];
  __device__ void init(int, int c4, long base) {
    float4 r = ald4<BF>(y, base * C + c4 * 4);
    ref[0] = r.x; ref[1] = r.y; ref[2] = r.z; ref[3] = r.w;
  }
  using Raw = float4;
  __device__ Raw load(long m, int c4) const { return ald4<BF>(y, m * C + c4 * 4); }
  __device__ void add(const Raw& v, float* a0, float* a1) const {
    float d[4] = {v.x - ref[0], v.y - ref[1], v.z - ref[2], v.w - ref[3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a0[j] += d[j];
      a1[j] += d[j] * d[j];
    }
  }
};

__global__ __launch_bounds__(256) void k_bn_moving_apply(const MovEntry* __restrict__ tab, float* __restrict__ W,
                                                         const double* __restrict__ s0,
                                                         const double* __restrict__ s1) {
  const MovEntry e = tab[blockIdx.x];
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= e.C) return;
  const long o = 2L * (e.off + c);
  // s1 == nullptr: one deferred pass (a prefetched first pass, phx_set_next)
  const float mm = moving_update(W[e.mm + c], s0[o]), mv = moving_update(W[e.mv + c], s0[o + 1]);
  W[e.mm + c] = s1 ? moving_update(mm, s1[o]) : mm;
  W[e.mv + c] = s1 ? moving_update(mv, s1[o + 1]) : mv;
}

void launch_bn_moving_apply(const MovEntry* tab, int n, int cmax, float* W, const double* side0,
                            const double* side1, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_bn_moving_apply, dim3(n, cdiv(cmax, 256)), dim3(256), 0, s, tab, W, side0, side1);
  PHX_LAUNCH_CHECK();
}

void launch_bn_stats(const float* y, long M, int C, double* part, float* mean, float* rstd,
                     const float* gamma, float* sc, float* mmean, float* mvar, float eps,
                     hipStream_t s, bool ybf, double* side) {
  StatsEpi e{y, M, mean, rstd, gamma, sc, mmean, mvar, eps, ybf ? 1 : 0, side};
  if (ybf) colred(StatsAcc<true>{y, C, {0, 0, 0, 0}}, e, M, C, 1, part, s);
  else colred(StatsAcc<false>{y, C, {0, 0, 0, 0}}, e, M, C, 1, part, s);
}

// ---- BN statistics from producer partials (StatSink / GradSink) ---------------------------
// One workgroup per channel: its P partials are contiguous (channel-major), each lane folds a
// strided subset into fp64, the 256 lane pairs meet in an LDS tree and the epilogue finishes the
// channel.  Forward (StatSink): partial = (sum, M2) of cnt[p] rows, folded as S1 = sum x and
// S2 = sum x^2 = M2 + sum^2/n.  Backward (GradSink): partial = (sum dz, sum dz*xhat), plain sums.
// Fixed summation order: bit-reproducible run to run.
// grouped: blockIdx.y = member (the per-level BNs of a head conv), each with its own partials
template <class E>
struct FinSeg {
  const float2* part;
  const float* cnt;
  int P;
  E e;
};
template <class E, int NS>  // NS argument slots: 1 (ordinary launch) or kMaxSeg
struct FinGroup {
  FinSeg<E> s[NS];
};

template <bool BWD, class E, int NS>
__global__ __launch_bounds__(256) void k_bn_finalize(FinGroup<E, NS> grp) {
  const FinSeg<E> sg = pick_seg(grp.s, NS == 1 ? 0 : (int)blockIdx.y);
  const float2* __restrict__ part = sg.part;
  const float* __restrict__ cnt = sg.cnt;
  const int P = sg.P;
  const E& e = sg.e;
  __shared__ double r1[256], r2[256];
  const int c = blockIdx.x, t = threadIdx.x;
  const float2* pc = part + (long)c * P;
  typename E::Pre pr{};
  if (t == 0) pr = e.pre(c);
  double s1 = 0.0, s2 = 0.0;
  auto fold = [&](float2 v, float n) {
    if (BWD) {
      s1 += (double)v.x;
      s2 += (double)v.y;
    } else if (n > 0.f) {
      s1 += (double)v.x;
      s2 += (double)v.y + (double)v.x * (double)v.x / (double)n;
    }
  };
  int p = t;
  for (; p + 768 < P; p += 1024) {
    float2 v[4];
    float n[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u] = pc[p + 256 * u];
      n[u] = BWD ? 1.f : cnt[p + 256 * u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) fold(v[u], n[u]);
  }
  // the remaining (at most three) partials of this lane: loads in flight together, folded in order
  if (P > 0) {
    float2 v[3];
    float n[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int pu = min(p + 256 * u, P - 1);
      v[u] = pc[pu];
      n[u] = BWD ? 1.f : cnt[pu];
    }
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (p + 256 * u < P) fold(v[u], n[u]);
  }
  r1[t] = s1;
  r2[t] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      r1[t] += r1[t + o];
      r2[t] += r2[t + o];
    }
    __syncthreads();
  }
  if (t == 0) e.fin(pr, c, r1[0], r2[0]);
}

// (a one-wave-per-channel form for P <= 64 — lanes strided over the partials, an xor-shuffle tree
// instead of the LDS tree — measured 0.04 ms/step slower on C2: the launch is latency-bound)
template <bool BWD, class E, int NS>
static void fin_launch(const FinGroup<E, NS>& g, int n, int C, int, hipStream_t s) {
  hipLaunchKernelGGL((k_bn_finalize<BWD, E, NS>), dim3(C, n), dim3(256), 0, s, g);
  PHX_LAUNCH_CHECK();
}
void launch_bn_finalize(const float2* part, const float* cnt, int P, long M, int C, float* mean,
                        float* rstd, const float* gamma, float* sc, float* mmean, float* mvar,
                        float eps, hipStream_t s, double* side) {
  // StatsEpi's shift is 0 here: S1, S2 are plain sums of x and x^2 in fp64
  FinGroup<StatsEpi, 1> g{};
  g.s[0] = FinSeg<StatsEpi>{part, cnt, P, StatsEpi{nullptr, M, mean, rstd, gamma, sc, mmean, mvar, eps, 0, side, C}};
  fin_launch<false>(g, 1, C, P, s);
}

void launch_bn_finalize_group(const BnFinSeg* segs, int n, int C, float eps, hipStream_t s) {
  if (n < 1 || n > kMaxSeg) throw std::runtime_error("bn finalize group: bad member count");
  FinGroup<StatsEpi, kMaxSeg> g{};
  int Pmax = 0;
  for (int i = 0; i < n; ++i) {
    const BnFinSeg& d = segs[i];
    g.s[i] = FinSeg<StatsEpi>{d.part, d.cnt, d.P,
                              StatsEpi{nullptr, d.M, d.mean, d.rstd, d.gamma, d.sc, d.mmean, d.mvar, eps, 0, d.side, C}};
    Pmax = std::max(Pmax, d.P);
  }
  fin_launch<false>(g, n, C, Pmax, s);
}

__global__ void k_bn_frozen_stats(const float* __restrict__ mm, const float* __restrict__ mv,
                                  float* __restrict__ mean, float* __restrict__ rstd,
                                  const float* __restrict__ gamma, float* __restrict__ sc, int C,
                                  float eps) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = mm[c];
  const double rs = 1.0 / sqrt((double)mv[c] + (double)eps);
  rstd[c] = (float)rs;
  sc[c] = (float)(rs * (double)gamma[c]);
}

void launch_bn_frozen_stats(const float* mmean, const float* mvar, float* mean, float* rstd,
                            const float* gamma, float* sc, int C, float eps, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_frozen_stats, dim3(cdiv(C, 256)), dim3(256), 0, s, mmean, mvar, mean,
                     rstd, gamma, sc, C, eps);
  PHX_LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void k_bn_apply(const float* __restrict__ y,
                                                  const float* __restrict__ mean,
                                                  const float* __restrict__ rstd,
                                                  const float* __restrict__ gamma,
                                                  const float* __restrict__ beta,
                                                  float* __restrict__ a, long n4, int C, int act) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  int c = (int)((i * 4) % C);
  float4 v = reinterpret_cast<const float4*>(y)[i];
  float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float z = (r[j] - mean[c + j]) * rstd[c + j] * gamma[c + j] + beta[c + j];
    r[j] = act_fwd(z, act);
  }
  reinterpret_cast<float4*>(a)[i] = make_float4(r[0], r[1], r[2], r[3]);
}

void launch_bn_apply(const float* y, const float* mean, const float* rstd, const float* gamma,
                     const float* beta, float* a, long M, int C, int act, hipStream_t s) {
  if (C % 4) throw std::runtime_error("bn_apply: C % 4");
  long n4 = M * C / 4;
  hipLaunchKernelGGL(k_bn_apply, dim3(cdiv(n4, 256)), dim3(256), 0, s, y, mean, rstd, gamma, beta,
                     a, n4, C, act);
  PHX_LAUNCH_CHECK();
}

// ---- BN backward ----------------------------------------------------------------------------
template <bool BF>
struct BwdAcc {
  const float* da;
  const float* y;
  const float* mean;
  const float* rstd;
  const float* gamma;
  const float* beta;
  int C, act;
  float mu[4], rs[4], ga[4], be[4];
  __device__ void init(int, int c4, long) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mu[j] = mean[c4 * 4 + j];
      rs[j] = rstd[c4 * 4 + j];
      ga[j] = gamma[c4 * 4 + j];
      be[j] = beta[c4 * 4 + j];
    }
  }
  struct Raw {
    float4 y, g;
  };
  __device__ Raw load(long m, int c4) const {
    return Raw{ald4<BF>(y, m * C + c4 * 4), *reinterpret_cast<const float4*>(da + m * C + c4 * 4)};
  }
  __device__ void add(const Raw& r, float* a0, float* a1) const {
    float ys[4] = {r.y.x, r.y.y, r.y.z, r.y.w};
    float gs[4] = {r.g.x, r.g.y, r.g.z, r.g.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float xh = (ys[j] - mu[j]) * rs[j];
      float dz = gs[j];
      if (act) dz *= act_grad(xh * ga[j] + be[j], act);
      a0[j] += dz;
      a1[j] += dz * xh;
    }
  }
};

// coef[c] = {gamma*rstd, mean(dz), mean(dz*xhat)}
struct BwdEpi {
  long M;
  const float* rstd;
  const float* gamma;
  float* coef;
  __device__ void operator()(int, int c, double s0, double s1) const {
    coef[c * 3 + 0] = gamma[c] * rstd[c];
    coef[c * 3 + 1] = (float)(s0 / (double)M);
    coef[c * 3 + 2] = (float)(s1 / (double)M);
  }
};

__global__ __launch_bounds__(256) void k_bn_bwd_apply(const float* __restrict__ da,
                                                      const float* __restrict__ y,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ rstd,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta,
                                                      const float* __restrict__ coef,
                                                      float* __restrict__ dy, long n4, int C,
                                                      int act, int frozen, int acc_flag) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  int c = (int)((i * 4) % C);
  float4 yv = reinterpret_cast<const float4*>(y)[i];
  float4 gv = reinterpret_cast<const float4*>(da)[i];
  float ys[4] = {yv.x, yv.y, yv.z, yv.w};
  float gs[4] = {gv.x, gv.y, gv.z, gv.w};
  float o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cc = c + j;
    float xh = (ys[j] - mean[cc]) * rstd[cc];
    float dz = gs[j];
    if (act) dz *= act_grad(xh * gamma[cc] + beta[cc], act);
    if (frozen)
      o[j] = gamma[cc] * rstd[cc] * dz;
    else
      o[j] = coef[cc * 3] * (dz - coef[cc * 3 + 1] - xh * coef[cc * 3 + 2]);
  }
  float4* op = reinterpret_cast<float4*>(dy) + i;
  if (acc_flag) {
    float4 p = *op;
    o[0] += p.x; o[1] += p.y; o[2] += p.z; o[3] += p.w;
  }
  *op = make_float4(o[0], o[1], o[2], o[3]);
}

void launch_bn_bwd_finalize(const float2* part, int P, long M, int C, float* mdz, float* mdzx,
                            hipStream_t s) {
  FinGroup<BwdEpi2, 1> g{};
  g.s[0] = FinSeg<BwdEpi2>{part, nullptr, P, BwdEpi2{M, mdz, mdzx, C}};
  fin_launch<true>(g, 1, C, P, s);
}

void launch_bn_bwd_finalize_group(const BnFinSeg* segs, int n, int C, hipStream_t s) {
  if (n < 1 || n > kMaxSeg) throw std::runtime_error("bn finalize group: bad member count");
  FinGroup<BwdEpi2, kMaxSeg> g{};
  int Pmax = 0;
  for (int i = 0; i < n; ++i) {
    g.s[i] = FinSeg<BwdEpi2>{segs[i].part, nullptr, segs[i].P, BwdEpi2{segs[i].M, segs[i].mdz, segs[i].mdzx, C}};
    Pmax = std::max(Pmax, segs[i].P);
  }
  fin_launch<true>(g, n, C, Pmax, s);
}

// bn=sync: the finalize's fold with an epilogue that keeps the fp64 sums (and the rows they cover)
struct SumsEpi {
  double* out;  // [C][3]
  double rows;
  const float* y = nullptr;  // StatsAcc's shift row (its sums are of x - y[c]): unshifted here
  int ybf = 0;
  struct Pre {};
  __device__ Pre pre(int) const { return Pre{}; }
  __device__ void fin(const Pre&, int c, double s0, double s1) const { (*this)(0, c, s0, s1); }
  __device__ void operator()(int, int c, double s0, double s1) const {
    if (y) {
      const double r = ybf ? (double)ald1<true>(y, c) : (double)y[c];
      s1 += 2.0 * r * s0 + rows * r * r;
      s0 += rows * r;
    }
    out[(long)c * 3 + 0] = rows;
    out[(long)c * 3 + 1] = s0;
    out[(long)c * 3 + 2] = s1;
  }
};

// bn=sync halves of the unfused reductions: the sums of one BN (forward sum x, sum x^2 over its
// input y; backward sum dz, sum dz*xhat) into sums[C][3], for the caller's all-reduce
void launch_bn_stats_sums(const float* y, long M, int C, double* part, double* sums, hipStream_t s, bool ybf) {
  const SumsEpi e{sums, (double)M, y, ybf ? 1 : 0};
  if (ybf) colred(StatsAcc<true>{y, C, {0, 0, 0, 0}}, e, M, C, 1, part, s);
  else colred(StatsAcc<false>{y, C, {0, 0, 0, 0}}, e, M, C, 1, part, s);
}

void launch_bn_fold_sums(const BnFinSeg* segs, int n, int C, bool bwd, double* sums, hipStream_t s) {
  if (n < 1 || n > kMaxSeg) throw std::runtime_error("bn fold: bad member count");
  FinGroup<SumsEpi, kMaxSeg> g{};
  for (int i = 0; i < n; ++i)
    g.s[i] = FinSeg<SumsEpi>{segs[i].part, segs[i].cnt, segs[i].P, SumsEpi{sums + (size_t)i * C * 3, (double)segs[i].M}};
  if (bwd) hipLaunchKernelGGL((k_bn_finalize<true, SumsEpi, kMaxSeg>), dim3(C, n), dim3(256), 0, s, g);
  else hipLaunchKernelGGL((k_bn_finalize<false, SumsEpi, kMaxSeg>), dim3(C, n), dim3(256), 0, s, g);
  PHX_LAUNCH_CHECK();
}

// one lane per (channel, member): StatsEpi / BwdEpi2 over the all-reduced sums (global row count)
template <bool BWD>
__global__ __launch_bounds__(256) void k_bn_from_sums(FinGroup<StatsEpi, kMaxSeg> fg, FinGroup<BwdEpi2, kMaxSeg> bg,
                                                      const double* __restrict__ sums, int C) {
  const int c = blockIdx.x * 256 + threadIdx.x, i = blockIdx.y;
  if (c >= C) return;
  const double* q = sums + ((size_t)i * C + c) * 3;
  const double rows = q[0];
  if constexpr (BWD) {
    BwdEpi2 e = pick_seg(bg.s, i).e;
    e.M = (long)rows;
    e(0, c, q[1], q[2]);
  } else {
    StatsEpi e = pick_seg(fg.s, i).e;
    e.M = (long)rows;
    e(0, c, q[1], q[2]);
  }
}

void launch_bn_from_sums(const BnFinSeg* segs, int n, int C, bool bwd, const double* sums, float eps,
                         hipStream_t s) {
  if (n < 1 || n > kMaxSeg) throw std::runtime_error("bn from sums: bad member count");
  FinGroup<StatsEpi, kMaxSeg> fg{};
  FinGroup<BwdEpi2, kMaxSeg> bg{};
  for (int i = 0; i < n; ++i) {
    const BnFinSeg& d = segs[i];
    if (bwd) bg.s[i].e = BwdEpi2{0, d.mdz, d.mdzx};
    else fg.s[i].e = StatsEpi{nullptr, 0, d.mean, d.rstd, d.gamma, d.sc, d.mmean, d.mvar, eps, 0, d.side};
  }
  if (bwd) hipLaunchKernelGGL(k_bn_from_sums<true>, dim3(cdiv(C, 256), n), dim3(256), 0, s, fg, bg, sums, C);
  else hipLaunchKernelGGL(k_bn_from_sums<false>, dim3(cdiv(C, 256), n), dim3(256), 0, s, fg, bg, sums, C);
  PHX_LAUNCH_CHECK();
}

template <bool BF>
__global__ __launch_bounds__(256) void k_gx_materialize(GradX g, float4* __restrict__ out, long n4,
                                                        int C) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  out[i] = gx_load4<BF>(g, i * 4, (int)((i * 4) % C));
}

void launch_bn_bwd_apply2(GradX g, float* out, long M, int C, hipStream_t s) {
  long n4 = M * C / 4;
  if (g.y && g.ybf)
    hipLaunchKernelGGL(k_gx_materialize<true>, dim3(cdiv(n4, 256)), dim3(256), 0, s, g, (float4*)out, n4, C);
  else
    hipLaunchKernelGGL(k_gx_materialize<false>, dim3(cdiv(n4, 256)), dim3(256), 0, s, g, (float4*)out, n4, C);
  PHX_LAUNCH_CHECK();
}

void launch_bn_bwd_reduce(const float* da, const float* y, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, long M, int C, int act,
                          double* part, float* mdz, float* mdzx, hipStream_t s, bool ybf) {
  if (ybf) colred(BwdAcc<true>{da, y, mean, rstd, gamma, beta, C, act, {}, {}, {}, {}}, BwdEpi2{M, mdz, mdzx}, M, C, 1, part, s);
  else colred(BwdAcc<false>{da, y, mean, rstd, gamma, beta, C, act, {}, {}, {}, {}}, BwdEpi2{M, mdz, mdzx}, M, C, 1, part, s);
}

void launch_bn_bwd_reduce_sums(const float* da, const float* y, const float* mean, const float* rstd,
                               const float* gamma, const float* beta, long M, int C, int act, double* part,
                               double* sums, hipStream_t s, bool ybf) {
  const SumsEpi e{sums, (double)M};
  if (ybf) colred(BwdAcc<true>{da, y, mean, rstd, gamma, beta, C, act, {}, {}, {}, {}}, e, M, C, 1, part, s);
  else colred(BwdAcc<false>{da, y, mean, rstd, gamma, beta, C, act, {}, {}, {}, {}}, e, M, C, 1, part, s);
}

void launch_bn_bwd(const float* da, const float* y, const float* mean, const float* rstd,
                   const float* gamma, const float* beta, float* dy, long M, int C, int act,
                   bool frozen, bool acc, double* part, float* coef, hipStream_t s) {
  if (C % 4) throw std::runtime_error("bn_bwd: C % 4");
  if (!frozen) {
    BwdAcc<false> f{da, y, mean, rstd, gamma, beta, C, act, {}, {}, {}, {}};
    BwdEpi e{M, rstd, gamma, coef};
    colred(f, e, M, C, 1, part, s);
  }
  long n4 = M * C / 4;
  hipLaunchKernelGGL(k_bn_bwd_apply, dim3(cdiv(n4, 256)), dim3(256), 0, s, da, y, mean, rstd, gamma,
                     beta, coef, dy, n4, C, act, frozen ? 1 : 0, acc ? 1 : 0);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// squeeze-excite (efficientnet_model.py:184-196)
// ------------------------------------------------------------------------------------------
// per-image channel sums: pool (sum x) and backward (sum dy*x) through the column reduction
template <bool BF>
struct SumAcc {
  InX x;
  const float* g;  // optional second factor
  int C;
  Chan4 ck;
  __device__ void init(int, int c4, long) {
    if (x.mu) ck = inx_chan4(x, c4 * 4);
  }
  struct Raw {
    float4 v, w;
  };
  __device__ Raw load(long m, int c4) const {
    Raw r;
    r.v = ald4<BF>(x.p, m * C + c4 * 4);
    if (g) r.w = *reinterpret_cast<const float4*>(g + m * C + c4 * 4);
    return r;
  }
  __device__ void add(const Raw& r, float* a0, float* a1) const {
    float4 v = r.v;
    if (x.mu) v = inx_apply4(x, ck, v);
    if (g) {
      v.x *= r.w.x; v.y *= r.w.y; v.z *= r.w.z; v.w *= r.w.w;
    }
    a0[0] += v.x; a0[1] += v.y; a0[2] += v.z; a0[3] += v.w;
    (void)a1;
  }
};

// The SE MLP ([B,C] -> [B,Cse] -> [B,C], efficientnet_model.py:184-196) runs in two launches after
// the per-image channel sums' chunk partials, both over (image, channel slice) workgroups:
//   k_se_squeeze  workgroup (b, s) folds the chunk partials of its channel slice in fp64 (fixed
//                 order), writes the slice's pool means and its share of the squeeze product,
//                 hp[b][s][j] = sum_{c in slice} v[c] * w[c][j] (lanes (j, channel group), rows of
//                 the [C][Cse] matrix read along j);
//   k_se_excite   workgroup (b, s) adds the shares in slice order (+ bias, activation) and writes
//                 the excitation of its channel slice (lanes (channel, j group), meeting in LDS).
// Backward runs the same pair on (sum dy*x) * s(1-s) with the transposed weights.  (One workgroup
// per image — the previous form — left D4's 4-image batch on 4 CUs, each folding and multiplying
// 2688 x 112 weights: latency-bound at ~34 us per SE.)
constexpr int kSeT = 256;

struct SePlan {
  int s1, cs1, s2, cs2;
};
static SePlan se_plan(int B, int C, int N) {
  SePlan p;
  const int want = std::max(1, 256 / B);
  // squeeze shares live in the tail of the colred scratch (B*C*2 doubles = B*C*4 floats)
  p.s1 = std::max(1, std::min(std::min(want, cdiv(C, 32)), 4 * C / std::max(N, 1)));
  p.cs1 = cdiv(C, p.s1);
  p.s1 = cdiv(C, p.cs1);
  p.s2 = std::max(1, std::min(2 * want, cdiv(C, 32)));
  p.cs2 = cdiv(C, p.s2);
  p.s2 = cdiv(C, p.cs2);
  return p;
}

// BWD = 0: v = mean over HW; BWD = 1: v = (sum dy*x) * s * (1 - s)
template <int BWD>
__global__ __launch_bounds__(kSeT) void k_se_squeeze(const double* __restrict__ part, int chunks, int C, int N,
                                                     int cs, const float* __restrict__ w, float inv,
                                                     const float* __restrict__ scale, float* __restrict__ pool,
                                                     float* __restrict__ hp) {
  extern __shared__ float sq_v[];  // [cs]
  __shared__ double redd[kSeT];
  __shared__ float redf[kSeT];
  const int b = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
  const int c0 = s * cs, n = min(cs, C - c0);
  const double* pb = part + (long)b * chunks * C * 2;
  // fold: lanes (channel, chunk group), every partial load of a lane issued before any is added
  if (n <= kSeT / 2) {
    const int kg = min(chunks, kSeT / n);
    const int c = t % n, g = t / n;
    if (g < kg) {
      double acc = 0.0;
      int k = g;
      for (; k + 7 * kg < chunks; k += 8 * kg) {
        double p8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) p8[u] = pb[((long)(k + u * kg) * C + c0 + c) * 2];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += p8[u];
      }
      for (; k < chunks; k += kg) acc += pb[((long)k * C + c0 + c) * 2];
      redd[g * n + c] = acc;
    }
    __syncthreads();
    if (t < n) {
      double acc = 0.0;
      for (int g2 = 0; g2 < kg; ++g2) acc += redd[g2 * n + t];
      sq_v[t] = (float)acc;
    }
  } else {
    for (int c = t; c < n; c += kSeT) {
      double acc = 0.0;
      int k = 0;
      for (; k + 3 < chunks; k += 4) {
        double p4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) p4[u] = pb[((long)(k + u) * C + c0 + c) * 2];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += p4[u];
      }
      for (; k < chunks; ++k) acc += pb[((long)k * C + c0 + c) * 2];
      sq_v[c] = (float)acc;
    }
  }
  __syncthreads();
  for (int c = t; c < n; c += kSeT) {
    float x = sq_v[c];
    if (BWD) {
      const float sg = scale[(long)b * C + c0 + c];
      x = x * sg * (1.f - sg);
    } else {
      x = x * inv;  // mean over HW
      pool[(long)b * C + c0 + c] = x;
    }
    sq_v[c] = x;
  }
  __syncthreads();
  // the slice's share of the squeeze product
  const int ng = kSeT / N;
  const int j = t % N, g = t / N;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (g < ng) {
    int c = g;
    for (; c + 7 * ng < n; c += 8 * ng) {
      float wv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) wv[u] = w[(long)(c0 + c + u * ng) * N + j];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = fmaf(sq_v[c + u * ng], wv[u], a[u]);
    }
    for (; c < n; c += ng) a[0] = fmaf(sq_v[c], w[(long)(c0 + c) * N + j], a[0]);
  }
  redf[t] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (t < N) {
    float h = 0.f;
    for (int g2 = 0; g2 < ng; ++g2) h += redf[g2 * N + t];
    hp[((long)b * gridDim.y + s) * N + t] = h;
  }
}

// BWD = 0: hidden = b1 + sum of shares (stored pre-activation), scale[c] = sigmoid(b2[c] +
//          sum_j act(hidden[j]) * w2[j][c]);
// BWD = 1: dh = (sum of shares) * act'(hidden), dpool[c] = sum_j dh[j] * w1[c][j]
template <int BWD>
__global__ __launch_bounds__(kSeT) void k_se_excite(const float* __restrict__ hp, int s1, int C, int N, int cs,
                                                    const float* __restrict__ b1, const float* __restrict__ w,
                                                    const float* __restrict__ b2, int act,
                                                    float* __restrict__ hidden, float* __restrict__ out) {
  __shared__ float hs[kSeT];
  __shared__ float redf[kSeT];
  const int b = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
  {
    // the shares: lanes (j, share group), 8 loads in flight per lane
    const int G = kSeT / N;
    const int j = t % N, g = t / N;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (g < G) {
      int k = g;
      for (; k + 7 * G < s1; k += 8 * G) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] += hp[((long)b * s1 + k + u * G) * N + j];
      }
      for (; k < s1; k += G) a[0] += hp[((long)b * s1 + k) * N + j];
    }
    redf[t] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  }
  __syncthreads();
  if (t < N) {
    float h = BWD ? 0.f : b1[t];
    for (int g = 0; g < kSeT / N; ++g) h += redf[g * N + t];
    if (BWD) {
      hs[t] = h * act_grad(hidden[(long)b * N + t], act);
    } else {
      if (s == 0) hidden[(long)b * N + t] = h;  // pre-activation, kept for backward
      hs[t] = act_fwd(h, act);
    }
  }
  __syncthreads();
  const int c0 = s * cs, n = min(cs, C - c0);
  const int jg = n >= kSeT ? 1 : min(8, kSeT / n);
  for (int cb = 0; cb < n; cb += kSeT) {
    const int c = cb + t % min(n, kSeT), g = t / min(n, kSeT);
    float e[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (g < jg && c < n) {
      const int cc = c0 + c;
      int j = g;
      for (; j + 7 * jg < N; j += 8 * jg) {
        float wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) wv[u] = BWD ? w[(long)cc * N + j + u * jg] : w[(long)(j + u * jg) * C + cc];
#pragma unroll
        for (int u = 0; u < 8; ++u) e[u] = fmaf(hs[j + u * jg], wv[u], e[u]);
      }
      for (; j < N; j += jg) e[0] = fmaf(hs[j], BWD ? w[(long)cc * N + j] : w[(long)j * C + cc], e[0]);
    }
    __syncthreads();
    redf[t] = ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
    __syncthreads();
    if (t < min(n - cb, kSeT) && jg >= 1) {
      const int cl = t;
      float v = 0.f;
      for (int g2 = 0; g2 < jg; ++g2) v += redf[g2 * min(n, kSeT) + cl];
      const int cc = c0 + cb + cl;
      out[(long)b * C + cc] = BWD ? v : sigmoidf_(b2[cc] + v);
    }
  }
}

template <int BWD>
static void se_mlp(const double* scratch, int chunks, int B, int C, int N, float inv, const float* wsq,
                   const float* b1, const float* wex, const float* b2, int act, const float* scale_in,
                   float* pool, float* hidden, float* out, hipStream_t s) {
  if (N > kSeT) throw std::runtime_error("se: squeeze width > 256");
  const SePlan p = se_plan(B, C, N);
  // shares after the chunk partials (the scratch tail colred_scratch_doubles reserves)
  float* hp = reinterpret_cast<float*>(const_cast<double*>(scratch) + (size_t)B * chunks * C * 2);
  hipLaunchKernelGGL((k_se_squeeze<BWD>), dim3(B, p.s1), dim3(kSeT), (size_t)p.cs1 * sizeof(float), s, scratch,
                     chunks, C, N, p.cs1, wsq, inv, scale_in, pool, hp);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL((k_se_excite<BWD>), dim3(B, p.s2), dim3(kSeT), 0, s, hp, p.s1, C, N, p.cs2, b1, wex, b2, act,
                     hidden, out);
  PHX_LAUNCH_CHECK();
}

void launch_se_fwd(InX x, float* y, int B, int HW, int C, int Cse, const float* w1,
                   const float* b1, const float* w2, const float* b2, int act, float* pool,
                   float* hidden, float* scale, hipStream_t s, double* scratch) {
  const int chunks = x.bf ? colred_parts(SumAcc<true>{x, nullptr, C, {}}, HW, C, B, scratch, s)
                          : colred_parts(SumAcc<false>{x, nullptr, C, {}}, HW, C, B, scratch, s);
  se_mlp<0>(scratch, chunks, B, C, Cse, 1.0f / (float)HW, w1, b1, w2, b2, act, nullptr, pool, hidden, scale, s);
  (void)y;  // the excitation is folded into the consuming GEMM's A load (rowscale)
}

// dx = dy * scale[b,c] + dpool[b,c] / HW (+ dx)
struct SeBwdApply {
  const float* dy;
  const float* scale;
  const float* dpool;
  float* dx;
  int C, acc;
  float inv;
  float4 sc, dp;
  using Raw = float4;
  __device__ void init(int seg, int c4) {
    sc = *reinterpret_cast<const float4*>(scale + (long)seg * C + c4 * 4);
    const float4 d = *reinterpret_cast<const float4*>(dpool + (long)seg * C + c4 * 4);
    dp = make_float4(d.x * inv, d.y * inv, d.z * inv, d.w * inv);
  }
  __device__ Raw load(long m, int c4) const { return *reinterpret_cast<const float4*>(dy + m * C + c4 * 4); }
  __device__ float4 out(const Raw& g, long m, int c4) const {
    float4 o = make_float4(fmaf(g.x, sc.x, dp.x), fmaf(g.y, sc.y, dp.y), fmaf(g.z, sc.z, dp.z), fmaf(g.w, sc.w, dp.w));
    float4* op = reinterpret_cast<float4*>(dx + m * C + c4 * 4);
    if (acc) {
      const float4 p = *op;
      o.x += p.x; o.y += p.y; o.z += p.z; o.w += p.w;
    }
    *op = o;
    return o;
  }
};

int launch_se_bwd(const float* dy, InX x, float* dx, int B, int HW, int C, int Cse,
                  const float* w1, const float* b1, const float* w2t, const float* b2, int act,
                  const float* pool, const float* hidden, const float* scale, float* gsum,
                  bool acc, hipStream_t s, double* scratch, GradSink gs) {
  (void)b1; (void)b2; (void)pool;
  // gsum[0 .. B*C): dpool
  const int chunks = x.bf ? colred_parts(SumAcc<true>{x, dy, C, {}}, HW, C, B, scratch, s)
                          : colred_parts(SumAcc<false>{x, dy, C, {}}, HW, C, B, scratch, s);
  se_mlp<1>(scratch, chunks, B, C, Cse, 1.f, w2t, nullptr, w1, nullptr, act, scale, nullptr,
            const_cast<float*>(hidden), gsum, s);
  return ew_gstats(SeBwdApply{dy, scale, gsum, dx, C, acc ? 1 : 0, 1.0f / (float)HW, {}, {}}, HW, C, B, gs, s);
}

// ------------------------------------------------------------------------------------------
// elementwise
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float4 drop_fwd4(const DropView& dv, long row, float4 u) {
  const float k = dv.keep[row / dv.rows];
  return make_float4(div_surv(u.x, dv.p) * k, div_surv(u.y, dv.p) * k, div_surv(u.z, dv.p) * k,
                     div_surv(u.w, dv.p) * k);
}
__device__ __forceinline__ float4 drop_bwd4(const DropView& dv, long row, float4 g) {
  const float k = dv.keep[row / dv.rows];
  return make_float4(div_surv(g.x * k, dv.p), div_surv(g.y * k, dv.p), div_surv(g.z * k, dv.p),
                     div_surv(g.w * k, dv.p));
}

template <bool BF>
__global__ void k_add(InX a, InX b, float* __restrict__ y, long n4, int C, DropView dv) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int c = (int)((i * 4) % C);
  float4 u = inx_load4<BF>(a, i * 4, c), v = inx_load4<BF>(b, i * 4, c);
  if (dv.keep) u = drop_fwd4(dv, i * 4 / C, u);
  ast4<BF>(y, i * 4, make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w));
}

void launch_add(InX a, InX b, float* y, long n, int C, hipStream_t s, DropView dv) {
  long n4 = n / 4;
  if (a.bf != b.bf) throw std::runtime_error("add: operands differ in storage type");
  if (a.bf) hipLaunchKernelGGL(k_add<true>, dim3(cdiv(n4, 256)), dim3(256), 0, s, a, b, y, n4, C, dv);
  else hipLaunchKernelGGL(k_add<false>, dim3(cdiv(n4, 256)), dim3(256), 0, s, a, b, y, n4, C, dv);
  PHX_LAUNCH_CHECK();
}

// widening copy of a bf16 activation (phx_debug_tap of a PHX_DTYPE_BF16 context)
__global__ void k_bf16_to_f32(const float* __restrict__ src, float* __restrict__ dst, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = ald1<true>(src, i);
}

void launch_bf16_to_f32(const float* src, float* dst, long n, hipStream_t s) {
  hipLaunchKernelGGL(k_bf16_to_f32, dim3(cdiv(n, 256)), dim3(256), 0, s, src, dst, n);
  PHX_LAUNCH_CHECK();
}

// PHX_CKSUM diagnostics: an order-independent hash of n 16-bit words (sum over i of a mix of
// (word, i), wrapping 64-bit integer adds), so the value does not depend on how the grid splits the
// buffer and any single changed bit changes it
__device__ __forceinline__ unsigned long long ck_mix(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}
__global__ void k_cksum(const uint16_t* __restrict__ p, long n, unsigned long long* __restrict__ out) {
  unsigned long long h = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    h += ck_mix(((unsigned long long)i << 16) ^ p[i] ^ 0x9e3779b97f4a7c15ull);
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd(out, h);
}

void launch_cksum(const void* p, size_t bytes, unsigned long long* out, hipStream_t s) {
  const long n = (long)(bytes / 2);
  if (!p || n == 0) return;
  hipLaunchKernelGGL(k_cksum, dim3((unsigned)std::min<long>(cdiv(n, 256), 2048)), dim3(256), 0, s,
                     reinterpret_cast<const uint16_t*>(p), n, out);
  PHX_LAUNCH_CHECK();
}

// drop connect keep flags: tf.floor(survival + tf.random.uniform([B,1,1,1])) per block and image
__global__ void k_drop_keep(const int* __restrict__ block, const float* __restrict__ p, int nd, int B,
                            uint64_t seed, int64_t step, int gimg0, int pass,
                            float* __restrict__ keep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nd * B) return;
  const int d = i / B, b = i - d * B;
  const u32x4 r = philox4x32_10(
      u32x4{(uint32_t)block[d], (uint32_t)pass, (uint32_t)(gimg0 + b),
            (uint32_t)((uint64_t)step << 8) | (uint32_t)RNG_DROP},
      (uint32_t)seed, (uint32_t)(seed >> 32));
  keep[i] = floorf(p[d] + u01(r.x));
}

void launch_drop_keep(const int* block, const float* p, int nd, int B, uint64_t seed, int64_t step,
                      int gimg0, int pass, float* keep, hipStream_t s) {
  hipLaunchKernelGGL(k_drop_keep, dim3(cdiv(nd * B, 256)), dim3(256), 0, s, block, p, nd, B, seed, step,
                     gimg0, pass, keep);
  PHX_LAUNCH_CHECK();
}

__global__ void k_copy_grad(const float4* __restrict__ src, float4* __restrict__ dst, long n4,
                            int acc, int C, DropView dv) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4 v = src[i];
  if (dv.keep) v = drop_bwd4(dv, i * 4 / C, v);
  if (acc) {
    float4 p = dst[i];
    v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
  }
  dst[i] = v;
}

struct CopyGrad {
  const float* src;
  float* dst;
  int C, acc;
  DropView dv;
  using Raw = float4;
  __device__ void init(int, int) {}
  __device__ Raw load(long m, int c4) const { return *reinterpret_cast<const float4*>(src + m * C + c4 * 4); }
  __device__ float4 out(const Raw& v0, long m, int c4) const {
    float4 v = v0;
    if (dv.keep) v = drop_bwd4(dv, m, v);
    float4* op = reinterpret_cast<float4*>(dst + m * C + c4 * 4);
    if (acc) {
      const float4 p = *op;
      v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
    }
    *op = v;
    return v;
  }
};

// GradSink sums of a gradient that is already in place (aliased add input): read only
struct ReadGrad {
  const float* src;
  int C;
  using Raw = float4;
  __device__ void init(int, int) {}
  __device__ Raw load(long m, int c4) const { return *reinterpret_cast<const float4*>(src + m * C + c4 * 4); }
  __device__ float4 out(const Raw& v, long, int) const { return v; }
};

int launch_grad_sums(const float* src, long n, int C, GradSink gs, hipStream_t s) {
  return ew_gstats(ReadGrad{src, C}, n / C, C, 1, gs, s);
}

int launch_copy_grad(const float* src, float* dst, long n, bool acc, hipStream_t s, int C,
                     GradSink gs, DropView dv) {
  if (gs.part) return ew_gstats(CopyGrad{src, dst, C, acc ? 1 : 0, dv}, n / C, C, 1, gs, s);
  long n4 = n / 4;
  hipLaunchKernelGGL(k_copy_grad, dim3(cdiv(n4, 256)), dim3(256), 0, s, (const float4*)src,
                     (float4*)dst, n4, acc ? 1 : 0, C, dv);
  PHX_LAUNCH_CHECK();
  return 0;
}

// max pool, TF SAME with -inf padding (efficientdet_keras.py:260-276).  The forward records, per
// output element, which window tap held the maximum (first in row-major scan order, the element
// TF's MaxPoolGrad routes the gradient to), so the backward is a gather of at most
// ceil(k/s)^2 dy values per input element with no window re-scan.
template <bool BF>
__global__ void k_maxpool_fwd(InX x, float* __restrict__ y, uint8_t* __restrict__ amax, int B, int H,
                              int W, int C, int Ho, int Wo, int k, int st, int pt, int pl) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * Ho * Wo * C;
  if (idx >= total) return;
  int c = (int)(idx % C);
  long p = idx / C;
  int ox = (int)(p % Wo);
  long t = p / Wo;
  int oy = (int)(t % Ho);
  int b = (int)(t / Ho);
  float m = -INFINITY;
  int am = 0;
  for (int i = 0; i < k; ++i) {
    int iy = oy * st - pt + i;
    if (iy < 0 || iy >= H) continue;
    for (int j = 0; j < k; ++j) {
      int ix = ox * st - pl + j;
      if (ix < 0 || ix >= W) continue;
      const float v = inx_load1<BF>(x, (((long)b * H + iy) * W + ix) * C + c, c);
      if (v > m || (am == 0 && m == -INFINITY)) {
        if (v > m) m = v;
        am = i * k + j + 1;
      }
    }
  }
  ast1<BF>(y, idx, m);
  amax[idx] = (uint8_t)(am - 1);
}

__global__ void k_maxpool_bwd(const uint8_t* __restrict__ amax, const float* __restrict__ dy,
                              float* __restrict__ dx, int B, int H, int W, int C, int Ho, int Wo,
                              int k, int st, int pt, int pl, int acc_flag) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * H * W * C;
  if (idx >= total) return;
  int c = (int)(idx % C);
  long p = idx / C;
  int ix = (int)(p % W);
  long t = p / W;
  int iy = (int)(t % H);
  int b = (int)(t / H);
  float g = 0.f;
  // windows containing (iy, ix): oy*st - pt <= iy < oy*st - pt + k
  const int oyl = max(0, (iy + pt - k + st) / st), oyh = min(Ho - 1, (iy + pt) / st);
  const int oxl = max(0, (ix + pl - k + st) / st), oxh = min(Wo - 1, (ix + pl) / st);
  for (int oy = oyl; oy <= oyh; ++oy) {
    const int i = iy - (oy * st - pt);
    if (i < 0 || i >= k) continue;
    for (int ox = oxl; ox <= oxh; ++ox) {
      const int j = ix - (ox * st - pl);
      if (j < 0 || j >= k) continue;
      const long o = (((long)b * Ho + oy) * Wo + ox) * C + c;
      if (amax[o] == i * k + j) g += dy[o];
    }
  }
  if (acc_flag) g += dx[idx];
  dx[idx] = g;
}

// Channel-quad forms (C % 4 == 0, every resample in the model tables): a lane owns 4 channels of
// one pixel — 16-B loads and stores, the BN view's parameters loaded once per lane, 32-bit index
// math — instead of one lane per element with 4-B accesses and 64-bit divisions (the scalar
// kernels above ran the D4 BiFPN resamples at a fraction of HBM bandwidth; they remain for C % 4).
__device__ __forceinline__ void quad_pos(int idx, int C4, int Wd, int Hd, int& c4, int& x, int& y, int& b) {
  c4 = idx % C4;
  const int p = idx / C4;
  x = p % Wd;
  const int q = p / Wd;
  y = q % Hd;
  b = q / Hd;
}

// max-pool: TF MaxPool picks the first maximum of the window (strict > after the first element)
template <bool BF>
__global__ __launch_bounds__(256) void k_maxpool_fwd4(InX x, float* __restrict__ y, uint32_t* __restrict__ amax,
                                                      int H, int W, int C4, int Ho, int Wo, int k, int st, int pt,
                                                      int pl, int total4) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total4) return;
  int c4, ox, oy, b;
  quad_pos(idx, C4, Wo, Ho, c4, ox, oy, b);
  const int C = C4 * 4;
  Chan4 ck;
  if (x.mu) ck = inx_chan4(x, c4 * 4);
  float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int am[4] = {-1, -1, -1, -1};
  for (int i = 0; i < k; ++i) {
    const int iy = oy * st - pt + i;
    if (iy < 0 || iy >= H) continue;
    for (int j = 0; j < k; ++j) {
      const int ix = ox * st - pl + j;
      if (ix < 0 || ix >= W) continue;
      float4 v4 = ald4<BF>(x.p, ((long)(b * H + iy) * W + ix) * C + c4 * 4);
      if (x.mu) v4 = inx_apply4(x, ck, v4);
      const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (am[e] < 0 || v[e] > m[e]) {
          m[e] = v[e];
          am[e] = i * k + j;
        }
    }
  }
  ast4<BF>(y, (long)idx * 4, make_float4(m[0], m[1], m[2], m[3]));
  amax[idx] = (uint32_t)(am[0] & 255) | ((uint32_t)(am[1] & 255) << 8) | ((uint32_t)(am[2] & 255) << 16) |
              ((uint32_t)(am[3] & 255) << 24);
}

__global__ __launch_bounds__(256) void k_maxpool_bwd4(const uint32_t* __restrict__ amax, const float4* __restrict__ dy,
                                                      float4* __restrict__ dx, int H, int W, int C4, int Ho, int Wo,
                                                      int k, int st, int pt, int pl, int acc_flag, int total4) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total4) return;
  int c4, ix, iy, b;
  quad_pos(idx, C4, W, H, c4, ix, iy, b);
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  const int oyl = max(0, (iy + pt - k + st) / st), oyh = min(Ho - 1, (iy + pt) / st);
  const int oxl = max(0, (ix + pl - k + st) / st), oxh = min(Wo - 1, (ix + pl) / st);
  for (int oy = oyl; oy <= oyh; ++oy) {
    const int i = iy - (oy * st - pt);
    if (i < 0 || i >= k) continue;
    for (int ox = oxl; ox <= oxh; ++ox) {
      const int j = ix - (ox * st - pl);
      if (j < 0 || j >= k) continue;
      const int o = ((b * Ho + oy) * Wo + ox) * C4 + c4;
      const uint32_t a = amax[o];
      const float4 d = dy[o];
      const float dv[4] = {d.x, d.y, d.z, d.w};
      const uint32_t want = (uint32_t)(i * k + j);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (((a >> (8 * e)) & 255u) == want) g[e] += dv[e];
    }
  }
  float4 r = make_float4(g[0], g[1], g[2], g[3]);
  if (acc_flag) {
    const float4 p = dx[idx];
    r.x += p.x; r.y += p.y; r.z += p.z; r.w += p.w;
  }
  dx[idx] = r;
}

static bool quad_ok(long total, int C) { return C % 4 == 0 && total / 4 < (1L << 31); }

void launch_maxpool_fwd(InX x, float* y, uint8_t* amax, int B, int H, int W, int C, int Ho, int Wo,
                        int k, int stride, int pt, int pl, hipStream_t s) {
  long total = (long)B * Ho * Wo * C;
  if (quad_ok(total, C)) {
    const int t4 = (int)(total / 4);
    if (x.bf)
      hipLaunchKernelGGL(k_maxpool_fwd4<true>, dim3(cdiv(t4, 256)), dim3(256), 0, s, x, y, (uint32_t*)amax, H, W,
                         C / 4, Ho, Wo, k, stride, pt, pl, t4);
    else
      hipLaunchKernelGGL(k_maxpool_fwd4<false>, dim3(cdiv(t4, 256)), dim3(256), 0, s, x, y, (uint32_t*)amax, H, W,
                         C / 4, Ho, Wo, k, stride, pt, pl, t4);
  } else if (x.bf) {
    hipLaunchKernelGGL(k_maxpool_fwd<true>, dim3(cdiv(total, 256)), dim3(256), 0, s, x, y, amax, B, H, W, C, Ho,
                       Wo, k, stride, pt, pl);
  } else {
    hipLaunchKernelGGL(k_maxpool_fwd<false>, dim3(cdiv(total, 256)), dim3(256), 0, s, x, y, amax, B, H, W, C, Ho,
                       Wo, k, stride, pt, pl);
  }
  PHX_LAUNCH_CHECK();
}

void launch_maxpool_bwd(const uint8_t* amax, const float* dy, float* dx, int B, int H, int W, int C,
                        int Ho, int Wo, int k, int stride, int pt, int pl, bool acc,
                        hipStream_t s) {
  long total = (long)B * H * W * C;
  if (quad_ok(total, C) && quad_ok((long)B * Ho * Wo * C, C)) {
    const int t4 = (int)(total / 4);
    hipLaunchKernelGGL(k_maxpool_bwd4, dim3(cdiv(t4, 256)), dim3(256), 0, s, (const uint32_t*)amax,
                       (const float4*)dy, (float4*)dx, H, W, C / 4, Ho, Wo, k, stride, pt, pl, acc ? 1 : 0, t4);
  } else {
    hipLaunchKernelGGL(k_maxpool_bwd, dim3(cdiv(total, 256)), dim3(256), 0, s, amax, dy, dx, B, H, W, C,
                       Ho, Wo, k, stride, pt, pl, acc ? 1 : 0);
  }
  PHX_LAUNCH_CHECK();
}

// nearest neighbour, legacy (align_corners=False, half_pixel_centers=False):
// src = min(floor(dst * (in/out)), in-1)  (efficientdet_keras.py:278-287)
__device__ __forceinline__ int nn_src(int d, float scale, int in) {
  int s = (int)floorf((float)d * scale);
  return s < in - 1 ? s : in - 1;
}

template <bool BF>
__global__ void k_upsample_fwd(InX x, float* __restrict__ y, int B, int H,
                               int W, int C, int Ho, int Wo) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * Ho * Wo * C;
  if (idx >= total) return;
  int c = (int)(idx % C);
  long p = idx / C;
  int ox = (int)(p % Wo);
  long t = p / Wo;
  int oy = (int)(t % Ho);
  int b = (int)(t / Ho);
  int sy = nn_src(oy, (float)H / (float)Ho, H);
  int sx = nn_src(ox, (float)W / (float)Wo, W);
  ast1<BF>(y, idx, inx_load1<BF>(x, (((long)b * H + sy) * W + sx) * C + c, c));
}

__global__ void k_upsample_bwd(const float* __restrict__ dy, float* __restrict__ dx, int B, int H,
                               int W, int C, int Ho, int Wo, int acc_flag) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * H * W * C;
  if (idx >= total) return;
  int c = (int)(idx % C);
  long p = idx / C;
  int ix = (int)(p % W);
  long t = p / W;
  int iy = (int)(t % H);
  int b = (int)(t / H);
  const float sy = (float)H / (float)Ho, sx = (float)W / (float)Wo;
  // candidate outputs: those whose src equals (iy, ix)
  int oy0 = (int)floorf((float)iy / sy) - 1, oy1 = (int)ceilf((float)(iy + 1) / sy) + 1;
  int ox0 = (int)floorf((float)ix / sx) - 1, ox1 = (int)ceilf((float)(ix + 1) / sx) + 1;
  oy0 = max(oy0, 0); ox0 = max(ox0, 0); oy1 = min(oy1, Ho - 1); ox1 = min(ox1, Wo - 1);
  float g = 0.f;
  for (int oy = oy0; oy <= oy1; ++oy) {
    if (nn_src(oy, sy, H) != iy) continue;
    for (int ox = ox0; ox <= ox1; ++ox) {
      if (nn_src(ox, sx, W) != ix) continue;
      g += dy[(((long)b * Ho + oy) * Wo + ox) * C + c];
    }
  }
  if (acc_flag) g += dx[idx];
  dx[idx] = g;
}

template <bool BF>
__global__ __launch_bounds__(256) void k_upsample_fwd4(InX x, float* __restrict__ y, int H, int W, int C4, int Ho,
                                                       int Wo, int total4) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total4) return;
  int c4, ox, oy, b;
  quad_pos(idx, C4, Wo, Ho, c4, ox, oy, b);
  const int sy = nn_src(oy, (float)H / (float)Ho, H);
  const int sx = nn_src(ox, (float)W / (float)Wo, W);
  ast4<BF>(y, (long)idx * 4, inx_load4<BF>(x, ((long)(b * H + sy) * W + sx) * (C4 * 4) + c4 * 4, c4 * 4));
}

__global__ __launch_bounds__(256) void k_upsample_bwd4(const float4* __restrict__ dy, float4* __restrict__ dx, int H,
                                                       int W, int C4, int Ho, int Wo, int acc_flag, int total4) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total4) return;
  int c4, ix, iy, b;
  quad_pos(idx, C4, W, H, c4, ix, iy, b);
  const float sy = (float)H / (float)Ho, sx = (float)W / (float)Wo;
  int oy0 = (int)floorf((float)iy / sy) - 1, oy1 = (int)ceilf((float)(iy + 1) / sy) + 1;
  int ox0 = (int)floorf((float)ix / sx) - 1, ox1 = (int)ceilf((float)(ix + 1) / sx) + 1;
  oy0 = max(oy0, 0); ox0 = max(ox0, 0); oy1 = min(oy1, Ho - 1); ox1 = min(ox1, Wo - 1);
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int oy = oy0; oy <= oy1; ++oy) {
    if (nn_src(oy, sy, H) != iy) continue;
    for (int ox = ox0; ox <= ox1; ++ox) {
      if (nn_src(ox, sx, W) != ix) continue;
      const float4 d = dy[((b * Ho + oy) * Wo + ox) * C4 + c4];
      g.x += d.x; g.y += d.y; g.z += d.z; g.w += d.w;
    }
  }
  if (acc_flag) {
    const float4 p = dx[idx];
    g.x += p.x; g.y += p.y; g.z += p.z; g.w += p.w;
  }
  dx[idx] = g;
}

void launch_upsample_fwd(InX x, float* y, int B, int H, int W, int C, int Ho, int Wo,
                         hipStream_t s) {
  long total = (long)B * Ho * Wo * C;
  if (quad_ok(total, C)) {
    const int t4 = (int)(total / 4);
    if (x.bf)
      hipLaunchKernelGGL(k_upsample_fwd4<true>, dim3(cdiv(t4, 256)), dim3(256), 0, s, x, y, H, W, C / 4, Ho, Wo, t4);
    else
      hipLaunchKernelGGL(k_upsample_fwd4<false>, dim3(cdiv(t4, 256)), dim3(256), 0, s, x, y, H, W, C / 4, Ho, Wo, t4);
  } else if (x.bf) {
    hipLaunchKernelGGL(k_upsample_fwd<true>, dim3(cdiv(total, 256)), dim3(256), 0, s, x, y, B, H, W, C, Ho, Wo);
  } else {
    hipLaunchKernelGGL(k_upsample_fwd<false>, dim3(cdiv(total, 256)), dim3(256), 0, s, x, y, B, H, W, C, Ho, Wo);
  }
  PHX_LAUNCH_CHECK();
}

void launch_upsample_bwd(const float* dy, float* dx, int B, int H, int W, int C, int Ho, int Wo,
                         bool acc, hipStream_t s) {
  long total = (long)B * H * W * C;
  if (quad_ok(total, C) && quad_ok((long)B * Ho * Wo * C, C)) {
    const int t4 = (int)(total / 4);
    hipLaunchKernelGGL(k_upsample_bwd4, dim3(cdiv(t4, 256)), dim3(256), 0, s, (const float4*)dy, (float4*)dx, H, W,
                       C / 4, Ho, Wo, acc ? 1 : 0, t4);
  } else {
    hipLaunchKernelGGL(k_upsample_bwd, dim3(cdiv(total, 256)), dim3(256), 0, s, dy, dx, B, H, W, C, Ho,
                       Wo, acc ? 1 : 0);
  }
  PHX_LAUNCH_CHECK();
}

// BiFPN fuse (FNode.fuse_features, efficientdet_keras.py:75-121) followed by the
// OpAfterCombine activation (:214-216).  fastattn: n_i = x_i * relu(w_i) / (sum relu(w) + 1e-4),
// summed in order (add_n, :31-39).
struct FuseArgs {
  InX x[3];
  float* dx[3];
  int acc[3];
};


template <bool BF>
__global__ void k_fuse_fwd(FuseArgs fa, int nin, const float* __restrict__ w0,
                           const float* __restrict__ w1, const float* __restrict__ w2, int method,
                           int act, float* __restrict__ y, long n, int C) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float wv[3], den;
  fuse_weights(w0, w1, w2, nin, method, wv, &den);
  const int c = (int)(i % C);
  const float x0 = inx_load1<BF>(fa.x[0], i, c), x1 = inx_load1<BF>(fa.x[1], i, c);
  const float x2 = nin > 2 ? inx_load1<BF>(fa.x[2], i, c) : 0.f;
  ast1<BF>(y, i, fuse_combine(x0, x1, x2, nin, method, wv, den, act));
}

template <bool BF>
__global__ void k_fuse_bwd(FuseArgs fa, int nin, const float* __restrict__ w0,
                           const float* __restrict__ w1, const float* __restrict__ w2, int method,
                           int act, const float* __restrict__ dy, long n, int C) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float wv[3], den;
  fuse_weights(w0, w1, w2, nin, method, wv, &den);
  const int c = (int)(i % C);
  const float x0 = inx_load1<BF>(fa.x[0], i, c), x1 = inx_load1<BF>(fa.x[1], i, c);
  const float x2 = nin > 2 ? inx_load1<BF>(fa.x[2], i, c) : 0.f;
  float v;
  if (method == 0) {
    v = x0 * wv[0] / den;
    v = v + x1 * wv[1] / den;
    if (nin > 2) v = v + x2 * wv[2] / den;
  } else {
    v = x0 + x1;
    if (nin > 2) v = v + x2;
  }
  float dv = dy[i] * act_grad(v, act);
  for (int k = 0; k < nin; ++k) {
    if (!fa.dx[k]) continue;
    float g = method == 0 ? (dv / den) * wv[k] : dv;
    if (fa.acc[k]) g += fa.dx[k][i];
    fa.dx[k][i] = g;
  }
}

// channel-quad form of k_fuse_bwd (C % 4 == 0): identical per-element arithmetic, 16-B accesses
template <bool BF>
__global__ __launch_bounds__(256) void k_fuse_bwd4(FuseArgs fa, int nin, const float* __restrict__ w0,
                                                   const float* __restrict__ w1, const float* __restrict__ w2,
                                                   int method, int act, const float4* __restrict__ dy, long n4,
                                                   int C) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float wv[3], den;
  fuse_weights(w0, w1, w2, nin, method, wv, &den);
  const int c = (int)((i * 4) % C);
  const float4 a0 = inx_load4<BF>(fa.x[0], i * 4, c), a1 = inx_load4<BF>(fa.x[1], i * 4, c);
  const float4 a2 = nin > 2 ? inx_load4<BF>(fa.x[2], i * 4, c) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 d4 = dy[i];
  const float x0[4] = {a0.x, a0.y, a0.z, a0.w}, x1[4] = {a1.x, a1.y, a1.z, a1.w}, x2[4] = {a2.x, a2.y, a2.z, a2.w};
  const float dd[4] = {d4.x, d4.y, d4.z, d4.w};
  float dv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float v;
    if (method == 0) {
      v = x0[e] * wv[0] / den;
      v = v + x1[e] * wv[1] / den;
      if (nin > 2) v = v + x2[e] * wv[2] / den;
    } else {
      v = x0[e] + x1[e];
      if (nin > 2) v = v + x2[e];
    }
    dv[e] = dd[e] * act_grad(v, act);
  }
  for (int k = 0; k < nin; ++k) {
    if (!fa.dx[k]) continue;
    float g[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) g[e] = method == 0 ? (dv[e] / den) * wv[k] : dv[e];
    float4* o = reinterpret_cast<float4*>(fa.dx[k]) + i;
    float4 r = make_float4(g[0], g[1], g[2], g[3]);
    if (fa.acc[k]) {
      const float4 p = *o;
      r.x += p.x; r.y += p.y; r.z += p.z; r.w += p.w;
    }
    *o = r;
  }
}

void launch_fuse_fwd(const InX* xs, int nin, const float* wsm0, const float* wsm1,
                     const float* wsm2, int method, int act, float* y, long n, int C,
                     hipStream_t s) {
  FuseArgs fa{};
  for (int i = 0; i < nin; ++i) fa.x[i] = xs[i];
  if (xs[0].bf)
    hipLaunchKernelGGL(k_fuse_fwd<true>, dim3(cdiv(n, 256)), dim3(256), 0, s, fa, nin, wsm0, wsm1, wsm2,
                       method, act, y, n, C);
  else
    hipLaunchKernelGGL(k_fuse_fwd<false>, dim3(cdiv(n, 256)), dim3(256), 0, s, fa, nin, wsm0, wsm1, wsm2,
                       method, act, y, n, C);
  PHX_LAUNCH_CHECK();
}

void launch_fuse_bwd(const InX* xs, int nin, const float* wsm0, const float* wsm1,
                     const float* wsm2, int method, int act, const float* dy, float* const* dxs,
                     const bool* acc, long n, int C, hipStream_t s) {
  FuseArgs fa{};
  for (int i = 0; i < nin; ++i) {
    fa.x[i] = xs[i];
    fa.dx[i] = dxs[i];
    fa.acc[i] = acc[i] ? 1 : 0;
  }
  if (C % 4 == 0 && xs[0].bf)
    hipLaunchKernelGGL(k_fuse_bwd4<true>, dim3(cdiv(n / 4, 256)), dim3(256), 0, s, fa, nin, wsm0, wsm1, wsm2,
                       method, act, (const float4*)dy, n / 4, C);
  else if (C % 4 == 0)
    hipLaunchKernelGGL(k_fuse_bwd4<false>, dim3(cdiv(n / 4, 256)), dim3(256), 0, s, fa, nin, wsm0, wsm1, wsm2,
                       method, act, (const float4*)dy, n / 4, C);
  else if (xs[0].bf)
    hipLaunchKernelGGL(k_fuse_bwd<true>, dim3(cdiv(n, 256)), dim3(256), 0, s, fa, nin, wsm0, wsm1, wsm2,
                       method, act, dy, n, C);
  else
    hipLaunchKernelGGL(k_fuse_bwd<false>, dim3(cdiv(n, 256)), dim3(256), 0, s, fa, nin, wsm0, wsm1, wsm2,
                       method, act, dy, n, C);
  PHX_LAUNCH_CHECK();
}

}  // namespace phx
