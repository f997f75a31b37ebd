// dw_stage.hpp — staging sources shared by the depthwise kernels (kernels_dw.hip) and the fused
// separable-conv kernels (kernels_sep.hip): how a kernel that stages an activation window into LDS sees
// its input — a BN view (InX), a BiFPN node fuse computed on load (FuseView) or a BN-backward gradient
// view (GradX) — plus the XCD-aware work split.
#pragma once
#include <type_traits>

#include "common.hpp"

namespace phx {

// XCD-aware work split: the ntiles*ncg (tile, channel slice) items, tile-major, are cut into
// 8 contiguous ranges of `per` items, one per XCD (dispatch is round-robin: block L -> XCD L%8),
// so the ncg slices of a tile run back to back on one XCD and share its L2, and every XCD gets
// work even when a level has fewer than 8 tiles.  Returns false for the padding blocks.
__device__ __forceinline__ bool dw_block_map(int L, int per, int ncg, int nwork, int* tile,
                                             int* cg) {
  const int w = (L & 7) * per + (L >> 3);
  if ((L >> 3) >= per || w >= nwork) return false;
  *tile = w / ncg;
  *cg = w - *tile * ncg;
  return true;
}

// ---- staging sources (BF: the activation tensors hold bf16) --------------------------------
template <bool BF>
struct StageInX {
  using Raw = float4;
  InX v;
  Chan4 k;
  bool f;
  __device__ __forceinline__ void init(const InX& x, int c) {
    v = x;
    f = x.mu != nullptr;
    if (f) k = inx_chan4(x, c);
  }
  __device__ __forceinline__ Raw zero() const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ Raw load(long e) const { return ald4<BF>(v.p, e); }
  __device__ __forceinline__ float4 finish(const Raw& x) const {
    return f ? inx_apply4(v, k, x) : x;
  }
  // the view's activation as a compile-time constant (dw_stage dispatches once per launch)
  static constexpr bool kActT = true;
  __device__ __forceinline__ int act() const { return v.act; }
  template <int ACT>
  __device__ __forceinline__ float4 finish_t(const Raw& x) const {
    InX c = v;
    c.act = ACT;
    return f ? inx_apply4(c, k, x) : x;
  }
};

template <bool BF>
struct StageFuse {
  struct Raw {
    float4 v[3];
  };
  FuseView f;
  Chan4 k[3];
  float wv[3], den;
  __device__ __forceinline__ void init(const FuseView& fv, int c) {
    f = fv;
    for (int i = 0; i < 3; ++i)
      if (i < f.nin && f.x[i].mu) k[i] = inx_chan4(f.x[i], c);
    fuse_weights(f.w[0], f.w[1], f.w[2], f.nin, f.method, wv, &den);
  }
  __device__ __forceinline__ Raw zero() const {
    Raw r;
    r.v[0] = r.v[1] = r.v[2] = make_float4(0.f, 0.f, 0.f, 0.f);
    return r;
  }
  __device__ __forceinline__ Raw load(long e) const {
    Raw r;
    r.v[0] = ald4<BF>(f.x[0].p, e);
    r.v[1] = ald4<BF>(f.x[1].p, e);
    r.v[2] = f.nin > 2 ? ald4<BF>(f.x[2].p, e) : make_float4(0.f, 0.f, 0.f, 0.f);
    return r;
  }
  __device__ __forceinline__ float4 finish(const Raw& r) const {
    float4 a[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) a[i] = (i < f.nin && f.x[i].mu) ? inx_apply4(f.x[i], k[i], r.v[i]) : r.v[i];
    return make_float4(fuse_combine(a[0].x, a[1].x, a[2].x, f.nin, f.method, wv, den, f.act),
                       fuse_combine(a[0].y, a[1].y, a[2].y, f.nin, f.method, wv, den, f.act),
                       fuse_combine(a[0].z, a[1].z, a[2].z, f.nin, f.method, wv, den, f.act),
                       fuse_combine(a[0].w, a[1].w, a[2].w, f.nin, f.method, wv, den, f.act));
  }
  static constexpr bool kActT = false;
  __device__ __forceinline__ int act() const { return 0; }
  template <int ACT>
  __device__ __forceinline__ float4 finish_t(const Raw& r) const { return finish(r); }
};

template <bool BF>
struct StageGradX {
  struct Raw {
    float4 d, y;
  };
  GradX g;
  GChan4 k;
  __device__ __forceinline__ void init(const GradX& x, int c) {
    g = x;
    if (g.y) k = gx_chan4(g, c);
  }
  __device__ __forceinline__ Raw zero() const {
    return Raw{make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
  }
  __device__ __forceinline__ Raw load(long e) const {
    Raw r;
    r.d = *reinterpret_cast<const float4*>(g.da + e);
    if (g.y) r.y = ald4<BF>(g.y, e);
    return r;
  }
  __device__ __forceinline__ float4 finish(const Raw& r) const {
    return g.y ? gx_apply4(g, k, r.d, r.y) : r.d;
  }
  static constexpr bool kActT = true;
  __device__ __forceinline__ int act() const { return g.y ? g.act : 0; }
  template <int ACT>
  __device__ __forceinline__ float4 finish_t(const Raw& r) const {
    GradX c = g;
    c.act = ACT;
    return g.y ? gx_apply4(c, k, r.d, r.y) : r.d;
  }
};

__device__ __forceinline__ void fma4(float4& a, const float4& x, const float4& w) {
  a.x = fmaf(x.x, w.x, a.x);
  a.y = fmaf(x.y, w.y, a.y);
  a.z = fmaf(x.z, w.z, a.z);
  a.w = fmaf(x.w, w.w, a.w);
}

}  // namespace phx
