// gemm2_kernel.hpp — the 1x1-convolution GEMM kernel template of the victim forward and data-gradient on the
// fp32 matrix cores (v_mfma_f32_32x32x2_f32, exact f32).
//
//   C[M,N] (+)= A'[M,K] * Bt[N,K]^T (+ bias)      A' = A through an InX view (BN + activation on
//                                                 load), optionally x SE rowscale, or a GradX view
//
// Design (MI355X):
//  * 256-thread workgroup = WM x WN waves, each wave owns TM x TN tiles of 32x32; block tile
//    BM x BN = (32*WM*TM) x (32*WN*TN), K advanced in BK = 16 chunks through a double-buffered
//    LDS image (unpadded rows, 16-B units XOR-swizzled: g2_off).  Operand fragments are ds_read_b128: lane l feeds
//    k = 4*(l>>5) + s of its row/column at MFMA step s, so one 16-B read serves 4 MFMAs (the k
//    order is permuted identically for A and B, so the products are unchanged).
//  * Workgroups are persistent along M: the (m-tile, k-chunk) steps of all the tiles a workgroup
//    owns form one software pipeline — the global loads of step s+1 are in flight while step s
//    runs its MFMAs and (on a tile's last chunk) its epilogue, so streaming shapes (K <= 64,
//    one chunk per tile) still overlap load, compute and store.
//  * The A view (BN, activation, SE scale, BN backward) is applied once per element when the
//    prefetched registers are written to LDS; a thread's channel quad is fixed within a chunk, so
//    its per-channel parameters are three (six) float4 loads per chunk.
//  * Epilogue straight from the accumulators: in the 32x32 C/D layout the 32 lanes of a half-wave
//    hold 32 consecutive columns of one row, so every store instruction writes two 128-B row
//    segments.  STATS: the consumer BN's batch statistics (StatSink) are reduced per tile in
//    registers (two passes, xor-32 shuffle), merged across the WM waves in LDS and folded across
//    the workgroup's tiles (Chan), one partial row per workgroup.
//  * Split-K (blockIdx.z) writes fp32 partial slabs reduced by k_gemm_splitk_reduce(_stats).
//  * MODE 4 (implicit im2col): A[m][k] is gathered from an NHWC tensor — the column matrix of a 3x3
//    convolution, k = (ky*3 + kx)*C + c — with the geometry packed into Gemm2Args::rpi (g2_geo):
//    power-of-2 channel and spatial sizes, so a row's pixel and a quad's (tap, channel) are shifts
//    and masks.  A 16-B quad never straddles a tap (C >= 4).
//  * Grouped launch: up to kMaxSeg GEMMs with the same B operand, N and K but their own A, C, M and
//    statistics sinks (the per-level members of a class/box-head conv, whose weights are shared
//    across pyramid levels) run as one grid; blockIdx.z = segment * splits + split.
#pragma once
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace phx {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct Gemm2Args {
  InX A;
  GradX G;
  const float* Bt;
  const float* bias;
  float* C;
  int M, N, K, acc;
  const float* rowscale;
  int rpi;
  int kslice;
  float* partial;
  StatSink sink;
  int mtiles;
  GradSink gsk;
};

// NS = argument slots: 1 for ordinary launches (small kernarg: ~1 us per launch is at stake),
// kMaxSeg for grouped ones
template <int NS>
struct Gemm2Group {
  Gemm2Args a[NS];
  int n;
};

// BF: bf16 matrix cores (v_mfma_f32_32x32x16_bf16, fp32 accumulation) — the A view is applied in
// fp32 and rounded to bf16 when the chunk is written to LDS, B (the weights) likewise; K advances in
// 32-deep chunks (two MFMAs per tile pair).  fp32 (BF = 0): v_mfma_f32_32x32x2_f32, 16-deep chunks.
#ifndef PHX_GEMM_BK_F32
#define PHX_GEMM_BK_F32 16
#endif
#ifndef PHX_GEMM_BK_BF16
#define PHX_GEMM_BK_BF16 32
#endif
template <int WM, int TM, int TN, int MODE, bool BF = false>
struct G2 {
  static constexpr int WN = 4 / WM;
  static constexpr int BM = WM * TM * 32, BN = WN * TN * 32, BK = BF ? PHX_GEMM_BK_BF16 : PHX_GEMM_BK_F32;
  static constexpr int LD = BK;                       // LDS row pitch in elements (unpadded; g2_off swizzles)
  static constexpr int KQ = BK / 4;                   // float4 per tile row per chunk
  static constexpr int RPP = 256 / KQ;                // tile rows loaded per pass of the 256 lanes
  static constexpr int NA = (BM + RPP - 1) / RPP;     // A float4 per thread per chunk
  static constexpr int NB = (BN + RPP - 1) / RPP;     // B float4 per thread per chunk
  static constexpr int ESZ = BF ? 2 : 4;              // bytes per LDS element
  static constexpr int LDS_FLOATS = 2 * (BM + BN) * LD * ESZ / 4;
};

// MODE 4 gather geometry, packed into 26 bits of Gemm2Args::rpi: log2 C | log2 Wo | log2 Ho | log2 W |
// log2 H | stride - 1 | pad top | pad left | gather mode (0 conv: x[oy*s + ky - pt][ox*s + kx - pl];
// 1 stride-2 transposed conv: x[(oy - ky) / 2][(ox - kx) / 2] when both are even)
struct G2Geo {
  int lC, lWo, lHo, lW, lH, s, pt, pl, mode;
};
__host__ __device__ __forceinline__ G2Geo g2_geo(uint32_t q) {
  return G2Geo{(int)(q & 15), (int)((q >> 4) & 15), (int)((q >> 8) & 15), (int)((q >> 12) & 15),
               (int)((q >> 16) & 15), (int)((q >> 20) & 1) + 1, (int)((q >> 21) & 3), (int)((q >> 23) & 3),
               (int)((q >> 25) & 1)};
}

template <int WM, int TM, int TN, int MODE, bool BF = false>
struct G2Regs {
  using P = G2<WM, TM, TN, MODE, BF>;
  float4 a[P::NA];
  bool gok[MODE == 4 ? P::NA : 1];
  float4 y[MODE == 3 ? P::NA : 1];
  float4 rs[MODE == 2 ? P::NA : 1];
  float4 b[P::NB];
  Chan4 ck;
  GChan4 gk;
};

// Branch-free: out-of-range rows / columns / k quads load from a clamped (valid) address and are
// zeroed when g2_store writes the chunk to LDS (a select here would wait for each load at once).
// A load under an exec-mask branch makes hipcc's wait counting conservative (vmcnt(0) right
// after the first conditional load), which exposed a full HBM round trip per K step before the
// MFMAs of the staged chunk could issue.
// ST (activation storage, PHX_DTYPE_BF16): 0 every tensor fp32; 1 forward — A and C are bf16
// activations; 2 data gradient — A and C are fp32 gradients, the BN input y (gradient view,
// GradSink) a bf16 activation
template <int WM, int TM, int TN, int MODE, bool BF, int ST>
__device__ __forceinline__ void g2_load(G2Regs<WM, TM, TN, MODE, BF>& r, const Gemm2Args& a, int m0, int n0,
                                        int k0, int kend) {
  using P = G2<WM, TM, TN, MODE, BF>;
  const int t = threadIdx.x;
  const int c4 = t % P::KQ;
  const int kk = k0 + 4 * c4;
  const bool kok = kk < kend;
  const int kc = kok ? kk : kend - 4;  // kend >= 4, K % 4 == 0
  if (MODE == 1 || MODE == 2) r.ck = inx_chan4(a.A, kc);
  if (MODE == 3) r.gk = gx_chan4(a.G, kc);
  if constexpr (MODE == 4) {
    const G2Geo g = g2_geo((uint32_t)a.rpi);
    const int tap = kc >> g.lC, c = kc & ((1 << g.lC) - 1);
    const int ky = (tap * 11) >> 5, kx = tap - 3 * ky;  // tap / 3 for tap < 9
#pragma unroll
    for (int u = 0; u < P::NA; ++u) {
      const int row = min(m0 + (t + 256 * u) / P::KQ, a.M - 1);
      const int ox = row & ((1 << g.lWo) - 1), oy = (row >> g.lWo) & ((1 << g.lHo) - 1);
      const int b = row >> (g.lWo + g.lHo);
      int iy, ix;
      bool ok = kok && tap < 9;
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
      const int row = m0 + (t + 256 * u) / P::KQ;
      const long e = (long)min(row, a.M - 1) * a.K + kc;
      if (MODE == 3) {
        r.a[u] = *reinterpret_cast<const float4*>(a.G.da + e);
        r.y[u] = ald4<ST == 2>(a.G.y, e);
      } else {
        r.a[u] = ald4<ST == 1>(a.A.p, e);
        if (MODE == 2)
          r.rs[u] = *reinterpret_cast<const float4*>(a.rowscale + (long)(min(row, a.M - 1) / a.rpi) * a.K + kc);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < P::NB; ++u) {
    const int idx = t + 256 * u;
    const int col = n0 + idx / P::KQ;
    const int kb = k0 + 4 * (idx % P::KQ);
    r.b[u] = *reinterpret_cast<const float4*>(a.Bt + (long)min(col, a.N - 1) * a.K + (kb < kend ? kb : kend - 4));
  }
}

// Element offset of (row, k) in an A / B tile: unpadded rows of U = BK*ESZ/16 16-B units with the
// unit index XORed by (row / (16/U)) mod U.  ds_read_b128 banks over a 256-B row in 16-lane groups
// whose 16 rows (r32 of each half-wave) cover every residue mod 16, so the 16 rows of a group land
// on 16 distinct 16-B slots for any fixed k: conflict-free.  The chunk stores (ds_write_b128 fp32 /
// ds_write_b64 bf16, banked over 128 B in 8 / 16 contiguous lanes = two rows of U = 4 units) also
// land on distinct slots.  The padded layout (pitch BK + 16 B) had conflict-free reads but 2-way
// conflicts in every store group (0.6-1.2 M conflict cycles per launch).
template <class P>
__device__ __forceinline__ int g2_off(int row, int k) {
  constexpr int EPU = 16 / P::ESZ;  // elements per 16-B unit
  constexpr int U = P::BK / EPU;    // units per row
  static_assert(U == 1 || U == 2 || U == 4 || U == 8 || U == 16, "g2_off: row of 1-16 units");
  const int f = (row / (16 / U)) & (U - 1);
  return row * P::LD + (((k / EPU) ^ f) * EPU) + k % EPU;
}

// element (row, k) of the A / B tile of LDS buffer `buf` (fp32 or bf16 elements)
template <class P>
__device__ __forceinline__ char* g2_tile(float* sm, int buf, bool b, int row, int k) {
  char* base = reinterpret_cast<char*>(sm) + (size_t)buf * (P::BM + P::BN) * P::LD * P::ESZ;
  if (b) base += (size_t)P::BM * P::LD * P::ESZ;
  return base + (size_t)g2_off<P>(row, k) * P::ESZ;
}

template <class P>
__device__ __forceinline__ void g2_put4(float* sm, int buf, bool b, int row, int k, float4 v) {
  if constexpr (P::ESZ == 2) *reinterpret_cast<uint2*>(g2_tile<P>(sm, buf, b, row, k)) = pack_bf16x4(v);
  else *reinterpret_cast<float4*>(g2_tile<P>(sm, buf, b, row, k)) = v;
}

// The activation of the A view is a compile-time constant inside the store pass (one dispatch per
// chunk instead of a branch tree per element).
template <int WM, int TM, int TN, int MODE, bool BF, int ACT>
__device__ __forceinline__ void g2_store_act(const G2Regs<WM, TM, TN, MODE, BF>& r, const Gemm2Args& a,
                                             float* sm, int buf, int m0, int n0, int k0, int kend) {
  using P = G2<WM, TM, TN, MODE, BF>;
  const int t = threadIdx.x;
  const int c4 = t % P::KQ;
  const bool kok = k0 + 4 * c4 < kend;
  InX ax = a.A;
  ax.act = ACT;
  GradX gx = a.G;
  gx.act = ACT;
#pragma unroll
  for (int u = 0; u < P::NA; ++u) {
    if (t + 256 * u >= P::BM * P::KQ) continue;
    const int rl = (t + 256 * u) / P::KQ;
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
    g2_put4<P>(sm, buf, false, rl, 4 * c4, v);
  }
#pragma unroll
  for (int u = 0; u < P::NB; ++u) {
    const int idx = t + 256 * u;
    if (idx < P::BN * P::KQ) {
      const bool ok = n0 + idx / P::KQ < a.N && k0 + 4 * (idx % P::KQ) < kend;
      g2_put4<P>(sm, buf, true, idx / P::KQ, 4 * (idx % P::KQ), ok ? r.b[u] : make_float4(0.f, 0.f, 0.f, 0.f));
    }
  }
}

template <int WM, int TM, int TN, int MODE, bool BF>
__device__ __forceinline__ void g2_store(const G2Regs<WM, TM, TN, MODE, BF>& r, const Gemm2Args& a, float* sm,
                                         int buf, int m0, int n0, int k0, int kend) {
  const int act = MODE == 0 ? 0 : MODE == 3 ? a.G.act : a.A.act;
  if (act == 1) g2_store_act<WM, TM, TN, MODE, BF, 1>(r, a, sm, buf, m0, n0, k0, kend);
  else if (act == 2) g2_store_act<WM, TM, TN, MODE, BF, 2>(r, a, sm, buf, m0, n0, k0, kend);
  else g2_store_act<WM, TM, TN, MODE, BF, 0>(r, a, sm, buf, m0, n0, k0, kend);
}

// every staging register of r used here (an empty asm reading it), so the loads that fill them are
// waited for at this point on every control path
template <int WM, int TM, int TN, int MODE, bool BF>
__device__ __forceinline__ void g2_consume(const G2Regs<WM, TM, TN, MODE, BF>& r) {
  using P = G2<WM, TM, TN, MODE, BF>;
#pragma unroll
  for (int u = 0; u < P::NA; ++u) asm volatile("" ::"v"(r.a[u].x), "v"(r.a[u].y), "v"(r.a[u].z), "v"(r.a[u].w));
#pragma unroll
  for (int u = 0; u < P::NB; ++u) asm volatile("" ::"v"(r.b[u].x), "v"(r.b[u].y), "v"(r.b[u].z), "v"(r.b[u].w));
  if constexpr (MODE == 3) {
#pragma unroll
    for (int u = 0; u < P::NA; ++u) asm volatile("" ::"v"(r.y[u].x), "v"(r.y[u].y), "v"(r.y[u].z), "v"(r.y[u].w));
  }
  if constexpr (MODE == 2) {
#pragma unroll
    for (int u = 0; u < P::NA; ++u) asm volatile("" ::"v"(r.rs[u].x), "v"(r.rs[u].y), "v"(r.rs[u].z), "v"(r.rs[u].w));
  }
}

// SK: 0 plain, 1 StatSink (BN statistics of C), 2 GradSink (BN-backward sums of a dgrad's C)
#ifndef PHX_GEMM_PF2
#define PHX_GEMM_PF2 0
#endif
#ifndef PHX_G2_XCD_TILES
#define PHX_G2_XCD_TILES 1
#endif
template <int WM, int TM, int TN, int MODE, int SK, int NS, bool BF, int ST>
__global__ __launch_bounds__(256, 2) void k_gemm2(Gemm2Group<NS> grp) {
  constexpr bool CBF = ST == 1;  // C holds bf16 activations (split-K partial slabs stay fp32)
  // two-deep prefetch for the fp32 forward GEMMs (the dgrad's gradient view and the bf16 chunks
  // hold twice the staging registers: one set keeps them clear of spills)
  constexpr bool PF2 = PHX_GEMM_PF2 && !BF && MODE != 3;
  const int zper = NS == 1 ? (int)gridDim.z : (int)gridDim.z / grp.n;
  const int seg = NS == 1 ? 0 : (int)blockIdx.z / zper;
  const int zs = (int)blockIdx.z - seg * zper;
  const Gemm2Args a = pick_seg(grp.a, seg);
  constexpr bool STATS = SK == 1;
  using P = G2<WM, TM, TN, MODE, BF>;
  constexpr int BM = P::BM, BN = P::BN, BK = P::BK;
  __shared__ __attribute__((aligned(16))) float sm[P::LDS_FLOATS];
  __shared__ float2 wst[SK ? 4 : 1][SK ? TN * 32 : 1];
  __shared__ float wcn[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int r32 = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * BN;
  const int kbeg = zs * a.kslice;
  const int kend = min(a.K, kbeg + a.kslice);
  const int ksteps = (kend - kbeg + BK - 1) / BK;
  const bool split = a.partial != nullptr;
  float* out = split ? a.partial + (long)zs * a.M * a.N : a.C;

  // running statistics of this workgroup's columns (wave wm == 0, lanes < 32)
  // (GradSink: smean = running sum dz, sm2 = running sum dz*xhat)
  float sn = 0.f, smean[TN], sm2[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) smean[j] = sm2[j] = 0.f;

  // bias of this workgroup's columns, read once (a load in the epilogue would wait behind the
  // prefetch of the next chunk: the wait counter is in order)
  float bias[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
    bias[j] = (!split && a.bias) ? a.bias[min(n0 + wn * TN * 32 + j * 32 + r32, a.N - 1)] : 0.f;

  // MODE 4 (the implicit im2col of a 3x3 conv): XCD-aware M-tile ranges — workgroup j runs on XCD
  // j % 8 (gridDim.x a multiple of 8), and each XCD sweeps a contiguous range of M tiles, so the input
  // rows a 3x3 gather shares between neighbouring tiles are read through one L2.  Every other mode
  // strides the tiles over the whole grid.  Each tile's arithmetic is the same either way.
  const bool xr = MODE == 4 && PHX_G2_XCD_TILES && gridDim.x >= 8 && (gridDim.x & 7) == 0;
  const int tstep = xr ? (int)(gridDim.x >> 3) : (int)gridDim.x;
  const int tper = xr ? (a.mtiles + 7) / 8 : a.mtiles;
  const int tbeg = xr ? (int)(blockIdx.x & 7) * tper : 0;
  const int tend = xr ? min(a.mtiles, tbeg + tper) : a.mtiles;
  int tile = tbeg + (xr ? (int)(blockIdx.x >> 3) : (int)blockIdx.x);
  if (tile < tend && ksteps > 0) {
    // PF2: two register sets, the loads of chunk s+2 are issued while chunk s is multiplied and
    // written to LDS at the end of step s+1 (two steps of latency cover; the HBM bytes a
    // workgroup keeps in flight double).  PF1: one set, loads one step ahead.
    G2Regs<WM, TM, TN, MODE, BF> rgA, rgB;
    g2_load<WM, TM, TN, MODE, BF, ST>(rgA, a, tile * BM, n0, kbeg, kend);
    g2_store<WM, TM, TN, MODE, BF>(rgA, a, sm, 0, tile * BM, n0, kbeg, kend);
    int buf = 0, kc = 0;
    // the chunk after (tile, kc): the following chunk of this tile, or the first of the next
    auto advance = [&](int t, int k, int& tn, int& kn) {
      tn = t;
      kn = k + 1;
      if (kn == ksteps) {
        tn = t + tstep;
        kn = 0;
      }
    };
    int t1, k1;
    advance(tile, 0, t1, k1);
    bool h1 = t1 < tend;
    if constexpr (PF2) g2_load<WM, TM, TN, MODE, BF, ST>(rgB, a, (h1 ? t1 : tile) * BM, n0, kbeg + (h1 ? k1 : 0) * BK, kend);
    __syncthreads();
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    // one pipeline step: L receives the loads issued now, S holds the chunk stored at its end
    auto step = [&](G2Regs<WM, TM, TN, MODE, BF>& L, G2Regs<WM, TM, TN, MODE, BF>& S) -> bool {
      int t2 = 0, k2 = 0;
      bool h2 = false;
      // (issued unconditionally — past the end a step re-loads its own chunk — so no branch joins
      // the loads and the MFMAs below do not wait for them)
      if constexpr (PF2) {
        advance(t1, k1, t2, k2);
        h2 = h1 && t2 < tend;
        g2_load<WM, TM, TN, MODE, BF, ST>(L, a, (h2 ? t2 : tile) * BM, n0, kbeg + (h2 ? k2 : kc) * BK, kend);
      } else {
        g2_load<WM, TM, TN, MODE, BF, ST>(L, a, (h1 ? t1 : tile) * BM, n0, kbeg + (h1 ? k1 : kc) * BK, kend);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the MFMAs
      // MFMAs on the staged chunk
      if constexpr (BF) {
        // lane (r32, h) feeds row / column r32 with k = 16*kk + 8*h .. +7 (one ds_read_b128 each)
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
          bf16x8_t fa[TM], fb[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i)
            fa[i] = *reinterpret_cast<const bf16x8_t*>(g2_tile<P>(sm, buf, false, wm * TM * 32 + i * 32 + r32, 16 * kk + 8 * h));
#pragma unroll
          for (int j = 0; j < TN; ++j)
            fb[j] = *reinterpret_cast<const bf16x8_t*>(g2_tile<P>(sm, buf, true, wn * TN * 32 + j * 32 + r32, 16 * kk + 8 * h));
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
      } else {
        const float* As = reinterpret_cast<const float*>(g2_tile<P>(sm, buf, false, 0, 0));
        const float* Bs = As + BM * P::LD;
        // k rows of this chunk that exist (a K of 24 or 40 leaves a last chunk of 8: its upper half
        // is zero-filled and its MFMAs would add exact zeros)
        const int kvalid = kend - (kbeg + kc * BK);
#pragma unroll
        for (int s8 = 0; s8 < BK / 8; ++s8) {
          if (s8 > 0 && 8 * s8 >= kvalid) break;  // wave-uniform
          float4 fa[TM], fb[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i)
            fa[i] = *reinterpret_cast<const float4*>(As + g2_off<P>(wm * TM * 32 + i * 32 + r32, 8 * s8 + 4 * h));
#pragma unroll
          for (int j = 0; j < TN; ++j)
            fb[j] = *reinterpret_cast<const float4*>(Bs + g2_off<P>(wn * TN * 32 + j * 32 + r32, 8 * s8 + 4 * h));
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].x, fb[j].x, acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].y, fb[j].y, acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].z, fb[j].z, acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].w, fb[j].w, acc[i][j], 0, 0, 0);
            }
        }
      }
      // The next chunk goes into the other LDS buffer before this tile's epilogue: its loads are then
      // the youngest memory operations when their wait is issued (the epilogue's stores come after it,
      // so the wait does not wait for them — in-order vmcnt), and every staging register is consumed
      // on every path, so the loop head needs no wait either (before, the compiler's conservative
      // counts made each tile wait for its own epilogue stores at the next chunk).
      if (h1) {
        g2_store<WM, TM, TN, MODE, BF>(PF2 ? S : L, a, sm, buf ^ 1, t1 * BM, n0, kbeg + k1 * BK, kend);
        g2_consume(PF2 ? S : L);
      }
      if (kc == ksteps - 1) {
        // ---- epilogue of `tile` ----
        // In the 32x32 C/D layout lane (r32, h) holds column r32, rows (e&3) + 8*(e>>2) + 4*h.
        // A wave whose 32*TM x 32*TN block lies inside C (`full`, wave-uniform) runs without
        // per-element bounds checks, and an accumulating store reads its 16 old values per tile
        // before adding (a per-element conditional load waits vmcnt(0) each time).
        const int mrow0 = tile * BM + wm * TM * 32;
        const int ncol0 = n0 + wn * TN * 32;
        const bool full = mrow0 + TM * 32 <= a.M && ncol0 + TN * 32 <= a.N;
        const bool accum = !split && a.acc;
        const bool cbf = CBF && !split;  // split-K partial slabs stay fp32
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = ncol0 + j * 32 + r32;
          const bool cok = col < a.N;
          const float bv = bias[j];
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const long cbase = (long)(mrow0 + i * 32 + 4 * h) * a.N + col;
            if (full) {
              float old[16];
              if (accum) {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                  const long ce = cbase + (long)((e & 3) + 8 * (e >> 2)) * a.N;
                  old[e] = cbf ? ald1<true>(out, ce) : out[ce];
                }
              }
#pragma unroll
              for (int e = 0; e < 16; ++e) {
                float v = acc[i][j][e] + bv;
                acc[i][j][e] = v;
                if (accum) v += old[e];
                const long ce = cbase + (long)((e & 3) + 8 * (e >> 2)) * a.N;
                if (cbf) ast1<true>(out, ce, v);
                else out[ce] = v;
                if (SK == 2) acc[i][j][e] = v;
                if (CBF && STATS) acc[i][j][e] = round_bf16(v);  // statistics of the stored values
              }
            } else {
#pragma unroll
              for (int e = 0; e < 16; ++e) {
                const int row = mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                float v = acc[i][j][e] + bv;
                acc[i][j][e] = v;
                if (cok && row < a.M) {
                  const long ce = (long)row * a.N + col;
                  if (accum) v += cbf ? ald1<true>(out, ce) : out[ce];
                  if (cbf) ast1<true>(out, ce, v);
                  else out[ce] = v;
                  if (SK == 2) acc[i][j][e] = v;
                }
                if (CBF && STATS) acc[i][j][e] = round_bf16(v);
              }
            }
          }
        }
        if constexpr (STATS) {
          // per-wave column statistics of this tile's TM*32 rows (two passes in registers), folded
          // into the wave's running statistics; the WM waves sharing these columns are merged once,
          // after the last tile (a per-tile workgroup barrier here stalled the pipeline)
          const float nw = (float)max(0, min(TM * 32, a.M - mrow0));
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int e = 0; e < 16; ++e)
                if (full || mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h < a.M) s += acc[i][j][e];
            s += __shfl_xor(s, 32);
            const float mean = nw > 0.f ? s / nw : 0.f;
            float q = 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int e = 0; e < 16; ++e)
                if (full || mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h < a.M) {
                  const float d = acc[i][j][e] - mean;
                  q = fmaf(d, d, q);
                }
            q += __shfl_xor(q, 32);
            float n_ = sn;
            chan_merge(n_, smean[j], sm2[j], nw, mean, q);
          }
          sn += nw;
        }
        if constexpr (SK == 2) {
          // BN-backward sums of the finished gradient tile (BN input y at the same elements)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * TN * 32 + j * 32 + r32;
            float s1 = 0.f, s2 = 0.f;
            {
              // BN input y at the tile's elements, loaded unconditionally from clamped addresses
              const int cc = min(col, a.N - 1);
              const float mu = a.gsk.mu[cc], rs = a.gsk.rstd[cc], sc = a.gsk.sc[cc], be = a.gsk.be[cc];
#pragma unroll
              for (int i = 0; i < TM; ++i) {
                float yv[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                  const int row = min(mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h, a.M - 1);
                  yv[e] = ald1<ST == 2>(a.gsk.y, (long)row * a.N + cc);
                }
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                  const int row = mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                  if (col < a.N && row < a.M) gs_one(acc[i][j][e], yv[e], mu, rs, sc, be, a.gsk.act, s1, s2);
                }
              }
            }
            s1 += __shfl_xor(s1, 32);
            s2 += __shfl_xor(s2, 32);
            smean[j] += s1;
            sm2[j] += s2;
          }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
      }
      if (!h1) return false;
      __syncthreads();
      buf ^= 1;
      tile = t1;
      kc = k1;
      if constexpr (PF2) {
        t1 = t2;
        k1 = k2;
        h1 = h2;
      } else {
        advance(tile, kc, t1, k1);
        h1 = t1 < tend;
      }
      return true;
    };
    if constexpr (PF2) {
      while (step(rgA, rgB) && step(rgB, rgA)) {
      }
    } else {
      while (step(rgA, rgA)) {
      }
    }
  }
  if constexpr (SK != 0) {
    // merge the running statistics / sums of the WM waves that share each column (fixed order)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      if (h == 0) wst[wave][j * 32 + r32] = make_float2(smean[j], sm2[j]);
    if (lane == 0) wcn[wave] = sn;
    __syncthreads();
    if (wm == 0 && h == 0) {
      float ntot = 0.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * TN * 32 + j * 32 + r32;
        float tn = 0.f, tm = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          const int wv = wn * WM + w;
          const float2 v = wst[wv][j * 32 + r32];
          if constexpr (STATS) {
            chan_merge(tn, tm, t2, wcn[wv], v.x, v.y);
          } else {
            tm += v.x;
            t2 += v.y;
          }
        }
        ntot = tn;
        if (col < a.N) {
          if constexpr (STATS) sink_put(a.sink, blockIdx.x, col, tn, tm, t2);
          else gsink_put(a.gsk, blockIdx.x, col, tm, t2);
        }
      }
      if constexpr (STATS)
        if (blockIdx.y == 0 && wn == 0 && lane == 0) sink_cnt(a.sink, blockIdx.x, ntot);
    }
  }
}

// ---- A-resident variant (k_gemm2r) ---------------------------------------------------------
// The workgroup's M tile of A' — its view (BN + activation, SE scale, BN backward) applied once per
// element — stays in LDS chunk by chunk while the workgroup sweeps every N tile over it, instead of
// each N tile re-loading A and re-applying the view (exp / rcp per element, which serialises with the
// fp32 MFMAs and dominates the bf16 ones).  Grid (gx, 1, segments), persistent along M; B chunks
// double-buffered behind the resident A tile (dynamic LDS: ksteps * BM * BK + 2 * BN * BK elements).
// One pipeline over the (M tile, N tile, k chunk) steps: the loads of step s+1 (A only while the
// first N tile of an M tile is swept) are in flight while step s multiplies.  The statistics /
// BN-backward sums go out per (M tile, wave row): partial row tile * WM + wm of the sink (no
// cross-wave merge; the finalize folds them in a fixed order).  No split-K; ksteps >= 2 (the next M
// tile's chunk 0 is written while the last chunk is read).  Few M tiles: blockIdx.y splits the N
// tiles into runs of Gemm2Args::kslice (unused without split-K) N tiles, one run per workgroup.
template <class P>
__device__ __forceinline__ void g2r_put(char* base, int row, int k, float4 v) {
  char* p = base + (size_t)g2_off<P>(row, k) * P::ESZ;
  if constexpr (P::ESZ == 2) *reinterpret_cast<uint2*>(p) = pack_bf16x4(v);
  else *reinterpret_cast<float4*>(p) = v;
}

template <int WM, int TM, int TN, int MODE, bool BF, int ST>
__device__ __forceinline__ void g2r_load_a(G2Regs<WM, TM, TN, MODE, BF>& r, const Gemm2Args& a, int m0, int k0) {
  using P = G2<WM, TM, TN, MODE, BF>;
  const int t = threadIdx.x;
  const int kk = k0 + 4 * (t % P::KQ);
  const int kc = kk < a.K ? kk : a.K - 4;
  if (MODE == 1 || MODE == 2) r.ck = inx_chan4(a.A, kc);
  if (MODE == 3) r.gk = gx_chan4(a.G, kc);
#pragma unroll
  for (int u = 0; u < P::NA; ++u) {
    const int row = min(m0 + (t + 256 * u) / P::KQ, a.M - 1);
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

template <int WM, int TM, int TN, int MODE, bool BF>
__device__ __forceinline__ void g2r_load_b(G2Regs<WM, TM, TN, MODE, BF>& r, const Gemm2Args& a, int n0, int k0) {
  using P = G2<WM, TM, TN, MODE, BF>;
#pragma unroll
  for (int u = 0; u < P::NB; ++u) {
    const int idx = threadIdx.x + 256 * u;
    const int kb = k0 + 4 * (idx % P::KQ);
    r.b[u] = *reinterpret_cast<const float4*>(a.Bt + (long)min(n0 + idx / P::KQ, a.N - 1) * a.K +
                                              (kb < a.K ? kb : a.K - 4));
  }
}

template <int WM, int TM, int TN, int MODE, bool BF, int ACT>
__device__ __forceinline__ void g2r_store_a_act(const G2Regs<WM, TM, TN, MODE, BF>& r, const Gemm2Args& a, char* base,
                                                int m0, int k0) {
  using P = G2<WM, TM, TN, MODE, BF>;
  const int t = threadIdx.x;
  const int c4 = t % P::KQ;
  const bool kok = k0 + 4 * c4 < a.K;
  InX ax = a.A;
  ax.act = ACT;
  GradX gx = a.G;
  gx.act = ACT;
#pragma unroll
  for (int u = 0; u < P::NA; ++u) {
    if (t + 256 * u >= P::BM * P::KQ) continue;
    const int rl = (t + 256 * u) / P::KQ;
    float4 v = r.a[u];
    if (kok && m0 + rl < a.M) {
      if (MODE == 1 || MODE == 2) v = inx_apply4(ax, r.ck, v);
      if (MODE == 2) {
        v.x *= r.rs[u].x; v.y *= r.rs[u].y; v.z *= r.rs[u].z; v.w *= r.rs[u].w;
      }
      if (MODE == 3) v = gx_apply4(gx, r.gk, v, r.y[u]);
    } else {
      v = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    g2r_put<P>(base, rl, 4 * c4, v);
  }
}

template <int WM, int TM, int TN, int MODE, bool BF>
__device__ __forceinline__ void g2r_store_a(const G2Regs<WM, TM, TN, MODE, BF>& r, const Gemm2Args& a, char* base,
                                            int m0, int k0) {
  const int act = MODE == 0 ? 0 : MODE == 3 ? a.G.act : a.A.act;
  if (act == 1) g2r_store_a_act<WM, TM, TN, MODE, BF, 1>(r, a, base, m0, k0);
  else if (act == 2) g2r_store_a_act<WM, TM, TN, MODE, BF, 2>(r, a, base, m0, k0);
  else g2r_store_a_act<WM, TM, TN, MODE, BF, 0>(r, a, base, m0, k0);
}

template <int WM, int TM, int TN, int MODE, bool BF>
__device__ __forceinline__ void g2r_store_b(const G2Regs<WM, TM, TN, MODE, BF>& r, const Gemm2Args& a, char* base,
                                            int n0, int k0) {
  using P = G2<WM, TM, TN, MODE, BF>;
#pragma unroll
  for (int u = 0; u < P::NB; ++u) {
    const int idx = threadIdx.x + 256 * u;
    if (idx < P::BN * P::KQ) {
      const bool ok = n0 + idx / P::KQ < a.N && k0 + 4 * (idx % P::KQ) < a.K;
      g2r_put<P>(base, idx / P::KQ, 4 * (idx % P::KQ), ok ? r.b[u] : make_float4(0.f, 0.f, 0.f, 0.f));
    }
  }
}

// dynamic LDS bytes of k_gemm2r for K
template <int WM, int TM, int TN, bool BF>
constexpr size_t g2r_lds_bytes(int K) {
  using P = G2<WM, TM, TN, 1, BF>;
  return ((size_t)((K + P::BK - 1) / P::BK) * P::BM + 2 * P::BN) * P::LD * P::ESZ;
}

template <int WM, int TM, int TN, int MODE, int SK, int NS, bool BF, int ST>
__global__ __launch_bounds__(256, 2) void k_gemm2r(Gemm2Group<NS> grp) {
  constexpr bool CBF = ST == 1;
  const Gemm2Args a = pick_seg(grp.a, NS == 1 ? 0 : (int)blockIdx.z);
  using P = G2<WM, TM, TN, MODE, BF>;
  constexpr int BM = P::BM, BN = P::BN, BK = P::BK;
  constexpr size_t ACH = (size_t)BM * P::LD * P::ESZ, BCH = (size_t)BN * P::LD * P::ESZ;
  extern __shared__ __attribute__((aligned(16))) float g2r_sm[];
  const int ksteps = (a.K + BK - 1) / BK;
  const int nt0 = (int)blockIdx.y * a.kslice;                        // this workgroup's N tiles
  const int nte = min((a.N + BN - 1) / BN, nt0 + a.kslice);
  char* const Ares = reinterpret_cast<char*>(g2r_sm);
  char* const Bb = Ares + (size_t)ksteps * ACH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int r32 = lane & 31, h = lane >> 5;
  int tile = blockIdx.x;
  if (tile >= a.mtiles || nt0 >= nte) return;  // workgroup-uniform, before any barrier
  G2Regs<WM, TM, TN, MODE, BF> rg;
  g2r_load_a<WM, TM, TN, MODE, BF, ST>(rg, a, tile * BM, 0);
  g2r_load_b(rg, a, nt0 * BN, 0);
  g2r_store_a(rg, a, Ares, tile * BM, 0);
  g2r_store_b(rg, a, Bb, nt0 * BN, 0);
  int buf = 0, nt = nt0, kc = 0;
  auto advance = [&](int t, int n, int k, int& t2, int& n2, int& k2) {
    t2 = t;
    n2 = n;
    k2 = k + 1;
    if (k2 == ksteps) {
      k2 = 0;
      if (++n2 == nte) {
        n2 = nt0;
        t2 = t + gridDim.x;
      }
    }
  };
  // the loads of step (tl, nl, kl) into R (A only on the first N tile of a run)
  auto load = [&](G2Regs<WM, TM, TN, MODE, BF>& R, int tl, int nl, int kl) {
    if (nl == nt0) g2r_load_a<WM, TM, TN, MODE, BF, ST>(R, a, tl * BM, kl * BK);
    g2r_load_b(R, a, nl * BN, kl * BK);
  };
  int t1, n1, k1;
  advance(tile, nt0, 0, t1, n1, k1);
  bool h1 = t1 < a.mtiles;
  auto load_bias = [&](float (&bv)[TN], int n0) {
#pragma unroll
    for (int j = 0; j < TN; ++j) bv[j] = a.bias ? a.bias[min(n0 + wn * TN * 32 + j * 32 + r32, a.N - 1)] : 0.f;
  };
  float bias[TN];
  load_bias(bias, nt0 * BN);
  __syncthreads();
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // one pipeline step: the loads of the next step go out first (unconditionally: past the end a
  // step re-loads its own chunk), then this step's MFMAs (and epilogue), then the next chunk's store.
  // (A two-deep register prefetch measured no faster on C2 / C4: 28.60 vs 28.56 ms on C4.)
  auto step = [&]() -> bool {
    load(rg, h1 ? t1 : tile, h1 ? n1 : nt, h1 ? k1 : kc);
    __builtin_amdgcn_sched_barrier(0);
      // MFMAs: A chunk kc of the resident tile, B chunk of buffer buf
      {
        char* const Ab = Ares + (size_t)kc * ACH;
        char* const Bc = Bb + (size_t)buf * BCH;
        if constexpr (BF) {
  #pragma unroll
          for (int kk = 0; kk < BK / 16; ++kk) {
            bf16x8_t fa[TM], fb[TN];
  #pragma unroll
            for (int i = 0; i < TM; ++i)
              fa[i] = *reinterpret_cast<const bf16x8_t*>(Ab + (size_t)g2_off<P>(wm * TM * 32 + i * 32 + r32, 16 * kk + 8 * h) * 2);
  #pragma unroll
            for (int j = 0; j < TN; ++j)
              fb[j] = *reinterpret_cast<const bf16x8_t*>(Bc + (size_t)g2_off<P>(wn * TN * 32 + j * 32 + r32, 16 * kk + 8 * h) * 2);
  #pragma unroll
            for (int i = 0; i < TM; ++i)
  #pragma unroll
              for (int j = 0; j < TN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
          }
        } else {
          const float* As = reinterpret_cast<const float*>(Ab);
          const float* Bs = reinterpret_cast<const float*>(Bc);
          const int kvalid = a.K - kc * BK;
  #pragma unroll
          for (int s8 = 0; s8 < BK / 8; ++s8) {
            if (s8 > 0 && 8 * s8 >= kvalid) break;  // wave-uniform
            float4 fa[TM], fb[TN];
  #pragma unroll
            for (int i = 0; i < TM; ++i)
              fa[i] = *reinterpret_cast<const float4*>(As + g2_off<P>(wm * TM * 32 + i * 32 + r32, 8 * s8 + 4 * h));
  #pragma unroll
            for (int j = 0; j < TN; ++j)
              fb[j] = *reinterpret_cast<const float4*>(Bs + g2_off<P>(wn * TN * 32 + j * 32 + r32, 8 * s8 + 4 * h));
  #pragma unroll
            for (int i = 0; i < TM; ++i)
  #pragma unroll
              for (int j = 0; j < TN; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].x, fb[j].x, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].y, fb[j].y, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].z, fb[j].z, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].w, fb[j].w, acc[i][j], 0, 0, 0);
              }
          }
        }
      }
      if (kc == ksteps - 1) {
        // ---- epilogue of (tile, nt): lane (r32, h) holds column r32, rows (e&3) + 8*(e>>2) + 4*h ----
        const int mrow0 = tile * BM + wm * TM * 32;
        const int ncol0 = nt * BN + wn * TN * 32;
        const bool full = mrow0 + TM * 32 <= a.M && ncol0 + TN * 32 <= a.N;
        const bool accum = a.acc != 0;
  #pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = ncol0 + j * 32 + r32;
          const bool cok = col < a.N;
          const float bv = bias[j];
  #pragma unroll
          for (int i = 0; i < TM; ++i) {
            if (full) {
              const long cbase = (long)(mrow0 + i * 32 + 4 * h) * a.N + col;
              float old[16];
              if (accum) {
  #pragma unroll
                for (int e = 0; e < 16; ++e) {
                  const long ce = cbase + (long)((e & 3) + 8 * (e >> 2)) * a.N;
                  old[e] = CBF ? ald1<true>(a.C, ce) : a.C[ce];
                }
              }
  #pragma unroll
              for (int e = 0; e < 16; ++e) {
                float v = acc[i][j][e] + bv;
                acc[i][j][e] = v;
                if (accum) v += old[e];
                const long ce = cbase + (long)((e & 3) + 8 * (e >> 2)) * a.N;
                if (CBF) ast1<true>(a.C, ce, v);
                else a.C[ce] = v;
                if (SK == 2) acc[i][j][e] = v;
                if (CBF && SK == 1) acc[i][j][e] = round_bf16(v);  // statistics of the stored values
              }
            } else {
  #pragma unroll
              for (int e = 0; e < 16; ++e) {
                const int row = mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                float v = acc[i][j][e] + bv;
                acc[i][j][e] = v;
                if (cok && row < a.M) {
                  const long ce = (long)row * a.N + col;
                  if (accum) v += CBF ? ald1<true>(a.C, ce) : a.C[ce];
                  if (CBF) ast1<true>(a.C, ce, v);
                  else a.C[ce] = v;
                  if (SK == 2) acc[i][j][e] = v;
                }
                if (CBF && SK == 1) acc[i][j][e] = round_bf16(v);
              }
            }
          }
        }
        const long prow = (long)tile * WM + wm;  // this wave's partial row of the sink
        if constexpr (SK == 1) {
          const float nw = (float)max(0, min(TM * 32, a.M - mrow0));
  #pragma unroll
          for (int j = 0; j < TN; ++j) {
            float s = 0.f;
  #pragma unroll
            for (int i = 0; i < TM; ++i)
  #pragma unroll
              for (int e = 0; e < 16; ++e)
                if (full || mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h < a.M) s += acc[i][j][e];
            s += __shfl_xor(s, 32);
            const float mean = nw > 0.f ? s / nw : 0.f;
            float q = 0.f;
  #pragma unroll
            for (int i = 0; i < TM; ++i)
  #pragma unroll
              for (int e = 0; e < 16; ++e)
                if (full || mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h < a.M) {
                  const float d = acc[i][j][e] - mean;
                  q = fmaf(d, d, q);
                }
            q += __shfl_xor(q, 32);
            const int col = ncol0 + j * 32 + r32;
            if (h == 0 && col < a.N) sink_put(a.sink, prow, col, nw, mean, q);
          }
          if (nt == nt0 && blockIdx.y == 0 && wn == 0 && lane == 0) sink_cnt(a.sink, prow, nw);
        }
        if constexpr (SK == 2) {
  #pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = ncol0 + j * 32 + r32;
            const int cc = min(col, a.N - 1);
            const float mu = a.gsk.mu[cc], rs = a.gsk.rstd[cc], sc = a.gsk.sc[cc], be = a.gsk.be[cc];
            float s1 = 0.f, s2 = 0.f;
  #pragma unroll
            for (int i = 0; i < TM; ++i) {
              float yv[16];
  #pragma unroll
              for (int e = 0; e < 16; ++e) {
                const int row = min(mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h, a.M - 1);
                yv[e] = ald1<ST == 2>(a.gsk.y, (long)row * a.N + cc);
              }
  #pragma unroll
              for (int e = 0; e < 16; ++e) {
                const int row = mrow0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (col < a.N && row < a.M) gs_one(acc[i][j][e], yv[e], mu, rs, sc, be, a.gsk.act, s1, s2);
              }
            }
            s1 += __shfl_xor(s1, 32);
            s2 += __shfl_xor(s2, 32);
            if (h == 0 && col < a.N) gsink_put(a.gsk, prow, col, s1, s2);
          }
        }
  #pragma unroll
        for (int i = 0; i < TM; ++i)
  #pragma unroll
          for (int j = 0; j < TN; ++j)
  #pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
      }
    if (!h1) return false;
    if (n1 == nt0) g2r_store_a(rg, a, Ares + (size_t)k1 * ACH, t1 * BM, k1 * BK);
    g2r_store_b(rg, a, Bb + (size_t)(buf ^ 1) * BCH, n1 * BN, k1 * BK);
    if (k1 == 0) load_bias(bias, n1 * BN);  // the epilogue above has used this (tile, N tile)'s
    __syncthreads();
    buf ^= 1;
    tile = t1;
    nt = n1;
    kc = k1;
    advance(tile, nt, kc, t1, n1, k1);
    h1 = t1 < a.mtiles;
    return true;
  };
  while (step()) {
  }
}

// st: activation storage variant (ST of k_gemm2).  A bf16 context stores bf16 activations, so its
// forward modes run ST 1 and its gradient views ST 2; an fp32 context always ST 0.
template <int WM, int TM, int TN, int MODE, int SK, int NS>
static void g2_go(dim3 g, hipStream_t s, const Gemm2Group<NS>& a, bool bf, int st) {
  if constexpr (MODE == 4) {  // the implicit im2col: fp32 only
    if (bf || st) throw std::logic_error("gemm2: the implicit im2col runs in fp32");
    PHX_TLAUNCH((k_gemm2<WM, TM, TN, 4, 0, NS, false, 0>), g, dim3(256), 0, s, a);
    return;
  }
  if (!bf) {
    if (st) throw std::logic_error("gemm2: bf16 storage needs the bf16 compute type");
    PHX_TLAUNCH((k_gemm2<WM, TM, TN, MODE, SK, NS, false, 0>), g, dim3(256), 0, s, a);
    return;
  }
  constexpr bool fwd_only = MODE == 1 || MODE == 2 || SK == 1;
  constexpr bool dgrad_only = MODE == 3 || SK == 2;
  if constexpr (fwd_only) {
    if (st != 1) throw std::logic_error("gemm2: bf16 forward without bf16 activations");
    PHX_TLAUNCH((k_gemm2<WM, TM, TN, MODE, SK, NS, true, 1>), g, dim3(256), 0, s, a);
  } else if constexpr (dgrad_only) {
    if (st != 2) throw std::logic_error("gemm2: bf16 gradient view without bf16 activations");
    PHX_TLAUNCH((k_gemm2<WM, TM, TN, MODE, SK, NS, true, 2>), g, dim3(256), 0, s, a);
  } else {  // raw A: a forward activation (ST 1) or a plain gradient (ST 0)
    if (st == 1) PHX_TLAUNCH((k_gemm2<WM, TM, TN, MODE, SK, NS, true, 1>), g, dim3(256), 0, s, a);
    else if (st == 0) PHX_TLAUNCH((k_gemm2<WM, TM, TN, MODE, SK, NS, true, 0>), g, dim3(256), 0, s, a);
    else throw std::logic_error("gemm2: raw dgrad with a bf16 y");
  }
}
// The A-resident kernel of a tile (k_gemm2r), storage variants as g2_go; lds = its dynamic LDS bytes
template <int WM, int TM, int TN>
constexpr bool g2r_cfg() {
  return (WM == 2 && TM == 2 && TN == 2) || (WM == 4 && TM == 1 && (TN == 3 || TN == 5)) || (WM == 2 && TM == 1 && TN == 2);
}

template <auto KFN>
static void g2r_attr() {
  static const bool ok = [] {
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(KFN)) != hipSuccess) return false;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(KFN), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(160 * 1024 - fa.sharedSizeBytes)) == hipSuccess;
  }();
  if (!ok) throw std::runtime_error("gemm2r: cannot raise the dynamic LDS limit");
}

template <int WM, int TM, int TN, int MODE, int SK, int NS>
static void g2r_go(dim3 g, hipStream_t s, const Gemm2Group<NS>& a, bool bf, int st, size_t lds) {
  if constexpr (MODE == 4) {
    throw std::logic_error("gemm2r: no implicit im2col");
  } else if (!bf) {
    if (st) throw std::logic_error("gemm2r: bf16 storage needs the bf16 compute type");
    g2r_attr<&k_gemm2r<WM, TM, TN, MODE, SK, NS, false, 0>>();
    PHX_TLAUNCH((k_gemm2r<WM, TM, TN, MODE, SK, NS, false, 0>), g, dim3(256), lds, s, a);
  } else {
    constexpr bool fwd_only = MODE == 1 || MODE == 2 || SK == 1;
    constexpr bool dgrad_only = MODE == 3 || SK == 2;
    if constexpr (fwd_only) {
      if (st != 1) throw std::logic_error("gemm2r: bf16 forward without bf16 activations");
      g2r_attr<&k_gemm2r<WM, TM, TN, MODE, SK, NS, true, 1>>();
      PHX_TLAUNCH((k_gemm2r<WM, TM, TN, MODE, SK, NS, true, 1>), g, dim3(256), lds, s, a);
    } else if constexpr (dgrad_only) {
      if (st != 2) throw std::logic_error("gemm2r: bf16 gradient view without bf16 activations");
      g2r_attr<&k_gemm2r<WM, TM, TN, MODE, SK, NS, true, 2>>();
      PHX_TLAUNCH((k_gemm2r<WM, TM, TN, MODE, SK, NS, true, 2>), g, dim3(256), lds, s, a);
    } else {
      if (st == 1) {
        g2r_attr<&k_gemm2r<WM, TM, TN, MODE, SK, NS, true, 1>>();
        PHX_TLAUNCH((k_gemm2r<WM, TM, TN, MODE, SK, NS, true, 1>), g, dim3(256), lds, s, a);
      } else if (st == 0) {
        g2r_attr<&k_gemm2r<WM, TM, TN, MODE, SK, NS, true, 0>>();
        PHX_TLAUNCH((k_gemm2r<WM, TM, TN, MODE, SK, NS, true, 0>), g, dim3(256), lds, s, a);
      } else {
        throw std::logic_error("gemm2r: raw dgrad with a bf16 y");
      }
    }
  }
}

template <int WM, int TM, int TN, int NS>
static void g2r_launch(int mode, int sk, dim3 g, hipStream_t s, const Gemm2Group<NS>& a, bool bf, int st, size_t lds) {
  if constexpr (!g2r_cfg<WM, TM, TN>()) {
    throw std::logic_error("gemm2r: no A-resident kernel for this tile");
  } else {
    switch (mode) {
      case 0:
        if (sk == 1) g2r_go<WM, TM, TN, 0, 1, NS>(g, s, a, bf, st, lds);
        else if (sk == 2) g2r_go<WM, TM, TN, 0, 2, NS>(g, s, a, bf, st, lds);
        else g2r_go<WM, TM, TN, 0, 0, NS>(g, s, a, bf, st, lds);
        break;
      case 1:
        sk == 1 ? g2r_go<WM, TM, TN, 1, 1, NS>(g, s, a, bf, st, lds) : g2r_go<WM, TM, TN, 1, 0, NS>(g, s, a, bf, st, lds);
        break;
      case 2:
        sk == 1 ? g2r_go<WM, TM, TN, 2, 1, NS>(g, s, a, bf, st, lds) : g2r_go<WM, TM, TN, 2, 0, NS>(g, s, a, bf, st, lds);
        break;
      case 3:
        sk == 2 ? g2r_go<WM, TM, TN, 3, 2, NS>(g, s, a, bf, st, lds) : g2r_go<WM, TM, TN, 3, 0, NS>(g, s, a, bf, st, lds);
        break;
      default:
        throw std::logic_error("gemm2r: no implicit im2col");
    }
  }
}

// sk: 1 forward statistics (modes 0-2), 2 BN-backward sums (dgrad modes 0, 3).  Each (WM, TM, TN, NS)
// is instantiated in its own translation unit (kernels_gemm_cfg*.hip) so the variants compile in
// parallel.
// res_lds > 0: the A-resident kernel (k_gemm2r) with that much dynamic LDS.
template <int WM, int TM, int TN, int NS>
void g2_launch_cfg(int mode, int sk, dim3 g, hipStream_t s, const Gemm2Group<NS>& a, bool bf, int st, size_t res_lds);

#define PHX_G2_DEFINE_LAUNCH_CFG                                                                                 \
  template <int WM, int TM, int TN, int NS>                                                                     \
  void g2_launch_cfg(int mode, int sk, dim3 g, hipStream_t s, const Gemm2Group<NS>& a, bool bf, int st,  \
                     size_t res_lds) {                                                                          \
    if (res_lds) return g2r_launch<WM, TM, TN, NS>(mode, sk, g, s, a, bf, st, res_lds);                       \
    switch (mode) {                                                                                             \
      case 0:                                                                                                   \
        if (sk == 1) g2_go<WM, TM, TN, 0, 1, NS>(g, s, a, bf, st);                                          \
        else if (sk == 2) g2_go<WM, TM, TN, 0, 2, NS>(g, s, a, bf, st);                                     \
        else g2_go<WM, TM, TN, 0, 0, NS>(g, s, a, bf, st);                                                  \
        break;                                                                                                  \
      case 1:                                                                                                   \
        sk == 1 ? g2_go<WM, TM, TN, 1, 1, NS>(g, s, a, bf, st) : g2_go<WM, TM, TN, 1, 0, NS>(g, s, a, bf, st); \
        break;                                                                                                  \
      case 2:                                                                                                   \
        sk == 1 ? g2_go<WM, TM, TN, 2, 1, NS>(g, s, a, bf, st) : g2_go<WM, TM, TN, 2, 0, NS>(g, s, a, bf, st); \
        break;                                                                                                  \
      case 4:                                                                                                   \
        if constexpr (NS == 1) g2_go<WM, TM, TN, 4, 0, NS>(g, s, a, bf, st);                                  \
        else throw std::logic_error("gemm2: no grouped implicit im2col");                                      \
        break;                                                                                                  \
      default:                                                                                                  \
        sk == 2 ? g2_go<WM, TM, TN, 3, 2, NS>(g, s, a, bf, st) : g2_go<WM, TM, TN, 3, 0, NS>(g, s, a, bf, st); \
        break;                                                                                                  \
    }                                                                                                           \
  }

}  // namespace phx
