// kernels_gemm.hip — the 1x1-convolution GEMM of the victim forward and data-gradient on the
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
//  * Grouped launch: up to kMaxSeg GEMMs with the same B operand, N and K but their own A, C, M and
//    statistics sinks (the per-level members of a class/box-head conv, whose weights are shared
//    across pyramid levels) run as one grid; blockIdx.z = segment * splits + split.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "gemm2_kernel.hpp"

namespace phx {

// ---- host --------------------------------------------------------------------------------
struct G2Cfg {
  int wm, tm, tn;
  int bm() const { return wm * tm * 32; }
  int bn() const { return (4 / wm) * tn * 32; }
};

// Wide outputs: a column tile that divides N wastes no matrix-core columns (tools/gemm_bench sweeps,
// BN + swish view: N = 672 and 192 on 96-column tiles, N = 320 on 160-column tiles); the
// class-head predict conv (N = 810, K = 64: store-heavy) runs fastest on 64x128 tiles.
static G2Cfg g2_pick(int N, int K, bool bf16) {
  if (N <= 32) return {4, 1, 1};
  if (N <= 64) return {4, 1, 2};
  if (N <= 96) return {4, 1, 3};
  if (N <= 128) return {2, 2, 2};
  if (N <= 160) return {4, 1, 5};
  static const bool waste = [] {
    const char* e = std::getenv("PHX_G2PICK");
    return !(e && e[0] == '0');
  }();
  if (waste && !bf16) {  // fp32 only: the bf16 tiles measured slightly slower with it (D4 C4)
    if (N % 128 != 0 && N % 96 == 0) return {4, 1, 3};
    if (N % 128 != 0 && N % 160 == 0) return {4, 1, 5};
    if (N >= 512 && K <= 64) return {2, 1, 2};
  }
  return {2, 2, 2};
}

// configuration forced by tools/gemm_bench sweeps (never set by the product)
static int g_force[4] = {0, 0, 0, 0};
void gemm2_force_cfg(int wm, int tm, int tn, int splits) {
  g_force[0] = wm; g_force[1] = tm; g_force[2] = tn; g_force[3] = splits;
}
static int g_force_wsk[2] = {0, 0};
void gemm2_force_wsk(int tm, int tn) {
  g_force_wsk[0] = tm; g_force_wsk[1] = tn;
}

// Wave-split-K tile (k_gemm2k) for a shape k_gemm2 would split across workgroups: the largest
// per-workgroup MFMA work that still spreads over the chip.  Cost model in units of one 32x32 MFMA
// tile's chunk work per wave: a CU runs its cdiv(wgs, 256) workgroups' TM*TN tiles plus a fixed
// per-chunk overhead of about two tiles (load wait, view, LDS store, barrier) each.
static int wsk_pick(int M, int N) {
  static const int cand[5][2] = {{2, 2}, {1, 3}, {2, 1}, {1, 2}, {1, 1}};
  int best = 0;
  long bc = 0;
  for (auto& c : cand) {
    const long wgs = (long)cdiv(M, 32 * c[0]) * cdiv(N, 32 * c[1]);
    const long cost = (long)cdiv(wgs, 256) * (c[0] * c[1] + 2);
    if (!best || cost < bc) {
      best = c[0] * 10 + c[1];
      bc = cost;
    }
  }
  return best;
}

Gemm2Plan plan_gemm2(int M, int N, int K, int target_wgs, bool bf16, bool allow_res, bool allow_wsk) {
  Gemm2Plan p;
  G2Cfg c = g2_pick(N, K, bf16);
  if (g_force[0]) {
    p.wm = g_force[0]; p.tm = g_force[1]; p.tn = g_force[2];
    c = G2Cfg{p.wm, p.tm, p.tn};
    p.mtiles = cdiv(M, c.bm());
    p.gy = cdiv(N, c.bn());
    const int bk = bf16 ? PHX_GEMM_BK_BF16 : PHX_GEMM_BK_F32;
    p.splits = std::max(1, g_force[3]);
    p.kslice = ((K + p.splits - 1) / p.splits + bk - 1) / bk * bk;
    p.splits = (K + p.kslice - 1) / p.kslice;
    const long want = std::max<long>(1, target_wgs / ((long)p.gy * p.splits));
    p.gx = (int)std::min<long>(p.mtiles, want);
    if (p.gy > 1 && p.gx > 8) p.gx = p.gx / 8 * 8;
    p.P = p.gx;
    p.res_lds = 0;
    return p;
  }
  // few 128x128 tiles (small M, wide N, no split-K): 64-row tiles double the workgroups so
  // every CU gets MFMA work
  static const bool half_rows = [] {
    const char* e = std::getenv("PHX_G212");
    return !(e && e[0] == '0');
  }();
  if (half_rows) {
    auto wgs = [&](const G2Cfg& q) { return (long)cdiv(M, q.bm()) * cdiv(N, q.bn()); };
    static const bool tiles_first = [] {
      const char* e = std::getenv("PHX_TILES_FIRST");
      return e && e[0] == '1';
    }();
    const bool splits = !tiles_first && wgs(c) < 256 && K >= 256;  // split-K covers these
    if (!splits) {
      if (c.wm == 4 && c.tm == 1 && c.tn == 2 && wgs(c) < 512) c = G2Cfg{2, 1, 1};
      if (c.wm == 2 && c.tm == 2 && c.tn == 2 && wgs(c) < 512) c = G2Cfg{2, 1, 2};
      if (c.wm == 2 && c.tm == 1 && c.tn == 2 && wgs(c) < 512) c = G2Cfg{1, 1, 1};
    }
  }
  p.wm = c.wm; p.tm = c.tm; p.tn = c.tn;
  p.mtiles = cdiv(M, c.bm());
  p.gy = cdiv(N, c.bn());
  const long tiles = (long)p.mtiles * p.gy;
  p.splits = 1;
  static const long split_below = [] {
    const char* e = std::getenv("PHX_SPLIT_TILES");
    return e ? std::atol(e) : 256L;
  }();
  if (tiles < split_below && K >= 256)
    p.splits = std::max(1, std::min<int>((int)((2 * split_below + tiles - 1) / tiles), K / 128));
  const int bk = bf16 ? PHX_GEMM_BK_BF16 : PHX_GEMM_BK_F32;  // K chunk of the kernel variant
  p.kslice = ((K + p.splits - 1) / p.splits + bk - 1) / bk * bk;
  p.splits = (K + p.kslice - 1) / p.kslice;
  // deep K over few tiles: split K across the waves of a workgroup instead (k_gemm2k; PHX_GEMM_WSK=0
  // keeps the cross-workgroup split)
  static const bool wsk_on = [] {
    const char* e = std::getenv("PHX_GEMM_WSK");
    return !(e && e[0] == '0');
  }();
  // the bf16 compute type takes k_gemm2k too (C4 27.80 -> 27.52-27.59 ms; PHX_GEMM_WSK_BF16=0 keeps the
  // split).  Its first affected layer differs from the split kernels' in 8e-5 of the stored bf16
  // values, each by one quantum (fp32 summation order); deeper, both builds are draws of the same
  // bf16 storage noise, equally far from the emulation oracle ("bf16 wave-split-K,
  // diagnosed"; scripts/diag_bf16_wsk_layers.py)
  static const bool wsk_bf16 = [] {
    const char* e = std::getenv("PHX_GEMM_WSK_BF16");
    return !(e && e[0] == '0');
  }();
  // bf16: the A view (fp32 VALU, once per N tile) outweighs the cheap bf16 MFMAs, so a split tile that
  // spans all of N exactly (one view pass: N = 160 on 128x160) stays faster than the narrower
  // wave-split tiles (tools/gemm_bench GEMM_WSK sweeps, D4 shapes)
  const bool bf16_keep = bf16 && p.gy == 1 && N % c.bn() == 0;
  const bool wsk_forced = g_force_wsk[0] > 0;
  // (not for the implicit im2col, nor for the U-Net's explicit column matrices that must match it
  // bit for bit: there the inference-mode U-Net amplifies a changed summation order past
  // test_eval_step_matches_oracle's bound, for 0.03 ms of C5)
  // also the few-tile shapes k_gemm2 runs unsplit on under 128 workgroups (the BiFPN's P5-P7 level
  // convs, K 64: 6.1 -> 3.8 us at M 4096, tools/gemm_bench GEMM_WSK; C2 11.55 -> 11.47 ms).  Round 5
  // kept it off for a metric-row bound that was tighter than the per-image bound it sums (DESIGN.md
  // section 5); with check_metric_row's bounds derived from the per-image ones it is on (PHX_GEMM_WSK_SMALL=0
  // turns it off)
  static const bool wsk_small = [] {
    const char* e = std::getenv("PHX_GEMM_WSK_SMALL");
    return !(e && e[0] == '0');
  }();
  const bool few = wsk_small && p.splits == 1 && (long)p.mtiles * p.gy < 128;
  if (allow_res && allow_wsk && g_force_wsk[0] >= 0 &&
      (wsk_forced || (wsk_on && (p.splits > 1 || few) && (!bf16 || (wsk_bf16 && !bf16_keep))))) {
    p.wsk = wsk_forced ? g_force_wsk[0] * 10 + g_force_wsk[1] : wsk_pick(M, N);
    p.tm = p.wsk / 10;
    p.tn = p.wsk % 10;
    p.wm = 0;
    p.mtiles = cdiv(M, 32 * p.tm);
    p.gx = p.mtiles;
    p.gy = cdiv(N, 32 * p.tn);
    p.splits = 1;
    p.kslice = K;
    p.P = p.mtiles * p.tm;
    p.res_lds = 0;
    return p;
  }
  const long want = std::max<long>(1, target_wgs / ((long)p.gy * p.splits));
  p.gx = (int)std::min<long>(p.mtiles, want);
  // with several N tiles, a multiple of 8 workgroups along M puts the gy workgroups that stream
  // the same A rows on one XCD (dispatch is round-robin over the 8 XCDs), so A is read from HBM
  // once per XCD L2 instead of once per N tile
  static const bool xcd8 = [] {
    const char* e = std::getenv("PHX_GX8");
    return !(e && e[0] == '0');
  }();
  if (xcd8 && p.gy > 1 && p.gx > 8) p.gx = p.gx / 8 * 8;
  p.P = p.gx;
  p.res_lds = 0;
  // A-resident sweeps (k_gemm2r): a workgroup keeps its M tile of A' in LDS for a run of N tiles, so
  // the A view is applied once per run instead of once per N tile.  Runs are as long as the grid
  // stays >= ~512 workgroups allows; at least 2 N tiles per run, K of at least 2 chunks, no split-K.
  static const bool res_on = [] {
    const char* e = std::getenv("PHX_GEMM_RES");
    return !(e && e[0] == '0');
  }();
  const bool res_tile = (c.wm == 2 && c.tm == 2 && c.tn == 2) || (c.wm == 4 && c.tm == 1 && (c.tn == 3 || c.tn == 5)) ||
                        (c.wm == 2 && c.tm == 1 && c.tn == 2);
  const int ksteps = (K + bk - 1) / bk;
  const int esz = bf16 ? 2 : 4;
  const size_t lds = ((size_t)ksteps * c.bm() + 2 * c.bn()) * bk * esz;
  if (allow_res && res_on && res_tile && p.splits == 1 && p.gy >= 2 && ksteps >= 2 && lds <= 160 * 1024) {
    const int per_cu = std::max(1, std::min(2, (int)((160 * 1024) / lds)));
    const int runs_want = (int)std::max<long>(1, std::min<long>(p.gy, cdiv(512, p.mtiles)));
    const int nper = cdiv(p.gy, runs_want);
    if (nper >= 2) {
      const int runs = cdiv(p.gy, nper);
      p.res_lds = lds;
      p.kslice = nper;
      p.gy = runs;
      p.gx = (int)std::min<long>(p.mtiles, std::max<long>(1, (long)256 * per_cu / runs));
      p.P = p.mtiles * c.wm;
    }
  }
  return p;
}

// storage variant of a launch (see g2_go): A (raw / BN view) bf16 -> 1; a bf16 y (gradient view or
// GradSink) -> 2
static int g2_storage(const InX& A, const GradX& G, const GradSink& gsk) {
  if (A.bf) return 1;
  if ((G.y && G.ybf) || (gsk.part && gsk.ybf)) return 2;
  return 0;
}

int gemm2_run(int mode, InX A, GradX G, const float* Bt, const float* bias, float* C, int M, int N,
              int K, bool acc, const float* rowscale, int rows_per_img, hipStream_t s,
              float* partial, StatSink sink, int target_wgs, GradSink gsk, bool bf16, bool allow_wsk) {
  if (K % 4 != 0) throw std::runtime_error("gemm: K must be a multiple of 4");
  // the operands each mode's loads dereference (checked here: a null view pointer faults the device)
  if (mode == 3 ? !(G.da && G.y && G.mu && G.rstd && G.sc && G.be && G.mdz && G.mdzx) : !A.p)
    throw std::invalid_argument("gemm: missing A operand");
  if ((mode == 1 || mode == 2) && !(A.mu && A.sc && A.be)) throw std::invalid_argument("gemm: BN view without parameters");
  if (mode == 2 && !rowscale) throw std::invalid_argument("gemm: SE mode without a row scale");
  if (!Bt || !C) throw std::invalid_argument("gemm: missing B or C");
  if (gsk.part && !(gsk.y && gsk.mu && gsk.rstd && gsk.sc && gsk.be)) throw std::invalid_argument("gemm: GradSink without its BN");
  const Gemm2Plan p = plan_gemm2(M, N, K, target_wgs, bf16, mode != 4, allow_wsk);
  const bool stats = sink.part != nullptr;
  if (stats && (acc || mode == 3 || (N & 3) || (p.splits > 1 && N > 1024)))
    throw std::runtime_error("gemm: unsupported statistics epilogue");
  if (p.splits > 1 && !partial) throw std::runtime_error("gemm: split-K needs a partial buffer");
  const bool kstats = stats && p.splits == 1;
  if (stats) sink.P = p.splits > 1 ? gemm_splitk_stats_partials(M, N) : p.P;
  const bool gs = gsk.part != nullptr;
  if (gs && (p.splits > 1 || mode == 1 || mode == 2)) throw std::runtime_error("gemm: unsupported GradSink");
  gsk.P = p.P;
  const int sk = kstats ? 1 : gs ? 2 : 0;
  if (p.wsk) {
    const Gemm2Args w{A, G, Bt, bias, C, M, N, K, acc ? 1 : 0, rowscale, (mode == 2 || mode == 4) ? rows_per_img : 1, K,
                      nullptr, sink, p.mtiles, gsk};
    g2k_launch(p.tm, p.tn, mode, sk, dim3(p.gx, p.gy, 1), s, w, bf16, g2_storage(A, G, gsk));
    PHX_LAUNCH_CHECK();
    return p.P;
  }
  Gemm2Group<1> a{};
  a.n = 1;
  if (mode == 4 && (stats || gs)) throw std::runtime_error("gemm: the implicit im2col has no fused sinks");
  // rpi: rows per image of the SE row scale (mode 2) or the packed gather geometry (mode 4, g2_geo)
  a.a[0] = Gemm2Args{A, G, Bt, bias, C, M, N, K, acc ? 1 : 0, rowscale, (mode == 2 || mode == 4) ? rows_per_img : 1,
                     p.kslice, p.splits > 1 ? partial : nullptr, sink, p.mtiles, gsk};
  dim3 g(p.gx, p.gy, p.splits);
  const int st = g2_storage(A, G, gsk);
  const int key = p.wm * 100 + p.tm * 10 + p.tn;
  switch (key) {
    case 411: g2_launch_cfg<4, 1, 1, 1>(mode, sk, g, s, a, bf16, st, p.res_lds); break;
    case 412: g2_launch_cfg<4, 1, 2, 1>(mode, sk, g, s, a, bf16, st, p.res_lds); break;
    case 413: g2_launch_cfg<4, 1, 3, 1>(mode, sk, g, s, a, bf16, st, p.res_lds); break;
    case 415: g2_launch_cfg<4, 1, 5, 1>(mode, sk, g, s, a, bf16, st, p.res_lds); break;
    case 222: g2_launch_cfg<2, 2, 2, 1>(mode, sk, g, s, a, bf16, st, p.res_lds); break;
    case 212: g2_launch_cfg<2, 1, 2, 1>(mode, sk, g, s, a, bf16, st, p.res_lds); break;
    case 211: g2_launch_cfg<2, 1, 1, 1>(mode, sk, g, s, a, bf16, st, p.res_lds); break;
    case 111: g2_launch_cfg<1, 1, 1, 1>(mode, sk, g, s, a, bf16, st, p.res_lds); break;
    default: throw std::runtime_error("gemm2: no kernel for this configuration");
  }
  PHX_LAUNCH_CHECK();
  if (p.splits > 1) return gemm_splitk_finish(partial, p.splits, M, N, bias, C, acc, sink, s, st == 1);
  return p.P;
}

bool gemm_group_ok(const int* M, int n, int N, int K, bool bf16) {
  if (n < 1 || n > kMaxSeg || gemm_impl_for(N, bf16) != 2) return false;
  for (int i = 0; i < n; ++i) {
    // (the members' own plans without the wave-split kernel: a grouped launch beats separate ones)
    const Gemm2Plan p = plan_gemm2(M[i], N, K, gemm2_target_wgs(), bf16, true, false);
    if (p.splits != 1 || p.wsk) return false;
  }
  return true;
}

int gemm_group_run(int mode, const GemmSeg* segs, int n, const float* Bt, int N, int K, hipStream_t s,
                   bool bf16, int* P_out, long max_part_rows) {
  std::vector<int> M(n);
  for (int i = 0; i < n; ++i) M[i] = segs[i].M;
  if (!gemm_group_ok(M.data(), n, N, K, bf16)) throw std::runtime_error("gemm group: unsupported shapes");
  if (K % 4 != 0) throw std::runtime_error("gemm: K must be a multiple of 4");
  const bool stats = segs[0].sink.part != nullptr, gs = segs[0].gsk.part != nullptr;
  if (stats && (mode == 3 || (N & 3))) throw std::runtime_error("gemm group: unsupported statistics");
  if (gs && (mode == 1 || mode == 2)) throw std::runtime_error("gemm group: unsupported GradSink");
  Gemm2Group<kMaxSeg> a{};
  a.n = n;
  int gx = 1, P = 1;
  Gemm2Plan p0{};
  for (int i = 0; i < n; ++i) {
    const Gemm2Plan p = plan_gemm2(M[i], N, K, gemm2_target_wgs(), bf16, true, false);
    if (i == 0) p0 = p;
    gx = std::max(gx, p.gx);
  }
  // the A-resident sweep when the first (largest) member takes it: every member runs p0's N-tile runs
  // and writes one partial row per (M tile, wave row)
  const int kslice = p0.res_lds ? p0.kslice : K;
  std::vector<int> Pm(n);  // partial rows of each member's sinks
  for (int i = 0; i < n; ++i) {
    Pm[i] = p0.res_lds ? cdiv(M[i], p0.wm * p0.tm * 32) * p0.wm : gx;
    P = std::max(P, Pm[i]);
    if (P_out) P_out[i] = Pm[i];
  }
  // every member's partial rows must fit its region of the caller's partial buffer (sized from each
  // op's own plan): a member planned with another member's tile must not spill into the next region,
  // where two workgroups of this launch would then race for the same partials
  if ((stats || gs) && max_part_rows >= 0 && P > max_part_rows)
    throw std::logic_error("gemm group: a member's partial rows exceed its region");
  for (int i = 0; i < n; ++i) {
    const GemmSeg& g = segs[i];
    if ((g.sink.part != nullptr) != stats || (g.gsk.part != nullptr) != gs)
      throw std::runtime_error("gemm group: members differ in their sinks");
    StatSink sink = g.sink;
    sink.P = Pm[i];
    GradSink gsk = g.gsk;
    gsk.P = Pm[i];
    a.a[i] = Gemm2Args{g.A, g.G, Bt, g.bias, g.C, g.M, N, K, g.acc ? 1 : 0, nullptr, 1, kslice, nullptr, sink,
                       cdiv(g.M, p0.wm * p0.tm * 32), gsk};
  }
  const int sk = stats ? 1 : gs ? 2 : 0;
  const int st = g2_storage(segs[0].A, segs[0].G, segs[0].gsk);
  dim3 grid(gx, p0.gy, n);
  const int key = p0.wm * 100 + p0.tm * 10 + p0.tn;
  switch (key) {
    case 411: g2_launch_cfg<4, 1, 1, kMaxSeg>(mode, sk, grid, s, a, bf16, st, p0.res_lds); break;
    case 412: g2_launch_cfg<4, 1, 2, kMaxSeg>(mode, sk, grid, s, a, bf16, st, p0.res_lds); break;
    case 413: g2_launch_cfg<4, 1, 3, kMaxSeg>(mode, sk, grid, s, a, bf16, st, p0.res_lds); break;
    case 415: g2_launch_cfg<4, 1, 5, kMaxSeg>(mode, sk, grid, s, a, bf16, st, p0.res_lds); break;
    case 222: g2_launch_cfg<2, 2, 2, kMaxSeg>(mode, sk, grid, s, a, bf16, st, p0.res_lds); break;
    case 212: g2_launch_cfg<2, 1, 2, kMaxSeg>(mode, sk, grid, s, a, bf16, st, p0.res_lds); break;
    case 211: g2_launch_cfg<2, 1, 1, kMaxSeg>(mode, sk, grid, s, a, bf16, st, p0.res_lds); break;
    case 111: g2_launch_cfg<1, 1, 1, kMaxSeg>(mode, sk, grid, s, a, bf16, st, p0.res_lds); break;
    default: throw std::runtime_error("gemm2: no kernel for this configuration");
  }
  PHX_LAUNCH_CHECK();
  return P;
}

}  // namespace phx
