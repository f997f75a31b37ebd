// kernels.hpp — host launchers of the phx HIP kernels.  All launches are asynchronous on the
// given stream and never allocate.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstddef>
#include <cstdint>

#include "common.hpp"

namespace phx {

// Launch-group timing by the kernels' own dispatch timestamps (the library profiler's GEMM
// groups, so the live roofline times kernels as rocprofv3 does, without the gaps two
// hipEventRecord packets add): while ext_timing() is set, a kernel launched through PHX_TLAUNCH
// records its start event (the group's first kernel) and its stop event (every kernel; the last
// one counts).
struct ExtTiming {
  hipEvent_t a = nullptr, b = nullptr;
  bool used = false;
};
ExtTiming*& ext_timing();
#define PHX_TLAUNCH(K, G, BL, SHM, S, ...)                                                              \
  do {                                                                                                 \
    if (::phx::ExtTiming* t_ = ::phx::ext_timing()) {                                                  \
      hipExtLaunchKernelGGL(K, G, BL, SHM, S, t_->used ? nullptr : t_->a, t_->b, 0, __VA_ARGS__);      \
      t_->used = true;                                                                                 \
    } else {                                                                                           \
      hipLaunchKernelGGL(K, G, BL, SHM, S, __VA_ARGS__);                                               \
    }                                                                                                  \
  } while (0)


// ---- convolutions (kernels_conv.hip) ------------------------------------------------------
// 3x3 stride-2 stem, Cin = 3: x [B,H,W,3] -> y [B,Ho,Wo,Co]; w [3,3,3,Co] (HWIO)
// returns the number of StatSink partial rows written (sink.part == nullptr: no statistics)
// ybf: y in bf16 storage (a PHX_DTYPE_BF16 context's activations; the statistics are taken over
// the stored values)
int launch_stem_fwd(const float* x, const float* w, float* y, int B, int H, int W, int Ho, int Wo,
                    int Co, int pt, int pl, hipStream_t s, StatSink sink = StatSink{}, bool ybf = false);
// dx [B,H,W,3] (+)= conv_transpose(dy); dy is a materialised gradient [B,Ho,Wo,Co]
void launch_stem_bwd(const float* dy, const float* w, float* dx, int B, int H, int W, int Ho,
                     int Wo, int Co, int pt, int pl, bool acc, hipStream_t s);
// dx [B,H,W,3] = conv_transpose(gx(dy)) through the stem BN's gradient view, only at pixels some
// paste owns (owner [B,H,W,3] >= 0; nullptr = everywhere), zero elsewhere; overwrites dx
bool stem_bwd_gx_supported(int Co);
void launch_stem_bwd_gx(GradX g, const float* w, const int16_t* owner, float* dx, int B, int H, int W,
                        int Ho, int Wo, int Co, int pt, int pl, hipStream_t s);
// C[M,N] (+)= A[M,K] * B + bias ; B given as Bt[N][K].  rowscale (optional): A[m,k] is
// multiplied by rowscale[(m / rows_per_img) * K + k] (SE excitation folded into the load).
struct GemmPlan {
  int nt, wm, gx, gy, splits, kslice;
};
GemmPlan plan_gemm(int M, int N, int K);
// bf16: the 1x1 convs with N > 16 run on the bf16 matrix cores (A view applied in fp32, rounded to
// bf16 in LDS; fp32 accumulation and epilogue) — the C4 configuration's compute type
size_t gemm_partial_floats(int M, int N, int K, bool bf16 = false);
// returns the StatSink partial rows written (see gemm_stat_partials)
int launch_gemm(InX A, const float* Bt, const float* bias, float* C, int M, int N, int K,
                bool acc, const float* rowscale, int rows_per_img, hipStream_t s,
                float* partial, StatSink sink = StatSink{}, bool bf16 = false);
int gemm_stat_partials(int M, int N, int K, bool bf16 = false);
// the two GEMM implementations behind launch_gemm (gemm_impl(): PHX_GEMM env, default 2)
struct Gemm2Plan {
  int wm, tm, tn, mtiles, gx, gy, splits, kslice;
  int P;           // statistics / BN-backward-sum partial rows the launch writes
  size_t res_lds;  // > 0: the A-resident kernel (k_gemm2r) with this much dynamic LDS; kslice then
                   // counts the N tiles of one workgroup's sweep and gy the sweeps
  int wsk = 0;     // > 0: the wave-split-K kernel (k_gemm2k, kernels_gemm_wsk.hip) with tile tm x tn
};
Gemm2Plan plan_gemm2(int M, int N, int K, int target_wgs, bool bf16 = false, bool allow_res = true,
                     bool allow_wsk = true);
void gemm2_force_cfg(int wm, int tm, int tn, int splits);  // tools/gemm_bench sweeps only (0 = off)
void gemm2_force_wsk(int tm, int tn);                       // tools/gemm_bench sweeps only (0 = off, -1 = never)
struct Gemm2Args;
void g2k_launch(int tm, int tn, int mode, int sk, dim3 g, hipStream_t s, const Gemm2Args& a, bool bf16, int st);
int gemm_impl();
int gemm_impl_for(int N, bool bf16 = false);
int gemm2_target_wgs();
int gemm1_run(int mode, InX A, GradX G, const float* Bt, const float* bias, float* C, int M, int N,
              int K, bool acc, const float* rowscale, int rows_per_img, hipStream_t s,
              float* partial, StatSink sink, GradSink gsk = GradSink{});
int gemm2_run(int mode, InX A, GradX G, const float* Bt, const float* bias, float* C, int M, int N,
              int K, bool acc, const float* rowscale, int rows_per_img, hipStream_t s,
              float* partial, StatSink sink, int target_wgs, GradSink gsk = GradSink{}, bool bf16 = false,
              bool allow_wsk = true);
int gemm_splitk_stats_partials(int M, int N);
// cbf: C holds bf16 activations (the partial slabs are fp32)
int gemm_splitk_finish(const float* partial, int splits, int M, int N, const float* bias, float* C,
                       bool acc, StatSink sink, hipStream_t s, bool cbf = false);
// 3x3 convolution GEMM over an implicitly gathered column matrix (kernels_conv.hip)
bool gemm_gather_ok(int B, int H, int W, int C, int Ho, int Wo, int K, int mode, int s, int pt, int pl);
int launch_gemm_gather(const float* x, int B, int H, int W, int C, int Ho, int Wo, int mode, int s, int pt, int pl,
                       const float* Bt, const float* bias, float* out, int N, int K, hipStream_t st, float* partial);
// dgrad GEMM whose A operand is a gradient view (BN backward applied on load)
// with a GradSink, the BN-backward sums of the dgrad's result (returns the partial rows)
int launch_gemm_dgrad(GradX A, const float* Bt, float* C, int M, int N, int K, bool acc,
                      hipStream_t s, float* partial, GradSink gs = GradSink{}, bool bf16 = false);
int gemm_dgrad_gsink_partials(int M, int N, int K, bool bf16 = false);
// the launch of this shape runs a kernel with the in-launch BN finalize (k_gemm2 / k_gemm2r, no split-K)
bool gemm_fold_ok(int M, int N, int K, bool bf16);
// Grouped GEMM: members share Bt [N][K] (weights shared across pyramid levels) and differ in A,
// C, M and sinks.  mode as gemm2 (0 raw, 1 BN view, 3 gradient view).  No split-K: see
// gemm_group_ok.  Returns the most partial rows any member's sinks get; P_out[i] = member i's
// (the same for all members, except on the A-resident sweep: one row per (M tile, wave row)).
struct GemmSeg {
  InX A;
  GradX G;
  const float* bias;
  float* C;
  int M;
  bool acc;
  StatSink sink;
  GradSink gsk;
};
bool gemm_group_ok(const int* M, int n, int N, int K, bool bf16 = false);
// max_part_rows >= 0: the partial rows one member's region holds (throws before launching if any
// member would write more)
int gemm_group_run(int mode, const GemmSeg* segs, int n, const float* Bt, int N, int K, hipStream_t s,
                   bool bf16 = false, int* P_out = nullptr, long max_part_rows = -1);
// depthwise k x k, stride s, TF SAME: x [B,H,W,C] -> y [B,Ho,Wo,C]; w [k,k,C]
int launch_dw_fwd(InX x, const float* w, float* y, int B, int H, int W, int C, int Ho,
                  int Wo, int k, int stride, int pt, int pl, hipStream_t s,
                  StatSink sink = StatSink{});
int dw_stat_partials(int B, int H, int W, int C, int Ho, int Wo, int k, int stride, int pt, int pl);
int launch_dw_bwd(GradX dy, const float* w, float* dx, int B, int H, int W, int C, int Ho,
                  int Wo, int k, int stride, int pt, int pl, bool acc, hipStream_t s,
                  GradSink gs = GradSink{});
int dw_bwd_partials(int B, int H, int W, int C, int Ho, int Wo, int k, int stride, int pt, int pl);
// grouped depthwise convs (same taps w, C, k, stride; per-member tensors and sinks); H, W are the
// conv input, Ho, Wo its output; out = y (forward) or dx (backward); nps[i] = partial rows
struct DwSeg {
  InX x;          // forward input view
  GradX gv;       // backward: gradient view of the conv output
  float* out;
  int H, W, Ho, Wo, pt, pl;
  bool acc;       // backward: accumulate into dx
  StatSink sink;  // forward
  GradSink gs;    // backward
};
void launch_dw_fwd_group(const DwSeg* segs, int n, int B, int C, const float* w, int k, int stride,
                         hipStream_t s, int* nps);
// ---- fused separable conv (kernels_sep.hip) ---------------------------------------------------
// keras SeparableConv2D(3x3, SAME, depth_multiplier 1) + bias: y [B,H,W,N] = pw(dw(view(x))) + bias,
// the depthwise output never stored.  Members share the taps wd [3][3][C], the transposed pointwise
// kernel bt [N][C], the bias and C, N (the per-level copies of a head conv); each has its input view —
// a BN view (x) or a BiFPN node fuse computed on load (f, fuse = true; ungrouped only) — output and
// StatSink (the consumer BN's batch statistics of y; part == nullptr: none).  nps[i]: member i's
// partial rows (sep_stat_partials)
struct SepMember {
  InX x;
  FuseView f;
  bool fuse;
  float* y;
  int H, W;
  StatSink sink;
};
bool sep_supported(int C, int N, bool bf16);
int sep_stat_partials(int B, int H, int W);
void launch_sep_fwd(const SepMember* m, int n, int B, int C, int N, const float* wd, const float* bt,
                    const float* bias, hipStream_t s, int* nps);
// its backward through the depthwise input: dx [B,H,W,C] (+)= dw^T(gv(dy) W^T), the pointwise data
// gradient never stored.  gv: the pointwise output's gradient view (the consumer BN's backward applied
// on load); wp: the pointwise kernel HWIO [C][N]; gs: the BN-backward sums of the BN whose output the
// depthwise conv reads (part == nullptr: none), nps[i] = member i's partial rows (sep_stat_partials)
struct SepBwdMember {
  GradX gv;
  float* dx;
  int H, W;
  bool acc;
  GradSink gs;
};
bool sep_bwd_supported(int C, int N, bool bf16);
void launch_sep_bwd(const SepBwdMember* m, int n, int B, int C, int N, const float* wd, const float* wp,
                    hipStream_t s, int* nps);
// depthwise 3x3 s1 whose input is a BiFPN fuse computed on load (FuseView); no statistics
void launch_dw_fwd_fused(const FuseView& fv, const float* w, float* y, int B, int H, int W, int C, int Ho,
                         int Wo, int k, int stride, int pt, int pl, hipStream_t s);
void launch_dw_bwd_group(const DwSeg* segs, int n, int B, int C, const float* w, int k, int stride,
                         hipStream_t s, int* nps);
void launch_transpose(const float* in, float* out, int rows, int cols, hipStream_t s);

// ---- normalisation / elementwise (kernels_norm.hip) ---------------------------------------
// Per-channel batch statistics of y [M,C]: writes mean/rstd (float) and updates moving stats
// (momentum 0.99, util_keras.py:33-35) when mmean != nullptr.  part: scratch (doubles).
size_t bn_stats_scratch_doubles(long M, int C);
// side != nullptr: the moving statistics are not touched; (mean, Bessel-corrected variance) go to
// side[2c], side[2c+1] in fp64 for launch_bn_moving_apply (a step whose two passes run concurrently)
void launch_bn_stats(const float* y, long M, int C, double* part, float* mean, float* rstd,
                     const float* gamma, float* sc, float* mmean, float* mvar, float eps,
                     hipStream_t s, bool ybf = false, double* side = nullptr);
// training-mode BN statistics from the P producer partials of a StatSink (k_bn_finalize)
void launch_bn_finalize(const float2* part, const float* cnt, int P, long M, int C, float* mean,
                        float* rstd, const float* gamma, float* sc, float* mmean, float* mvar,
                        float eps, hipStream_t s, double* side = nullptr);
// grouped finalize (one launch for the per-level BNs of a head conv, each its own partials)
struct BnFinSeg {
  const float2* part;
  const float* cnt;  // forward only
  int P;
  long M;
  float *mean, *rstd;
  const float* gamma;
  float *sc, *mmean, *mvar;
  float *mdz, *mdzx;  // backward
  double* side = nullptr;  // forward: deferred moving statistics (see launch_bn_stats)
};
// The moving-statistics updates of two passes, in pass order (m <- m - (m - batch) * 0.01 twice,
// each rounded to float as the in-finalize update does): for every entry, channels c < C of
// W[mm + c] / W[mv + c] from side0 / side1 + off (fp64 (mean, var) pairs)
struct MovEntry {
  long mm, mv;
  int C, off;
};
void launch_bn_moving_apply(const MovEntry* tab, int n, int cmax, float* W, const double* side0,
                            const double* side1, hipStream_t s);
void launch_bn_finalize_group(const BnFinSeg* segs, int n, int C, float eps, hipStream_t s);
// bn=sync halves of a finalize: fold each member's partials into sums[i][C][3] = (rows, S1, S2) in
// fp64 (forward: sum x, sum x^2; backward: sum dz, sum dz*xhat), then — after the caller's
// all-reduce of the sums — the statistics / backward means from the global sums
void launch_bn_fold_sums(const BnFinSeg* segs, int n, int C, bool bwd, double* sums, hipStream_t s);
void launch_bn_from_sums(const BnFinSeg* segs, int n, int C, bool bwd, const double* sums, float eps,
                         hipStream_t s);
void launch_bn_stats_sums(const float* y, long M, int C, double* part, double* sums, hipStream_t s, bool ybf);
void launch_bn_bwd_reduce_sums(const float* da, const float* y, const float* mean, const float* rstd,
                               const float* gamma, const float* beta, long M, int C, int act, double* part,
                               double* sums, hipStream_t s, bool ybf);
void launch_bn_bwd_finalize_group(const BnFinSeg* segs, int n, int C, hipStream_t s);
// frozen BN: mean/rstd from moving statistics
void launch_bn_frozen_stats(const float* mmean, const float* mvar, float* mean, float* rstd,
                            const float* gamma, float* sc, int C, float eps, hipStream_t s);
// a = act(gamma * (y - mean) * rstd + beta)
void launch_bn_apply(const float* y, const float* mean, const float* rstd, const float* gamma,
                     const float* beta, float* a, long M, int C, int act, hipStream_t s);
// BN backward, training mode.  Sums over M of dz and dz*xhat (dz = da * act'(z)) then
// dy (+)= gamma*rstd*(dz - mean(dz) - xhat*mean(dz*xhat)).  frozen: dy = gamma*rstd*dz.
void launch_bn_bwd(const float* da, const float* y, const float* mean, const float* rstd,
                   const float* gamma, const float* beta, float* dy, long M, int C, int act,
                   bool frozen, bool acc, double* part, float* coef, hipStream_t s);
// materialise a gradient view: out[M,C] = gx(view)
void launch_bn_bwd_apply2(GradX g, float* out, long M, int C, hipStream_t s);
// reduction half of the BN backward: mdz[c] = mean(dz), mdzx[c] = mean(dz*xhat); the apply
// half runs inside the consumer through a GradX view
void launch_bn_bwd_reduce(const float* da, const float* y, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, long M, int C, int act,
                          double* part, float* mdz, float* mdzx, hipStream_t s, bool ybf = false);
// squeeze-excite forward: pool[B,C] = mean_hw(x); scale[B,C]; y = x * scale
void launch_se_fwd(InX x, float* y, int B, int HW, int C, int Cse, const float* w1,
                   const float* b1, const float* w2, const float* b2, int act, float* pool,
                   float* hidden, float* scale, hipStream_t s, double* scratch);
// w2t: the expand kernel transposed to [C][Cse]
// returns the GradSink partial rows written (gs.part == nullptr: no BN-backward sums)
int launch_se_bwd(const float* dy, InX x, float* dx, int B, int HW, int C, int Cse,
                  const float* w1, const float* b1, const float* w2t, const float* b2, int act,
                  const float* pool, const float* hidden, const float* scale, float* gsum,
                  bool acc, hipStream_t s, double* scratch, GradSink gs = GradSink{});
int ew_gstats_partials(long seg_rows, int C, int nseg);
// mdz = mean(dz), mdzx = mean(dz*xhat) from the P GradSink partials
void launch_bn_bwd_finalize(const float2* part, int P, long M, int C, float* mdz, float* mdzx,
                            hipStream_t s);
size_t colred_scratch_doubles(long seg_rows, int C, int nseg);
// drop connect (utils.py:329-344) on one operand: v' = (v / p) * keep[image], forward, and
// (g * keep[image]) / p for its gradient
struct DropView {
  const float* keep = nullptr;  // [B] 0 / 1 per image (launch_drop_keep); nullptr = off
  float p = 1.f;                // survival probability of the block
  long rows = 1;                // rows (pixels) per image
};
// keep[d*B + b] = floor(p[d] + U), U = u01(Philox(seed; block[d], pass, gimg0 + b, step<<8|RNG_DROP))
void launch_drop_keep(const int* block, const float* p, int nd, int B, uint64_t seed, int64_t step,
                      int gimg0, int pass, float* keep, hipStream_t s);
// dst[n] (fp32) = src[n] (bf16 storage)
void launch_bf16_to_f32(const float* src, float* dst, long n, hipStream_t s);
// *out += an order-independent 64-bit hash of the bytes (PHX_CKSUM diagnostics; *out zeroed by the
// caller)
void launch_cksum(const void* p, size_t bytes, unsigned long long* out, hipStream_t s);
// y = drop(a) + b
void launch_add(InX a, InX b, float* y, long n, int C, hipStream_t s, DropView dv = DropView{});
// dst (+)= drop'(src); with a GradSink (C channels) the BN-backward sums of the result come along
int launch_copy_grad(const float* src, float* dst, long n, bool acc, hipStream_t s, int C = 4,
                     GradSink gs = GradSink{}, DropView dv = DropView{});
// GradSink sums of src [n/C, C] without writing anything (src is already the BN output's gradient)
int launch_grad_sums(const float* src, long n, int C, GradSink gs, hipStream_t s);
// amax: per output element, the window tap (row-major) holding the maximum; the backward
// routes each dy there (TF MaxPoolGrad)
void launch_maxpool_fwd(InX x, float* y, uint8_t* amax, int B, int H, int W, int C, int Ho, int Wo,
                        int k, int stride, int pt, int pl, hipStream_t s);
void launch_maxpool_bwd(const uint8_t* amax, const float* dy, float* dx, int B, int H, int W, int C,
                        int Ho, int Wo, int k, int stride, int pt, int pl, bool acc,
                        hipStream_t s);
void launch_upsample_fwd(InX x, float* y, int B, int H, int W, int C, int Ho, int Wo,
                         hipStream_t s);
void launch_upsample_bwd(const float* dy, float* dx, int B, int H, int W, int C, int Ho, int Wo,
                         bool acc, hipStream_t s);
// BiFPN fuse: y = act(sum_i x_i * w_i / (sum_j w_j + 1e-4)) (fastattn, w = relu(wsm)) or
// act(sum_i x_i) (method 1)
void launch_fuse_fwd(const InX* xs, int nin, const float* wsm0, const float* wsm1,
                     const float* wsm2, int method, int act, float* y, long n, int C,
                     hipStream_t s);
void launch_fuse_bwd(const InX* xs, int nin, const float* wsm0, const float* wsm1,
                     const float* wsm2, int method, int act, const float* dy, float* const* dxs,
                     const bool* acc, long n, int C, hipStream_t s);

// ---- detection post-processing (kernels_post.hip) -----------------------------------------
struct LevelDesc {
  long cls_off;   // float offset of the level's class output (relative to base)
  long box_off;
  int h, w;
  int anchor0;    // first anchor index of this level
  int tile0;      // first pre_nms tile of this level
};
int pre_nms_tiles(int h, int w, int na);
// soft-NMS candidates appended by pre_nms: list [B][A] anchor indices, count [B] (zero on entry,
// reset to zero by the k_soft_nms that consumes them); mask selects keep bits (2: first pass,
// 1: second pass), thresh = the NMS score threshold.  list == nullptr: no list.
struct NmsCand {
  int* list = nullptr;
  int* count = nullptr;
  int mask = 0;
  float thresh = 0.f;
};
// pre_nms (postprocess.py:119-156) + person/validity filter (attacker.py:69-89, 105-113)
// outputs per anchor: score, class, box; keep flag (bit0 = person&valid, bit1 = >= thresh)
void launch_pre_nms(const float* cls_base, const float* box_base, const LevelDesc* lev_dev,
                    int nlev, const float* anchors, int A, int B, int nclass, int na,
                    float img_h, float img_w, float thresh, float* scores, int* classes,
                    float* boxes, uint8_t* keep, int ntiles, hipStream_t s, NmsCand cand = NmsCand{},
                    bool bf = false);  // bf: class / box outputs in bf16 storage
// soft-NMS (NonMaxSuppressionV5, gaussian) per image over candidates selected by keep&mask
void launch_soft_nms(const float* boxes, const float* scores, const uint8_t* keep, int keep_mask,
                     const int* count, int B, int N, float score_thresh, float soft_sigma,
                     int max_out, float clip_hi, float* out_boxes, float* out_scores,
                     int* out_count, float* work, hipStream_t s, NmsCand cand = NmsCand{});
// work floats of launch_soft_nms (compacted candidate boxes, spilled queue keys, anchors, visits)
size_t soft_nms_work_floats(int B, int N);
// per-image m_b = max(max_{keep} score, 0), tie count, and loss-gradient coefficient
void launch_image_max(const float* scores, const uint8_t* keep, int B, int A, float* m,
                      int* argmax, int* nties, int* scratch, hipStream_t s);
size_t image_max_scratch_ints(int B);

// ---- input pipeline (kernels_data.hip, train_data_generator.py) -----------------------------
// DataSequence._map_fn for B packed uint8 RGB images (offsets [B] bytes, dims [B,2] = (h, w), device)
// -> out [B,oh,ow,3] normalised, cv2-INTER_LINEAR-resized, top-left letterboxed, zero padded
void launch_letterbox(const uint8_t* src, const int64_t* offsets, const int32_t* dims, int B,
                      const float* mean, const float* stdv, int oh, int ow, float* out, hipStream_t s);
// flip -> RandomFlip -> RandomContrast(.2) -> random_brightness(.2) -> clip; in/out [B,H,W,3]
size_t augment_scratch_doubles(int B);
void launch_augment(const float* in, float* out, int B, int H, int W, uint64_t seed, int64_t step,
                    int gimg0, double* scratch, hipStream_t s);
// ---- inference compositor (kernels_advpatch.hip, adv_patch.py) ------------------------------
struct ApBox {
  int valid;      // this image has a box in this round
  int y, x;       // patch origin (AdversarialPatch._create)
  int ph, pw;     // patch size (square)
};
// printed = (raw + 127) >> 1 per byte ([P,P,3]); *ysum = sum of its Y (zeroed first)
void launch_ap_print(const uint8_t* raw, uint8_t* printed, int P, unsigned long long* ysum, hipStream_t s);
// ysum[b] = sum of Y over the out_h x out_w rescale of image b (its sh x sw content + grey letterbox)
void launch_ap_ysum(const uint8_t* img, int B, int H, int W, int out_h, int out_w, int sh, int sw,
                    unsigned long long* ysum, hipStream_t s);
// paste round `slot`: boxes[b] for every image (device), max_pix = largest ph * pw of the round
void launch_ap_paste(uint8_t* img, int B, int H, int W, const uint8_t* printed, int P, const ApBox* boxes,
                     int max_pix, int slot, const unsigned long long* ysum, const unsigned long long* ysrc, int out_h,
                     int out_w, uint64_t seed, int64_t step, int gimg0, hipStream_t s);
}  // namespace phx
