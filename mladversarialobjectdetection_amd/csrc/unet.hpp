// unet.hpp — launchers of the defender step (kernels_unet.hip) and the victim-side helper the
// defender's first pass uses (api.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

struct phx_ctx;

namespace phx {

// ---- gathers and weight matrices (kernels_unet.hip) ----------------------------------------
// col [B*Ho*Wo, Kp]: mode 0 conv (stride s, pads pt / pl), mode 1 transposed conv (stride 2)
void un_im2col(const float* x, float* col, int B, int H, int W, int C, int Ho, int Wo, int Kp, int mode, int s,
               int pt, int pl, hipStream_t st);
// out [B*Ho*Wo, N] = col (gathered as un_im2col's mode / stride / pads, never stored) x Bt^T + bias,
// for the few-channel levels (N <= 32, Kp <= 288); false = shape not covered (use im2col + GEMM)
bool un_conv3_small(const float* x, const float* Bt, const float* bias, float* out, int B, int H, int W, int C,
                    int Ho, int Wo, int N, int Kp, int mode, int s, int pt, int pl, hipStream_t st);
// GEMM B operands from Keras kernels: kind 0 conv fwd, 1 conv dgrad, 2 tconv fwd, 3 tconv dgrad,
// 4 1x1 fwd, 5 1x1 dgrad (bt [N][Kp])
void un_wprep(const float* w, float* bt, int kind, int ci, int co, int Kp, hipStream_t st);
// weight gradient of (dy [M][Co], col [M][Kp]) into the Keras layout of g (kind 0 conv, 2 tconv,
// 4 1x1); part: un_wgrad_slices(M, Co, Kp) * Co * Kp floats.  The column matrix is gathered on the
// fly from x: src 0 = x itself [M][ldx]; src 1 = 3x3 conv (stride 1, pads 1) over x [B,H,W,C];
// src 2 = stride-2 transposed conv over x [B,H/2,W/2,C] (rows = the B*H*W outputs)
int un_wgrad_slices(long M, int Co, int Kp);
void un_wgrad(const float* dy, int ldy, const float* x, int ldx, int src, int B, int H, int W, int C, long M,
              int Co, int Kp, int Kin, int taps, int kind, float* part, float* g, hipStream_t st);

// ---- BN (training) and column sums: fp64 partials (un_colred_doubles) ----------------------
size_t un_colred_doubles(long M, int C);
void un_bn_stats(const float* y, long M, int C, const float* gamma, float* mean, float* rstd, float* sc,
                 float* mmean, float* mvar, double* part, hipStream_t st);
// BN backward through act (1 leaky, 0 identity): dy and the gamma / beta gradients
void un_bn_bwd(const float* da, const float* y, long M, int C, const float* mu, const float* rstd, const float* sc,
               const float* be, int act, float* mdz, float* mdzx, float* dgamma, float* dbeta, float* dy,
               double* part, hipStream_t st);
void un_colsum(const float* v, long M, int C, float* out, double* part, hipStream_t st);
void un_bnact(const float* y, const float* mu, const float* sc, const float* be, float* a, long M, int C, int act,
              hipStream_t st);

// ---- pooling, dropout, attention, output ----------------------------------------------------
// layer < 0: inference (no Dropout), also for un_att_cat
void un_pool_drop(const float* x, float* out, uint8_t* arg, int B, int H, int W, int C, uint64_t seed, int64_t step,
                  int gimg0, int layer, hipStream_t st);
void un_pool_drop_bwd(const float* dout, const uint8_t* arg, float* dx, int B, int H, int W, int C, uint64_t seed,
                      int64_t step, int gimg0, int layer, bool acc, hipStream_t st);
void un_att_s(const float* g, const float* x, const float* mu1, const float* sc1, const float* be1, const float* mu2,
              const float* sc2, const float* be2, float* s, long M, int C, hipStream_t st);
void un_att_t(const float* s, const float* w, const float* b, float* t, long M, int C, hipStream_t st);
void un_att_cat(const float* up, const float* skip, const float* t, const float* mu3, const float* sc3,
                const float* be3, float* cat, int B, long HW, int C, uint64_t seed, int64_t step, int gimg0, int layer,
                hipStream_t st);
void un_att_cat_bwd(const float* dcat, const float* skip, const float* t, const float* mu3, const float* sc3,
                    const float* be3, float* dup, float* dskip, float* dz3, int B, long HW, int C, uint64_t seed,
                    int64_t step, int gimg0, int layer, hipStream_t st);
void un_att_s_bwd(const float* dt, const float* w3, const float* g, const float* x, const float* mu1,
                  const float* sc1, const float* be1, const float* mu2, const float* sc2, const float* be2,
                  float* dsum, long M, int C, hipStream_t st);
int un_loss_blocks(long M);
void un_out_loss(const float* x, const float* w, const float* b, const float* tgt, float* upd, float* dz,
                 double* lpart, float* loss, long M, long HW, int C, hipStream_t st);
void un_small_dgrad(const float* dz, const float* w, float* dx, long M, int C, int O, bool acc, hipStream_t st);
void un_add(float* a, const float* b, long n, hipStream_t st);

// ---- Masker extras ---------------------------------------------------------------------------
// info [B][3] = (source image, flip lr, flip ud); crops [B][P][P][3]
void def_perm_crops(const float* images, int* info, float* crops, int B, int H, int W, int P, uint64_t seed,
                    int64_t step, int gimg0, hipStream_t st);
// filter_valid_boxes (attack_detection.py:79-94); os (optional) receives the kept scores
void def_filter(const float* nb, const float* ns, const int* nc, int B, int maxo, float H, float W, float thresh,
                float* ob, int* oc, hipStream_t st, float* os = nullptr);

// ---- victim side (api.cpp) -----------------------------------------------------------------
// odet_model (attack_detection.py:96-127): frozen-BN forward, person anchors, soft-NMS, clip and
// filter_valid_boxes; boxes [B][100][4], count [B]
// train: the call's training flag (drop connect), pass: drop-connect key (0 first, 1 second);
// score_thresh >= 0: odet_model(images, score_thresh) — the soft-NMS threshold only (0 -> 0.001);
// scores (optional): the kept boxes' scores [B][100]
void def_first_pass(phx_ctx* ctx, const float* images, int B, int64_t step, int gimg0, float* boxes, int* count,
                    hipStream_t s, bool train = true, int pass = 0, float score_thresh = -1.f,
                    float* scores = nullptr);
int ctx_image_size(const phx_ctx* ctx);
// a launch group on the victim context's profiler (phx_profile / phx_profile_report): events on
// `s` around the group, with its algorithmic FLOPs / bytes; a no-op while profiling is off
struct ProfScope {
  void* p;
  size_t idx;
  hipStream_t s;
};
ProfScope prof_begin(phx_ctx* ctx, const char* kind, double flops, double bytes, hipStream_t s);
void prof_end(const ProfScope& r);
bool ctx_profiling(const phx_ctx* ctx);  // phx_profile is on (launch groups timed one at a time)
uint64_t ctx_seed(const phx_ctx* ctx);
int ctx_device(const phx_ctx* ctx);
// what a frozen first pass of the victim depends on besides its inputs: the weights / moving-statistics
// version (bumped by every load and training pass) and the score thresholds — a prefetched first pass
// made at another generation is stale
uint64_t ctx_generation(const phx_ctx* ctx);

}  // namespace phx
