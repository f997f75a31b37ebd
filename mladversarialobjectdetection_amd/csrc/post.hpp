// post.hpp — launchers for post-processing, loss and EOT kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"
#include "phx.h"
#include <cfloat>

#define PHX_MAX_OUT_DEV 100
#define PHX_NPATCH_DEV (640 * 640 * 3)
#define PHX_PATCH_DEV 640

namespace phx {

// loss + metrics (PHX_M_LOSS, _SCALE_LOSS, _SUM_M, _SUM_M2, _NIMG), dL/dm per image, dL/dscale
void launch_loss(const float* mraw, int B, const float* params, float* dm, float* dscale,
                 float* metrics, hipStream_t s);
void launch_cls_scatter(const float* scores, const uint8_t* keep, const float* mraw,
                        const int* nties, const float* dm, const float* cls_base,
                        const LevelDesc* lev, int nlev, int A, int B, int nclass, int na,
                        const float* wpred, int K, float* dx_base, const long* dx_off,
                        hipStream_t s, bool bf = false);  // bf: cls_base holds bf16 logits
void launch_count_ge(const float* sc, const int* cnt, int B, int maxo, float th, float* out,
                     hipStream_t s);
// zero up to kZeroSegs buffers (16-B aligned, sizes multiples of 16 B) in one launch
constexpr int kZeroSegs = 8;
void launch_zero_segs(char* const* ptr, const size_t* bytes, int n, hipStream_t s);
// the step's prologue in one launch: the metric row zeroed and, with caller boxes ([B,maxb,4],
// count [B]), the injected-placement slots [B,100,4] (slots past maxb zero) and counts staged
void launch_step_prologue(float* metrics, int nmetric, const float* boxes, const int32_t* count, int B, int maxb,
                          float* inj_boxes, int* inj_count, hipStream_t s);

// ---- EOT (kernels_eot.hip) ------------------------------------------------------------------
struct BoxPlace {
  int valid;        // ps*ps > min_patch_area (attacker.py:391-394)
  int ymin, xmin;   // int32-truncated placement (attacker.py:418)
  int ps, diag, pad;
  float angle, delta;
  float fwd[6];     // tfa rotate projective transform (output -> input)
  float inv[6];     // its inverse (TF-registered gradient, fill 0)
  long roff;        // offset (floats) of this box's ps*ps*3 block in the R storage
};

struct ImgParams {
  float w[3], b[3];  // print variation (attacker.py:365-372)
};

struct SpanEntry {
  int start, end;     // source span [start, end)
  float inv_total;    // 1 / sum of raw triangle weights
  float sample_f;     // span centre in source pixel units
};

struct EotDims {
  int B, H, W;        // images
  int maxb;           // box slots per image
  int P;              // patch side (640)
  int span_stride;    // SpanEntry entries per box slot (>= max ps)
  long rcap;          // R storage capacity (floats)
};

// placement rule: the attacker's Patcher.create (attacker.py:448-488: centre tolerance 0.2, the
// trained scale params[NPATCH]) or the defender's Masker.create in training (attack_detection.py:
// 450-483: tolerance 0.5, scale U(0.3, 0.5) per box)
struct PlaceRule {
  float tol = 0.2f;
  int random_scale = 0;
  float scale_lo = 0.f, scale_hi = 0.f;
};
// placement + per-image print parameters (+ R offsets).  boxes [B,maxb,4], count [B].
void launch_eot_place(const EotDims& d, const float* boxes, const int* count, const float* params,
                      uint64_t seed, int64_t step, int gimg0, ImgParams* img, BoxPlace* place,
                      SpanEntry* spans, int* err, hipStream_t s, PlaceRule rule = PlaceRule{});
// brightness matcher: out[b] = match(print(patch, img[b]), tgt[b]); mean scratch doubles [B*2*64]
void launch_eot_match(const EotDims& d, const float* patch, const ImgParams* img, const float* tgt,
                      float* matched, double* ysum, float* ymean, bool apply_print,
                      hipStream_t s);
// brightness matcher over one printed source per image (the defender's Masker: src [B,P,P,3])
void launch_eot_match_batch(const EotDims& d, const float* src, const ImgParams* img, const float* tgt,
                            float* matched, double* ysum, float* ymean, hipStream_t s);
// per box: pre = resize(matched[b]) + U(-amp, amp) noise + delta  (pre-clip values)
void launch_eot_resize(const EotDims& d, const float* matched, const BoxPlace* place,
                       const SpanEntry* spans, uint64_t seed, int64_t step, int gimg0,
                       float* rstore, hipStream_t s, float noise_amp = 0.01f);
// composite: out = paste of every valid box, owner map for the gradient; mask (optional, the
// defender's target): img_in - out on every pixel some box's region covers, 0 elsewhere
void launch_eot_composite(const EotDims& d, const float* img_in, const BoxPlace* place,
                          const float* rstore, float* img_out, int16_t* owner, hipStream_t s,
                          float* mask = nullptr);
// backward: dR (pre-clip) per box from dimg via TF's inverse-warp rotation gradient
void launch_eot_rot_bwd(const EotDims& d, const float* dimg, const int16_t* owner,
                        const BoxPlace* place, const float* rstore, float* dstore,
                        hipStream_t s);
// backward: dmatched[b] = sum_k resize^T(dR_k); tstore: eot_resize_scratch_floats(d) floats
void launch_eot_resize_bwd(const EotDims& d, const BoxPlace* place, const SpanEntry* spans,
                           const float* dstore, float* tstore, float* dmatched, hipStream_t s);
long eot_resize_scratch_floats(const EotDims& d);
// backward through brightness matcher + print variation, summed over images, + 1e-5 TV grad.
void launch_eot_patch_bwd(const EotDims& d, const float* patch, const ImgParams* img,
                          const float* ymean, const float* dmatched, double* dsum, float* grad,
                          bool add_tv, hipStream_t s);
// TV value (tf.image.total_variation) into metrics[PHX_M_TV] and 1e-5*TV added to loss
void launch_tv(const float* patch, int P, double* scratch, float* metrics, bool add_to_loss,
               hipStream_t s);
void launch_eot_count(const EotDims& d, const BoxPlace* place, float* metrics, hipStream_t s);

// Adam + clip constraints
void launch_adam_clip(float* params, const float* grad, float* m, float* v, long n, float lr,
                      int64_t t, hipStream_t s);
// plain Keras Adam (no constraints): the defender's U-Net variables
void launch_adam(float* params, const float* grad, float* m, float* v, long n, float lr, int64_t t, hipStream_t s);

}  // namespace phx
