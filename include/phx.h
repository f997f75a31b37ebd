/*
 * phx.h — C ABI of libphx.so, the MI355X-native (gfx950) adversarial-patch optimisation step.
 *
 * This is the drop-in boundary for the inner step of tiiuae/MLAdversarialObjectDetection's
 * attacker_train.py.  Each entry point replaces one reference interface; the reference
 * file:line it stands in for is given next to it (paths relative to the reference root).
 *
 * Conventions
 *  - Plain pointers and sizes only.  Device pointers are HIP device memory (e.g. PyTorch-ROCm
 *    tensors' data_ptr()); every launch is enqueued on the caller's stream (`stream`, a
 *    hipStream_t passed as void*; NULL = the null stream).  No entry point synchronises the
 *    device unless its comment says so.
 *  - Layouts: images NHWC float32 [B,H,W,3] in the victim's normalised space; boxes
 *    [ymin,xmin,ymax,xmax] float32 pixels; the trainable parameter buffer is the contiguous
 *    float32 vector [patch 640*640*3 | scale 1] (`PHX_NPARAM` floats), gradients use the same
 *    layout (the reference's `_trainable_variables = [scale, patch]`, attacker.py:63, in a
 *    flat order that lets one RCCL all-reduce cover both).
 *  - Errors: every int-returning call returns 0 on success and a negative PHX_E* code on
 *    failure; phx_last_error() returns the message.  No C++ exception crosses the ABI.
 */
#ifndef PHX_H_
#define PHX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PHX_ABI_VERSION 2

#define PHX_PATCH_SIZE 640                               /* attacker.py:43 */
#define PHX_NPATCH (PHX_PATCH_SIZE * PHX_PATCH_SIZE * 3)
#define PHX_NPARAM (PHX_NPATCH + 1)                      /* [patch | scale] */
#define PHX_MAX_OUT 100                                  /* nms max_output_size, hparams_config.py:264 */

enum {
  PHX_OK = 0,
  PHX_EINVAL = -1,   /* bad argument / shape */
  PHX_EHIP = -2,     /* HIP runtime error */
  PHX_ESTATE = -3,   /* call order (e.g. weights not loaded) */
  PHX_ECAP = -4,     /* capacity exceeded (batch > max_batch, ...) */
};

/* BN modes.  LOCAL = training-mode batch statistics over the rank's batch, as
 * the reference's attack step (victim inherits training=True, attacker.py:172); FROZEN =
 * inference BN with moving statistics (attacker.py:325 test_step); SYNC = training-mode
 * statistics over the global batch of all ranks (SyncBN: the per-channel [n, sum x, sum x^2]
 * of every BN forward and [n, sum dz, sum dz*xhat] of every BN backward are SUM-reduced through
 * the caller's collective, phx_set_allreduce), equal to one reference step on the whole batch. */
enum { PHX_BN_LOCAL = 0, PHX_BN_FROZEN = 1, PHX_BN_SYNC = 2 };

/* Arithmetic of the victim's 1x1 convolutions ("C4: bf16 act, fp32 acc").
 * F32: fp32 matrix cores (the reference's precision, BASELINE configs 1-3).  BF16: bf16 matrix
 * cores with fp32 accumulation; BN statistics, depthwise convs, EOT and the loss stay fp32. */
enum { PHX_DTYPE_F32 = 0, PHX_DTYPE_BF16 = 1 };

typedef struct phx_config {
  const char* model_name;   /* "efficientdet-d0" ... "-d7", "efficientdet-lite0".."-lite4"
                               (hparams_config.py:301-467)                                  */
  int image_size;           /* 0 = model default; square images only                         */
  int max_batch;            /* per-rank batch capacity (workspace is sized for it)            */
  int bn_mode;              /* PHX_BN_LOCAL / PHX_BN_FROZEN / PHX_BN_SYNC                     */
  float score_thresh;       /* nms_configs.score_thresh (hparams_config.py:258-266 default 0;
                               attacker_train.py:31 override 0.5).  As the reference: the first
                               pass keeps scores >= it (attacker.py:83-84) and gaussian soft-NMS
                               keeps scores > (it, or 0.001 when it is 0) (postprocess.py:186-188) */
  uint64_t seed;            /* Philox key for all EOT randomness                              */
  int compute_dtype;        /* PHX_DTYPE_F32 / PHX_DTYPE_BF16                                  */
} phx_config;

typedef struct phx_ctx phx_ctx;

/* bn=sync's collective: SUM-reduce n doubles at device address buf across the ranks, in place,
 * ordered on `stream` after the library's work so far and before its next launch (an RCCL
 * all-reduce enqueued on the stream, or a blocking one).  Returns 0 on success.  The library calls
 * it from phx_step_grad / phx_detect / phx_first_pass of a PHX_BN_SYNC context, once per BN (per
 * head group) and pass; every rank must run the same steps.  Replaces the cross-replica sums of
 * the reference's SyncBatchNormalization (automl/efficientdet/utils.py:205-241). */
typedef int (*phx_allreduce_fn)(void* user, double* buf, size_t n, void* stream);
int phx_set_allreduce(phx_ctx* ctx, phx_allreduce_fn fn, void* user);

/* Per-step metrics written by phx_step_grad (host-readable device or host memory, PHX_NMETRIC
 * floats), the reference's add_metric set, attacker.py:196-207. */
enum {
  PHX_M_LOSS = 0,        /* sum_b m_b^2 + scale_loss (+ 1e-5*TV on the rank that owns TV)  */
  PHX_M_SCALE_LOSS = 1,  /* sum_b (m_b - s)^2                                              */
  PHX_M_TV = 2,          /* total_variation(patch) (written by the rank that owns TV, else 0)  */
  PHX_M_SUM_M = 3,       /* sum_b m_b      (mean_max_score = SUM_M / B)                    */
  PHX_M_SUM_M2 = 4,      /* sum_b m_b^2    (std_max_score)                                 */
  PHX_M_ASR_NUM = 5,     /* #second-pass boxes >= 0.5 after soft-NMS                       */
  PHX_M_ASR_DEN = 6,     /* #first-pass boxes >= 0.5                                       */
  PHX_M_NBOX = 7,        /* #patches pasted                                                */
  PHX_M_NIMG = 8,        /* #images of the step (B): the metric row is SUM-all-reducible     */
  PHX_NMETRIC = 9
};

/* ---- lifetime --------------------------------------------------------------------------- */
/* Replaces util.get_victim_model (util.py:177) + infer_lib.KerasDriver.__init__
 * (infer_lib.py:385-403): builds the EfficientDet program for `cfg` on `device`. */
int phx_create(const phx_config* cfg, int device, phx_ctx** out);
void phx_destroy(phx_ctx* ctx);
/* ctx == NULL: the message of this thread's last failed phx_create. */
const char* phx_last_error(const phx_ctx* ctx);
int phx_abi_version(void);
/* The effective model configuration as JSON (hparams_config.get_efficientdet_config,
 * hparams_config.py:301-480, + the BiFPN node list of fpn_configs.get_fpn_config,
 * tf2/fpn_configs.py:166-176): name, backbone_name, image_size, fpn_num_filters,
 * fpn_cell_repeats, box_class_repeats, anchor_scale, num_scales, aspect_ratios, min_level,
 * max_level, act_type, fpn_weight_method, mean_rgb, stddev_rgb, num_classes, survival_prob,
 * fpn_nodes, score_thresh, nms_score_thresh.  Buffer protocol as phx_weight_manifest. */
int phx_model_info(const phx_ctx* ctx, char* buf, size_t cap, size_t* needed);
/* Config.override({'nms_configs': {'score_thresh': t}}) (hparams_config.py:91-109) after
 * creation: first-pass filter >= t, soft-NMS threshold t (0.001 when t == 0, method gaussian). */
int phx_set_score_thresh(phx_ctx* ctx, float score_thresh);

/* JSON list of the victim's tensors in blob order: [{"name","shape","offset","kind"}...].
 * kind: "kernel","bias","gamma","beta","moving_mean","moving_variance","wsm".
 * Writes at most `cap` bytes (NUL-terminated); *needed = full length + 1. */
int phx_weight_manifest(const phx_ctx* ctx, char* buf, size_t cap, size_t* needed);
size_t phx_weight_count(const phx_ctx* ctx);   /* floats in the blob */
/* Copies a host float32 blob laid out per the manifest (restore_ckpt, util_keras.py:108). */
int phx_load_weights(phx_ctx* ctx, const float* host_blob, size_t nfloats);
/* Copies the (possibly updated) BN moving statistics back into a host blob. */
int phx_read_weights(phx_ctx* ctx, float* host_blob, size_t nfloats);

/* ---- victim ----------------------------------------------------------------------------- */
/* EfficientDetModel.call(images, pre_mode=None, post_mode=None) (efficientdet_keras.py:966)
 * followed by postprocess.pre_nms (postprocess.py:119): per anchor max logit score (sigmoid),
 * argmax class and decoded box.  scores [B,A], classes [B,A] int32, boxes [B,A,4].
 * A = phx_num_anchors(). BN statistics per cfg.bn_mode (moving stats are updated in LOCAL). */
int phx_detect(phx_ctx* ctx, const float* images, int B, float* scores, int32_t* classes,
               float* boxes, void* stream);
int phx_num_anchors(const phx_ctx* ctx);
int phx_image_size(const phx_ctx* ctx);
/* Device bytes of the executor for batch B (activations, gradients, statistics, EOT and
 * post-processing buffers); builds (allocates) it if it does not exist yet.  SURVEY §8b's
 * phx_workspace_bytes; the library owns the workspace, no step allocates. */
int phx_workspace_bytes(phx_ctx* ctx, int B, size_t* bytes);

/* PatchAttacker.first_pass (attacker.py:91-116): detect + person/valid/threshold filter +
 * gaussian soft-NMS (postprocess.nms, postprocess.py:159-205 → NonMaxSuppressionV5) +
 * clip_boxes.  out_boxes [B,100,4], out_scores [B,100], out_count [B] (device). */
int phx_first_pass(phx_ctx* ctx, const float* images, int B, float* out_boxes,
                   float* out_scores, int32_t* out_count, void* stream);

/* Soft-NMS alone over caller-provided candidates (postprocess.nms with padded=True):
 * boxes [B,N,4], scores [B,N], count [B] valid candidates per row. */
int phx_soft_nms(phx_ctx* ctx, const float* boxes, const float* scores, const int32_t* count,
                 int B, int N, float* out_boxes, float* out_scores, int32_t* out_count,
                 void* stream);

/* ---- EOT patch pipeline ----------------------------------------------------------------- */
/* BrightnessMatcher.call((src, tgt)) (brightness_matcher.py:43-73) for one src per image:
 * src [B,P,P,3], tgt [B,H,W,3] -> out [B,P,P,3]. */
int phx_brightness_match(phx_ctx* ctx, const float* src, int P, const float* tgt, int H, int W,
                         int B, float* out, void* stream);

/* Patcher.call([boxes, images]) (attacker.py:490-498): print variation, brightness match,
 * placement, antialiased resize, noise, brightness jitter, ±20° rotate, composite, paste.
 * boxes [B,maxb,4] with count [B]; params = [patch | scale]; `step` keys the RNG.
 * Also returns per-box placements [B,maxb,8] (ymin,xmin,ps,diag,angle,delta,valid,-) if
 * `placements` is non-NULL. */
int phx_patch_images(phx_ctx* ctx, const float* images, int B, const float* boxes,
                     const int32_t* count, int maxb, const float* params, int64_t step,
                     int global_image_offset, float* out_images, float* placements,
                     void* stream);

/* ---- the step --------------------------------------------------------------------------- */
/* PatchAttacker.call(images, training=True) (attacker.py:172-219): first pass (or the
 * caller's boxes when `boxes` != NULL: "injected" placement), EOT paste, second pass, loss,
 * and the gradient of the loss w.r.t. [patch | scale] written to `grad` (PHX_NPARAM floats,
 * overwritten).  `add_tv` = 1 adds the 1e-5*TV term (rank 0 only under data parallelism).
 * metrics: PHX_NMETRIC floats (device pointer).  `global_image_offset` = rank * B keys the
 * RNG so draws are independent of the GPU count. */
int phx_step_grad(phx_ctx* ctx, const float* images, int B, const float* boxes,
                  const int32_t* count, int maxb, const float* params, int64_t step,
                  int global_image_offset, int add_tv, float* grad, float* metrics,
                  void* stream);
/* Cross-step first-pass prefetch (first-pass placement, bn=local).  The clean first pass of a step
 * depends on its images, the step (drop connect) and the image offset, not on the patch, so the
 * training loop (attacker_train.py's fit, whose generator has the next batch ready) may name the
 * next batch: the next phx_step_grad without caller boxes then also runs the first pass of
 * next_images — for step + 1 at global_image_offset — on a stream of its own beside its second pass
 * and backward, deferring that pass's BN moving-statistics updates; the phx_step_grad call for
 * exactly those images, B, step and offset applies them (after the previous step's, as in the
 * one-stream order) and places its patches by those detections (attacker.py:180-184), bit for bit
 * the result of running the first pass itself.  next_images must keep its contents until then.
 * NULL withdraws a named batch and also a first pass already prefetched for it (a caller that
 * refilled that device buffer in place: the Python mirror does this when the tensor's version
 * counter moved); the next phx_step_grad consumes a prefetch either way (one with caller boxes
 * drops it).  phx_load_weights and phx_set_score_thresh drop a pending prefetch; phx_sync makes
 * `stream` wait for one. */
int phx_set_next(phx_ctx* ctx, const float* next_images, int B, int32_t global_image_offset);
int phx_sync(phx_ctx* ctx, void* stream);

/* PatchAttacker.call(images, training=False) as run by test_step (attacker.py:318-326): the
 * victim in inference mode (BN from the moving statistics, no drop connect, moving statistics
 * unchanged), first pass (or injected boxes), EOT paste, second pass, loss and the metric row; no
 * gradient.  Optional outputs (NULL = skip): the second pass's soft-NMS person boxes / scores /
 * counts ([B,100,4], [B,100], [B]) that call returns as (boxes_pred, scores_pred). */
int phx_eval_step(phx_ctx* ctx, const float* images, int B, const float* boxes,
                  const int32_t* count, int maxb, const float* params, int64_t step,
                  int global_image_offset, int add_tv, float* metrics, float* out_boxes,
                  float* out_scores, int32_t* out_count, void* stream);

/* Keras Adam (ResourceApplyAdam, beta1 .9, beta2 .999, eps 1e-7; attacker_train.py:38) on
 * [patch | scale] followed by the variable constraints clip(patch,-1,1), clip(scale,0,1)
 * (attacker.py:51-54).  m, v: PHX_NPARAM floats each.  t = 1-based iteration. */
int phx_adam_clip(phx_ctx* ctx, float* params, const float* grad, float* m, float* v,
                  float lr, int64_t t, void* stream);

/* ---- input pipeline (off the attack step) ----------------------------- */
/* DataSequence._map_fn (train_data_generator.py:55-77) for a batch of decoded RGB uint8 images:
 * (x - mean_rgb) / stddev_rgb, resize by min(out_h/h, out_w/w) to (int(h*s), int(w*s)) with
 * cv2.resize INTER_LINEAR semantics, pasted at the top-left of a zero [out_h,out_w,3] canvas.
 * src: packed HWC uint8 images; offsets [B] int64 byte offsets into src; dims [B,2] int32
 * (h, w) — all three device pointers.  mean_rgb / stddev_rgb: 3 floats each (host).
 * out [B,out_h,out_w,3] float32 (device); out_h*out_w*3 must be a multiple of 4. */
int phx_letterbox(phx_ctx* ctx, const uint8_t* src, const int64_t* offsets, const int32_t* dims, int B,
                  const float* mean_rgb, const float* stddev_rgb, int out_h, int out_w, float* out,
                  void* stream);
/* The train-set map chain of partition() (train_data_generator.py:201-204, 222-225):
 * tf.image.random_flip_left_right -> RandomFlip('horizontal') -> RandomContrast(0.2) ->
 * tf.image.random_brightness(0.2) -> clip [-1, 1], on in [B,H,W,3] -> out (must not alias).
 * Flips are drawn per image (Philox keyed by ctx seed, step, global image index), the contrast
 * factor and brightness delta once per step (shared by every rank).  The first call for a
 * batch size allocates a small scratch (synchronous). */
int phx_augment(phx_ctx* ctx, const float* in, int B, int H, int W, int64_t step, int global_image_offset,
                float* out, void* stream);

/* Inference-time patch compositor: AdversarialPatch.add_adv_to_img (adv_patch.py:16-201) for a batch
 * of uint8 RGB images [B,H,W,3] on the device, modified in place.  boxes / count are HOST arrays:
 * boxes [B][max_boxes][4] (ymin, xmin, ymax, xmax in pixels), count [B].  patch [P,P,3] uint8
 * (device) is the unprinted patch (patch.png); the library prints it (print_patch, :40-58).  Boxes
 * are pasted in order, each brightness-matched (cv2 YUV, :110-131) against the image as patched so
 * far rescaled into out_h x out_w (:93-108), resized to the box's patch (cv2 INTER_AREA down,
 * INTER_CUBIC up, :151-164), with U(-0.01, 0.01) noise (:140-149; Philox keyed by ctx seed, step,
 * global image index, box slot).  A patch side below 1 or beyond the image is PHX_EINVAL (the
 * reference's cv2 / numpy raise there).  The first call allocates a small scratch (synchronous). */
int phx_adv_patch(phx_ctx* ctx, uint8_t* images, int B, int H, int W, const float* boxes, const int32_t* count,
                  int max_boxes, const uint8_t* patch, int patch_size, double scale, int out_h, int out_w,
                  int64_t step, int global_image_offset, void* stream);

/* Per-launch-group device timing (HIP events on the launch stream).  enable=1 clears and
 * starts recording; phx_profile_report synchronises and writes JSON
 * {kind: {count, ms, flops, bytes}} with the algorithmic FLOPs / bytes of the launches. */
int phx_profile(phx_ctx* ctx, int enable);
int phx_profile_report(phx_ctx* ctx, char* buf, size_t cap, size_t* needed);

/* Debug / test hooks (parity tests call these; not on the timed path).
 * phx_debug_last_patched: copies the last step's patched images [B,H,W,3] (device->device). */
int phx_debug_last_patched(phx_ctx* ctx, float* out, void* stream);
/* Last step's per-image max scores m_b [B] and loss-anchor index [B] (device->device). */
int phx_debug_last_maxscores(phx_ctx* ctx, float* m, int32_t* anchor, void* stream);
/* Last step's second-pass pre_nms outputs (postprocess.pre_nms, postprocess.py:119-156): per-anchor
 * scores [B,A], classes [B,A] and decoded boxes [B,A,4] (ymin, xmin, ymax, xmax px) — the values
 * the loss's person / validity masks read (attacker.py:118-141).  Any pointer may be NULL
 * (device->device). */
int phx_debug_last_detections(phx_ctx* ctx, float* scores, int32_t* classes, float* boxes, void* stream);
/* Last step's d loss / d patched images [B,H,W,3] as the EOT backward reads it (the stem dgrad
 * writes it only at pixels a paste owns; elsewhere 0) (device->device). */
int phx_debug_last_image_grad(phx_ctx* ctx, float* out, void* stream);
/* Per-layer diagnostics of the last step.  `op_name` names an op of the program: a batch norm by
 * its weight prefix (e.g. "efficientnet-b0/blocks_3/tpu_batch_normalization_1"), a BiFPN fuse as
 * "<node>/fuse", a resampling max-pool / upsample as "<resample prefix>/max_pool" / "/upsample".
 * which = 0 copies the op's output (for a batch norm, which is never materialised: its input), which
 * = 1 the loss gradient w.r.t. its output (a batch norm's after its activation); NHWC [B,h,w,C] =
 * nfloats floats (device->device).  PHX_EINVAL if the name or size is wrong, or no gradient exists. */
int phx_debug_tap(phx_ctx* ctx, const char* op_name, int which, float* out, size_t nfloats, void* stream);
/* Stream-hazard diagnostics.  With PHX_CKSUM=1 in the environment (read per call), every
 * phx_step_grad takes an order-independent 64-bit hash of each tensor / statistics slot an op
 * writes, on the op's stream right after it.  This copies the last step's list ("name\thex\n" lines,
 * launch order) of the executor with `tag` (0: the step's, 1: the concurrent first pass's) into buf
 * (synchronising); *needed = bytes including the NUL.  Two steps on the same inputs must give the
 * same list; the first differing line names the launch that broke. */
int phx_debug_checksums(phx_ctx* ctx, int tag, char* buf, size_t cap, size_t* needed);
/* The raw storage (bf16 words in a PHX_DTYPE_BF16 context) of op `op_index`'s output (which = 0) or
 * input which - 1 in the last step's executor `tag`; nbytes must equal its size (device->device). */
int phx_debug_tensor(phx_ctx* ctx, int tag, int op_index, int which, void* out, size_t nbytes, void* stream);

/* ---- defender step (BASELINE C5) ------------------------------------------
 * attack_detection.PatchAttackDefender (attack_detection.py:31-206, training) over a frozen
 * victim ctx: first pass (inference BN, person anchors, soft-NMS, filter_valid_boxes), Masker
 * (self-supervised patches, attack_detection.py:321-498), 2 * PatchNeutralizer(images)
 * (generator.py:17-277: attention U-Net, n_filters 8, dropout 0.2, batch norm) and
 * loss = sum_b mean((targets - updates)^2) with its gradient w.r.t. the U-Net variables.
 * The variables are one flat float buffer in phx_def_manifest order (Keras shapes and layouts:
 * conv kernels [k,k,in,out], transposed-conv kernels [k,k,out,in]); the library owns the BN moving
 * statistics (updated by every step, as Keras training-mode BN).  Replaces generator.define_model
 * + PatchAttackDefender.__init__ (attack_detection.py:34-71). */
typedef struct phx_def phx_def;
/* the U-Net at the victim's image size (a multiple of 16, >= 240); seed keys the Masker's and
 * Dropout's Philox draws */
int phx_def_create(phx_ctx* victim, int max_batch, uint64_t seed, phx_def** out);
void phx_def_destroy(phx_def* d);
/* d == NULL: the message of this thread's last failed phx_def_create. */
const char* phx_def_last_error(phx_def* d);
int64_t phx_def_num_params(phx_def* d);
int64_t phx_def_num_moving(phx_def* d);
/* JSON {n_params, n_moving, params: [{name, shape, offset}], bn: [{name, channels, moving_mean,
 * moving_variance}]} (offsets in floats) */
int phx_def_manifest(phx_def* d, char* buf, size_t cap, size_t* needed);
/* BN moving statistics: src != NULL loads them, dst != NULL copies them out (any memory) */
int phx_def_moving(phx_def* d, float* dst, const float* src, void* stream);
/* Device bytes of the batch-B workspace a training step uses (built if needed). */
int phx_def_workspace_bytes(phx_def* d, int B, size_t* bytes);
/* Device bytes the first phx_def_eval_step at batch B adds to that workspace (the evaluation
 * Masker's matched patches and worst-case resized-patch store, reserved on first use and freed with
 * the workspace); a run that only trains never holds them. */
int phx_def_eval_workspace_bytes(phx_def* d, int B, size_t* bytes);
/* PatchAttackDefender.call(images, training=True) + tape.gradient (attack_detection.py:168-206).
 * boxes [B,100,4] + count [B] (device) place the patches; NULL = the victim's first pass.
 * grad: num_params floats followed by the metric row [loss] (SUM-all-reducible). */
int phx_def_step_grad(phx_def* d, const float* images, int B, const float* boxes, const int32_t* count,
                      const float* params, float* grad, int64_t step, int32_t global_image_offset, void* stream);
/* Cross-step first-pass prefetch.  The first pass of a training step depends only on its images
 * (the protege is frozen), so the host loop (defender_train.py's fit over the generator, which has
 * the next batch ready) may name the next batch: the next phx_def_step_grad then also runs the
 * victim's first pass of next_images — for step + 1 at global_image_offset — on the defender's own
 * stream beside its U-Net work, into a second box buffer, and the phx_def_step_grad call for exactly
 * those images, B, step and offset (without caller boxes) uses those boxes instead of running the
 * first pass (attack_detection.py:174-178: the same boxes either way).  next_images must keep its
 * contents until that call; NULL withdraws it, and a prefetch already made (a refilled buffer).  A
 * prefetch made at another victim generation (a weight load, a training pass or new score thresholds
 * on the victim ctx since) is not used.  A prefetch ties up the victim ctx until it
 * finishes: the defender's own calls wait for it, other users of the victim ctx call phx_def_sync
 * on their stream first. */
int phx_def_set_next(phx_def* d, const float* next_images, int B, int32_t global_image_offset);
/* makes `stream` wait for the first pass a phx_def_set_next prefetch has in flight */
int phx_def_sync(phx_def* d, void* stream);
/* PatchAttackDefender.call(images, training=False) as test_step runs it (attack_detection.py:168-198,
 * 320-326): first pass (or the caller's boxes), the Masker's evaluation branch with the attacker's
 * trained patch — eval_patch = [patch 640*640*3 | scale] (device; the PatchAttackDefender eval_patch
 * directory's patch.tiff / scale.txt, :57-61) — print variation, brightness match, centred placement
 * at the fixed scale (:454-456), the second detector pass odet_model(images, score_thresh=0.)
 * (:185-187, soft-NMS threshold 0.001, filter_valid_boxes at the config's threshold), updates =
 * 2 * PatchNeutralizer(images, training=False) (inference BN, no Dropout) and the loss.  metrics:
 * [loss] (1 float, device).  out_boxes [B,100,4] / out_scores [B,100] / out_count [B]: the second
 * pass's detections (NULL = skip).  No variable or moving statistic changes. */
int phx_def_eval_step(phx_def* d, const float* images, int B, const float* boxes, const int32_t* count,
                      const float* params, const float* eval_patch, float* metrics, float* out_boxes,
                      float* out_scores, int32_t* out_count, int64_t step, int32_t global_image_offset,
                      void* stream);
/* debug copies of the last step (device->device): patched images / targets / updates [B,H,W,3],
 * first-pass boxes [B,100,4], counts [B] (int32 bits) */
enum { PHX_DEF_PATCHED = 0, PHX_DEF_TARGETS = 1, PHX_DEF_UPDATES = 2, PHX_DEF_BOXES = 3, PHX_DEF_COUNTS = 4 };
int phx_def_debug(phx_def* d, int what, float* dst, size_t nfloats, void* stream);
/* Keras Adam without constraints (the defender's optimizer, defender_train.py:35) */
int phx_adam(float* params, const float* grad, float* m, float* v, int64_t n, float lr, int64_t t, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PHX_H_ */
