// kernels_post.hip — detection post-processing on the attack path:
//   pre_nms            automl/efficientdet/tf2/postprocess.py:67-156 (level merge, per-anchor class
//                      max/argmax, box decode anchors.py:30-58, sigmoid)
//   person/valid mask  attacker.py:69-89, 105-113, 132-140
//   soft-NMS           postprocess.py:159-205 -> tf.raw_ops.NonMaxSuppressionV5 (gaussian),
//                      restated from TF's non_max_suppression_op.cc [TF-recall]
//   loss               attacker.py:189-193 and its gradient (ragged reduce_max, maximum(.,0))
// Arithmetic that decides discrete outcomes (masks, thresholds, argmax) is kept in TF's fp32
// operation order with FMA contraction disabled.
#include <algorithm>

#include "common.hpp"
#include "kernels.hpp"
#include "post.hpp"

#pragma clang fp contract(off)

namespace phx {

__device__ __forceinline__ float sigmoid_exact(float x) { return 1.0f / (1.0f + expf(-x)); }

// ------------------------------------------------------------------------------------------
// soft-NMS candidate lists, appended by pre_nms: every (image, anchor) with keep & mask and a
// score above the NMS threshold (NonMaxSuppressionV5 drops the rest up front).  A workgroup counts
// its tile's candidates, reserves a range of the image's list with one atomic, and writes the anchor
// indices in anchor order; ranges of different tiles land in any order, so k_soft_nms breaks score
// ties by anchor index (the order of the reference's ragged candidate list), which makes its
// result independent of the list order.  k_soft_nms resets the count after reading it.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void nms_cand_append(const NmsCand& c, int b, int A, bool want, int a) {
  __shared__ int wcount[4], wbase[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(want);
  if (lane == 0) wcount[wave] = __popcll(bal);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = wcount[0] + wcount[1] + wcount[2] + wcount[3];
    const int base = tot ? atomicAdd(c.count + b, tot) : 0;
    wbase[0] = base;
    wbase[1] = base + wcount[0];
    wbase[2] = wbase[1] + wcount[1];
    wbase[3] = wbase[2] + wcount[2];
  }
  __syncthreads();
  if (want) {
    const int pos = wbase[wave] + __popcll(bal & ((1ull << lane) - 1ull));
    if (pos < A) c.list[(long)b * A + pos] = a;  // a list never holds more than the image's anchors
  }
}

// ------------------------------------------------------------------------------------------
// pre_nms + masks.  A workgroup owns a tile of 128 consecutive anchors of one (image, level):
// their 128 x 90 logits are one contiguous 46 KB run, staged into LDS with float4 loads, then
// lane t reduces anchor t's 90 classes (max, first argmax) and decodes its box.
// ------------------------------------------------------------------------------------------
constexpr int kPreTile = 128;

// BF: the class / box outputs are bf16 activations (PHX_DTYPE_BF16); widened to fp32 when staged
template <bool BF>
__global__ __launch_bounds__(256) void k_pre_nms(const float* __restrict__ cls_base,
                                                 const float* __restrict__ box_base,
                                                 const LevelDesc* __restrict__ lev, int nlev,
                                                 const float* __restrict__ anchors, int A, int B,
                                                 int nclass, int na, float img_h, float img_w,
                                                 float thresh, float* __restrict__ scores,
                                                 int* __restrict__ classes,
                                                 float* __restrict__ boxes,
                                                 uint8_t* __restrict__ keep, NmsCand cand) {
  extern __shared__ float4 smem4[];
  float* lg_s = reinterpret_cast<float*>(smem4);
  const int b = blockIdx.y;
  int l = 0;
  while (l + 1 < nlev && (int)blockIdx.x >= lev[l + 1].tile0) ++l;
  const LevelDesc L = lev[l];
  const int nloc = L.h * L.w * na;                      // anchors of this level per image
  const int a0 = ((int)blockIdx.x - L.tile0) * kPreTile;  // first local anchor of the tile
  const int n = min(kPreTile, nloc - a0);
  const long run = ((long)b * nloc + a0) * nclass;      // element offset of the tile's logits
  const int nf = n * nclass;
  const int nf4 = nf >> 2;
  if constexpr (BF) {
    const long e0 = L.cls_off + run;
    const uint16_t* src = reinterpret_cast<const uint16_t*>(cls_base) + e0;
    if ((e0 & 3) == 0) {
      const uint2* src4 = reinterpret_cast<const uint2*>(src);
      int i = threadIdx.x;
      for (; i + 768 < nf4; i += 1024) {
        uint2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = src4[i + 256 * u];
#pragma unroll
        for (int u = 0; u < 4; ++u) smem4[i + 256 * u] = unpack_bf16x4(v[u]);
      }
      for (; i < nf4; i += blockDim.x) smem4[i] = unpack_bf16x4(src4[i]);
      for (int j = (nf4 << 2) + threadIdx.x; j < nf; j += blockDim.x) lg_s[j] = ald1<true>(cls_base, e0 + j);
    } else {
      for (int j = threadIdx.x; j < nf; j += blockDim.x) lg_s[j] = ald1<true>(cls_base, e0 + j);
    }
  } else {
  const float* src = cls_base + L.cls_off + run;
  const float4* src4 = reinterpret_cast<const float4*>(src);
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    // staging: four 16-B loads in flight per lane before any LDS store (all of a lane's loads at
    // once — 12 — measured slower: 99 -> 125 us, the staging registers cost occupancy)
    int i = threadIdx.x;
    for (; i + 768 < nf4; i += 1024) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = src4[i + 256 * u];
#pragma unroll
      for (int u = 0; u < 4; ++u) smem4[i + 256 * u] = v[u];
    }
    for (; i < nf4; i += blockDim.x) smem4[i] = src4[i];
    for (int j = (nf4 << 2) + threadIdx.x; j < nf; j += blockDim.x) lg_s[j] = src[j];
  } else {
    // a run that starts off a 16-B boundary (an image of a level with an odd pixel count, e.g. a
    // 1x1 or 5x5 P7: h*w*9*90 floats per image): scalar staging
    for (int j = threadIdx.x; j < nf; j += blockDim.x) lg_s[j] = src[j];
  }
  }
  __syncthreads();
  // two lanes per anchor (lanes t and t + 128 of the block are in different waves, so the halves
  // meet in LDS): each scans half the classes for (max, first argmax); the second half wins only
  // when strictly greater, which keeps the first-occurrence argmax of the sequential scan
  const int t = threadIdx.x & (kPreTile - 1), half = threadIdx.x >> 7;
  const int hc = (nclass + 1) / 2;
  const int c0 = half * hc, c1 = min(nclass, c0 + hc);
  float m = -INFINITY;
  int am = c0;
  if (t < n && c0 < c1) {
    const float* lg = lg_s + t * nclass;
    m = lg[c0];
    for (int c = c0 + 1; c < c1; ++c) {
      float v = lg[c];
      if (v > m) { m = v; am = c; }
    }
  }
  __shared__ float hm[kPreTile];
  __shared__ int ha_[kPreTile];
  if (half == 1) {
    hm[t] = m;
    ha_[t] = am;
  }
  __syncthreads();
  // the candidate append below is a workgroup collective (ballots + barriers): every thread reaches
  // it exactly once, at the same program point, so nothing returns early
  const bool live = half == 0 && t < n;
  bool want = false;
  const int a = L.anchor0 + a0 + t;
  if (live) {
  if (c0 + hc < nclass && hm[t] > m) {
    m = hm[t];
    am = ha_[t];
  }
  const long idx = (long)b * A + a;
  const float4 bx = ald4<BF>(box_base, L.box_off + ((long)b * nloc + a0 + t) * 4);
  const float4 an = *reinterpret_cast<const float4*>(anchors + (long)a * 4);
  float yca = (an.x + an.z) / 2.0f;
  float xca = (an.y + an.w) / 2.0f;
  float ha = an.z - an.x;
  float wa = an.w - an.y;
  float w = expf(bx.w) * wa;
  float h = expf(bx.z) * ha;
  float yc = bx.x * ha + yca;
  float xc = bx.y * wa + xca;
  float ymin = yc - h / 2.0f, xmin = xc - w / 2.0f, ymax = yc + h / 2.0f, xmax = xc + w / 2.0f;
  float sc = sigmoid_exact(m);
  scores[idx] = sc;
  classes[idx] = am;
  *reinterpret_cast<float4*>(boxes + idx * 4) = make_float4(ymin, xmin, ymax, xmax);
  // filter_valid_boxes (attacker.py:69-89): boxes_h/w from the decoded box
  float bh = ymax - ymin, bw = xmax - xmin;
  float area = bh * bw;
  bool valid = (bw / img_w <= 1.0f) && (bh / img_h <= 1.0f) && (area > 100.0f);
  uint8_t kf = 0;
  if (am == 0 && valid) {
    kf = 1;
    if (sc >= thresh) kf |= 2;
  }
  if (am == 0) kf |= 4;  // person, before the validity filter (the defender's odet_model)
  keep[idx] = kf;
  want = (kf & cand.mask) != 0 && sc > cand.thresh;
  }
  if (cand.list) nms_cand_append(cand, b, A, want, a);
}

void launch_pre_nms(const float* cls_base, const float* box_base, const LevelDesc* lev_dev,
                    int nlev, const float* anchors, int A, int B, int nclass, int na,
                    float img_h, float img_w, float thresh, float* scores, int* classes,
                    float* boxes, uint8_t* keep, int ntiles, hipStream_t s, NmsCand cand, bool bf) {
  size_t shm = (size_t)kPreTile * nclass * sizeof(float);
  if (bf)
    hipLaunchKernelGGL(k_pre_nms<true>, dim3(ntiles, B), dim3(256), shm, s, cls_base, box_base, lev_dev, nlev,
                       anchors, A, B, nclass, na, img_h, img_w, thresh, scores, classes, boxes, keep, cand);
  else
    hipLaunchKernelGGL(k_pre_nms<false>, dim3(ntiles, B), dim3(256), shm, s, cls_base, box_base, lev_dev, nlev,
                       anchors, A, B, nclass, na, img_h, img_w, thresh, scores, classes, boxes, keep, cand);
  PHX_LAUNCH_CHECK();
}

int pre_nms_tiles(int h, int w, int na) { return (h * w * na + kPreTile - 1) / kPreTile; }

// ------------------------------------------------------------------------------------------
// soft-NMS: one workgroup per image.  Exact restatement of NonMaxSuppressionV5's lazy
// priority queue: pop the (score desc, candidate order asc) maximum, decay it by every box
// selected since its last visit (newest first, early exit at <= thresh), select if unchanged,
// else re-queue while > thresh.  Candidate order = ragged (anchor) order.
//
// Layout (one image, dynamic LDS up to 160 KB):
//  * candidates are compacted in anchor order (a bitmap of the candidate anchors, then a
//    workgroup scan), so the candidate position IS the tie order and the queue key of position
//    c is the 64-bit (score bits << 32 | ~c): scores are positive floats, so an unsigned max
//    picks the higher score and, among equals, the lower position.  Removed = key 0.
//  * the candidates' boxes are copied to a compacted global array (one load per pop);
//  * score bits and last-visit counts live in LDS for the first `cap` positions, in global
//    memory beyond; per-chunk maxima (chunks of 64*m positions) and per-group maxima (groups of
//    64 chunks) in LDS, so a pop is one group scan, and a re-queue one chunk + one group rescan.
//  * the pop loop runs in wave 0 alone (no workgroup barriers); its state is wave-uniform.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float tf_iou(const float* bi, const float* bj) {
  const float ymin_i = fminf(bi[0], bi[2]), xmin_i = fminf(bi[1], bi[3]);
  const float ymax_i = fmaxf(bi[0], bi[2]), xmax_i = fmaxf(bi[1], bi[3]);
  const float ymin_j = fminf(bj[0], bj[2]), xmin_j = fminf(bj[1], bj[3]);
  const float ymax_j = fmaxf(bj[0], bj[2]), xmax_j = fmaxf(bj[1], bj[3]);
  const float area_i = (ymax_i - ymin_i) * (xmax_i - xmin_i);
  const float area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j);
  if (area_i <= 0.f || area_j <= 0.f) return 0.f;
  const float iy0 = fmaxf(ymin_i, ymin_j), ix0 = fmaxf(xmin_i, xmin_j);
  const float iy1 = fminf(ymax_i, ymax_j), ix1 = fminf(xmax_i, xmax_j);
  const float inter = fmaxf(iy1 - iy0, 0.f) * fmaxf(ix1 - ix0, 0.f);
  return inter / (area_i + area_j - inter);
}

constexpr int kNmsThreads = 256;
constexpr int kNmsLdsBytes = 160 * 1024;
constexpr int kNmsGroups = 64;  // group maxima (<= 64 groups of 64 chunks)

struct NmsPlan {
  int m;        // chunk = 64*m positions
  int nchunk;   // chunks for N positions
  int ck_bytes; // chunk-key region (also the bitmap of N bits during compaction)
  int cap;      // positions whose key / visit count live in LDS
  int lds;      // dynamic LDS bytes
  int lp;       // top-list sort size of the fast path (power of 2, <= kNmsTopMax)
  int qrows;    // re-queue rows of the fast path (0: general queue only)
};

// Fast path (k_soft_nms phases F1-F4): batches of the highest-scoring unlisted candidates — at least
// kNmsTopWant each, all of them when fewer are left — sorted by queue key, their boxes in LDS.  Every
// candidate outside the batch scores below the batch, so a pop is exact whenever the batch or the
// re-queue set holds the maximum; the next batch is built when neither does.  Wave 0 takes the batch
// 64 candidates at a time (a "row", lane j = the row's j-th candidate) and visits all of them at
// once, one per lane, against every selection so far (the per-lane product in TF's newest-first
// order); a row candidate's visit stays exact until a later selection overlaps it (a decay factor
// other than exactly 1 would come first in TF's product), which marks it for a fresh visit at its
// pop.  Popping a fresh candidate is then a handful of scalar operations.  Visited candidates that
// stay above the threshold are re-queued in place (the row's lanes); a used-up row moves its
// re-queued entries to a free row of the re-queue set in LDS (qrows rows of 64, one max per row in a
// lane of wave 0).  The general queue (phases 3-5) runs instead when a batch or the re-queue set
// overflows its LDS capacity.
constexpr int kNmsTopWant = 960;  // a batch of ~1000 sorts at 1024 entries
constexpr int kNmsTopMax = 4096;
constexpr int kNmsHistBins = 4096;
constexpr int kNmsRowBytes = 64 * (8 + 16 + 4);  // a re-queue row: keys | boxes | last-visit counts
constexpr int kNmsFl = 24;  // decay factors other than 1 kept per row candidate (its product's terms)
constexpr int kNmsSelBytes = PHX_MAX_OUT_DEV * 16 + (PHX_MAX_OUT_DEV * 4 + 15) / 16 * 16 + kNmsFl * 64 * 4;

static NmsPlan nms_plan(int N) {
  NmsPlan p;
  p.m = std::max(1, cdiv(N, 64L * 64 * kNmsGroups));
  p.nchunk = cdiv(N, 64L * p.m);
  const int bitmap = cdiv(N, 64) * 8;
  p.ck_bytes = (std::max(p.nchunk * 8, bitmap) + 15) / 16 * 16;
  const int fixed = kNmsGroups * 8 + PHX_MAX_OUT_DEV * 16 + PHX_MAX_OUT_DEV * 4 + kNmsThreads * 4 + 64;
  int cap = (kNmsLdsBytes - fixed - p.ck_bytes) / 5 / 64 * 64;
  p.cap = std::max(0, std::min(cap, (N + 63) / 64 * 64));
  p.lds = fixed + p.ck_bytes + p.cap * 5;
  // fast path scratch after the fixed region: sort keys (u64; the score histogram before) | sort
  // payload (u32) | list boxes (float4) | normalised selected boxes + areas | re-queue rows
  p.lp = 4;  // >= 4: the list boxes after the u32 payload stay 16-B aligned
  while (p.lp < std::min(N, kNmsTopMax)) p.lp <<= 1;
  const int fast = std::max(p.lp * 8, kNmsHistBins * 4) + p.lp * 4 + p.lp * 16 + kNmsSelBytes;
  // PHX_NMS_FAST=0: the general queue only (A/B and diagnosis; read per call, so one process can
  // compare both paths bit for bit)
  const char* fe = std::getenv("PHX_NMS_FAST");
  const bool fast_on = !(fe && fe[0] == '0');
  p.qrows = fast_on ? std::max(0, std::min(64, (kNmsLdsBytes - fixed - p.ck_bytes - fast) / kNmsRowBytes)) : 0;
  p.lds = std::max(p.lds, fixed + p.ck_bytes + fast + p.qrows * kNmsRowBytes);
  p.lds = (p.lds + 15) / 16 * 16;
  return p;
}

// Wave-wide max of a 64-bit key, on the queue's critical path (a dependent chain per pop): the max
// of the high words, then of the low words among the lanes holding it — each within 16-lane rows by
// DPP (quad xor 1, xor 2, half-row mirror, row mirror: one v_max with a DPP operand per step), the
// four row maxima by readlane.  A shuffle (ds_bpermute) per step cost ~6x as much.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, false));  // row_mirror
  const uint32_t a = max((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16));
  const uint32_t c = max((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48));
  return max(a, c);
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
  const uint32_t mh = wave_max_u32(hi);
  const uint32_t ml = wave_max_u32(hi == mh ? lo : 0u);
  return ((uint64_t)mh << 32) | ml;
}

// sc = orig * f(newest) * f(next) * ... in that order (lane l holds the factor of selection
// nsel-1-l in f0 and of nsel-65-l in f1; lanes past the visit's selections hold 1).  TF stops at the
// first product <= thresh; every factor lies in (0, 1], so the full product is <= thresh as well and
// the outcome is the same — the chain runs without a per-factor test.  A factor of exactly 1 (a
// selected box that does not overlap: exp(0)) leaves the product unchanged, so only the lanes whose
// factor differs from 1 are multiplied in, in lane order: a short dependent chain of scalar
// multiplies instead of one per selection.
__device__ __forceinline__ float decay_chain(float orig, float f0, float f1) {
  float sc = orig;
  unsigned long long m0 = __ballot(f0 != 1.f), m1 = __ballot(f1 != 1.f);
  while (m0) {
    const int l = __ffsll(m0) - 1;
    m0 &= m0 - 1ull;
    sc *= __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(f0), l));
  }
  while (m1) {
    const int l = __ffsll(m1) - 1;
    m1 &= m1 - 1ull;
    sc *= __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(f1), l));
  }
  return sc;
}

__device__ __forceinline__ uint64_t nms_key(uint32_t sbits, int pos) {
  return sbits ? (((uint64_t)sbits << 32) | (uint32_t)~(uint32_t)pos) : 0ull;
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

__device__ __forceinline__ float4 readlane_f4(float4 v, int l) {
  return make_float4(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), l)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), l)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.z), l)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.w), l)));
}

// A visit of one candidate (box cb4, queue score orig) by the whole wave: the decay factors of the
// selections [from, nsel) — lane l computes selection nsel-1-l (and nsel-65-l) — and TF's product.
__device__ __forceinline__ float nms_visit(float4 cb4, float orig, int from, int nsel, const float4* s_sel,
                                           float scale, int lane) {
  const float cb[4] = {cb4.x, cb4.y, cb4.z, cb4.w};
  const int nf = nsel - from;
  float f0 = 1.f, f1 = 1.f;
  if (lane < nf) {
    const float4 s4 = s_sel[nsel - 1 - lane];
    const float sbx[4] = {s4.x, s4.y, s4.z, s4.w};
    const float sim = tf_iou(cb, sbx);
    f0 = expf(scale * sim * sim);
  }
  if (lane + 64 < nf) {
    const float4 s4 = s_sel[nsel - 65 - lane];
    const float sbx[4] = {s4.x, s4.y, s4.z, s4.w};
    const float sim = tf_iou(cb, sbx);
    f1 = expf(scale * sim * sim);
  }
  return decay_chain(orig, f0, f1);
}

// tf_iou's operands with the corners ordered and the area taken (the same operations in the same
// order, so nms_factor(norm(i), norm(j)) == expf(scale * iou^2) of tf_iou(i, j) bit for bit)
struct NmsNBox {
  float y0, x0, y1, x1, a;
};

__device__ __forceinline__ NmsNBox nms_norm(float4 b) {
  NmsNBox n;
  n.y0 = fminf(b.x, b.z);
  n.x0 = fminf(b.y, b.w);
  n.y1 = fmaxf(b.x, b.z);
  n.x1 = fmaxf(b.y, b.w);
  n.a = (n.y1 - n.y0) * (n.x1 - n.x0);
  return n;
}

__device__ __forceinline__ NmsNBox nms_sel_at(const float4* s_seln, const float* s_sela, int k) {
  const float4 v = s_seln[k];
  return NmsNBox{v.x, v.y, v.z, v.w, s_sela[k]};
}

// whether candidate c and selection s intersect; when not, their decay factor is exactly 1
__device__ __forceinline__ bool nms_overlap(const NmsNBox& c, const NmsNBox& s) {
  return fminf(c.y1, s.y1) > fmaxf(c.y0, s.y0) && fminf(c.x1, s.x1) > fmaxf(c.x0, s.x0);
}

__device__ __forceinline__ float nms_factor(const NmsNBox& c, const NmsNBox& s, float scale) {
  if (c.a <= 0.f || s.a <= 0.f) return 1.f;
  const float iy0 = fmaxf(c.y0, s.y0), ix0 = fmaxf(c.x0, s.x0);
  const float iy1 = fminf(c.y1, s.y1), ix1 = fminf(c.x1, s.x1);
  const float inter = fmaxf(iy1 - iy0, 0.f) * fmaxf(ix1 - ix0, 0.f);
  const float sim = inter / (c.a + s.a - inter);
  return expf(scale * sim * sim);
}

// nms_visit on the normalised selections: the factors of the selections that do not intersect the
// candidate are exactly 1 and skipped without the division and exponential
__device__ __forceinline__ float nms_visit_n(const NmsNBox& cn, float orig, int from, int nsel, const float4* s_seln,
                                             const float* s_sela, float scale, int lane) {
  const int nf = nsel - from;
  float f0 = 1.f, f1 = 1.f;
  if (lane < nf) {
    const NmsNBox sn = nms_sel_at(s_seln, s_sela, nsel - 1 - lane);
    if (nms_overlap(cn, sn)) f0 = nms_factor(cn, sn, scale);
  }
  if (lane + 64 < nf) {
    const NmsNBox sn = nms_sel_at(s_seln, s_sela, nsel - 65 - lane);
    if (nms_overlap(cn, sn)) f1 = nms_factor(cn, sn, scale);
  }
  return decay_chain(orig, f0, f1);
}

__global__ __launch_bounds__(kNmsThreads) void k_soft_nms(
    const float* __restrict__ boxes, const float* __restrict__ scores,
    const uint8_t* __restrict__ keep, int keep_mask, const int* __restrict__ count, int N,
    float score_thresh, float scale, int max_out, float clip_hi, float* __restrict__ out_boxes,
    float* __restrict__ out_scores, int* __restrict__ out_count, float4* __restrict__ cbox_all,
    uint32_t* __restrict__ gkey_all, int* __restrict__ gwi_all, uint8_t* __restrict__ gwb_all,
    NmsCand cand, NmsPlan pl, int dbg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char nms_smem[];
  const int b = blockIdx.x;
  // wave: readfirstlane makes it (and everything decided in wave 0's queue loop) uniform to the
  // compiler, so the loop's state lives in scalar registers and its branches are scalar
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const float* bb = boxes + (long)b * N * 4;
  const float* sb = scores + (long)b * N;
  float4* cbox = cbox_all + (long)b * N;
  uint32_t* gkey = gkey_all + (long)b * N;
  int* gwi = gwi_all + (long)b * N;
  uint8_t* gwb = gwb_all + (long)b * N;

  uint64_t* s_ck = reinterpret_cast<uint64_t*>(nms_smem);       // chunk maxima (or the bitmap)
  uint32_t* s_bm = reinterpret_cast<uint32_t*>(nms_smem);
  uint64_t* s_gk = reinterpret_cast<uint64_t*>(nms_smem + pl.ck_bytes);
  float4* s_sel = reinterpret_cast<float4*>(s_gk + kNmsGroups);
  float* s_sels = reinterpret_cast<float*>(s_sel + PHX_MAX_OUT_DEV);
  int* s_scan = reinterpret_cast<int*>(s_sels + PHX_MAX_OUT_DEV);
  int* s_misc = s_scan + kNmsThreads;
  uint32_t* s_key = reinterpret_cast<uint32_t*>(s_misc + 16);
  uint8_t* s_wb = reinterpret_cast<uint8_t*>(s_key + pl.cap);
  const int cap = pl.cap;

  // PHX_NMS_STATS: phase times (100 MHz realtime clock; stamps only when dbg)
  auto stamp = [&]() -> uint64_t { return dbg ? __builtin_amdgcn_s_memrealtime() : 0ull; };
  const uint64_t ts0 = stamp();
  // 1. bitmap of the candidate anchors (or count-prefix positions)
  const int nbits = N;
  const int nwords = (nbits + 63) / 64 * 2;
  for (int w = t; w < nwords; w += kNmsThreads) s_bm[w] = 0u;
  if (cand.list && t == 0) s_misc[0] = min(cand.count[b], N);
  __syncthreads();
  if (cand.list) {
    // candidates appended by pre_nms (score > thresh and keep & mask already applied)
    const int nl = s_misc[0];
    const int* lst = cand.list + (long)b * N;
    for (int i = t; i < nl; i += kNmsThreads) {
      const int a = lst[i];
      atomicOr(&s_bm[a >> 5], 1u << (a & 31));
    }
    __syncthreads();
    if (t == 0) cand.count[b] = 0;  // consumed: the next pre_nms appends from 0
  } else {
    const int n_in = count ? min(count[b], N) : N;
    for (int base = 0; base < n_in; base += 4 * kNmsThreads) {
      bool ok[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = base + u * kNmsThreads + t;
        const int ic = min(i, N - 1);
        bool o = sb[ic] > score_thresh;
        if (keep) o = o && ((keep[(long)b * N + ic] & keep_mask) != 0);
        ok[u] = o && i < n_in;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const unsigned long long bal = __ballot(ok[u]);
        const int w0 = (base + u * kNmsThreads + wave * 64) >> 5;
        if (lane == 0 && w0 < nwords) {
          s_bm[w0] = (uint32_t)bal;
          s_bm[w0 + 1] = (uint32_t)(bal >> 32);
        }
      }
    }
  }
  __syncthreads();

  // 2. ordered compaction: thread t owns words [t*per, (t+1)*per); a workgroup scan of their
  //    popcounts places the anchors in order (written to gwi)
  const int per = (nwords + kNmsThreads - 1) / kNmsThreads;
  const int w_lo = min(nwords, t * per), w_hi = min(nwords, w_lo + per);
  int cnt = 0;
  for (int w = w_lo; w < w_hi; ++w) cnt += __popc(s_bm[w]);
  s_scan[t] = cnt;
  __syncthreads();
  for (int off = 1; off < kNmsThreads; off <<= 1) {
    const int v = t >= off ? s_scan[t - off] : 0;
    __syncthreads();
    s_scan[t] += v;
    __syncthreads();
  }
  {
    int pos = s_scan[t] - cnt;
    for (int w = w_lo; w < w_hi; ++w) {
      uint32_t bits = s_bm[w];
      while (bits) {
        const int bit = __ffs(bits) - 1;
        bits &= bits - 1;
        gwi[pos++] = w * 32 + bit;
      }
    }
  }
  const int n = __builtin_amdgcn_readfirstlane(s_scan[kNmsThreads - 1]);
  __syncthreads();  // gwi complete (global writes of this workgroup, visible after the barrier)

  // ---- fast path -------------------------------------------------------------------------
  // Batches of the highest-scoring candidates not yet listed (>= kNmsTopWant each, or all that are
  // left), sorted by queue key with their boxes in LDS; wave 0 pops from the batch's rows and from
  // the re-queue set (rows of 64 in LDS) and asks for the next batch when the batch is used up while
  // an unlisted candidate could be next.  The general queue below runs instead (from scratch) when a
  // batch or the re-queue set overflows.
  bool fast_done = false;
  if (pl.qrows > 0) {
    unsigned char* fbase = reinterpret_cast<unsigned char*>(s_key);
    uint32_t* hist = reinterpret_cast<uint32_t*>(fbase);                    // [kNmsHistBins]
    uint64_t* lkey = reinterpret_cast<uint64_t*>(fbase);                    // [lp] (after the histograms)
    uint32_t* lpay = reinterpret_cast<uint32_t*>(fbase + max(pl.lp * 8, kNmsHistBins * 4));  // [lp]
    float4* lbox = reinterpret_cast<float4*>(reinterpret_cast<unsigned char*>(lpay) + pl.lp * 4);  // [lp]
    float4* s_seln = lbox + pl.lp;                                           // [PHX_MAX_OUT_DEV]
    float* s_sela = reinterpret_cast<float*>(s_seln + PHX_MAX_OUT_DEV);      // [PHX_MAX_OUT_DEV]
    float* flist = s_sela + (PHX_MAX_OUT_DEV + 3) / 4 * 4;                     // [kNmsFl][64]
    unsigned char* qbase = reinterpret_cast<unsigned char*>(s_seln) + kNmsSelBytes;
    uint64_t* qkey = reinterpret_cast<uint64_t*>(qbase);                     // [qrows][64]
    float4* qbox = reinterpret_cast<float4*>(qkey + pl.qrows * 64);           // [qrows][64]
    int* qfrom = reinterpret_cast<int*>(qbox + pl.qrows * 64);                // [qrows][64]
    // F1. every candidate's score bits (positive floats: integer order = float order) to gkey,
    //     eight gathers in flight per lane
    for (int p0 = 0; p0 < n; p0 += 8 * kNmsThreads) {
      int a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = gwi[min(p0 + u * kNmsThreads + t, n - 1)];
      uint32_t k[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) k[u] = __float_as_uint(sb[a[u]]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (p0 + u * kNmsThreads + t < n) gkey[p0 + u * kNmsThreads + t] = k[u];
    }
    __syncthreads();
    // wave 0's queue state, kept across batches: the selections, and the re-queue rows' maxima
    // (lane r: row r's largest key, 0 = a free row) with their overall maximum
    int nsel = 0;
    uint64_t rmax = 0ull, cmax = 0ull;
    int crow = 0;
    int npop = 0, nrq = 0, nbatch = 0;  // PHX_NMS_STATS counts and phase times
    int ndirty = 0;
    uint64_t tsel = 0, tlist = 0, tsort = 0, tpop = 0, tsa = stamp();
    const uint64_t ts1 = tsa;
    uint32_t hi = 0xffffffffu;  // candidates with score bits < hi are not listed yet
    int rem = n;                // how many
    int state = 0;              // 0 next batch, 1 done, 2 fall back
    while (state == 0) {
      // F2. the batch: unlisted keys with key >> 8 >= thr24, the largest 24-bit prefix whose count
      //     reaches min(rem, kNmsTopWant) (two histogram passes: bits 31..20, then 19..8 inside the
      //     crossing bin); thr24 = 0 lists every remaining candidate
      uint32_t thr24 = 0;
      if (rem > kNmsTopWant) {
        uint32_t prefix = 0;
        int need = kNmsTopWant;
        for (int pass = 0; pass < 2; ++pass) {
          for (int i = t; i < kNmsHistBins; i += kNmsThreads) hist[i] = 0u;
          __syncthreads();
          for (int p0 = 0; p0 < n; p0 += 8 * kNmsThreads) {
            uint32_t k[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) k[u] = gkey[min(p0 + u * kNmsThreads + t, n - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              if (p0 + u * kNmsThreads + t >= n || k[u] >= hi) continue;
              if (pass == 0) atomicAdd(&hist[k[u] >> 20], 1u);
              else if ((k[u] >> 20) == prefix) atomicAdd(&hist[(k[u] >> 8) & 4095u], 1u);
            }
          }
          __syncthreads();
          // suffix counts from the top bin down: thread t owns bins [4095 - 16t - 15, 4095 - 16t]
          int cnt = 0;
          for (int i = 0; i < 16; ++i) cnt += (int)hist[4095 - 16 * t - i];
          s_scan[t] = cnt;
          __syncthreads();
          for (int off = 1; off < kNmsThreads; off <<= 1) {
            const int v = t >= off ? s_scan[t - off] : 0;
            __syncthreads();
            s_scan[t] += v;
            __syncthreads();
          }
          const int before = s_scan[t] - cnt;  // candidates in higher bins
          if (before < need && before + cnt >= need) {
            int acc = before, bin = 4095 - 16 * t;
            for (int i = 0; i < 16; ++i) {
              acc += (int)hist[4095 - 16 * t - i];
              bin = 4095 - 16 * t - i;
              if (acc >= need) break;
            }
            s_misc[4] = bin;
            s_misc[5] = need - (acc - (int)hist[bin]);  // still needed inside the crossing bin
          }
          __syncthreads();
          const uint32_t bin = (uint32_t)__builtin_amdgcn_readfirstlane(s_misc[4]);
          need = __builtin_amdgcn_readfirstlane(s_misc[5]);
          prefix = pass == 0 ? bin : ((prefix << 12) | bin);
          __syncthreads();
        }
        thr24 = prefix;
      }
      const uint32_t lo = thr24 << 8;  // unlisted after this batch: score bits < lo
      uint64_t tsb = stamp();
      tsel += tsb - tsa;
      // F3. the batch's keys and boxes (any order; the sort below orders them by queue key)
      if (t == 0) s_misc[6] = 0;
      __syncthreads();
      for (int p0 = 0; p0 < n; p0 += 8 * kNmsThreads) {
        uint32_t k[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) k[u] = gkey[min(p0 + u * kNmsThreads + t, n - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int p = p0 + u * kNmsThreads + t;
          if (p < n && k[u] < hi && (k[u] >> 8) >= thr24) {
            const int j = atomicAdd(&s_misc[6], 1);
            if (j < pl.lp) {
              lkey[j] = nms_key(k[u], p);
              lbox[j] = *reinterpret_cast<const float4*>(bb + (long)gwi[p] * 4);
            }
          }
        }
      }
      __syncthreads();
      const int L = __builtin_amdgcn_readfirstlane(s_misc[6]);
      if (L > pl.lp) {
        state = 2;
        break;
      }
      rem -= L;
      ++nbatch;
      tsa = stamp();
      tlist += tsa - tsb;
      int ls = 1;  // sort size: the batch rounded up to a power of 2
      while (ls < L) ls <<= 1;
      for (int j = t; j < ls; j += kNmsThreads) {
        lpay[j] = (uint32_t)j;
        if (j >= L) lkey[j] = 0ull;
      }
      __syncthreads();
      // bitonic sort, descending by key (keys are unique: the low word is ~position)
      for (int k = 2; k <= ls; k <<= 1) {
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          for (int i = t; i < ls; i += kNmsThreads) {
            const int ix = i ^ jj;
            if (ix > i) {
              const uint64_t a = lkey[i], b2 = lkey[ix];
              const bool desc = (i & k) == 0;
              if (desc ? (a < b2) : (a > b2)) {
                lkey[i] = b2;
                lkey[ix] = a;
                const uint32_t pa = lpay[i];
                lpay[i] = lpay[ix];
                lpay[ix] = pa;
              }
            }
          }
          __syncthreads();
        }
      }
      // F4. the lazy queue over the batch's rows + the re-queue set, wave 0 alone
      tsb = stamp();
      tsort += tsb - tsa;
      if (wave == 0) {
        int f = 0, st = 1;
        int rown = 0, jn = 0;       // the row's candidates, the next one not popped yet
        uint64_t ck = 0ull;         // lane j: the row's j-th candidate's key
        float4 cbx = make_float4(0.f, 0.f, 0.f, 0.f);  // its box
        NmsNBox cn = nms_norm(cbx);
        float cs = 0.f;             // its score: the product over every selection so far
        int fc = 0;                 // its decay factors other than 1 (flist[0..fc), oldest first)
        bool dirty = false;         // more than kNmsFl of them: a full visit at its pop
        uint64_t rk = 0ull;         // its re-queue key once popped (0: not in the queue)
        int rfrom = 0;              // selections at that pop
        uint64_t qmax = 0ull;       // max of rk
        // TF's product of a row candidate: its score times its factors, newest first (factors of
        // exactly 1 leave it unchanged and are not kept)
        auto product = [&](bool on) {
          if (on) {
            float sc = __uint_as_float((uint32_t)(ck >> 32));
            for (int q = min(fc, kNmsFl) - 1; q >= 0; --q) sc *= flist[q * 64 + lane];
            cs = sc;
          }
        };
        // a factor other than 1 of a new selection for the lanes `on`: appended, the product redone
        auto add_factor = [&](bool on, float g) {
          if (on) {
            if (fc < kNmsFl) flist[fc * 64 + lane] = g;
            else dirty = true;
            ++fc;
          }
          product(on && !dirty);
        };
        // a new selection: lane 0 records it; the row's candidates not popped yet (lanes >= j0) take
        // its decay factor into their product
        auto select = [&](float4 b4, float sc, int j0) {
          const NmsNBox sn = nms_norm(b4);
          if (lane == 0) {
            s_sel[nsel] = b4;
            s_sels[nsel] = sc;
            s_seln[nsel] = make_float4(sn.y0, sn.x0, sn.y1, sn.x1);
            s_sela[nsel] = sn.a;
          }
          ++nsel;
          const bool ov = lane >= j0 && lane < rown && nms_overlap(cn, sn);
          if (__ballot(ov)) {
            const float g = ov ? nms_factor(cn, sn, scale) : 1.f;
            if (__ballot(g != 1.f)) add_factor(g != 1.f, g);
          }
        };
        while (nsel < max_out) {
          if (jn >= rown) {
            // the row is used up: its re-queued candidates move to a free row of the set
            if (qmax) {
              const unsigned long long fr = __ballot(lane < pl.qrows && rmax == 0ull);
              if (!fr) { st = 2; break; }
              const int r = __ffsll(fr) - 1;
              qkey[r * 64 + lane] = rk;
              qbox[r * 64 + lane] = cbx;
              qfrom[r * 64 + lane] = rfrom;
              if (lane == r) rmax = qmax;
              if (qmax > cmax) { cmax = qmax; crow = r; }
              rk = 0ull;
              qmax = 0ull;
            }
            rown = 0;
            if (f < L) {
              // the next row, visited against every selection so far, one candidate per lane
              const int j = f + lane;
              ck = j < L ? lkey[j] : 0ull;
              cbx = j < L ? lbox[lpay[j]] : make_float4(0.f, 0.f, 0.f, 0.f);
              cn = nms_norm(cbx);
              rown = min(64, L - f);
              f += rown;
              jn = 0;
              dirty = false;
              fc = 0;
              // the factors other than 1, oldest selection first, then the product newest first
              for (int k = 0; k < nsel; ++k) {
                const NmsNBox sn = nms_sel_at(s_seln, s_sela, k);
                const bool ov = lane < rown && nms_overlap(cn, sn);
                if (__ballot(ov)) {
                  const float g = ov ? nms_factor(cn, sn, scale) : 1.f;
                  if (g != 1.f) {
                    if (fc < kNmsFl) flist[fc * 64 + lane] = g;
                    else dirty = true;
                    ++fc;
                  }
                }
              }
              product(!dirty);
            }
          }
          const uint64_t fk = jn < rown ? readlane_u64(ck, jn) : 0ull;
          const uint64_t rtop = qmax > cmax ? qmax : cmax;
          if (f >= L && jn >= rown && rem > 0 && (uint32_t)(rtop >> 32) < lo) { st = 0; break; }  // an unlisted one could be next
          const uint64_t top = rtop > fk ? rtop : fk;
          if (top == 0ull) break;
          const float orig = __uint_as_float((uint32_t)(top >> 32));
          if (!(orig > score_thresh)) break;
          const int pos = (int)~(uint32_t)top;
          ++npop;
          if (rtop > fk) {
            // a re-queued candidate: in this row (qmax) or in row crow of the set
            ++nrq;
            const bool cur = qmax > cmax;
            uint64_t rowk = 0ull;
            int owner, from;
            float4 b4;
            if (cur) {
              owner = __ffsll(__ballot(rk == qmax)) - 1;
              from = __builtin_amdgcn_readlane(rfrom, owner);
              b4 = readlane_f4(cbx, owner);
            } else {
              rowk = qkey[crow * 64 + lane];
              owner = __ffsll(__ballot(rowk == cmax)) - 1;
              from = qfrom[crow * 64 + owner];
              b4 = qbox[crow * 64 + owner];
            }
            const float sc = nms_visit_n(nms_norm(b4), orig, from, nsel, s_seln, s_sela, scale, lane);
            uint64_t nk = 0ull;
            if (sc == orig) select(b4, sc, jn);
            else if (sc > score_thresh) nk = nms_key(__float_as_uint(sc), pos);
            if (cur) {
              if (lane == owner) {
                rk = nk;
                rfrom = nsel;
              }
              qmax = wave_max_u64(rk);
            } else {
              if (lane == owner) {
                rowk = nk;
                qkey[crow * 64 + owner] = nk;
                qfrom[crow * 64 + owner] = nsel;
              }
              const uint64_t m = wave_max_u64(rowk);
              if (lane == crow) rmax = m;
              cmax = wave_max_u64(rmax);
              crow = cmax ? __ffsll(__ballot(rmax == cmax)) - 1 : 0;
            }
          } else {
            // the row's next candidate: its row-wide visit holds unless a later selection overlaps it
            const int j = jn++;
            float sc;
            if ((__ballot(dirty) >> j) & 1ull) {
              sc = nms_visit_n(nms_norm(readlane_f4(cbx, j)), orig, 0, nsel, s_seln, s_sela, scale, lane);
              ++ndirty;
            } else sc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cs), j));
            if (sc == orig) {
              select(readlane_f4(cbx, j), sc, jn);
            } else if (sc > score_thresh) {
              const uint64_t nk = nms_key(__float_as_uint(sc), pos);
              if (lane == j) {
                rk = nk;
                rfrom = nsel;
              }
              if (nk > qmax) qmax = nk;
            }
          }
        }
        if (lane == 0) {
          s_misc[1] = nsel;
          s_misc[2] = st;
        }
      }
      __syncthreads();
      state = __builtin_amdgcn_readfirstlane(s_misc[2]);  // workgroup-uniform
      hi = lo;
      tsa = stamp();
      tpop += tsa - tsb;
      __syncthreads();    // the next batch rewrites the list
    }
    if (dbg && t == 0)
      printf("nms image %d: %d candidates, %d batch(es), %d pops (%d re-queued), %d selected -> %s | us: "
             "compaction + scores %.1f, batch select %.1f list %.1f sort %.1f, pops %.1f; %d full visits of row "
             "candidates\n", b, n, nbatch, npop,
             nrq, s_misc[1], state == 1 ? "fast path" : "general queue", (ts1 - ts0) * 0.01, tsel * 0.01,
             tlist * 0.01, tsort * 0.01, tpop * 0.01, ndirty);
    fast_done = state == 1;
  }
  if (!fast_done) {

  // 3. gather keys and boxes in candidate order (coalesced over positions)
  for (int p0 = 0; p0 < n; p0 += 4 * kNmsThreads) {
    int a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = gwi[min(p0 + u * kNmsThreads + t, n - 1)];
    float sc[4];
    float4 bx[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sc[u] = sb[a[u]];
      bx[u] = *reinterpret_cast<const float4*>(bb + (long)a[u] * 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + u * kNmsThreads + t;
      if (p < n) {
        cbox[p] = bx[u];
        const uint32_t k = __float_as_uint(sc[u]);
        if (p < cap) {
          s_key[p] = k;
          s_wb[p] = 0;
        } else {
          gkey[p] = k;
          gwb[p] = 0;
        }
      }
    }
  }
  __syncthreads();

  // 4. chunk and group maxima
  const int CH = 64 * pl.m;
  const int nch = (n + CH - 1) / CH;
  const int ngr = (nch + 63) / 64;
  // spilled keys / visit counts are re-read after wave 0 rewrote them: volatile (L1-bypassing) loads
  volatile const uint32_t* vgkey = gkey;
  volatile const uint8_t* vgwb = gwb;
  auto key_at = [&](int p) -> uint32_t { return p < cap ? s_key[p] : vgkey[p]; };
  auto chunk_max = [&](int ch) -> uint64_t {
    uint64_t v = 0;
    for (int j = 0; j < pl.m; ++j) {
      const int p = ch * CH + j * 64 + lane;
      if (p < n) {
        const uint64_t k = nms_key(key_at(p), p);
        v = k > v ? k : v;
      }
    }
    return wave_max_u64(v);
  };
  for (int ch = wave; ch < nch; ch += kNmsThreads / 64) {
    const uint64_t v = chunk_max(ch);
    if (lane == 0) s_ck[ch] = v;
  }
  __syncthreads();
  for (int g = wave; g < ngr; g += kNmsThreads / 64) {
    const int ch = g * 64 + lane;
    const uint64_t v = wave_max_u64(ch < nch ? s_ck[ch] : 0ull);
    if (lane == 0) s_gk[g] = v;
  }
  __syncthreads();

  // 5. the lazy priority queue, wave 0 only
  if (wave == 0) {
    const uint32_t tbits = __float_as_uint(score_thresh);
    int nsel = 0;
    while (nsel < max_out) {
      const uint64_t top = wave_max_u64(lane < ngr ? s_gk[lane] : 0ull);
      if (top == 0ull) break;
      const uint32_t vbits = (uint32_t)(top >> 32);
      if (!(__uint_as_float(vbits) > score_thresh)) break;
      (void)tbits;
      const int c = (int)~(uint32_t)top;
      const float orig = __uint_as_float(vbits);
      const int from = c < cap ? (int)s_wb[c] : (int)vgwb[c];
      // decay factors of the selections since the last visit, newest first; TF's decay order,
      // exact-1 factors skipped
      const float4 cb4 = cbox[c];
      const float sc = nms_visit(cb4, orig, from, nsel, s_sel, scale, lane);
      uint32_t nk;
      if (sc == orig) {
        if (lane == 0) {
          s_sel[nsel] = cb4;
          s_sels[nsel] = sc;
        }
        ++nsel;
        nk = 0u;
      } else {
        nk = sc > score_thresh ? __float_as_uint(sc) : 0u;
      }
      // the candidate's new key and visit count (wb = selections at this visit)
      const int wbnew = (sc == orig) ? nsel - 1 : nsel;
      if (lane == 0) {
        if (c < cap) {
          s_key[c] = nk;
          s_wb[c] = (uint8_t)wbnew;
        } else {
          gkey[c] = nk;
          gwb[c] = (uint8_t)wbnew;
        }
      }
      // rescan c's chunk (c's own value from registers) and its group
      const int ch = c / CH;
      uint64_t v = 0;
      for (int j = 0; j < pl.m; ++j) {
        const int p = ch * CH + j * 64 + lane;
        if (p < n) {
          const uint64_t k = p == c ? nms_key(nk, p) : nms_key(key_at(p), p);
          v = k > v ? k : v;
        }
      }
      const uint64_t cmax = wave_max_u64(v);
      const int g = ch >> 6;
      const int chl = g * 64 + lane;
      uint64_t gv = chl == ch ? cmax : (chl < nch ? s_ck[chl] : 0ull);
      gv = wave_max_u64(gv);
      if (lane == 0) {
        s_ck[ch] = cmax;
        s_gk[g] = gv;
      }
    }
    if (lane == 0) s_misc[1] = nsel;
  }
  }  // general queue
  __syncthreads();
  // 6. outputs: padded to max_out, boxes clipped to [0, image_size] (postprocess.py:61-64)
  const int nsel = s_misc[1];
  for (int k = t; k < max_out; k += kNmsThreads) {
    float* ob = out_boxes + ((long)b * max_out + k) * 4;
    if (k < nsel) {
      const float4 s4 = s_sel[k];
      ob[0] = fminf(fmaxf(s4.x, 0.0f), clip_hi);
      ob[1] = fminf(fmaxf(s4.y, 0.0f), clip_hi);
      ob[2] = fminf(fmaxf(s4.z, 0.0f), clip_hi);
      ob[3] = fminf(fmaxf(s4.w, 0.0f), clip_hi);
      out_scores[(long)b * max_out + k] = s_sels[k];
    } else {
      ob[0] = ob[1] = ob[2] = ob[3] = 0.f;
      out_scores[(long)b * max_out + k] = 0.f;
    }
  }
  if (t == 0) out_count[b] = nsel;
}

size_t soft_nms_work_floats(int B, int N) { return (size_t)B * N * 7; }

// PHX_NMS_STATS=1: each image's soft-NMS reports its candidate count, list size, pops and path
static int nms_debug() {
  static const int v = [] {
    const char* e = std::getenv("PHX_NMS_STATS");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return v;
}

void launch_soft_nms(const float* boxes, const float* scores, const uint8_t* keep, int keep_mask,
                     const int* count, int B, int N, float score_thresh, float soft_sigma,
                     int max_out, float clip_hi, float* out_boxes, float* out_scores,
                     int* out_count, float* work, hipStream_t s, NmsCand cand) {
  if (max_out > PHX_MAX_OUT_DEV || max_out > 128) throw std::runtime_error("soft_nms: max_out too large");
  const NmsPlan pl = nms_plan(N);
  if (pl.lds > kNmsLdsBytes || pl.nchunk > 64 * kNmsGroups) throw std::runtime_error("soft_nms: too many candidates");
  // TF: scale = -0.5 / soft_nms_sigma (soft_nms_sigma = sigma / 2, postprocess.py:191-200)
  float scale = soft_sigma > 0.f ? -0.5f / soft_sigma : 0.f;
  // work (soft_nms_work_floats): compacted boxes [B][N] float4 | keys [B][N] | anchors [B][N] |
  // visit counts [B][N] bytes
  const long BN = (long)B * N;
  float4* cbox = reinterpret_cast<float4*>(work);
  uint32_t* gkey = reinterpret_cast<uint32_t*>(work + 4 * BN);
  int* gwi = reinterpret_cast<int*>(work + 5 * BN);
  uint8_t* gwb = reinterpret_cast<uint8_t*>(work + 6 * BN);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_soft_nms),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kNmsLdsBytes) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(k_soft_nms, dim3(B), dim3(kNmsThreads), pl.lds, s, boxes, scores, keep, keep_mask,
                     count, N, score_thresh, scale, max_out, clip_hi, out_boxes, out_scores, out_count,
                     cbox, gkey, gwi, gwb, cand, pl, nms_debug());
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// per-image max over kept anchors (attacker.py:190): raw max (lowest() if empty) + ties
// ------------------------------------------------------------------------------------------
// per-image max over kept anchors in two launches: grid (kImaxChunks, B) workgroups each reduce
// a contiguous anchor chunk to (max, first index, #elements equal to the chunk max); one lane
// per image then merges its chunks (ties across chunks: counts of chunks whose max equals the
// image max add up; the first index is the smallest among them).
constexpr int kImaxChunks = 48;

__global__ __launch_bounds__(256) void k_image_max_part(const float* __restrict__ scores,
                                                        const uint8_t* __restrict__ keep, int A,
                                                        float* __restrict__ pm,
                                                        int* __restrict__ pi,
                                                        int* __restrict__ pc) {
  const int b = blockIdx.y, ch = blockIdx.x, t = threadIdx.x;
  const int per = (A + gridDim.x - 1) / gridDim.x;
  const int a0 = ch * per, a1 = min(A, a0 + per);
  __shared__ float rs[256];
  __shared__ int ri[256];
  __shared__ int rc[256];
  float best = -FLT_MAX;
  int bi = 0x7fffffff;
  for (int a = a0 + t; a < a1; a += 256) {
    const long e = (long)b * A + a;
    if (keep[e] & 1) {
      const float v = scores[e];
      if (v > best || (v == best && a < bi)) { best = v; bi = a; }
    }
  }
  rs[t] = best;
  ri[t] = bi;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) {
      const float v = rs[t + off];
      const int j = ri[t + off];
      if (v > rs[t] || (v == rs[t] && j < ri[t])) { rs[t] = v; ri[t] = j; }
    }
    __syncthreads();
  }
  const float mx = rs[0];
  const int mi = ri[0];
  int cnt = 0;
  if (mi != 0x7fffffff)
    for (int a = a0 + t; a < a1; a += 256) {
      const long e = (long)b * A + a;
      if ((keep[e] & 1) && scores[e] == mx) ++cnt;
    }
  __syncthreads();
  rc[t] = cnt;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) rc[t] += rc[t + off];
    __syncthreads();
  }
  if (t == 0) {
    const int o = b * gridDim.x + ch;
    pm[o] = mx;
    pi[o] = mi;
    pc[o] = rc[0];
  }
}

__global__ void k_image_max_merge(const float* __restrict__ pm, const int* __restrict__ pi,
                                  const int* __restrict__ pc, int S, int B, float* __restrict__ m,
                                  int* __restrict__ argm, int* __restrict__ nties) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float mx = -FLT_MAX;
  int mi = 0x7fffffff, cnt = 0;
  // 16 chunks' loads in flight per round, merged in chunk order (a load-use chain per chunk before)
  for (int k0 = 0; k0 < S; k0 += 16) {
    float pv[16];
    int pj[16], pn[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int o = b * S + min(k0 + u, S - 1);
      pj[u] = pi[o];
      pv[u] = pm[o];
      pn[u] = pc[o];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (k0 + u >= S) break;
      const int j = pj[u];
      if (j == 0x7fffffff) continue;
      const float v = pv[u];
      if (mi == 0x7fffffff || v > mx) {
        mx = v; mi = j; cnt = pn[u];
      } else if (v == mx) {
        mi = min(mi, j);
        cnt += pn[u];
      }
    }
  }
  m[b] = mi == 0x7fffffff ? -FLT_MAX : mx;
  argm[b] = mi == 0x7fffffff ? -1 : mi;
  nties[b] = mi == 0x7fffffff ? 0 : cnt;
}

size_t image_max_scratch_ints(int B) { return (size_t)B * kImaxChunks * 3; }

void launch_image_max(const float* scores, const uint8_t* keep, int B, int A, float* m, int* argmax,
                      int* nties, int* scratch, hipStream_t s) {
  float* pm = reinterpret_cast<float*>(scratch);
  int* pi = scratch + (size_t)B * kImaxChunks;
  int* pc = pi + (size_t)B * kImaxChunks;
  hipLaunchKernelGGL(k_image_max_part, dim3(kImaxChunks, B), dim3(256), 0, s, scores, keep, A, pm, pi, pc);
  PHX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_image_max_merge, dim3(cdiv(B, 64)), dim3(64), 0, s, pm, pi, pc, kImaxChunks, B, m,
                     argmax, nties);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// loss (attacker.py:189-193) + per-image dL/dm coefficient + dscale + metrics.  One block.
//   m_b = max(raw_b, 0); loss = sum m_b^2 + sum (m_b - s)^2 (+ 1e-5 TV added by the TV kernel)
//   dL/draw_b = (4 m_b - 2 s) if raw_b >= 0 (tf.maximum grad goes to x on ties), else 0
// ------------------------------------------------------------------------------------------
__global__ void k_loss(const float* __restrict__ mraw, int B, const float* __restrict__ params,
                       int npatch, float* __restrict__ dm, float* __restrict__ dscale,
                       float* __restrict__ metrics) {
  if (threadIdx.x != 0) return;
  const float s = params[npatch];
  float sum_sq = 0.f, scale_loss = 0.f, sm = 0.f, sm2 = 0.f, dsc = 0.f;
  for (int b = 0; b < B; ++b) {
    float raw = mraw[b];
    float mb = fmaxf(raw, 0.0f);
    float d = mb - s;
    sum_sq += mb * mb;
    scale_loss += d * d;
    sm += mb;
    sm2 += mb * mb;
    dsc += -2.0f * d;
    dm[b] = raw >= 0.0f ? (2.0f * mb + 2.0f * d) : 0.0f;
  }
  *dscale = dsc;
  metrics[PHX_M_LOSS] = sum_sq + scale_loss;
  metrics[PHX_M_SCALE_LOSS] = scale_loss;
  metrics[PHX_M_SUM_M] = sm;
  metrics[PHX_M_SUM_M2] = sm2;
  metrics[PHX_M_NIMG] = (float)B;
}

void launch_loss(const float* mraw, int B, const float* params, float* dm, float* dscale,
                 float* metrics, hipStream_t s) {
  hipLaunchKernelGGL(k_loss, dim3(1), dim3(64), 0, s, mraw, B, params, PHX_NPATCH_DEV, dm, dscale,
                     metrics);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// sparse class-head backward: for every kept anchor whose score equals the image max, route
// dL/dm through sigmoid and the class reduce_max (ties split, TF _MaxGrad) into the input of
// the class-predict pointwise conv: dx[pixel, :] += W[:, k*ncls + c] * dlogit.
// One lane per (image, pixel): it walks the pixel's anchors and their tied classes in a fixed
// order and accumulates into its own dx row, so several contributions to one pixel (tied scores
// of its anchors: frequent with bf16 logits) always add in the same order.  (Float atomics here
// made the sum depend on the workgroup schedule, e.g. on work running on another stream.)
// ------------------------------------------------------------------------------------------
template <bool BF>
__global__ __launch_bounds__(256) void k_cls_scatter(
    const float* __restrict__ scores, const uint8_t* __restrict__ keep,
    const float* __restrict__ mraw, const int* __restrict__ nties, const float* __restrict__ dm,
    const float* __restrict__ cls_base, const LevelDesc* __restrict__ lev, int nlev, int A, int B,
    int nclass, int na, const float* __restrict__ wpred /*[K][na*ncls]*/, int K,
    float* __restrict__ dx_base, const long* __restrict__ dx_off) {
  const int PT = A / na;  // pixels per image over all levels
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * PT) return;
  const int b = (int)(idx / PT), p = (int)(idx % PT);
  if (dm[b] == 0.0f) return;
  int l = 0;
  while (l + 1 < nlev && p * na >= lev[l + 1].anchor0) ++l;
  const LevelDesc L = lev[l];
  const int pix = p - L.anchor0 / na;
  const float mx = mraw[b];
  const float ds = dm[b] / (float)nties[b];
  const long prow = (long)b * L.h * L.w + pix;
  float* dx = dx_base + dx_off[l] + prow * K;
  const int N = na * nclass;
  // the pixel's anchors that carry the image max: every keep / score load in flight at once
  const long abase = (long)b * A + L.anchor0 + (long)pix * na;
  constexpr int kNA = 16;
  uint32_t win = 0;
  if (na <= kNA) {
    uint8_t kp[kNA];
    float sv[kNA];
#pragma unroll
    for (int k = 0; k < kNA; ++k) {
      kp[k] = keep[abase + min(k, na - 1)];
      sv[k] = scores[abase + min(k, na - 1)];
    }
#pragma unroll
    for (int k = 0; k < kNA; ++k)
      if (k < na && (kp[k] & 1) && sv[k] == mx) win |= 1u << k;
  } else {
    for (int k = 0; k < na && k < 32; ++k)
      if ((keep[abase + k] & 1) && scores[abase + k] == mx) win |= 1u << k;
  }
  if (!win) return;
  for (int k = 0; k < na; ++k) {
    if (!(win >> k & 1)) continue;
    const float s = scores[abase + k];
    const float dl = ds * s * (1.0f - s);  // SigmoidGrad: y * (1 - y) * dy
    const long lg = L.cls_off + prow * (na * nclass) + (long)k * nclass;  // element offset (BF: bf16)
    // the anchor's logits: all loads issued at once (a scan that loaded them one by one, three times,
    // was a chain of ~270 round trips), the max and its ties (a class bit mask, ascending) from registers
    constexpr int kNC = 96;
    uint32_t tie[kNC / 32] = {0u, 0u, 0u};
    int nt = 0;
    float m;
    if (nclass <= kNC) {
      float v[kNC];
#pragma unroll
      for (int q = 0; q < kNC; ++q) v[q] = ald1<BF>(cls_base, lg + min(q, nclass - 1));
      m = v[0];
#pragma unroll
      for (int q = 1; q < kNC; ++q)
        if (q < nclass) m = fmaxf(m, v[q]);
#pragma unroll
      for (int q = 0; q < kNC; ++q)
        if (q < nclass && v[q] == m) {
          tie[q >> 5] |= 1u << (q & 31);
          ++nt;
        }
    } else {
      m = ald1<BF>(cls_base, lg);
      for (int c = 1; c < nclass; ++c) m = fmaxf(m, ald1<BF>(cls_base, lg + c));
      for (int c = 0; c < nclass; ++c) nt += (ald1<BF>(cls_base, lg + c) == m);
    }
    const float dlc = dl / (float)nt;
    for (int c = 0; c < nclass; ++c) {
      if (nclass <= kNC) {
        const int wd = c >> 5;
        const uint32_t rest = (wd == 0 ? tie[0] : wd == 1 ? tie[1] : tie[2]) >> (c & 31);  // next tie at or after c
        if (!rest) {
          c = ((c >> 5) + 1) * 32 - 1;  // (none left in this word)
          continue;
        }
        c += __builtin_ctz(rest);
        if (c >= nclass) break;
      } else if (ald1<BF>(cls_base, lg + c) != m) {
        continue;
      }
      const int col = k * nclass + c;
      // 64 kernel-column loads and 64 dx values in flight per round (one lane does this for its
      // image's winning anchor: a dependent chain of K round trips was ~40 us of the step)
      for (int j0 = 0; j0 < K; j0 += 64) {
        float w[64], o[64];
#pragma unroll
        for (int u = 0; u < 64; ++u) {
          const int j = min(j0 + u, K - 1);
          w[u] = wpred[(long)j * N + col];
          o[u] = dx[j];
        }
#pragma unroll
        for (int u = 0; u < 64; ++u)
          if (j0 + u < K) dx[j0 + u] = o[u] + w[u] * dlc;
      }
    }
  }
}

void launch_cls_scatter(const float* scores, const uint8_t* keep, const float* mraw,
                        const int* nties, const float* dm, const float* cls_base,
                        const LevelDesc* lev, int nlev, int A, int B, int nclass, int na,
                        const float* wpred, int K, float* dx_base, const long* dx_off,
                        hipStream_t s, bool bf) {
  if (A % na) throw std::runtime_error("cls_scatter: anchors not a multiple of anchors per pixel");
  if (na > 32) throw std::runtime_error("cls_scatter: more than 32 anchors per pixel");
  const long n = (long)B * (A / na);
  if (bf)
    hipLaunchKernelGGL(k_cls_scatter<true>, dim3(cdiv(n, 256)), dim3(256), 0, s, scores, keep, mraw, nties,
                       dm, cls_base, lev, nlev, A, B, nclass, na, wpred, K, dx_base, dx_off);
  else
    hipLaunchKernelGGL(k_cls_scatter<false>, dim3(cdiv(n, 256)), dim3(256), 0, s, scores, keep, mraw, nties,
                       dm, cls_base, lev, nlev, A, B, nclass, na, wpred, K, dx_base, dx_off);
  PHX_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// ASR counts (attacker.py:238-255): boxes with score >= 0.5 among soft-NMS outputs
// ------------------------------------------------------------------------------------------
__global__ void k_count_ge(const float* __restrict__ sc, const int* __restrict__ cnt, int B,
                           int maxo, float th, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  int n = 0;
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < cnt[b]; ++k) n += sc[(long)b * maxo + k] >= th;
  *out = (float)n;
}

void launch_count_ge(const float* sc, const int* cnt, int B, int maxo, float th, float* out,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_count_ge, dim3(1), dim3(64), 0, s, sc, cnt, B, maxo, th, out);
  PHX_LAUNCH_CHECK();
}

// ---- launch merges: buffer zeroing and the step prologue (each replaced several memset / copy
// packets of ~5 us apiece on the step's stream) ----
struct ZeroSegs {
  float4* p[kZeroSegs];
  long n4[kZeroSegs];  // float4 count
  long off[kZeroSegs + 1];
  int n;
};

__global__ __launch_bounds__(256) void k_zero_segs(ZeroSegs z) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < z.off[z.n]; i += stride) {
    int k = 0;
#pragma unroll
    for (int j = 1; j < kZeroSegs; ++j)
      if (j < z.n && i >= z.off[j]) k = j;
    float4* p = z.p[0];
    long o = z.off[0];
#pragma unroll
    for (int j = 1; j < kZeroSegs; ++j)
      if (j == k) {
        p = z.p[j];
        o = z.off[j];
      }
    p[i - o] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

void launch_zero_segs(char* const* ptr, const size_t* bytes, int n, hipStream_t s) {
  if (n <= 0) return;
  if (n > kZeroSegs) throw std::invalid_argument("zero_segs: too many buffers");
  ZeroSegs z{};
  z.n = n;
  z.off[0] = 0;
  for (int k = 0; k < n; ++k) {
    if ((reinterpret_cast<uintptr_t>(ptr[k]) | bytes[k]) & 15) throw std::invalid_argument("zero_segs: alignment");
    z.p[k] = reinterpret_cast<float4*>(ptr[k]);
    z.n4[k] = (long)(bytes[k] / 16);
    z.off[k + 1] = z.off[k] + z.n4[k];
  }
  const long blocks = std::min<long>(cdiv(z.off[n], 256L), 4096L);
  hipLaunchKernelGGL(k_zero_segs, dim3((unsigned)std::max<long>(blocks, 1)), dim3(256), 0, s, z);
  PHX_LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void k_step_prologue(float* metrics, int nmetric, const float4* boxes,
                                                       const int32_t* count, int B, int maxb, float4* inj_boxes,
                                                       int* inj_count) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < nmetric) metrics[i] = 0.f;
  if (!boxes) return;
  if (i < B * PHX_MAX_OUT_DEV) {
    const int b = i / PHX_MAX_OUT_DEV, j = i - b * PHX_MAX_OUT_DEV;
    inj_boxes[i] = j < maxb ? boxes[(long)b * maxb + j] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (i < B) inj_count[i] = count[i];
}

void launch_step_prologue(float* metrics, int nmetric, const float* boxes, const int32_t* count, int B, int maxb,
                          float* inj_boxes, int* inj_count, hipStream_t s) {
  if (boxes && (maxb < 0 || maxb > PHX_MAX_OUT_DEV)) throw std::out_of_range("maxb > 100");
  if (boxes && (reinterpret_cast<uintptr_t>(boxes) & 15)) throw std::invalid_argument("boxes: 16-B alignment");
  const int n = std::max(nmetric, boxes ? B * PHX_MAX_OUT_DEV : 0);
  hipLaunchKernelGGL(k_step_prologue, dim3(cdiv(n, 256)), dim3(256), 0, s, metrics, nmetric,
                     reinterpret_cast<const float4*>(boxes), count, B, maxb, reinterpret_cast<float4*>(inj_boxes),
                     inj_count);
  PHX_LAUNCH_CHECK();
}

}  // namespace phx
