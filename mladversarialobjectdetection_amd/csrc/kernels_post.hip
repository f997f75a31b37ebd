// kernels_post.hip — detection post-processing on the attack path:
//   pre_nms            automl/efficientdet/tf2/postprocess.py:67-156 (level merge, per-anchor class
//                      max/argmax, box decode anchors.py:30-58, sigmoid)
//   person/valid mask  attacker.py:69-89, 105-113, 132-140
//   soft-NMS           postprocess.py:159-205 -> tf.raw_ops.NonMaxSuppressionV5 (gaussian),
//                      restated from TF's non_max_suppression_op.cc [TF-recall]
//   loss               attacker.py:189-193 and its gradient (ragged reduce_max, maximum(.,0))
// Arithmetic that decides discrete outcomes (masks, thresholds, argmax) is kept in TF's fp32
// operation order with FMA contraction disabled.
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
  const long run = ((long)b * nloc + a0) * nclass;      // float offset of the tile's logits
  const float* src = cls_base + L.cls_off + run;
  const int nf = n * nclass;
  const int nf4 = nf >> 2;
  const float4* src4 = reinterpret_cast<const float4*>(src);
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    // staging: four 16-B loads in flight per lane before any LDS store
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
  const float4 bx = *reinterpret_cast<const float4*>(box_base + L.box_off + ((long)b * nloc + a0 + t) * 4);
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
  keep[idx] = kf;
  want = (kf & cand.mask) != 0 && sc > cand.thresh;
  }
  if (cand.list) nms_cand_append(cand, b, A, want, a);
}

void launch_pre_nms(const float* cls_base, const float* box_base, const LevelDesc* lev_dev,
                    int nlev, const float* anchors, int A, int B, int nclass, int na,
                    float img_h, float img_w, float thresh, float* scores, int* classes,
                    float* boxes, uint8_t* keep, int ntiles, hipStream_t s, NmsCand cand) {
  size_t shm = (size_t)kPreTile * nclass * sizeof(float);
  hipLaunchKernelGGL(k_pre_nms, dim3(ntiles, B), dim3(256), shm, s, cls_base, box_base, lev_dev, nlev,
                     anchors, A, B, nclass, na, img_h, img_w, thresh, scores, classes, boxes, keep, cand);
  PHX_LAUNCH_CHECK();
}

int pre_nms_tiles(int h, int w, int na) { return (h * w * na + kPreTile - 1) / kPreTile; }

// ------------------------------------------------------------------------------------------
// soft-NMS: one workgroup per image.  Exact restatement of NonMaxSuppressionV5's lazy
// priority queue: pop the (score desc, index asc) maximum, decay it by every box selected
// since its last visit (newest first, early exit at <= thresh), select if unchanged, else
// re-queue while > thresh.  Candidate order = ragged (anchor) order.
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

__global__ __launch_bounds__(kNmsThreads) void k_soft_nms(
    const float* __restrict__ boxes, const float* __restrict__ scores,
    const uint8_t* __restrict__ keep, int keep_mask, const int* __restrict__ count, int N,
    float score_thresh, float scale, int max_out, float clip_hi, float* __restrict__ out_boxes,
    float* __restrict__ out_scores, int* __restrict__ out_count, float* __restrict__ wscore,
    int* __restrict__ wsb, int* __restrict__ widx, NmsCand cand) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const float* bb = boxes + (long)b * N * 4;
  const float* sb = scores + (long)b * N;
  float* ws = wscore + (long)b * N;
  int* wb = wsb + (long)b * N;
  int* wi = widx + (long)b * N;
  const int n_in = count ? count[b] : N;

  __shared__ int s_n;
  __shared__ float sel_box[PHX_MAX_OUT_DEV][4];
  __shared__ float sel_score[PHX_MAX_OUT_DEV];
  __shared__ int s_nsel;
  __shared__ int red_i[kNmsThreads];
  __shared__ int s_done;

  if (cand.list) {
    // 1'. candidates appended by pre_nms (score > thresh and keep & mask already applied)
    if (t == 0) s_n = min(cand.count[b], N);
    __syncthreads();
    const int* lst = cand.list + (long)b * N;
    for (int i = t; i < s_n; i += kNmsThreads) {
      const int a = lst[i];
      wi[i] = a;
      ws[i] = sb[a];
      wb[i] = 0;
    }
    __syncthreads();
    if (t == 0) cand.count[b] = 0;  // consumed: the next pre_nms appends from 0
  } else {
  // 1. ordered compaction of candidates with score > thresh (and mask): every lane owns a
  //    contiguous segment, one workgroup scan of the segment counts places them
  auto ok_at = [&](int i) -> bool {
    bool ok = sb[i] > score_thresh;
    if (keep) ok = ok && ((keep[(long)b * N + i] & keep_mask) != 0);
    return ok;
  };
  const int per = (n_in + kNmsThreads - 1) / kNmsThreads;
  const int lo = min(n_in, t * per), hi = min(n_in, lo + per);
  int cnt = 0;
  for (int i = lo; i < hi; ++i) cnt += ok_at(i) ? 1 : 0;
  red_i[t] = cnt;
  __syncthreads();
  for (int off = 1; off < kNmsThreads; off <<= 1) {
    int v = (t >= off) ? red_i[t - off] : 0;
    __syncthreads();
    red_i[t] += v;
    __syncthreads();
  }
  {
    int pos = red_i[t] - cnt;
    for (int i = lo; i < hi; ++i) {
      if (ok_at(i)) {
        wi[pos] = i;
        ws[pos] = sb[i];
        wb[pos] = 0;
        ++pos;
      }
    }
  }
  if (t == kNmsThreads - 1) s_n = red_i[t];
  __syncthreads();
  }
  const int n = s_n;
  if (t == 0) { s_nsel = 0; s_done = 0; }
  __syncthreads();

  // 2. lazy priority-queue loop.  Lane t owns candidates t, t+256, ... and caches the best
  //    (score desc, index asc) of its subset; only the owner of the candidate an iteration changed
  //    rescans.  The decay factors of the selections since the candidate's last visit are computed
  //    by one wave in parallel, then applied newest-first in order by one lane (same product, same
  //    early exit as the sequential rule).
  // order: score desc, then anchor index asc (the reference's candidate order); myi = position
  auto better = [](float v, int a, float bv, int ba) { return v > bv || (v == bv && a < ba); };
  float myv = -INFINITY;
  int myi = 0x7fffffff, mya = 0x7fffffff;
  for (int i = t; i < n; i += kNmsThreads) {
    const float v = ws[i];
    const int a = wi[i];
    if (better(v, a, myv, mya)) { myv = v; myi = i; mya = a; }
  }
  __shared__ float wv_s[kNmsThreads / 64];
  __shared__ int wv_i[kNmsThreads / 64], wv_a[kNmsThreads / 64];
  __shared__ float fac[PHX_MAX_OUT_DEV];
  __shared__ int s_c, s_from;
  __shared__ float s_orig;
  const int lane = t & 63, wave = t >> 6;
  while (true) {
    if (s_nsel >= max_out) break;
    float v = myv;
    int i = myi, a = mya;
    for (int o = 32; o > 0; o >>= 1) {
      const float v2 = __shfl_xor(v, o);
      const int i2 = __shfl_xor(i, o);
      const int a2 = __shfl_xor(a, o);
      if (better(v2, a2, v, a)) { v = v2; i = i2; a = a2; }
    }
    if (lane == 0) { wv_s[wave] = v; wv_i[wave] = i; wv_a[wave] = a; }
    __syncthreads();
    if (t == 0) {
      float bv = wv_s[0];
      int bi = wv_i[0], ba = wv_a[0];
      for (int w = 1; w < kNmsThreads / 64; ++w)
        if (better(wv_s[w], wv_a[w], bv, ba)) { bv = wv_s[w]; bi = wv_i[w]; ba = wv_a[w]; }
      if (!(bv > score_thresh) || bi == 0x7fffffff) {
        s_done = 1;
      } else {
        s_c = bi;
        s_orig = bv;
        s_from = wb[bi];
      }
    }
    __syncthreads();
    if (s_done) break;
    const int c = s_c, from = s_from, nsel = s_nsel;
    const float* cb = bb + (long)wi[c] * 4;
    if (wave == 0)
      for (int j = from + lane; j < nsel; j += 64) {
        const float sim = tf_iou(cb, sel_box[j]);
        fac[j] = expf(scale * sim * sim);
      }
    __syncthreads();
    if (t == 0) {
      const float orig = s_orig;
      float sc = orig;
      for (int j = nsel - 1; j >= from; --j) {
        sc *= fac[j];
        if (sc <= score_thresh) break;
      }
      wb[c] = nsel;
      if (sc == orig) {
        sel_box[nsel][0] = cb[0]; sel_box[nsel][1] = cb[1];
        sel_box[nsel][2] = cb[2]; sel_box[nsel][3] = cb[3];
        sel_score[nsel] = sc;
        s_nsel = nsel + 1;
        ws[c] = -INFINITY;
      } else if (sc > score_thresh) {
        ws[c] = sc;
      } else {
        ws[c] = -INFINITY;
      }
    }
    __syncthreads();
    if (t == c % kNmsThreads) {
      myv = -INFINITY;
      myi = mya = 0x7fffffff;
      for (int k = t; k < n; k += kNmsThreads) {
        const float vv = ws[k];
        const int ak = wi[k];
        if (better(vv, ak, myv, mya)) { myv = vv; myi = k; mya = ak; }
      }
    }
  }
  __syncthreads();
  // 3. outputs: padded to max_out, boxes clipped to [0, image_size] (postprocess.py:61-64)
  const int nsel = s_nsel;
  for (int k = t; k < max_out; k += kNmsThreads) {
    float* ob = out_boxes + ((long)b * max_out + k) * 4;
    if (k < nsel) {
#pragma unroll
      for (int j = 0; j < 4; ++j) ob[j] = fminf(fmaxf(sel_box[k][j], 0.0f), clip_hi);
      out_scores[(long)b * max_out + k] = sel_score[k];
    } else {
      ob[0] = ob[1] = ob[2] = ob[3] = 0.f;
      out_scores[(long)b * max_out + k] = 0.f;
    }
  }
  if (t == 0) out_count[b] = nsel;
}

void launch_soft_nms(const float* boxes, const float* scores, const uint8_t* keep, int keep_mask,
                     const int* count, int B, int N, float score_thresh, float soft_sigma,
                     int max_out, float clip_hi, float* out_boxes, float* out_scores,
                     int* out_count, float* work_score, int* work_sb, hipStream_t s, NmsCand cand) {
  if (max_out > PHX_MAX_OUT_DEV) throw std::runtime_error("soft_nms: max_out too large");
  // TF: scale = -0.5 / soft_nms_sigma (soft_nms_sigma = sigma / 2, postprocess.py:191-200)
  float scale = soft_sigma > 0.f ? -0.5f / soft_sigma : 0.f;
  int* widx = work_sb + (long)B * N;
  hipLaunchKernelGGL(k_soft_nms, dim3(B), dim3(kNmsThreads), 0, s, boxes, scores, keep, keep_mask,
                     count, N, score_thresh, scale, max_out, clip_hi, out_boxes, out_scores,
                     out_count, work_score, work_sb, widx, cand);
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
  for (int k = 0; k < S; ++k) {
    const int o = b * S + k;
    const int j = pi[o];
    if (j == 0x7fffffff) continue;
    const float v = pm[o];
    if (mi == 0x7fffffff || v > mx) {
      mx = v; mi = j; cnt = pc[o];
    } else if (v == mx) {
      mi = min(mi, j);
      cnt += pc[o];
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
// the class-predict pointwise conv: dx[pixel, :] += W[:, k*ncls + c] * dlogit
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_cls_scatter(
    const float* __restrict__ scores, const uint8_t* __restrict__ keep,
    const float* __restrict__ mraw, const int* __restrict__ nties, const float* __restrict__ dm,
    const float* __restrict__ cls_base, const LevelDesc* __restrict__ lev, int nlev, int A, int B,
    int nclass, int na, const float* __restrict__ wpred /*[K][na*ncls]*/, int K,
    float* __restrict__ dx_base, const long* __restrict__ dx_off) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * A) return;
  const int b = (int)(idx / A), a = (int)(idx % A);
  if (!(keep[idx] & 1)) return;
  const float mx = mraw[b];
  if (scores[idx] != mx || dm[b] == 0.0f) return;
  const float ds = dm[b] / (float)nties[b];
  const float s = scores[idx];
  const float dl = ds * s * (1.0f - s);  // SigmoidGrad: y * (1 - y) * dy
  int l = 0;
  while (l + 1 < nlev && a >= lev[l + 1].anchor0) ++l;
  const LevelDesc L = lev[l];
  const int local = a - L.anchor0;
  const int pix = local / na, k = local % na;
  const long prow = (long)b * L.h * L.w + pix;
  const float* lg = cls_base + L.cls_off + prow * (na * nclass) + (long)k * nclass;
  float m = lg[0];
  for (int c = 1; c < nclass; ++c) m = fmaxf(m, lg[c]);
  int nt = 0;
  for (int c = 0; c < nclass; ++c) nt += (lg[c] == m);
  const float dlc = dl / (float)nt;
  float* dx = dx_base + dx_off[l] + prow * K;
  const int N = na * nclass;
  for (int c = 0; c < nclass; ++c) {
    if (lg[c] != m) continue;
    const int col = k * nclass + c;
    for (int j = 0; j < K; ++j) atomicAdd(dx + j, wpred[(long)j * N + col] * dlc);
  }
}

void launch_cls_scatter(const float* scores, const uint8_t* keep, const float* mraw,
                        const int* nties, const float* dm, const float* cls_base,
                        const LevelDesc* lev, int nlev, int A, int B, int nclass, int na,
                        const float* wpred, int K, float* dx_base, const long* dx_off,
                        hipStream_t s) {
  long n = (long)B * A;
  hipLaunchKernelGGL(k_cls_scatter, dim3(cdiv(n, 256)), dim3(256), 0, s, scores, keep, mraw, nties,
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

}  // namespace phx
