// DetectionIntentionLoss (loss.py:58-206) on device, with no host synchronisation:
//   1. best anchor per GT (torch max(dim=0): first index on ties)          [B x Gmax blocks]
//   2. per-anchor assignment (IoU thresholds 0.45/0.6, force-match, first-index argmax over
//      GTs), delta encoding, focal / Smooth-L1 / CE terms, per-block partial sums
//   3. deterministic final reduction + normalisation + NaN/Inf guard (loss.py:186-198)
//   4. backward: per-anchor analytic gradients scaled by the saved normalisers
#include "geom.h"

#pragma clang fp contract(off)

using namespace ivit;

namespace {

enum { ST_FOCAL = 0, ST_BOX, ST_CE, ST_NPOS, ST_KEEP, ST_LOSS, ST_CLS, ST_BOXL, ST_INT, ST_FINITE, ST_CDEN, ST_IDEN };
constexpr int NPART = 5;
constexpr int LB = 256;

struct LossWs {
  int* best_anchor;   // [B*G]
  float* best_iou;    // [B*G]
  int* tgt;           // [B*NA]: cls target in bits 0..1 (+1 offset), intent target << 2
  float* box_t;       // [B*NA*6]
  float* part;        // [nblk*NPART]
};

IVIT_DEV float iou_of(const float* a, const float* g, int rot) { return rot ? rotated_iou(a, g) : axis_iou(a, g); }

__global__ __launch_bounds__(256) void best_anchor_kernel(const float* __restrict__ anchors, long NA,
                                                          const float* __restrict__ gt, const int* __restrict__ ngt,
                                                          int G, int rot, int* best_anchor, float* best_iou) {
  const int b = blockIdx.x, g = blockIdx.y;
  if (g >= ngt[b]) return;
  const float* gb = gt + ((long)b * G + g) * 5;
  float bv = -1.f;
  long bi = 0;
  for (long a = threadIdx.x; a < NA; a += 256) {
    const float v = iou_of(anchors + a * 5, gb, rot);
    if (v > bv) { bv = v; bi = a; }
  }
  __shared__ float sv[256];
  __shared__ long si[256];
  sv[threadIdx.x] = bv;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float v2 = sv[threadIdx.x + o];
      const long i2 = si[threadIdx.x + o];
      if (v2 > sv[threadIdx.x] || (v2 == sv[threadIdx.x] && i2 < si[threadIdx.x])) {
        sv[threadIdx.x] = v2;
        si[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    best_anchor[b * G + g] = (int)si[0];
    best_iou[b * G + g] = sv[0];
  }
}

IVIT_DEV float focal_term(float x, float t, float alpha, float gamma) {
  // torchvision.ops.sigmoid_focal_loss, reduction='none'
  const float p = 1.f / (1.f + expf(-x));
  const float ce = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
  const float pt = p * t + (1.f - p) * (1.f - t);
  float l = ce * powf(1.f - pt, gamma);
  if (alpha >= 0.f) l = (alpha * t + (1.f - alpha) * (1.f - t)) * l;
  return l;
}
IVIT_DEV float focal_grad(float x, float t, float alpha, float gamma) {
  const float p = 1.f / (1.f + expf(-x));
  const float ce = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
  const float pt = p * t + (1.f - p) * (1.f - t);
  const float omp = 1.f - pt;
  float g = (p - t) * powf(omp, gamma) - ce * gamma * powf(omp, gamma - 1.f) * (2.f * t - 1.f) * p * (1.f - p);
  if (alpha >= 0.f) g *= alpha * t + (1.f - alpha) * (1.f - t);
  return g;
}
IVIT_DEV float sl1(float d, float beta) {
  const float a = fabsf(d);
  return a < beta ? 0.5f * d * d / beta : a - 0.5f * beta;
}
IVIT_DEV float sl1_grad(float d, float beta) {
  return fabsf(d) < beta ? d / beta : (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f));
}

__global__ __launch_bounds__(LB) void assign_loss_kernel(
    const float* __restrict__ cls, const float* __restrict__ box, const float* __restrict__ intent,
    const float* __restrict__ anchors, int B, long NA, int K, const float* __restrict__ gt,
    const int* __restrict__ ngt, const int* __restrict__ gint, int G, const float* __restrict__ keep,
    unsigned dom, int downs, const float* __restrict__ cw, float pos_thr, float neg_thr, float alpha, float gamma,
    float beta, int rot, LossWs ws) {
  const long i = (long)blockIdx.x * LB + threadIdx.x;  // b * NA + a
  float vals[NPART] = {0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < (long)B * NA) {
    const int b = (int)(i / NA);
    const long a = i - (long)b * NA;
    const int ng = ngt[b];
    int t = 0, it = -1;
    if (ng > 0) {
      const float* an = anchors + a * 5;
      float mx = -1.f;
      int arg = 0;
      for (int g = 0; g < ng; ++g) {
        const float v = iou_of(an, gt + ((long)b * G + g) * 5, rot);
        if (v > mx) { mx = v; arg = g; }
      }
      t = mx < neg_thr ? 0 : (mx >= pos_thr ? 1 : -1);
      for (int g = 0; g < ng; ++g)
        if (ws.best_anchor[b * G + g] == (int)a && ws.best_iou[b * G + g] >= neg_thr) t = 1;
      if (t == 1) {
        const float* gb = gt + ((long)b * G + arg) * 5;
        const float eps = 1e-6f;
        float* bt = ws.box_t + i * 6;
        bt[0] = (gb[0] - an[0]) / (an[2] + eps);
        bt[1] = (gb[1] - an[1]) / (an[3] + eps);
        bt[2] = logf(gb[2] / (an[2] + eps) + eps);
        bt[3] = logf(gb[3] / (an[3] + eps) + eps);
        bt[4] = sinf(gb[4] - an[4]);
        bt[5] = cosf(gb[4] - an[4]);
        it = gint[b * G + arg];
      }
    }
    ws.tgt[i] = (t + 1) | ((it + 1) << 2);
    if (t >= 0) vals[0] = focal_term(cls[i], (float)t, alpha, gamma);
    if (t == 1) {
      const float* bp = box + i * 6;
      const float* bt = ws.box_t + i * 6;
      float s = 0.f;
      for (int k = 0; k < 6; ++k) s += sl1(bp[k] - bt[k], beta);
      vals[1] = s;
      const float* lg = intent + i * K;
      float m = lg[0];
      for (int k = 1; k < K; ++k) m = fmaxf(m, lg[k]);
      float se = 0.f;
      for (int k = 0; k < K; ++k) se += expf(lg[k] - m);
      float ce = (logf(se) + m) - lg[it];
      float mk = 1.f;
      if (downs) {
        if ((dom >> it) & 1u) mk = keep ? keep[i] : 1.f;
      } else if (cw) {
        ce *= cw[it];
      }
      vals[2] = ce * mk;
      vals[3] = 1.f;
      vals[4] = mk;
    }
  }
  __shared__ float red[NPART][LB];
#pragma unroll
  for (int k = 0; k < NPART; ++k) red[k][threadIdx.x] = vals[k];
  __syncthreads();
  for (int o = LB / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o)
#pragma unroll
      for (int k = 0; k < NPART; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < NPART) ws.part[(long)blockIdx.x * NPART + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void loss_final_kernel(const float* __restrict__ part, int nblk, int downs, float wc, float wb, float wi,
                                  float* stats) {
  __shared__ double red[NPART][256];
  double s[NPART] = {0, 0, 0, 0, 0};
  for (int k = threadIdx.x; k < nblk; k += 256)
    for (int j = 0; j < NPART; ++j) s[j] += part[(long)k * NPART + j];
  for (int j = 0; j < NPART; ++j) red[j][threadIdx.x] = s[j];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      for (int j = 0; j < NPART; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x) return;
  const float focal = (float)red[0][0], boxs = (float)red[1][0], ces = (float)red[2][0];
  const float npos = (float)red[3][0], ks = (float)red[4][0];
  const float cden = fmaxf(1.f, npos);
  const float iden = downs ? fmaxf(1.f, ks) : fmaxf(1.f, npos);
  const float cl = focal / cden;
  const float bl = npos > 0.f ? boxs / cden : 0.f;
  const float il = npos > 0.f ? ces / iden : 0.f;
  const float tot = wc * cl + wb * bl + wi * il;
  const bool fin = isfinite(tot);
  stats[ST_FOCAL] = focal; stats[ST_BOX] = boxs; stats[ST_CE] = ces; stats[ST_NPOS] = npos; stats[ST_KEEP] = ks;
  stats[ST_LOSS] = fin ? tot : 0.f;
  stats[ST_CLS] = fin ? cl : 0.f;
  stats[ST_BOXL] = fin ? bl : 0.f;
  stats[ST_INT] = fin ? il : 0.f;
  stats[ST_FINITE] = fin ? 1.f : 0.f;
  stats[ST_CDEN] = cden;
  stats[ST_IDEN] = iden;
}

__global__ __launch_bounds__(LB) void loss_bwd_kernel(const float* __restrict__ cls, const float* __restrict__ box,
                                                      const float* __restrict__ intent, long total, int K,
                                                      const float* __restrict__ keep, unsigned dom, int downs,
                                                      const float* __restrict__ cw, float alpha, float gamma,
                                                      float beta, float wc, float wb, float wi,
                                                      const float* __restrict__ stats, const float* grad_loss,
                                                      const int* __restrict__ tgt, const float* __restrict__ box_t,
                                                      float* dcls, float* dbox, float* dint) {
  const long i = (long)blockIdx.x * LB + threadIdx.x;
  if (i >= total) return;
  if (stats[ST_FINITE] == 0.f) {
    // loss.py:190-198 returns a disconnected zero leaf: no gradient reaches the logits. Write
    // exact zeros (a non-finite per-anchor gradient times 0 would be NaN).
    dcls[i] = 0.f;
    for (int k = 0; k < 6; ++k) dbox[i * 6 + k] = 0.f;
    for (int k = 0; k < K; ++k) dint[i * K + k] = 0.f;
    return;
  }
  const float go = grad_loss ? grad_loss[0] : 1.f;
  const float cden = stats[ST_CDEN], iden = stats[ST_IDEN];
  const int code = tgt[i];
  const int t = (code & 3) - 1, it = (code >> 2) - 1;
  dcls[i] = t >= 0 ? go * wc * focal_grad(cls[i], (float)t, alpha, gamma) / cden : 0.f;
  for (int k = 0; k < 6; ++k)
    dbox[i * 6 + k] = t == 1 ? go * wb * sl1_grad(box[i * 6 + k] - box_t[i * 6 + k], beta) / cden : 0.f;
  const float* lg = intent + i * K;
  if (t == 1) {
    float mk = 1.f;
    if (downs) {
      if ((dom >> it) & 1u) mk = keep ? keep[i] : 1.f;
    } else if (cw) {
      mk = cw[it];
    }
    float m = lg[0];
    for (int k = 1; k < K; ++k) m = fmaxf(m, lg[k]);
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += expf(lg[k] - m);
    const float sc = go * wi * mk / iden;
    for (int k = 0; k < K; ++k) dint[i * K + k] = sc * (expf(lg[k] - m) / se - (k == it ? 1.f : 0.f));
  } else {
    for (int k = 0; k < K; ++k) dint[i * K + k] = 0.f;
  }
}

LossWs carve(void* work, long B, long NA, long G) {
  char* w = (char*)work;
  auto take = [&](long bytes) { char* p = w; w += (bytes + 255) / 256 * 256; return (void*)p; };
  LossWs ws;
  // targets first: their offsets must not depend on Gmax (the backward re-carves with G = 1)
  ws.tgt = (int*)take(B * NA * 4);
  ws.box_t = (float*)take(B * NA * 24);
  ws.part = (float*)take((long)ivit_cdiv(B * NA, LB) * NPART * 4);
  ws.best_anchor = (int*)take(B * G * 4);
  ws.best_iou = (float*)take(B * G * 4);
  return ws;
}

}  // namespace

extern "C" long ivit_det_loss_workspace(long B, long NA, long Gmax) {
  const long G = Gmax > 0 ? Gmax : 1;
  return (B * G * 4 + 255) / 256 * 256 * 2 + (B * NA * 4 + 255) / 256 * 256 + (B * NA * 24 + 255) / 256 * 256 +
         ((long)ivit_cdiv(B * NA, LB) * NPART * 4 + 255) / 256 * 256;
}

extern "C" int ivit_det_loss_fwd(const float* cls, const float* box, const float* intent, const float* anchors, long B,
                                 long NA, long K, const float* gt, const int* ngt, const int* gint, long Gmax,
                                 const float* keep, unsigned dominant_mask, int downsampling, const float* class_w,
                                 float pos_thr, float neg_thr, float alpha, float gamma, float beta, float w_cls,
                                 float w_box, float w_int, int use_rotated, float* stats, void* work, long work_bytes,
                                 void* stream) {
  IVIT_CHECK_ARG(work_bytes >= ivit_det_loss_workspace(B, NA, Gmax), "ivit_det_loss_fwd: workspace too small");
  IVIT_CHECK_ARG(K <= 32, "ivit_det_loss_fwd: K <= 32");
  hipStream_t st = ivit_stream(stream);
  const long G = Gmax > 0 ? Gmax : 1;
  LossWs ws = carve(work, B, NA, G);
  if (Gmax > 0)
    hipLaunchKernelGGL(best_anchor_kernel, dim3(B, Gmax), dim3(256), 0, st, anchors, NA, gt, ngt, (int)G, use_rotated,
                       ws.best_anchor, ws.best_iou);
  const int nblk = ivit_cdiv(B * NA, LB);
  hipLaunchKernelGGL(assign_loss_kernel, dim3(nblk), dim3(LB), 0, st, cls, box, intent, anchors, (int)B, NA, (int)K,
                     gt, ngt, gint, (int)G, keep, dominant_mask, downsampling, class_w, pos_thr, neg_thr, alpha, gamma,
                     beta, use_rotated, ws);
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, ws.part, nblk, downsampling, w_cls, w_box, w_int,
                     stats);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_det_loss_bwd(const float* cls, const float* box, const float* intent, long B, long NA, long K,
                                 const float* keep, unsigned dominant_mask, int downsampling, const float* class_w,
                                 float alpha, float gamma, float beta, float w_cls, float w_box, float w_int,
                                 const float* stats, const float* grad_loss, float* dcls, float* dbox, float* dintent,
                                 void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(work_bytes >= ivit_det_loss_workspace(B, NA, 1), "ivit_det_loss_bwd: workspace too small");
  hipStream_t st = ivit_stream(stream);
  LossWs ws = carve(work, B, NA, 1);  // the forward's workspace, passed back unchanged
  const long total = B * NA;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(ivit_cdiv(total, LB)), dim3(LB), 0, st, cls, box, intent, total, (int)K,
                     keep, dominant_mask, downsampling, class_w, alpha, gamma, beta, w_cls, w_box, w_int, stats,
                     grad_loss, ws.tgt, ws.box_t, dcls, dbox, dintent);
  IVIT_LAUNCH_CHECK();
  return 0;
}
