// Detection mAP / intention matching of eval_vit.py:191-292 + calculate_ap (utils.py:564-575)
// on the device. One workgroup per (sample, IoU threshold):
//   A  best GT per prediction (first index of the row max, torch.max) and the qualifying flag
//      best >= thr (f32 compare, as torch / numpy compare an f32 value with a Python float);
//      first[g] = the first qualifying prediction (score order) whose best GT is g
//      (LDS atomicMin). The reference's sequential walk marks prediction k a TP iff it
//      qualifies and no earlier qualifying prediction had the same best GT — i.e. k == first[best].
//   B  cumulative TP count (block scan) -> precision cum/(k+1) and recall cum/ngt in f32;
//   C  suffix max of precision (reverse block scan) and the VOC all-point sum
//      sum_k [tp_k] (rec_k - rec_{k-1}) * max(prec_k..) in f64 (calculate_ap's f64 arithmetic).
#include "ivit_common.h"

namespace {

constexpr int MT = 256;
constexpr int MAX_GT = 4096;

// inclusive block scan (sum or max) of one value per thread; every thread gets its prefix
template <bool MAX>
IVIT_DEV float block_scan(float v, float* sh) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float u = __shfl_up(v, o, 64);
    if (lane >= o) v = MAX ? fmaxf(v, u) : v + u;
  }
  if (lane == 63) sh[w] = v;
  __syncthreads();
  float c = MAX ? -INFINITY : 0.f;
  for (int i = 0; i < w; ++i) c = MAX ? fmaxf(c, sh[i]) : c + sh[i];
  __syncthreads();
  return MAX ? fmaxf(v, c) : v + c;
}

__global__ __launch_bounds__(MT) void det_match_kernel(const float* __restrict__ iou, const long* __restrict__ iou_off,
                                                       const int* __restrict__ npred, const int* __restrict__ ngt,
                                                       const long* __restrict__ pred_off, long ptot,
                                                       const float* __restrict__ thr, int T, double* __restrict__ ap,
                                                       int* __restrict__ best_out, unsigned char* __restrict__ tp_out,
                                                       float* __restrict__ prec_ws, int* __restrict__ cum_ws) {
  __shared__ int first[MAX_GT];
  __shared__ float sh[MT / 64];
  __shared__ double red[MT / 64];
  const int s = blockIdx.x, t = blockIdx.y, tid = threadIdx.x;
  const int P = npred[s], G = ngt[s];
  if (P == 0 || G == 0) {  // eval_vit.py:209-214
    if (tid == 0) ap[(long)s * T + t] = (P == 0 && G == 0) ? 1.0 : 0.0;
    return;
  }
  const float th = thr[t];
  const float* M = iou + iou_off[s];
  const long po = pred_off[s];
  unsigned char* tp = tp_out + (long)t * ptot + po;
  float* prec = prec_ws + (long)t * ptot + po;
  int* cum = cum_ws + (long)t * ptot + po;
  for (int g = tid; g < G; g += MT) first[g] = 0x7fffffff;
  __syncthreads();
  // A: best GT (first max) per prediction -> cum[p] (scratch), qualifying flag -> tp[p];
  //    first qualifying prediction per GT
  for (int p = tid; p < P; p += MT) {
    const float* row = M + (long)p * G;
    float bv = row[0];
    int bg = 0;
    for (int g = 1; g < G; ++g) {
      const float v = row[g];
      if (v > bv) { bv = v; bg = g; }  // strict: first index on ties; NaN never wins
    }
    const bool q = bv >= th;
    if (t == 0) best_out[po + p] = bg;
    cum[p] = bg;
    tp[p] = q;
    if (q) atomicMin(&first[bg], p);
  }
  __syncthreads();
  // B: TP flags, running TP count, precision (chunks of MT predictions in score order)
  __shared__ int tot;
  int carry = 0;
  for (int c0 = 0; c0 < P; c0 += MT) {
    const int p = c0 + tid;
    int f = 0;
    if (p < P) {
      f = tp[p] && first[cum[p]] == p;
      tp[p] = (unsigned char)f;
    }
    const int inc = (int)block_scan<false>((float)f, sh) + carry;  // counts <= 2^24: exact in f32
    if (p < P) {
      cum[p] = inc;
      prec[p] = (float)inc / ((float)(p + 1) + 1e-9f);  // eval_vit.py:252 (f32)
    }
    if (tid == MT - 1) tot = inc;
    __syncthreads();
    carry = tot;
    __syncthreads();
  }
  // C: suffix max of precision, VOC sum over the TP positions (f64)
  const float ng = (float)G + 1e-9f;  // eval_vit.py:251 (f32)
  float smax = 0.f;                   // mpre's trailing 0
  double acc = 0.0;
  const int nch = (P + MT - 1) / MT;
  for (int ch = nch - 1; ch >= 0; --ch) {
    // reverse order inside the chunk: thread i holds element c0 + MT-1-i
    const int p = ch * MT + (MT - 1 - tid);
    const float v = p < P ? prec[p] : 0.f;
    const float m = fmaxf(block_scan<true>(v, sh), smax);  // max over this element and everything after it
    if (p < P && tp[p]) {
      const int c = cum[p];
      const double r1 = (double)((float)c / ng), r0 = (double)((float)(c - 1) / ng);
      acc += (r1 - r0) * (double)m;
    }
    __shared__ float cmax;
    if (tid == MT - 1) cmax = m;  // the chunk's first element: max of the whole suffix
    __syncthreads();
    smax = cmax;
    __syncthreads();
  }
  // block sum of acc
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) {
    double a = 0.0;
    for (int i = 0; i < MT / 64; ++i) a += red[i];
    ap[(long)s * T + t] = a;
  }
}

}  // namespace

extern "C" int ivit_det_match(const float* iou, const long* iou_off, const int* npred, const int* ngt,
                              const long* pred_off, long n_samples, long total_pred, const float* thresholds,
                              long n_thr, double* ap, int* best_gt, unsigned char* tp, void* work, long work_bytes,
                              int max_gt, void* stream) {
  if (n_samples <= 0 || n_thr <= 0) return 0;
  IVIT_CHECK_ARG(max_gt <= MAX_GT, "ivit_det_match: at most %d GT boxes per sample (got %d)", MAX_GT, max_gt);
  IVIT_CHECK_ARG(n_samples < 2147483647L && n_thr < 65536, "ivit_det_match: grid too large");
  IVIT_CHECK_ARG(work_bytes >= 8 * n_thr * (total_pred > 0 ? total_pred : 1), "ivit_det_match: workspace too small");
  float* prec = (float*)work;
  int* cum = (int*)(prec + n_thr * total_pred);
  hipLaunchKernelGGL(det_match_kernel, dim3(n_samples, n_thr), dim3(MT), 0, ivit_stream(stream), iou, iou_off, npred,
                     ngt, pred_off, total_pred, thresholds, (int)n_thr, ap, best_gt, tp, prec, cum);
  IVIT_LAUNCH_CHECK();
  return 0;
}
