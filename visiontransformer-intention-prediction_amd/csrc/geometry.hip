// Eval-path geometry (utils.py): anchors, axis/rotated IoU matrices, delta decode and
// torchvision-CPU-exact non-maximum suppression.
#include "geom.h"

#include <rocprim/device/device_segmented_radix_sort.hpp>

#include <cmath>
#include <cstring>

#pragma clang fp contract(off)

using namespace ivit;

namespace {

// utils.py:519-562: centres x=(off_y - (s*gy + s/2))*voxel, y=((s*gx + s/2) - off_x)*voxel;
// rows location-major, anchor-minor.
__global__ void anchors_kernel(int fh, int fw, int stride, const float* cfgs, int A, float voxel, float off_x,
                               float off_y, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)fh * fw * A) return;
  const int a = (int)(i % A);
  const long loc = i / A;
  const int gy = (int)(loc / fw), gx = (int)(loc % fw);
  const float px = (float)(gx * stride) + (float)stride / 2.0f;
  const float py = (float)(gy * stride) + (float)stride / 2.0f;
  out[i * 5 + 0] = (off_y - py) * voxel;
  out[i * 5 + 1] = (px - off_x) * voxel;
  out[i * 5 + 2] = cfgs[a * 3 + 0];
  out[i * 5 + 3] = cfgs[a * 3 + 1];
  out[i * 5 + 4] = cfgs[a * 3 + 2];
}

__global__ void iou_matrix_kernel(const float* b1, long n1, const float* b2, long n2, float* out, int rotated) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n1 * n2) return;
  const long r = i / n2, c = i - r * n2;
  out[i] = rotated ? rotated_iou(b1 + r * 5, b2 + c * 5) : axis_iou(b1 + r * 5, b2 + c * 5);
}

// utils.py:227-257
__global__ void decode_kernel(const float* rel, const float* anchors, const long* idx, long n, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* d = rel + i * 6;
  const float* a = anchors + (idx ? idx[i] : i) * 5;
  float* o = out + i * 5;
  o[0] = d[0] * a[2] + a[0];
  o[1] = d[1] * a[3] + a[1];
  o[2] = expf(d[2]) * a[2];
  o[3] = expf(d[3]) * a[3];
  const float yaw = a[4] + atan2f(d[4], d[5]);
  o[4] = atan2f(sinf(yaw), cosf(yaw));
}

// ---- NMS (torchvision CPU nms_kernel_impl): stable descending sort; f32 corners/areas/IoU;
//      suppress j if (double)IoU > thr.
// rank by counting: rank(i) = #{j : s_j > s_i  or  (s_j == s_i and j < i)}
__global__ void nms_rank_kernel(const float* __restrict__ s, long n, int* __restrict__ order) {
  __shared__ float tile[256];
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const float si = i < n ? s[i] : 0.f;
  long rank = 0;
  for (long j0 = 0; j0 < n; j0 += 256) {
    __syncthreads();
    if (j0 + threadIdx.x < n) tile[threadIdx.x] = s[j0 + threadIdx.x];
    __syncthreads();
    const int lim = (int)min((long)256, n - j0);
    for (int k = 0; k < lim; ++k) {
      const float sj = tile[k];
      const long j = j0 + k;
      rank += (sj > si) || (sj == si && j < i);
    }
  }
  if (i < n) order[rank] = (int)i;
}

__global__ void nms_sorted_boxes_kernel(const float* __restrict__ b, const int* __restrict__ order, long n,
                                        float* __restrict__ sb) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const float* q = b + (long)order[p] * 5;
  const float x1 = q[0] - q[2] / 2.f, y1 = q[1] - q[3] / 2.f, x2 = q[0] + q[2] / 2.f, y2 = q[1] + q[3] / 2.f;
  sb[p * 5 + 0] = x1;
  sb[p * 5 + 1] = y1;
  sb[p * 5 + 2] = x2;
  sb[p * 5 + 3] = y2;
  sb[p * 5 + 4] = (x2 - x1) * (y2 - y1);
}

// torchvision's test, bit for bit: (double)RN32(inter / u) > thr with u = (area_i + area_j) - inter in
// f32, i.e. RN32(inter / u) >= t, t the smallest float whose double exceeds thr. The IEEE division is
// a ~10-instruction VALU sequence, and with divergent lanes the whole wave waits for it (anchors
// overlap their neighbours, so most 64-lane iterations had some lane dividing). Instead
// q = inter * rcp(u) (relative error < 2^-22) decides every pair whose q lies outside
// [t - 8 ulp, t + 8 ulp] (a margin of ~2^-20); the rest, and u <= 0 / non-finite operands / a
// threshold that is negative or below the normal floats, take the exact division. Disjoint pairs
// (inter = 0) are decided before any of it.
struct NmsThr {
  double thr;
  float lo, hi;
  int fast;
};
NmsThr nms_thr(double thr) {
  NmsThr r{thr, 0.f, 0.f, 0};
  if (!(thr >= 1e-30) || !(thr < 1e30)) return r;
  float t = (float)thr;
  while ((double)t <= thr) t = nextafterf(t, INFINITY);
  float tp;
  while ((double)(tp = nextafterf(t, -INFINITY)) > thr) t = tp;  // the smallest float above thr
  float lo = t, hi = t;
  for (int k = 0; k < 8; ++k) {
    lo = nextafterf(lo, -INFINITY);
    hi = nextafterf(hi, INFINITY);
  }
  r.lo = lo;
  r.hi = hi;
  r.fast = 1;
  return r;
}
IVIT_DEV bool nms_suppresses(float ix1, float iy1, float ix2, float iy2, float ia, float4 c, float ca,
                             const NmsThr& th) {
  // raw v_max / v_min: fmaxf / fminf on LDS values made the compiler canonicalise each operand
  // first (one more instruction per use); the corners are never NaN for finite decoded boxes
  auto vmax = [](float a, float b) { float d; asm("v_max_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b)); return d; };
  auto vmin = [](float a, float b) { float d; asm("v_min_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b)); return d; };
  const float xx1 = vmax(ix1, c.x), yy1 = vmax(iy1, c.y);
  const float xx2 = vmin(ix2, c.z), yy2 = vmin(iy2, c.w);
  const float w = vmax(0.f, xx2 - xx1), h = vmax(0.f, yy2 - yy1);
  const float inter = w * h;
  // disjoint boxes (most pairs): inter = 0 gives 0 / u = +-0 or NaN, never above a threshold >= 0
  if (th.fast && !(inter > 0.f)) return false;
  const float u = (ia + ca) - inter;
  if (th.fast && u >= 1.17549435e-38f && u < INFINITY && inter < INFINITY) {  // u normal: rcp(u) finite
    const float q = inter * __builtin_amdgcn_rcpf(u);
    if (q >= th.hi) return true;
    if (q <= th.lo) return false;
  }
  const float ovr = inter / u;
  return (double)ovr > th.thr;
}

// One 64-thread workgroup per (row block rb, chunk of NMS_CB column blocks >= rb): the rows' boxes
// stay in registers while the chunk's column blocks pass through LDS (corners as one float4, the
// area), each block's boxes loaded into registers one block ahead. A workgroup per (rb, cb) pair
// meant ~4 M one-wave workgroups per eval batch (half of them empty, below the diagonal).
constexpr int NMS_CB = 8;
IVIT_DEV void nms_mask_body(const float* __restrict__ sb, long n, int nw, const NmsThr& th,
                            unsigned long long* __restrict__ mask, int rb, int cb0) {
  __shared__ float4 cxy[2][64];
  __shared__ float car[2][64];
  const int t = threadIdx.x;
  const long i = (long)rb * 64 + t;
  const bool row_ok = i < n;
  float ix1 = 0.f, iy1 = 0.f, ix2 = 0.f, iy2 = 0.f, ia = 0.f;
  if (row_ok) {
    ix1 = sb[i * 5 + 0]; iy1 = sb[i * 5 + 1]; ix2 = sb[i * 5 + 2]; iy2 = sb[i * 5 + 3]; ia = sb[i * 5 + 4];
  }
  const int cbs = max(cb0, rb), cb1 = min(cb0 + NMS_CB, nw);
  float4 pxy = make_float4(0.f, 0.f, 0.f, 0.f);
  float pa = 0.f;
  auto fetch = [&](int cb) {
    const long cj = (long)cb * 64 + t;
    if (cj < n) {
      pxy = make_float4(sb[cj * 5 + 0], sb[cj * 5 + 1], sb[cj * 5 + 2], sb[cj * 5 + 3]);
      pa = sb[cj * 5 + 4];
    }
  };
  if (cbs < cb1) fetch(cbs);
  for (int cb = cbs; cb < cb1; ++cb) {
    const int buf = (cb - cbs) & 1;
    cxy[buf][t] = pxy;
    car[buf][t] = pa;
    if (cb + 1 < cb1) fetch(cb + 1);
    __syncthreads();  // one wave: publishes this block's boxes (the other buffer is the next one's)
    const int lim = (int)min((long)64, n - (long)cb * 64);
    // a wave-uniform loop; the diagonal block keeps only the bits of boxes after this one
    const unsigned long long keep_mask = cb == rb ? (t == 63 ? 0ull : ~0ull << (t + 1)) : ~0ull;
    unsigned long long bits = 0;
    for (int k = 0; k < lim; ++k)
      if (nms_suppresses(ix1, iy1, ix2, iy2, ia, cxy[buf][k], car[buf][k], th)) bits |= 1ull << k;
    if (row_ok) mask[i * nw + cb] = bits & keep_mask;
  }
}

// mask[p][w] bit k: sorted box 64w+k (> p) overlaps sorted box p with IoU > thr.
// grid (ceil(nw / NMS_CB), nw)
__global__ __launch_bounds__(64) void nms_mask_kernel(const float* __restrict__ sb, long n, int nw, NmsThr th,
                                                      unsigned long long* __restrict__ mask) {
  const int cb0 = blockIdx.x * NMS_CB, rb = blockIdx.y;
  if (cb0 + NMS_CB <= rb) return;
  nms_mask_body(sb, n, nw, th, mask, rb, cb0);
}

constexpr int NMS_MAXW = 1024;  // n <= 65536

// The greedy walk of torchvision's nms over the suppression mask (one workgroup per sample):
// column block c (64 sorted boxes) is settled by wave 0 on SCALAR registers (each diagonal word
// read by v_readlane; the serial 64-step chain runs on the scalar unit), then the kept boxes'
// mask rows are OR-ed into the removed words of the later columns, one owner thread per word with
// the kept rows' words loaded eight at a time (the earlier per-word loop over the kept bits waited
// for each load in turn).
IVIT_DEV void nms_scan_body(const unsigned long long* __restrict__ mask, long n, int nw, const int* __restrict__ order,
                            long* __restrict__ keep, long* __restrict__ count_out) {
  __shared__ unsigned long long removed[NMS_MAXW];
  __shared__ unsigned long long kept_s;
  __shared__ long cnt_s;
  __shared__ int kbit[64];
  for (int w = threadIdx.x; w < nw; w += 256) removed[w] = 0ull;
  if (threadIdx.x == 0) cnt_s = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  // wave 0 holds the next column's diagonal word and sorted index, loaded during the current
  // column's update (neither depends on it): the walk does not wait on a global load
  unsigned long long diag_n = 0ull;
  int ord_n = 0;
  if (threadIdx.x < 64 && lane < n) {
    diag_n = mask[(long)lane * nw];
    ord_n = order[lane];
  }
  for (int c = 0; c < nw; ++c) {
    if (threadIdx.x < 64) {
      const long row = (long)c * 64 + lane;
      const unsigned long long diag = diag_n;
      const int ord = ord_n;
      const unsigned dlo = (unsigned)diag, dhi = (unsigned)(diag >> 32);
      const unsigned long long r0 = removed[c];
      // (the builtins return int: widen through unsigned, or the low word sign-extends)
      unsigned long long w =
          ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(r0 >> 32)) << 32) |
          (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)r0);
      unsigned long long kept = 0ull;
      const int lim = (int)min((long)64, n - (long)c * 64);
      for (int i = 0; i < lim; ++i) {
        if (!((w >> i) & 1ull)) {
          kept |= 1ull << i;
          w |= ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(dhi, i) << 32) |
               (unsigned long long)(unsigned)__builtin_amdgcn_readlane(dlo, i);
        }
      }
      const long base = cnt_s;
      if ((kept >> lane) & 1ull) {
        const int rk = __popcll(lane ? (kept & ((1ull << lane) - 1ull)) : 0ull);
        keep[base + rk] = ord;
        kbit[rk] = lane;
      }
      if (lane == 0) {
        kept_s = kept;
        cnt_s = base + __popcll(kept);
      }
    }
    __syncthreads();
    if (threadIdx.x < 64 && c + 1 < nw) {
      const long row = (long)(c + 1) * 64 + lane;
      diag_n = row < n ? mask[row * nw + c + 1] : 0ull;
      ord_n = row < n ? order[row] : 0;
    }
    const int K = __popcll(kept_s);
    if (K) {
      // each later word has one owner thread (no atomics); its kept rows' words are loaded 8 at a time
      const unsigned long long* blk = mask + (long)c * 64 * nw;
      for (int wc = c + 1 + threadIdx.x; wc < nw; wc += 256) {
        unsigned long long acc = removed[wc];
        for (int b0 = 0; b0 < K; b0 += 8) {
          unsigned long long v[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = b0 + q < K ? blk[(long)kbit[b0 + q] * nw + wc] : 0ull;
#pragma unroll
          for (int q = 0; q < 8; ++q) acc |= v[q];
        }
        removed[wc] = acc;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *count_out = cnt_s;
}

__global__ __launch_bounds__(256) void nms_scan_kernel(const unsigned long long* __restrict__ mask, long n, int nw,
                                                       const int* __restrict__ order, long* __restrict__ keep,
                                                       long* __restrict__ count) {
  nms_scan_body(mask, n, nw, order, keep, count);
}

// ---- batched NMS: sample s owns rows seg[s] .. seg[s+1]-1 of every per-row array and the
// mask words mask_off[s] .. ; blockIdx.y (rank / sorted boxes / scan) or blockIdx.z (mask)
// selects the sample, so all samples' kernels run in one launch each (the single-workgroup
// scan of one sample no longer serialises the batch).
// keys / values of the segmented sort: the score (+0.0f: a -0 score ties with +0 as in torch's
// comparison sort) and the row's local index.
__global__ void nms_keys_b_kernel(const float* __restrict__ scores, const long* __restrict__ seg, float* __restrict__ key,
                                  int* __restrict__ idx) {
  const int sm = blockIdx.y;
  const long o = seg[sm], n = seg[sm + 1] - o;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  key[o + i] = scores[o + i] + 0.0f;
  idx[o + i] = (int)i;
}

__global__ void nms_sorted_boxes_b_kernel(const float* __restrict__ b, const int* __restrict__ order,
                                          const long* __restrict__ seg, float* __restrict__ sb) {
  const int sm = blockIdx.y;
  const long o = seg[sm], n = seg[sm + 1] - o;
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const float* q = b + (o + order[o + p]) * 5;
  const float x1 = q[0] - q[2] / 2.f, y1 = q[1] - q[3] / 2.f, x2 = q[0] + q[2] / 2.f, y2 = q[1] + q[3] / 2.f;
  float* d = sb + (o + p) * 5;
  d[0] = x1;
  d[1] = y1;
  d[2] = x2;
  d[3] = y2;
  d[4] = (x2 - x1) * (y2 - y1);
}

// grid (ceil(nwmax / NMS_CB), nwmax, samples)
__global__ __launch_bounds__(64) void nms_mask_b_kernel(const float* __restrict__ sb_all, const long* __restrict__ seg,
                                                        const long* __restrict__ mask_off, NmsThr th,
                                                        unsigned long long* __restrict__ mask_all) {
  const int sm = blockIdx.z;
  const long o = seg[sm], n = seg[sm + 1] - o;
  const int nw = (int)((n + 63) / 64);
  const int cb0 = blockIdx.x * NMS_CB, rb = blockIdx.y;
  if (cb0 >= nw || rb >= nw || cb0 + NMS_CB <= rb) return;
  nms_mask_body(sb_all + o * 5, n, nw, th, mask_all + mask_off[sm], rb, cb0);
}

__global__ __launch_bounds__(256) void nms_scan_b_kernel(const unsigned long long* __restrict__ mask_all,
                                                         const long* __restrict__ seg,
                                                         const long* __restrict__ mask_off,
                                                         const int* __restrict__ order_all,
                                                         long* __restrict__ keep_all, long* __restrict__ count) {
  const int sm = blockIdx.x;
  const long o = seg[sm], n = seg[sm + 1] - o;
  nms_scan_body(mask_all + mask_off[sm], n, (int)((n + 63) / 64), order_all + o, keep_all + o, count + sm);
}

}  // namespace

extern "C" int ivit_generate_anchors(long bev_h, long bev_w, long stride, const float* cfgs, long A, float voxel,
                                     float off_x, float off_y, float* out, void* stream) {
  IVIT_CHECK_ARG(stride > 0 && bev_h >= 0 && bev_w >= 0 && A >= 0, "ivit_generate_anchors: bad sizes (stride %ld)",
                 stride);
  const int fh = (int)(bev_h / stride), fw = (int)(bev_w / stride);
  const long n = (long)fh * fw * A;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(anchors_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, ivit_stream(stream), fh, fw, (int)stride,
                     cfgs, (int)A, voxel, off_x, off_y, out);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_axis_iou(const float* b1, long n1, const float* b2, long n2, float* out, void* stream) {
  if (n1 * n2 <= 0) return 0;
  hipLaunchKernelGGL(iou_matrix_kernel, dim3(ivit_cdiv(n1 * n2, 256)), dim3(256), 0, ivit_stream(stream), b1, n1, b2,
                     n2, out, 0);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_rotated_iou(const float* b1, long n1, const float* b2, long n2, float* out, void* stream) {
  if (n1 * n2 <= 0) return 0;
  hipLaunchKernelGGL(iou_matrix_kernel, dim3(ivit_cdiv(n1 * n2, 128)), dim3(128), 0, ivit_stream(stream), b1, n1, b2,
                     n2, out, 1);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_decode_boxes(const float* rel, const float* anchors, const long* idx, long n, float* out,
                                 void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(decode_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, ivit_stream(stream), rel, anchors, idx, n,
                     out);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" long ivit_nms_workspace(long n) {
  const long nw = (n + 63) / 64;
  return n * 4 + n * 5 * 4 + n * nw * 8 + 64;
}

extern "C" int ivit_nms(const float* boxes_xywha, const float* scores, long n, double iou_thr, long* keep, long* count,
                        void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(n <= 64L * NMS_MAXW, "ivit_nms: n=%ld exceeds %d", n, 64 * NMS_MAXW);
  IVIT_CHECK_ARG(work_bytes >= ivit_nms_workspace(n), "ivit_nms: workspace too small");
  hipStream_t st = ivit_stream(stream);
  if (n <= 0) {
    (void)hipMemsetAsync(count, 0, sizeof(long), st);
    IVIT_LAUNCH_CHECK();
    return 0;
  }
  const int nw = (int)((n + 63) / 64);
  char* w = (char*)work;
  int* order = (int*)w;
  w += (n * 4 + 15) / 16 * 16;
  float* sb = (float*)w;
  w += (n * 20 + 15) / 16 * 16;
  unsigned long long* mask = (unsigned long long*)w;
  hipLaunchKernelGGL(nms_rank_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, scores, n, order);
  hipLaunchKernelGGL(nms_sorted_boxes_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, boxes_xywha, order, n, sb);
  hipLaunchKernelGGL(nms_mask_kernel, dim3(ivit_cdiv(nw, NMS_CB), nw), dim3(64), 0, st, sb, n, nw, nms_thr(iou_thr),
                     mask);
  hipLaunchKernelGGL(nms_scan_kernel, dim3(1), dim3(256), 0, st, mask, n, nw, order, keep, count);
  IVIT_LAUNCH_CHECK();
  return 0;
}

// Batched torchvision-CPU-exact NMS (eval_vit.py:170 per sample, all samples in one launch per
// stage). seg: [S+1] int64 row offsets (device); mask_off: [S] int64 word offsets of each
// sample's [n_s, ceil(n_s/64)] suppression mask (device). keep[seg[s] ..] receives sample s's kept
// LOCAL indices in score order, count[s] their number. The score order is a stable descending
// segmented radix sort (rocPRIM; ties keep the row order, as torch's stable sort). Workspace:
// ivit_nms_batched_workspace(n_samples, total, mask_words) bytes.
namespace {
size_t nms_sort_temp_bytes(long n_samples, long total) {
  size_t bytes = 0;
  if (rocprim::segmented_radix_sort_pairs_desc(nullptr, bytes, (const float*)nullptr, (float*)nullptr,
                                               (const int*)nullptr, (int*)nullptr, (unsigned)total,
                                               (unsigned)n_samples, (const long*)nullptr, (const long*)nullptr) !=
      hipSuccess)
    return 0;
  return bytes;
}
long al16(long b) { return (b + 15) / 16 * 16; }
}  // namespace

extern "C" long ivit_nms_batched_workspace(long n_samples, long total, long mask_words) {
  if (n_samples <= 0 || total <= 0) return 64;
  return al16(4 * total) + al16(20 * total) + al16(8 * mask_words) + 2 * al16(4 * total) + al16(4 * total) +
         al16((long)nms_sort_temp_bytes(n_samples, total)) + 256 + 64;
}

extern "C" int ivit_nms_batched(const float* boxes_xywha, const float* scores, const long* seg, const long* mask_off,
                                long n_samples, long total, long max_n, long mask_words, double iou_thr, long* keep,
                                long* count, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(max_n <= 64L * NMS_MAXW, "ivit_nms_batched: n=%ld exceeds %d", max_n, 64 * NMS_MAXW);
  IVIT_CHECK_ARG(n_samples < 65536 && total < (1L << 31), "ivit_nms_batched: too many samples / rows (%ld, %ld)",
                 n_samples, total);
  IVIT_CHECK_ARG(work_bytes >= ivit_nms_batched_workspace(n_samples, total, mask_words),
                 "ivit_nms_batched: workspace too small");
  hipStream_t st = ivit_stream(stream);
  if (n_samples <= 0) return 0;
  if (max_n <= 0) {
    (void)hipMemsetAsync(count, 0, sizeof(long) * n_samples, st);
    IVIT_LAUNCH_CHECK();
    return 0;
  }
  const int nwmax = (int)((max_n + 63) / 64);
  char* w = (char*)(((uintptr_t)work + 15) & ~(uintptr_t)15);
  int* order = (int*)w;
  w += al16(4 * total);
  float* sb = (float*)w;
  w += al16(20 * total);
  unsigned long long* mask = (unsigned long long*)w;
  w += al16(8 * mask_words);
  float* key = (float*)w;
  w += al16(4 * total);
  float* key_sorted = (float*)w;
  w += al16(4 * total);
  int* idx = (int*)w;
  w += al16(4 * total);
  w = (char*)(((uintptr_t)w + 255) & ~(uintptr_t)255);
  size_t tb = nms_sort_temp_bytes(n_samples, total);
  const int gx = ivit_cdiv(max_n, 256);
  hipLaunchKernelGGL(nms_keys_b_kernel, dim3(gx, n_samples), dim3(256), 0, st, scores, seg, key, idx);
  const hipError_t e = rocprim::segmented_radix_sort_pairs_desc(w, tb, key, key_sorted, idx, order, (unsigned)total,
                                                               (unsigned)n_samples, seg, seg + 1, 0, 32, st);
  if (e != hipSuccess) {
    ivit_set_error("ivit_nms_batched: segmented sort: %s", hipGetErrorString(e));
    return (int)e;
  }
  hipLaunchKernelGGL(nms_sorted_boxes_b_kernel, dim3(gx, n_samples), dim3(256), 0, st, boxes_xywha, order, seg, sb);
  hipLaunchKernelGGL(nms_mask_b_kernel, dim3(ivit_cdiv(nwmax, NMS_CB), nwmax, n_samples), dim3(64), 0, st, sb, seg,
                     mask_off, nms_thr(iou_thr), mask);
  hipLaunchKernelGGL(nms_scan_b_kernel, dim3(n_samples), dim3(256), 0, st, mask, seg, mask_off, order, keep, count);
  IVIT_LAUNCH_CHECK();
  return 0;
}
