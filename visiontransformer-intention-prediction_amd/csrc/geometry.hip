// Eval-path geometry (utils.py): anchors, axis/rotated IoU matrices, delta decode and
// torchvision-CPU-exact non-maximum suppression.
#include "geom.h"

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
IVIT_DEV void decode_one(const float* d, const float* a, float* o) {
  o[0] = d[0] * a[2] + a[0];
  o[1] = d[1] * a[3] + a[1];
  o[2] = expf(d[2]) * a[2];
  o[3] = expf(d[3]) * a[3];
  const float yaw = a[4] + atan2f(d[4], d[5]);
  o[4] = atan2f(sinf(yaw), cosf(yaw));
}

__global__ void decode_kernel(const float* rel, const float* anchors, const long* idx, long n, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  decode_one(rel + i * 6, anchors + (idx ? idx[i] : i) * 5, out + i * 5);
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
  // u in [2^-126, 2^126): rcp(u) is a normal float too (at u >= 2^126 it would be subnormal, flushed
  // or imprecise, and q could land on the wrong side of the margin)
  if (th.fast && u >= 1.17549435e-38f && u < 0x1p126f && inter < INFINITY) {
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
    if (lim == 64) {
      // a full block: 8 boxes per group with constant bit positions and LDS offsets (the rolled loop
      // spent ~8 of its ~18 VALU per pair on the 64-bit variable shift, the select and the address)
      for (int k0 = 0; k0 < 64; k0 += 8) {
        unsigned by = 0;
        float4 cc[8];  // the group's corners read together (one LDS wait per group, not per pair)
#pragma unroll
        for (int e = 0; e < 8; ++e) cc[e] = cxy[buf][k0 + e];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (nms_suppresses(ix1, iy1, ix2, iy2, ia, cc[e], car[buf][k0 + e], th)) by |= 1u << e;
        bits |= (unsigned long long)by << k0;
      }
    } else {
      for (int k = 0; k < lim; ++k)
        if (nms_suppresses(ix1, iy1, ix2, iy2, ia, cxy[buf][k], car[buf][k], th)) bits |= 1ull << k;
    }
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

constexpr int NMS_MAXW = 2048;  // n <= 131072

// The greedy walk of torchvision's nms over the suppression mask, one workgroup per sample. Column
// block c (64 sorted boxes) is settled by wave 0 on scalar registers: starting from removed[c], it
// visits only the boxes still standing (find-first-one of ~w above the last kept box, each kept
// box's diagonal word read by v_readlane) — one step per KEPT box. The update of the later words
// no longer sits between two columns' walks. Column c's kept rows reach
//   * words c+1 and c+2 through wave 0 itself, right after its walk of c: it loaded those two words
//     of all 64 rows of column c two columns ahead (with the diagonal word; two register sets), and
//     each kept lane ORs its two into removed[] (LDS atomics);
//   * words >= c+3 through waves 1-3: their loads are issued in iteration c+1 (up to 8 kept rows in
//     flight per word, held across the barrier) and OR-ed into removed[] in iteration c+2,
// so the walk of column w finds every contribution of columns < w in removed[w], and an iteration
// costs one walk or one load issue, not a walk plus a global round trip. Kept-row lists are
// triple-buffered (column j in slot j % 3).
IVIT_DEV void nms_scan_body(const unsigned long long* __restrict__ mask, long n, int nw, const int* __restrict__ order,
                             long* __restrict__ keep, long* __restrict__ count_out) {
  __shared__ unsigned long long removed[NMS_MAXW];
  __shared__ unsigned long long kept_s[3];
  __shared__ long cnt_s;
  __shared__ int kbit[3][64];
  for (int w = threadIdx.x; w < nw; w += 256) removed[w] = 0ull;
  if (threadIdx.x == 0) cnt_s = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const bool w0 = threadIdx.x < 64;
  const int t = threadIdx.x - 64;  // bulk thread index (waves 1-3)
  // wave 0: column c's diagonal word, its two next words and the row's sorted index (lane = row),
  // four loads issued as inline asm so that the compiler's wait pass does not retire them early
  // (it cannot count them across the walk's loop and waited vmcnt(0), i.e. for the other set too);
  // rows / words past the end read clamped addresses, whose values no kept lane ever uses
  auto ld_row = [&](int c, unsigned long long& dg, unsigned long long& n1, unsigned long long& n2, int& od) {
    const int cc = min(c, nw - 1);
    const long row = min((long)cc * 64 + lane, n - 1);
    const unsigned long long* mr = mask + row * nw;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(dg) : "v"(mr + cc) : "memory");
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(n1) : "v"(mr + min(cc + 1, nw - 1)) : "memory");
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(n2) : "v"(mr + min(cc + 2, nw - 1)) : "memory");
    asm volatile("global_load_dword %0, %1, off" : "=v"(od) : "v"(order + row) : "memory");
  };
  // two register sets, A for even and B for odd columns: a set is reloaded (two columns ahead)
  // right after its column's walk, so each column's words are in flight for a whole iteration
  // (rotating one set through copies would make every copy wait for its load)
  struct Row { unsigned long long dg, n1, n2; int od; };
  Row ra{0ull, 0ull, 0ull, 0}, rb{0ull, 0ull, 0ull, 0};
  if (w0) {
    ld_row(0, ra.dg, ra.n1, ra.n2, ra.od);
    ld_row(1, rb.dg, rb.n1, rb.n2, rb.od);
  }
  // bulk: the held words of column c-1's kept rows (<= 8 per word), two words per thread
  unsigned long long held[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) held[i][q] = 0ull;
  auto iter = [&](int c, Row& r) {
    if (w0) {
      // this set's four loads retired: at most the other set's four (issued after them) remain,
      // or those and the previous column's keep[] store
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      asm volatile("" : "+v"(r.dg), "+v"(r.n1), "+v"(r.n2), "+v"(r.od));
      const unsigned dlo = (unsigned)r.dg, dhi = (unsigned)(r.dg >> 32);
      const unsigned long long r0 = removed[c];
      unsigned long long w =
          ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(r0 >> 32)) << 32) |
          (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)r0);
      unsigned long long kept = 0ull;
      const int lim = (int)min((long)64, n - (long)c * 64);
      // (the walk over all 64 bits took 2-3 x as long: scan 1332 -> 859 us per eval step)
      const unsigned long long valid = lim == 64 ? ~0ull : (1ull << lim) - 1ull;
      unsigned long long cand = ~w & valid;
      while (cand) {
        const int i = __builtin_ctzll(cand);
        kept |= 1ull << i;
        w |= ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(dhi, i) << 32) |
             (unsigned long long)(unsigned)__builtin_amdgcn_readlane(dlo, i);
        cand = ~w & valid & ((~0ull << i) << 1);
      }
      const long base = cnt_s;
      if ((kept >> lane) & 1ull) {
        const int rk = __popcll(lane ? (kept & ((1ull << lane) - 1ull)) : 0ull);
        keep[base + rk] = r.od;
        kbit[c % 3][rk] = lane;
        if (c + 1 < nw) atomicOr(&removed[c + 1], r.n1);
        if (c + 2 < nw) atomicOr(&removed[c + 2], r.n2);
      }
      if (lane == 0) {
        kept_s[c % 3] = kept;
        cnt_s = base + __popcll(kept);
      }
      ld_row(c + 2, r.dg, r.n1, r.n2, r.od);
    } else {
      if (c >= 2) {  // apply column c-2's held words (words >= c+1)
        const int j = c - 2, K = __popcll(kept_s[j % 3]);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int wc = j + 3 + t + 192 * i;
          if (wc < nw) {
            unsigned long long acc = 0ull;
#pragma unroll
            for (int q = 0; q < 8; ++q) acc |= held[i][q];
            for (int q = 8; q < K; ++q) acc |= mask[((long)j * 64 + kbit[j % 3][q]) * nw + wc];  // > 8 kept
            if (acc) atomicOr(&removed[wc], acc);
          }
        }
        for (int wc = j + 3 + 384 + t; wc < nw; wc += 192) {  // past the held words (n > 24 700)
          unsigned long long acc = 0ull;
          for (int q = 0; q < K; ++q) acc |= mask[((long)j * 64 + kbit[j % 3][q]) * nw + wc];
          if (acc) atomicOr(&removed[wc], acc);
        }
      }
      if (c >= 1) {  // issue column c-1's loads (words >= c+2)
        const int j = c - 1, K = __popcll(kept_s[j % 3]);
        long rbo[8];  // the kept rows' mask-row offsets, read from LDS before any load is issued
#pragma unroll
        for (int q = 0; q < 8; ++q) rbo[q] = ((long)j * 64 + kbit[j % 3][q]) * nw;  // q >= K: unused
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int wc = j + 3 + t + 192 * i;
#pragma unroll
          for (int q = 0; q < 8; ++q) held[i][q] = wc < nw && q < K ? mask[rbo[q] + wc] : 0ull;
        }
      }
    }
    __syncthreads();
  };
  for (int c = 0; c < nw; c += 2) {
    iter(c, ra);
    if (c + 1 < nw) iter(c + 1, rb);
  }
  if (threadIdx.x == 0) *count_out = cnt_s;
}

__global__ __launch_bounds__(256) void nms_scan_kernel(const unsigned long long* __restrict__ mask, long n, int nw,
                                                       const int* __restrict__ order, long* __restrict__ keep,
                                                       long* __restrict__ count) {
  nms_scan_body(mask, n, nw, order, keep, count);
}

// ---- batched NMS and the fused eval post-processing -------------------------------------------
// Sample s owns rows lo(s) .. lo(s) + n(s) - 1 of every per-row array and the mask words mo(s) ..:
// either host prefix offsets (seg [S+1], mask_off [S]: ivit_nms_batched) or a fixed capacity per
// sample with the row counts on the device (ivit_eval_post: nothing is read back before the NMS).
struct SegView {
  const long* seg;   // [S+1] row offsets, or null
  const long* moff;  // [S] mask word offsets (with seg)
  const int* cnt;    // [S] rows per sample (without seg)
  long row_stride, mask_stride;
  IVIT_DEV long lo(int s) const { return seg ? seg[s] : (long)s * row_stride; }
  IVIT_DEV long n(int s) const { return seg ? seg[s + 1] - seg[s] : (long)cnt[s]; }
  IVIT_DEV long mo(int s) const { return seg ? moff[s] : (long)s * mask_stride; }
};

// One sample per workgroup of PS_T threads (16 waves) for the selection and the score sort.
constexpr int PS_T = 1024;
constexpr int PS_D = 16;  // radix digits: 4 key bits per pass

// Ascending order of the key = torch's stable descending sort of the score: the IEEE order made
// unsigned, inverted; s + 0.0f makes -0 tie with +0 as torch's comparison sort does.
IVIT_DEV unsigned desc_key(float s) {
  const unsigned u = __float_as_uint(s + 0.0f);
  return ~(u ^ ((u >> 31) ? 0xffffffffu : 0x80000000u));
}

// Exclusive prefix of v over the workgroup in thread order; the total goes to wsum[16].
// wsum: 17 LDS words. The caller separates two calls by a barrier.
IVIT_DEV unsigned block_excl_scan(unsigned v, unsigned* wsum) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (wid == 0) {
    const unsigned w = lane < PS_T / 64 ? wsum[lane] : 0u;
    unsigned z = w;
#pragma unroll
    for (int o = 1; o < PS_T / 64; o <<= 1) {
      const unsigned y = __shfl_up(z, o, 64);
      if (lane >= o) z += y;
    }
    if (lane < PS_T / 64) wsum[lane] = z - w;
    if (lane == PS_T / 64 - 1) wsum[16] = z;
  }
  __syncthreads();
  return wsum[wid] + x - v;
}

// Stable LSD radix sort of n (key, value) pairs by ascending key, by one workgroup. Thread t owns
// the contiguous chunk [t*I, t*I + I), I = ceil(n / PS_T): it counts its chunk's digits into its
// own histogram column (hist[d * PS_T + t], no atomics), the digit-major exclusive scan of the
// columns gives every (digit, thread) its first slot, and the thread scatters its chunk in order —
// so equal digits keep their order and the sort is stable. Thread t scans entries 16t .. 16t + 15,
// which all belong to digit t / 64: wave d's sum is digit d's total, and a pass in which one digit
// holds all n keys moves nothing and is skipped (the scores of one eval sample share their top
// bits). Keys / values ping-pong between (k0, v0) and (k1, v1), global scratch that stays in L2;
// returns which pair holds the result. n < 2^31.
IVIT_DEV int block_radix_sort(unsigned* k0, int* v0, unsigned* k1, int* v1, int n, unsigned* hist, unsigned* wsum,
                              int* skip) {
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int I = (n + PS_T - 1) / PS_T;
  const int b0 = min(t * I, n), b1 = min(b0 + I, n);
  int cur = 0;
  for (int shift = 0; shift < 32; shift += 4) {
    const unsigned* ki = cur ? k1 : k0;
    const int* vi = cur ? v1 : v0;
    unsigned* ko = cur ? k0 : k1;
    int* vo = cur ? v0 : v1;
#pragma unroll
    for (int d = 0; d < PS_D; ++d) hist[d * PS_T + t] = 0u;
    if (t == 0) *skip = 0;
    // the chunk in groups of 8 keys, each group's loads issued together (one L2 latency per group,
    // not per key: the LDS counter updates after them are a dependent chain the compiler cannot
    // overlap with the next key's load)
    for (int g0 = b0; g0 < b1; g0 += 8) {
      unsigned kr[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) kr[e] = g0 + e < b1 ? ki[g0 + e] : 0u;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (g0 + e < b1) ++hist[((kr[e] >> shift) & 15u) * PS_T + t];
    }
    __syncthreads();
    unsigned c[PS_D], run = 0;
#pragma unroll
    for (int j = 0; j < PS_D; ++j) {
      c[j] = hist[t * PS_D + j];
      run += c[j];
    }
    unsigned x = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (wid == 0) {
      const unsigned w = lane < PS_D ? wsum[lane] : 0u;
      unsigned z = w;
#pragma unroll
      for (int o = 1; o < PS_D; o <<= 1) {
        const unsigned y = __shfl_up(z, o, 64);
        if (lane >= o) z += y;
      }
      if (lane < PS_D) {
        wsum[lane] = z - w;
        if (w == (unsigned)n) *skip = 1;
      }
    }
    __syncthreads();
    unsigned off = wsum[wid] + x - run;
#pragma unroll
    for (int j = 0; j < PS_D; ++j) {
      hist[t * PS_D + j] = off;
      off += c[j];
    }
    __syncthreads();
    if (!*skip) {
      for (int g0 = b0; g0 < b1; g0 += 8) {
        unsigned kr[8];
        int vr[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          kr[e] = g0 + e < b1 ? ki[g0 + e] : 0u;
          vr[e] = g0 + e < b1 ? vi[g0 + e] : 0;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (g0 + e < b1) {
            const unsigned slot = ((kr[e] >> shift) & 15u) * PS_T + t;
            const unsigned p = hist[slot];
            hist[slot] = p + 1u;
            ko[p] = kr[e];
            vo[p] = vr[e];
          }
        }
      }
      cur ^= 1;
    }
    __syncthreads();
  }
  return cur;
}

// torchvision's nms input for sorted row p: corners of box[order[p]] and the area (utils.py:266-272)
IVIT_DEV void sorted_corners(const float* q, float* d) {
  const float x1 = q[0] - q[2] / 2.f, y1 = q[1] - q[3] / 2.f, x2 = q[0] + q[2] / 2.f, y2 = q[1] + q[3] / 2.f;
  d[0] = x1;
  d[1] = y1;
  d[2] = x2;
  d[3] = y2;
  d[4] = (x2 - x1) * (y2 - y1);
}

// ivit_nms_batched, stage 1: one workgroup per sample — keys from the scores, the stable
// descending sort, the sorted corner boxes. k0/v0/k1/v1: [total] scratch.
__global__ __launch_bounds__(PS_T) void nms_sort_b_kernel(const float* __restrict__ b, const float* __restrict__ scores,
                                                          const long* __restrict__ seg, unsigned* k0, int* v0,
                                                          unsigned* k1, int* v1, int* __restrict__ order,
                                                          float* __restrict__ sb) {
  __shared__ unsigned hist[PS_D * PS_T];
  __shared__ unsigned wsum[20];
  __shared__ int skip;
  const int sm = blockIdx.x;
  const long o = seg[sm];
  const int n = (int)(seg[sm + 1] - o);
  for (int i = threadIdx.x; i < n; i += PS_T) {
    k0[o + i] = desc_key(scores[o + i]);
    v0[o + i] = i;
  }
  __syncthreads();
  const int r = block_radix_sort(k0 + o, v0 + o, k1 + o, v1 + o, n, hist, wsum, &skip);
  const int* ord = (r ? v1 : v0) + o;
  for (int p = threadIdx.x; p < n; p += PS_T) {
    const int q = ord[p];
    order[o + p] = q;
    sorted_corners(b + (o + q) * 5, sb + (o + p) * 5);
  }
}

// grid (ceil(nwmax / NMS_CB), nwmax, samples)
__global__ __launch_bounds__(64) void nms_mask_b_kernel(const float* __restrict__ sb_all, SegView sv, NmsThr th,
                                                        unsigned long long* __restrict__ mask_all) {
  const int sm = blockIdx.z;
  const long o = sv.lo(sm), n = sv.n(sm);
  const int nw = (int)((n + 63) / 64);
  const int cb0 = blockIdx.x * NMS_CB, rb = blockIdx.y;
  if (cb0 >= nw || rb >= nw || cb0 + NMS_CB <= rb) return;
  nms_mask_body(sb_all + o * 5, n, nw, th, mask_all + sv.mo(sm), rb, cb0);
}

__global__ __launch_bounds__(256) void nms_scan_b_kernel(const unsigned long long* __restrict__ mask_all, SegView sv,
                                                         const int* __restrict__ order_all,
                                                         long* __restrict__ keep_all, long* __restrict__ count) {
  const int sm = blockIdx.x;
  const long o = sv.lo(sm), n = sv.n(sm);
  nms_scan_body(mask_all + sv.mo(sm), n, (int)((n + 63) / 64), order_all + o, keep_all + o, count + sm);
}

// ---- eval post-processing (eval_vit.py:156-176) for a whole batch, capacity NA rows per sample.
struct PostWs {
  int* n;            // [S] rows passing the confidence threshold
  int* anchor;       // [S*NA] anchor index of compacted row p
  float* score;      // [S*NA]
  float* box;        // [S*NA*5] decoded (utils.py:227-257)
  unsigned *k0, *k1;  // sort scratch
  int *v0, *v1;
  int* order;        // [S*NA] stable descending score order (compacted-row indices)
  float* sb;         // [S*NA*5] sorted corners + area
  long* keep;        // [S*NA] kept compacted-row indices in score order
  unsigned long long* mask;
};

// torch's f32 sigmoid on the GPU: 1 / (1 + exp(-x)), IEEE division (UnarySpecialOpsKernel.cu)
IVIT_DEV float torch_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }

// eval_vit.py:159-168 for sample blockIdx.x: scores = sigmoid(cls); where(score >= conf) in anchor
// order (a workgroup-wide exclusive scan of per-thread counts: thread t owns anchors
// [t*I, t*I + I)); the compacted scores, anchor indices and decoded boxes; then apply_nms's stable
// descending score order and its sorted corner boxes. NaN logits fail the threshold, as in torch.
__global__ __launch_bounds__(PS_T) void post_select_kernel(const float* __restrict__ cls, const float* __restrict__ rel,
                                                           const float* __restrict__ anchors, int NA, float conf,
                                                           PostWs w) {
  __shared__ unsigned hist[PS_D * PS_T];
  __shared__ unsigned wsum[20];
  __shared__ int skip;
  const int sm = blockIdx.x, t = threadIdx.x;
  const long base = (long)sm * NA;
  const float* c = cls + base;
  const float* r = rel + base * 6;
  const int I = (NA + PS_T - 1) / PS_T;
  const int a0 = min(t * I, NA), a1 = min(a0 + I, NA);
  unsigned np = 0;
  for (int g0 = a0; g0 < a1; g0 += 8) {  // the logits of 8 anchors loaded together
    float lr[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) lr[e] = g0 + e < a1 ? c[g0 + e] : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) np += g0 + e < a1 && torch_sigmoid(lr[e]) >= conf;
  }
  unsigned p = block_excl_scan(np, wsum);
  const int n = (int)wsum[16];
  for (int g0 = a0; g0 < a1; g0 += 8) {
    float lr[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) lr[e] = g0 + e < a1 ? c[g0 + e] : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int a = g0 + e;
      const float s = torch_sigmoid(lr[e]);
      if (a < a1 && s >= conf) {
        const long q = base + p;
        w.anchor[q] = a;
        w.score[q] = s;
        w.k0[q] = desc_key(s);
        w.v0[q] = (int)p;
        decode_one(r + (long)a * 6, anchors + (long)a * 5, w.box + q * 5);
        ++p;
      }
    }
  }
  if (t == 0) w.n[sm] = n;
  __syncthreads();
  const int res = block_radix_sort(w.k0 + base, w.v0 + base, w.k1 + base, w.v1 + base, n, hist, wsum, &skip);
  const int* ord = (res ? w.v1 : w.v0) + base;
  for (int i = t; i < n; i += PS_T) {
    const int q = ord[i];
    w.order[base + i] = q;
    sorted_corners(w.box + (base + q) * 5, w.sb + (base + i) * 5);
  }
}

// eval_vit.py:172-175: kept row j of sample s (blockIdx.y) -> its score, decoded box and the
// argmax intention of its anchor (first maximum; a NaN is the maximum, the first NaN wins — torch's
// argmax), packed at s * NA + j.
__global__ void post_gather_kernel(const long* __restrict__ kcnt, const float* __restrict__ intent, int NA, int K,
                                   PostWs w, float* __restrict__ out_score, float* __restrict__ out_box,
                                   long* __restrict__ out_int) {
  const int sm = blockIdx.y;
  const long j = (long)blockIdx.x * 256 + threadIdx.x;
  if (j >= kcnt[sm]) return;
  const long base = (long)sm * NA, k = base + w.keep[base + j], q = base + j;
  out_score[q] = w.score[k];
#pragma unroll
  for (int e = 0; e < 5; ++e) out_box[q * 5 + e] = w.box[k * 5 + e];
  const float* lg = intent + (base + w.anchor[k]) * K;
  int best = 0;
  float bv = lg[0];
  for (int e = 1; e < K; ++e) {
    const float v = lg[e];
    if (bv == bv && (v > bv || v != v)) {
      bv = v;
      best = e;
    }
  }
  out_int[q] = best;
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
// sort (nms_sort_b_kernel: one workgroup per sample; ties keep the row order, as torch's stable
// sort). Workspace: ivit_nms_batched_workspace(n_samples, total, mask_words) bytes.
namespace {
long al16(long b) { return (b + 15) / 16 * 16; }
}  // namespace

extern "C" long ivit_nms_batched_workspace(long n_samples, long total, long mask_words) {
  if (n_samples <= 0 || total <= 0) return 64;
  return al16(4 * total) + al16(20 * total) + al16(8 * mask_words) + 4 * al16(4 * total) + 64;
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
  unsigned* k0 = (unsigned*)w;
  w += al16(4 * total);
  unsigned* k1 = (unsigned*)w;
  w += al16(4 * total);
  int* v0 = (int*)w;
  w += al16(4 * total);
  int* v1 = (int*)w;
  const SegView sv{seg, mask_off, nullptr, 0, 0};
  hipLaunchKernelGGL(nms_sort_b_kernel, dim3(n_samples), dim3(PS_T), 0, st, boxes_xywha, scores, seg, k0, v0, k1, v1,
                     order, sb);
  hipLaunchKernelGGL(nms_mask_b_kernel, dim3(ivit_cdiv(nwmax, NMS_CB), nwmax, n_samples), dim3(64), 0, st, sb, sv,
                     nms_thr(iou_thr), mask);
  hipLaunchKernelGGL(nms_scan_b_kernel, dim3(n_samples), dim3(256), 0, st, mask, sv, order, keep, count);
  IVIT_LAUNCH_CHECK();
  return 0;
}

// Eval post-processing for a batch (eval_vit.py:156-176): four launches, no host round trip.
namespace {
struct PostLayout {
  long bytes;
  long off[12];
};
PostLayout post_layout(long B, long NA) {
  const long R = B * NA, nw = (NA + 63) / 64;
  const long sz[12] = {4 * B, 4 * R, 4 * R, 20 * R, 4 * R, 4 * R, 4 * R, 4 * R, 4 * R, 20 * R, 8 * R, 8 * R * nw};
  PostLayout L{0, {}};
  for (int i = 0; i < 12; ++i) {
    L.off[i] = L.bytes;
    L.bytes += al16(sz[i]);
  }
  L.bytes += 16;  // alignment slack
  return L;
}
}  // namespace

extern "C" long ivit_eval_post_workspace(long B, long NA) {
  if (B <= 0 || NA <= 0) return 64;
  return post_layout(B, NA).bytes;
}

extern "C" int ivit_eval_post(const float* cls, const float* box_rel, const float* intent, const float* anchors, long B,
                              long NA, long K, float conf_thr, double iou_thr, float* out_scores, float* out_boxes,
                              long* out_intent, long* out_count, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(B >= 0 && B < 65536 && NA >= 0 && K >= 1, "ivit_eval_post: bad sizes (B %ld, NA %ld, K %ld)", B, NA,
                 K);
  IVIT_CHECK_ARG(NA <= 64L * NMS_MAXW, "ivit_eval_post: NA=%ld exceeds %d", NA, 64 * NMS_MAXW);
  IVIT_CHECK_ARG(work_bytes >= ivit_eval_post_workspace(B, NA), "ivit_eval_post: workspace too small");
  hipStream_t st = ivit_stream(stream);
  if (B == 0) return 0;
  if (NA == 0) {
    (void)hipMemsetAsync(out_count, 0, sizeof(long) * B, st);
    IVIT_LAUNCH_CHECK();
    return 0;
  }
  const PostLayout L = post_layout(B, NA);
  char* base = (char*)(((uintptr_t)work + 15) & ~(uintptr_t)15);
  PostWs w;
  w.n = (int*)(base + L.off[0]);
  w.anchor = (int*)(base + L.off[1]);
  w.score = (float*)(base + L.off[2]);
  w.box = (float*)(base + L.off[3]);
  w.k0 = (unsigned*)(base + L.off[4]);
  w.k1 = (unsigned*)(base + L.off[5]);
  w.v0 = (int*)(base + L.off[6]);
  w.v1 = (int*)(base + L.off[7]);
  w.order = (int*)(base + L.off[8]);
  w.sb = (float*)(base + L.off[9]);
  w.keep = (long*)(base + L.off[10]);
  w.mask = (unsigned long long*)(base + L.off[11]);
  const int nw = (int)((NA + 63) / 64);
  const SegView sv{nullptr, nullptr, w.n, NA, NA * nw};
  hipLaunchKernelGGL(post_select_kernel, dim3(B), dim3(PS_T), 0, st, cls, box_rel, anchors, (int)NA, conf_thr, w);
  hipLaunchKernelGGL(nms_mask_b_kernel, dim3(ivit_cdiv(nw, NMS_CB), nw, B), dim3(64), 0, st, w.sb, sv,
                     nms_thr(iou_thr), w.mask);
  hipLaunchKernelGGL(nms_scan_b_kernel, dim3(B), dim3(256), 0, st, w.mask, sv, w.order, w.keep, out_count);
  hipLaunchKernelGGL(post_gather_kernel, dim3(ivit_cdiv(NA, 256), B), dim3(256), 0, st, out_count, intent, (int)NA,
                     (int)K, w, out_scores, out_boxes, out_intent);
  IVIT_LAUNCH_CHECK();
  return 0;
}
