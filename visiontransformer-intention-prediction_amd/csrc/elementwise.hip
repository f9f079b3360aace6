// Small bandwidth-bound kernels: dtype casts, column-slice copies, the head output split
// (heads.py:18-25,39-43 view/permute + model_vit.py:181-184 reshape) and fused AdamW
// (torch.optim.AdamW as used at train_vit.py:130).
#include "ivit_common.h"

namespace {

IVIT_DEV float ldv(const void* p, int dt, long i) {
  return dt == IVIT_BF16 ? bf2f(((const bf16*)p)[i]) : ((const float*)p)[i];
}
IVIT_DEV void stv(void* p, int dt, long i, float v) {
  if (dt == IVIT_BF16) ((bf16*)p)[i] = f2bf(v);
  else ((float*)p)[i] = v;
}

__global__ void cast_kernel(const void* x, int xdt, void* y, int ydt, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) stv(y, ydt, i, ldv(x, xdt, i));
}

__global__ void add_act_grad_kernel(const void* a, int adt, const void* b, int bdt, const void* pre, int pdt,
                                    const float* rs, long re, void* out, int odt, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = ldv(a, adt, i);
  if (b) v += ldv(b, bdt, i);
  if (pre) v *= gelu_erf_grad(ldv(pre, pdt, i));
  if (rs) v *= rs[i / re];
  stv(out, odt, i, v);
}

// 8 elements per thread (n % 8 == 0, row_elems % 8 == 0, 16-B aligned operands): the same per-element
// arithmetic and order as add_act_grad_kernel, 16-B accesses
__global__ __launch_bounds__(256) void add_act_grad8_kernel(const void* a, int adt, const void* b, int bdt,
                                                           const void* pre, int pdt, const float* rs, long re,
                                                           void* out, int odt, long n) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  float v[8], w[8];
  ld8dt(a, adt, i, v);
  if (b) {
    ld8dt(b, bdt, i, w);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += w[e];
  }
  if (pre) {
    ld8dt(pre, pdt, i, w);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= gelu_erf_grad(w[e]);
  }
  if (rs) {
    const float r = rs[i / re];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= r;
  }
  st8dt(out, odt, i, v);
}

// standalone activation modules (nn.GELU exact erf / nn.ReLU) and their input gradients
__global__ void act_fwd_kernel(int act, const void* x, int xdt, void* y, int ydt, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = ldv(x, xdt, i);
  stv(y, ydt, i, act == IVIT_ACT_GELU ? gelu_erf(v) : (act == IVIT_ACT_RELU ? (v > 0.f ? v : 0.f) : v));
}
__global__ void act_bwd_kernel(int act, const void* dy, int dydt, const void* x, int xdt, void* dx, int dxdt,
                               long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float g = ldv(dy, dydt, i), v = ldv(x, xdt, i);
  stv(dx, dxdt, i, act == IVIT_ACT_GELU ? g * gelu_erf_grad(v) : (act == IVIT_ACT_RELU ? (v > 0.f ? g : 0.f) : g));
}

__global__ void copy_cols_kernel(const void* src, long lds, void* dst, long ldd, long rows, long cols, int dt) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  const long r = i / cols, c = i - r * cols;
  stv(dst, dt, r * ldd + c, ldv(src, dt, r * lds + c));
}

// head row m (one BEV cell), anchor a: det channel a*7 + j (j=0 cls, 1..6 box),
// intent channel A*7 + a*K + k.  Flat anchor index = m*A + a  (model_vit.py:183-184).
__global__ void split_heads_kernel(const float* __restrict__ h, long ldh, long M, int A, int K, float* cls,
                                   float* box, float* intent) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over M*A
  if (i >= M * A) return;
  const long m = i / A;
  const int a = (int)(i - m * A);
  const float* r = h + m * ldh;
  cls[i] = r[a * 7];
#pragma unroll
  for (int j = 0; j < 6; ++j) box[i * 6 + j] = r[a * 7 + 1 + j];
  for (int k = 0; k < K; ++k) intent[i * K + k] = r[A * 7 + a * K + k];
}

__global__ void merge_heads_kernel(const float* dcls, const float* dbox, const float* dint, long M, int A, int K,
                                   void* dh, long ldh, int dt) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over M*ldh
  if (i >= M * ldh) return;
  const long m = i / ldh;
  const int c = (int)(i - m * ldh);
  float v = 0.f;
  if (c < A * 7) {
    const int a = c / 7, j = c - a * 7;
    const long fa = m * A + a;
    v = j == 0 ? (dcls ? dcls[fa] : 0.f) : (dbox ? dbox[fa * 6 + j - 1] : 0.f);
  } else if (c < A * 7 + A * K) {
    const int cc = c - A * 7, a = cc / K, k = cc - a * K;
    v = dint ? dint[(m * A + a) * K + k] : 0.f;
  }
  stv(dh, dt, i, v);
}

// torch _multi_tensor_adamw (foreach=True, amsgrad=False, maximize=False):
//   p *= 1 - lr*wd ; m = lerp(m, g, 1-b1) ; v = v*b2 + (1-b2) g^2
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// shadows (optional): per tensor a bf16 copy of the updated parameter (nullptr: none) — the
// compute-dtype weights the next forward reads, refreshed here instead of by per-step casts.
// omb1 / omb2: the (1 - beta) weights of lerp / addcmul (torch computes them in f64 from its Python
// floats; the guarded entry point does the same).
// finite (optional, device): 0 = the loss guard fired (loss.py:190-198) — nothing is updated, as
// when the reference's step sees no grad.
// steps_in / steps_out (optional, device f32 per tensor): the step counts before / after this
// update. With them bc1 / bc2 come from steps_in[t] + 1 in f64 (what the host computes from its
// counter), and a skipped (finite = 0) update leaves the count where it was, so the NEXT update's
// bias correction is the one torch.optim.AdamW uses when that step never happened. The count is
// written to a second buffer (block 0 of the tensor) so that no block reads a count another
// block has already advanced; the caller swaps the two buffers.
// One element of the update. Contraction off: the two launch forms below (and any vector width)
// round identically, whatever the surrounding code lets the backend fuse.
IVIT_DEV void adamw_elem(float gi, float& pi, float& mi, float& vi, float keep, float omb1, float b2, float omb2,
                         float bc2s, float eps, float step) {
#pragma clang fp contract(off)
  pi = pi * keep;
  mi = mi + omb1 * (gi - mi);
  vi = vi * b2 + omb2 * gi * gi;
  const float den = sqrtf(vi) / bc2s + eps;
  pi = pi - step * (mi / den);
}

__global__ __launch_bounds__(256) void adamw_kernel(void* const* params, void* const* grads, void* const* ms,
                                                    void* const* vs, const long* sizes, float lr, float b1, float b2,
                                                    float eps, float wd, float bc1, float bc2s, void* const* shadows,
                                                    int sstride, const float* finite, const float* steps_in,
                                                    float* steps_out, double b1d, double b2d, float omb1,
                                                    float omb2) {
  const int t = blockIdx.y;
  const bool go = finite == nullptr || *finite != 0.f;
  const long n = sizes[t];
  if (steps_in != nullptr) {
    const float s0 = steps_in[t];
    if (blockIdx.x == 0 && threadIdx.x == 0) steps_out[t] = go ? s0 + 1.f : s0;
    // the grid is sized for the largest tensor: most blocks of a small one have no elements, and
    // must leave before the f64 pow (it made the launch 4x slower)
    if (!go || (long)blockIdx.x * blockDim.x >= n) return;
    const double s = (double)s0 + 1.0;
    bc1 = (float)(1.0 - pow(b1d, s));
    bc2s = (float)sqrt(1.0 - pow(b2d, s));
  }
  if (!go) return;
  float* p = (float*)params[t];
  const float* g = (const float*)grads[t];
  float* m = (float*)ms[t];
  float* v = (float*)vs[t];
  bf16* sh = shadows ? (bf16*)shadows[(long)sstride * t] : nullptr;
  const float step = lr / bc1, keep = 1.f - lr * wd;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_elem(g[i], pi, mi, vi, keep, omb1, b2, omb2, bc2s, eps, step);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (sh) sh[i] = (bf16)pi;
  }
}

// The same update over a flat list of fixed-size chunks (ivit_adamw_chunked): one workgroup per
// chunk of AW_CHUNK elements of one tensor (chunks[b] = (tensor, chunk index)), 16-B accesses where
// the tensor's four arrays allow them. The 2D form above launches max_size / 256 workgroups for EVERY
// tensor (335 k for IntentNetViT's 327 parameters, nearly all of them leaving at once), which kept
// the update at ~3.7 TB/s; this grid has exactly the ~15.7 k chunks there are. Same element update
// (adamw_elem): bit-identical results.
constexpr int AW_CHUNK = 4096;
__global__ __launch_bounds__(256) void adamw_chunk_kernel(void* const* params, void* const* grads, void* const* ms,
                                                          void* const* vs, const long* sizes, const int2* chunks,
                                                          float lr, float b2, float eps, float wd, float bc1,
                                                          float bc2s, void* const* shadows, const float* finite,
                                                          const float* steps_in, float* steps_out, double b1d,
                                                          double b2d, float omb1, float omb2) {
  const int2 ck = chunks[blockIdx.x];
  const int t = ck.x;
  const bool go = finite == nullptr || *finite != 0.f;
  if (steps_in != nullptr) {
    const float s0 = steps_in[t];
    if (ck.y == 0 && threadIdx.x == 0) steps_out[t] = go ? s0 + 1.f : s0;
    if (!go) return;
    const double s = (double)s0 + 1.0;
    bc1 = (float)(1.0 - pow(b1d, s));
    bc2s = (float)sqrt(1.0 - pow(b2d, s));
  }
  if (!go) return;
  const long off = (long)ck.y * AW_CHUNK;
  const long n = sizes[t];
  const int len = (int)min((long)AW_CHUNK, n - off);
  float* p = (float*)params[t] + off;
  const float* g = (const float*)grads[t] + off;
  float* m = (float*)ms[t] + off;
  float* v = (float*)vs[t] + off;
  bf16* sh = shadows && shadows[t] ? (bf16*)shadows[t] + off : nullptr;
  const float step = lr / bc1, keep = 1.f - lr * wd;
  auto upd = [&](float gi, float& pi, float& mi, float& vi) {
    adamw_elem(gi, pi, mi, vi, keep, omb1, b2, omb2, bc2s, eps, step);
  };
  const bool vec = ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0) &&
                   (((uintptr_t)sh & 7) == 0) && (len & 3) == 0;
  if (vec) {
    for (int i = threadIdx.x * 4; i < len; i += 1024) {
      const float4 gi = *(const float4*)(g + i);
      float4 pi = *(const float4*)(p + i), mi = *(const float4*)(m + i), vi = *(const float4*)(v + i);
      upd(gi.x, pi.x, mi.x, vi.x);
      upd(gi.y, pi.y, mi.y, vi.y);
      upd(gi.z, pi.z, mi.z, vi.z);
      upd(gi.w, pi.w, mi.w, vi.w);
      *(float4*)(p + i) = pi;
      *(float4*)(m + i) = mi;
      *(float4*)(v + i) = vi;
      if (sh) *(uint2*)(sh + i) = make_uint2(pk_bf16(pi.x, pi.y), pk_bf16(pi.z, pi.w));
    }
  } else {
    for (int i = threadIdx.x; i < len; i += 256) {
      float pi = p[i], mi = m[i], vi = v[i];
      upd(g[i], pi, mi, vi);
      p[i] = pi;
      m[i] = mi;
      v[i] = vi;
      if (sh) sh[i] = (bf16)pi;
    }
  }
}

}  // namespace

extern "C" int ivit_cast(const void* x, int x_dtype, void* y, int y_dtype, long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(cast_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, ivit_stream(stream), x, x_dtype, y, y_dtype,
                     n);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_add_act_grad(const void* a, int a_dtype, const void* b, int b_dtype, const void* pre,
                                 int pre_dtype, const float* row_scale, long row_elems, void* out, int out_dtype, long n,
                                 void* stream) {
  if (n <= 0) return 0;
  const long re = row_elems > 0 ? row_elems : 1;
  if (n % 8 == 0 && (!row_scale || re % 8 == 0) && hal16(a) && (!b || hal16(b)) && (!pre || hal16(pre)) && hal16(out))
    hipLaunchKernelGGL(add_act_grad8_kernel, dim3(ivit_cdiv(n / 8, 256)), dim3(256), 0, ivit_stream(stream), a, a_dtype,
                       b, b_dtype, pre, pre_dtype, row_scale, re, out, out_dtype, n);
  else
    hipLaunchKernelGGL(add_act_grad_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, ivit_stream(stream), a, a_dtype, b,
                       b_dtype, pre, pre_dtype, row_scale, re, out, out_dtype, n);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_copy_cols(const void* src, long lds, void* dst, long ldd, long rows, long cols, int dtype,
                              void* stream) {
  if (rows * cols <= 0) return 0;
  hipLaunchKernelGGL(copy_cols_kernel, dim3(ivit_cdiv(rows * cols, 256)), dim3(256), 0, ivit_stream(stream), src, lds,
                     dst, ldd, rows, cols, dtype);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_split_heads(const float* h, long ldh, long M, long A, long K, float* cls, float* box,
                                float* intent, void* stream) {
  IVIT_CHECK_ARG(ldh >= A * 7 + A * K, "ivit_split_heads: ldh too small");
  if (M <= 0) return 0;
  hipLaunchKernelGGL(split_heads_kernel, dim3(ivit_cdiv(M * A, 256)), dim3(256), 0, ivit_stream(stream), h, ldh, M,
                     (int)A, (int)K, cls, box, intent);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_merge_heads_grad(const float* dcls, const float* dbox, const float* dint, long M, long A, long K,
                                     void* dh, long ldh, int dh_dtype, void* stream) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(merge_heads_kernel, dim3(ivit_cdiv(M * ldh, 256)), dim3(256), 0, ivit_stream(stream), dcls, dbox,
                     dint, M, (int)A, (int)K, dh, ldh, dh_dtype);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_adamw(long n_tensors, void* const* params, void* const* grads, void* const* exp_avg,
                          void* const* exp_avg_sq, const long* sizes, long max_size, float lr, float beta1,
                          float beta2, float eps, float weight_decay, float bc1, float bc2_sqrt, void* stream) {
  if (n_tensors <= 0) return 0;
  IVIT_CHECK_ARG(n_tensors < 65536, "ivit_adamw: too many tensors");
  int gx = ivit_cdiv(max_size, 256);
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(adamw_kernel, dim3(gx, n_tensors), dim3(256), 0, ivit_stream(stream), params, grads, exp_avg,
                     exp_avg_sq, sizes, lr, beta1, beta2, eps, weight_decay, bc1, bc2_sqrt, (void* const*)nullptr, 1,
                     (const float*)nullptr, (const float*)nullptr, (float*)nullptr, 0.0, 0.0, 1.f - beta1, 1.f - beta2);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_adamw_shadow(long n_tensors, void* const* params, void* const* grads, void* const* exp_avg,
                                 void* const* exp_avg_sq, void* const* shadows, const long* sizes, long max_size,
                                 float lr, float beta1, float beta2, float eps, float weight_decay, float bc1,
                                 float bc2_sqrt, void* stream) {
  if (n_tensors <= 0) return 0;
  IVIT_CHECK_ARG(n_tensors < 65536, "ivit_adamw_shadow: too many tensors");
  IVIT_CHECK_ARG(shadows != nullptr, "ivit_adamw_shadow: shadow table is null");
  int gx = ivit_cdiv(max_size, 256);
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(adamw_kernel, dim3(gx, n_tensors), dim3(256), 0, ivit_stream(stream), params, grads, exp_avg,
                     exp_avg_sq, sizes, lr, beta1, beta2, eps, weight_decay, bc1, bc2_sqrt, shadows, 1,
                     (const float*)nullptr, (const float*)nullptr, (float*)nullptr, 0.0, 0.0, 1.f - beta1, 1.f - beta2);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_adamw_guarded(long n_tensors, void* const* params, void* const* grads, void* const* exp_avg,
                                  void* const* exp_avg_sq, void* const* shadows, const long* sizes, long max_size,
                                  float lr, double beta1, double beta2, float eps, float weight_decay, float bc1,
                                  float bc2_sqrt, const float* finite, const float* steps_in, float* steps_out,
                                  void* stream) {
  if (n_tensors <= 0) return 0;
  IVIT_CHECK_ARG(n_tensors < 65536, "ivit_adamw_guarded: too many tensors");
  IVIT_CHECK_ARG((steps_in == nullptr) == (steps_out == nullptr), "ivit_adamw_guarded: steps_in / steps_out pair");
  IVIT_CHECK_ARG(steps_in == nullptr || steps_in != steps_out, "ivit_adamw_guarded: steps_out aliases steps_in");
  int gx = ivit_cdiv(max_size, 256);
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(adamw_kernel, dim3(gx, n_tensors), dim3(256), 0, ivit_stream(stream), params, grads, exp_avg,
                     exp_avg_sq, sizes, lr, (float)beta1, (float)beta2, eps, weight_decay, bc1, bc2_sqrt, shadows, 1,
                     finite, steps_in, steps_out, beta1, beta2, (float)(1.0 - beta1), (float)(1.0 - beta2));
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" long ivit_adamw_chunk_elems() { return AW_CHUNK; }

extern "C" int ivit_adamw_chunked(long n_tensors, void* const* params, void* const* grads, void* const* exp_avg,
                                  void* const* exp_avg_sq, void* const* shadows, const long* sizes,
                                  const int* chunks, long n_chunks, float lr, double beta1, double beta2, float eps,
                                  float weight_decay, float bc1, float bc2_sqrt, const float* finite,
                                  const float* steps_in, float* steps_out, void* stream) {
  if (n_tensors <= 0 || n_chunks <= 0) return 0;
  IVIT_CHECK_ARG(chunks != nullptr && n_chunks < (1L << 31), "ivit_adamw_chunked: bad chunk table");
  IVIT_CHECK_ARG((steps_in == nullptr) == (steps_out == nullptr), "ivit_adamw_chunked: steps_in / steps_out pair");
  IVIT_CHECK_ARG(steps_in == nullptr || steps_in != steps_out, "ivit_adamw_chunked: steps_out aliases steps_in");
  IVIT_CHECK_ARG(((uintptr_t)chunks & 7) == 0, "ivit_adamw_chunked: misaligned chunk table");
  hipLaunchKernelGGL(adamw_chunk_kernel, dim3((unsigned)n_chunks), dim3(256), 0, ivit_stream(stream), params, grads,
                     exp_avg, exp_avg_sq, sizes, (const int2*)chunks, lr, (float)beta2, eps, weight_decay, bc1,
                     bc2_sqrt, shadows, finite, steps_in, steps_out, beta1, beta2, (float)(1.0 - beta1),
                     (float)(1.0 - beta2));
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_act_fwd(int act, const void* x, int x_dtype, void* y, int y_dtype, long n, void* stream) {
  IVIT_CHECK_ARG(act == IVIT_ACT_GELU || act == IVIT_ACT_RELU || act == IVIT_ACT_NONE, "ivit_act_fwd: bad act %d", act);
  if (n <= 0) return 0;
  hipLaunchKernelGGL(act_fwd_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, ivit_stream(stream), act, x, x_dtype, y,
                     y_dtype, n);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_act_bwd(int act, const void* dy, int dy_dtype, const void* x, int x_dtype, void* dx, int dx_dtype,
                            long n, void* stream) {
  IVIT_CHECK_ARG(act == IVIT_ACT_GELU || act == IVIT_ACT_RELU || act == IVIT_ACT_NONE, "ivit_act_bwd: bad act %d", act);
  if (n <= 0) return 0;
  hipLaunchKernelGGL(act_bwd_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, ivit_stream(stream), act, dy, dy_dtype, x,
                     x_dtype, dx, dx_dtype, n);
  IVIT_LAUNCH_CHECK();
  return 0;
}
