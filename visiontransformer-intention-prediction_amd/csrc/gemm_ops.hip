// C-ABI GEMM-shaped ops: linear fwd/dgrad/wgrad, patch embedding, NHWC convolutions.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include "gemm_engine.h"
#include "conv_panel.h"
#include "patch_embed.h"

using namespace ivit;

static thread_local char g_err[512];
static u64* g_stamp_buf = nullptr;
static long g_stamp_cap = 0;
u64* ivit_stamp_buffer(long blocks) { return g_stamp_buf && 8 * blocks <= g_stamp_cap ? g_stamp_buf : nullptr; }
extern "C" int ivit_debug_stamps(void* buf, long cap) {
  g_stamp_buf = (u64*)buf;
  g_stamp_cap = buf ? cap : 0;
  return 0;
}

void ivit_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
extern "C" const char* ivit_last_error(void) { return g_err; }

// Tuning knobs: defaults, then the IVIT_WIDE_EPI / IVIT_CONV_PANEL environment variables read ONCE
// when the library loads; ivit_set_knob changes them at run time (tests, A/B tools).
static int knob_env(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}
static int g_knobs[IVIT_KNOB_COUNT] = {knob_env("IVIT_WIDE_EPI", 0), knob_env("IVIT_CONV_PANEL", 1)};
int ivit_knob(int knob) { return knob >= 0 && knob < IVIT_KNOB_COUNT ? g_knobs[knob] : 0; }
extern "C" int ivit_set_knob(int knob, int value) {
  IVIT_CHECK_ARG(knob >= 0 && knob < IVIT_KNOB_COUNT, "ivit_set_knob: unknown knob %d", knob);
  IVIT_CHECK_ARG(knob != IVIT_KNOB_WIDE_EPI || (value >= 0 && value <= 2), "ivit_set_knob: wide epilogue form %d",
                 value);
  g_knobs[knob] = value;
  return 0;
}
extern "C" long ivit_get_knob(int knob) { return ivit_knob(knob); }
extern "C" const char* ivit_version(void) { return "ivit-hip 0.1 gfx950"; }

// ----------------------------------------------------------------------------- reductions
// Sum split-K slabs: out[i] (+)= sum_s slab[s][i]
__global__ void splitk_reduce_kernel(const float* __restrict__ slab, long n, int splits, float* __restrict__ out,
                                     int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += slab[(long)k * n + i];
  out[i] = accumulate ? out[i] + s : s;
}

// Two slab sets in one launch: i < n0 -> out0[i] (+)= sum_s slab0[s][i]; else out1[i - n0]
// (+)= sum_s slab1[s][i - n0] (weight gradient and its fused bias gradient).
__global__ void splitk_reduce2_kernel(const float* __restrict__ slab0, long n0, float* __restrict__ out0,
                                      const float* __restrict__ slab1, long n1, float* __restrict__ out1, int splits,
                                      int accumulate) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const float* sl = slab0;
  float* out = out0;
  long n = n0;
  if (i >= n0) {
    i -= n0;
    sl = slab1;
    out = out1;
    n = n1;
    if (i >= n1) return;
  }
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += sl[(long)k * n + i];
  out[i] = accumulate ? out[i] + s : s;
}

// The same with 16-B accesses (four consecutive outputs per thread, the splits' loads issued ahead
// of the in-order sums): n0, n1 multiples of 4, every pointer 16-B aligned. Same summation order.
__global__ void splitk_reduce2_v4_kernel(const float* __restrict__ slab0, long n0, float* __restrict__ out0,
                                         const float* __restrict__ slab1, long n1, float* __restrict__ out1,
                                         int splits, int accumulate) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const float* sl = slab0;
  float* out = out0;
  long n = n0;
  if (i >= n0) {
    i -= n0;
    sl = slab1;
    out = out1;
    n = n1;
    if (i >= n1) return;
  }
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int k = 0; k < splits; ++k) {
    const float4 v = *(const float4*)(sl + (long)k * n + i);
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  if (accumulate) {
    const float4 o = *(const float4*)(out + i);
    s.x = o.x + s.x;
    s.y = o.y + s.y;
    s.z = o.z + s.z;
    s.w = o.w + s.w;
  }
  *(float4*)(out + i) = s;
}

static int reduce_wgrad(hipStream_t st, const float* slab, long n, float* dW, const float* bslab, long nb, float* db,
                        int splits, int accumulate) {
  const long n1 = bslab ? nb : 0;
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (n % 4 == 0 && n1 % 4 == 0 && al16(slab) && al16(dW) && (!n1 || (al16(bslab) && al16(db))))
    hipLaunchKernelGGL(splitk_reduce2_v4_kernel, dim3(ivit_cdiv((n + n1) / 4, 256)), dim3(256), 0, st, slab, n, dW,
                       bslab, n1, db, splits, accumulate);
  else
    hipLaunchKernelGGL(splitk_reduce2_kernel, dim3(ivit_cdiv(n + n1, 256)), dim3(256), 0, st, slab, n, dW, bslab, n1,
                       db, splits, accumulate);
  IVIT_LAUNCH_CHECK();
  return 0;
}

// Column sums in two passes (deterministic): partial[chunk][col] then out[col].
constexpr int CS_ROWS = 256;
template <typename S>
__global__ void colsum_partial_kernel(const S* __restrict__ X, long ld, long rpb, long rstride, long roff, long M,
                                      long N, float* __restrict__ part) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;  // 4 row phases
  const long r0 = (long)blockIdx.y * CS_ROWS;
  float s = 0.f;
  if (col < N) {
    for (long r = r0 + ph; r < min(M, r0 + CS_ROWS); r += 4) {
      const long row = rpb ? (r / rpb) * rstride + roff + r % rpb : r;
      s += to_f32(X[row * ld + col]);
    }
  }
  __shared__ float red[4][64];
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph == 0 && col < N)
    part[(long)blockIdx.y * N + col] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

extern "C" long ivit_colsum_workspace(long M, long N) { return (long)ivit_cdiv(M, CS_ROWS) * N * 4; }

extern "C" int ivit_colsum(const void* X, int x_dtype, long ld, long rpb, long rstride, long roff, long M, long N,
                           float* out, int accumulate, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(work_bytes >= ivit_colsum_workspace(M, N), "ivit_colsum: workspace too small");
  if (M <= 0 || N <= 0) return 0;
  hipStream_t st = ivit_stream(stream);
  const int chunks = ivit_cdiv(M, CS_ROWS);
  dim3 g(ivit_cdiv(N, 64), chunks);
  if (x_dtype == IVIT_BF16)
    hipLaunchKernelGGL(colsum_partial_kernel<bf16>, g, dim3(256), 0, st, (const bf16*)X, ld, rpb, rstride, roff, M, N,
                       (float*)work);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<float>, g, dim3(256), 0, st, (const float*)X, ld, rpb, rstride, roff, M,
                       N, (float*)work);
  launch_colreduce(st, (const float*)work, chunks, N, (int)N, out, (int)N, nullptr, accumulate);
  IVIT_LAUNCH_CHECK();
  return 0;
}

// Split-K factor from a wave-quantisation cost model: with `slots` resident workgroups (two
// 128x128 workgroups per CU), time ~ rounds(tiles*s / slots) * (ktiles/s + c0), c0 ~ 4 K-tiles
// of per-workgroup prologue/epilogue. Measured on MI355X (tools/gemm_bench.py): one slightly
// over-full round costs more than a shorter, fuller one (e.g. 576 vs 288 workgroups).
static int splitk_choice(long tiles, long K, int bk) {
  static const long slots = [] {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus <= 0) cus = 256;
    return 2L * cus;
  }();
  const double kt = (double)((K + bk - 1) / bk);
  int best = 1;
  double best_cost = 1e30;
  for (int s = 1; s <= 128; ++s) {
    if (s > 1 && kt / s < 8.0) break;
    const double rounds = (double)((tiles * s + slots - 1) / slots);
    // + 4 K steps of fixed cost per workgroup: 1 / 12 / 32 measured alike on the bench (48.65-48.83 ms)
    const double cost = rounds * (kt / s + 4.0);
    if (cost < best_cost - 1e-9) { best_cost = cost; best = s; }
  }
  return best;
}

// ----------------------------------------------------------------------------- linear
template <typename S, typename O>
static int linear_fwd_t(const void* X, long ldx, const void* W, const float* bias, long M, long N, long K, int act,
                        void* Y, long ldy, void* Ypre, const float* resid, long ldr, const float* rs, long rps,
                        hipStream_t st, long qcols = 0, float qscale = 1.f) {
  const bool bf = sizeof(S) == 2;
  LdDense<S> la{(const S*)X, ldx, (int)M, (int)K, 0, 0, 0, {}};
  LdDense<S> lb{(const S*)W, K, (int)N, (int)K, 0, 0, 0, {}};
  if (resid) {
    EpiResid e{(float*)Y, ldy, resid, ldr, bias, rs, (int)(rps > 0 ? rps : 1)};
    return launch_gemm<true, true>(bf, la, lb, e, M, N, K, 1, 1, st);
  }
  EpiStore<O> e{(O*)Y, ldy, {}, bias, act, (O*)Ypre, 1.f, (int)qcols, qscale};
  return launch_gemm<true, true>(bf, la, lb, e, M, N, K, 1, 1, st);
}

extern "C" int ivit_linear_fwd_qs(int dtype, const void* X, long ldx, const void* W, const float* bias, long M, long N,
                                  long K, void* Y, long ldy, int y_dtype, long scale_cols, float col_scale,
                                  void* stream) {
  IVIT_CHECK_ARG(K % 8 == 0 && ldx % 8 == 0, "ivit_linear_fwd_qs: K and ldx must be multiples of 8");
  IVIT_CHECK_ARG(scale_cols >= 0 && scale_cols <= N && scale_cols % 8 == 0,
                 "ivit_linear_fwd_qs: scale_cols must be a multiple of 8 in [0, N] (got %ld)", scale_cols);
  hipStream_t st = ivit_stream(stream);
  int rc;
  if (dtype == IVIT_BF16)
    rc = y_dtype == IVIT_BF16 ? linear_fwd_t<bf16, bf16>(X, ldx, W, bias, M, N, K, IVIT_ACT_NONE, Y, ldy, nullptr,
                                                         nullptr, 0, nullptr, 0, st, scale_cols, col_scale)
                              : linear_fwd_t<bf16, float>(X, ldx, W, bias, M, N, K, IVIT_ACT_NONE, Y, ldy, nullptr,
                                                          nullptr, 0, nullptr, 0, st, scale_cols, col_scale);
  else
    rc = linear_fwd_t<float, float>(X, ldx, W, bias, M, N, K, IVIT_ACT_NONE, Y, ldy, nullptr, nullptr, 0, nullptr, 0,
                                    st, scale_cols, col_scale);
  if (rc) return rc;
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_linear_fwd(int dtype, const void* X, long ldx, const void* W, const float* bias, long M, long N,
                               long K, int act, void* Y, long ldy, int y_dtype, void* Ypre, const float* resid, long ldr,
                               const float* row_scale, long rows_per_scale, void* stream) {
  IVIT_CHECK_ARG(K % 8 == 0 && ldx % 8 == 0, "ivit_linear_fwd: K and ldx must be multiples of 8");
  IVIT_CHECK_ARG(!resid || y_dtype == IVIT_F32, "ivit_linear_fwd: residual output must be f32");
  hipStream_t st = ivit_stream(stream);
  int rc;
  if (dtype == IVIT_BF16)
    rc = y_dtype == IVIT_BF16
             ? linear_fwd_t<bf16, bf16>(X, ldx, W, bias, M, N, K, act, Y, ldy, Ypre, resid, ldr, row_scale, rows_per_scale, st)
             : linear_fwd_t<bf16, float>(X, ldx, W, bias, M, N, K, act, Y, ldy, Ypre, resid, ldr, row_scale, rows_per_scale, st);
  else
    rc = linear_fwd_t<float, float>(X, ldx, W, bias, M, N, K, act, Y, ldy, Ypre, resid, ldr, row_scale, rows_per_scale, st);
  if (rc) return rc;
  IVIT_LAUNCH_CHECK();
  return 0;
}

template <typename S, typename O>
static int linear_dgrad_t(const void* dY, long lddy, const void* W, long M, long N, long K, void* dX, long lddx,
                          const void* pre, long ldpre, hipStream_t st) {
  const bool bf = sizeof(S) == 2;
  LdDense<S> la{(const S*)dY, lddy, (int)M, (int)N, 0, 0, 0, {}};   // A[m][n], reduce over n
  LdDense<S> lb{(const S*)W, K, (int)N, (int)K, 0, 0, 0, {}};       // B[n][k] MN-contiguous
  if (pre) {
    EpiGeluGrad<O, S> e{(O*)dX, lddx, (const S*)pre, ldpre};
    return launch_gemm<true, false>(bf, la, lb, e, M, K, N, 1, 1, st);
  }
  EpiStore<O> e{(O*)dX, lddx, {}, nullptr, IVIT_ACT_NONE, nullptr, 1.f};
  return launch_gemm<true, false>(bf, la, lb, e, M, K, N, 1, 1, st);
}

extern "C" int ivit_linear_dgrad(int dtype, const void* dY, long lddy, const void* W, long M, long N, long K, void* dX,
                                 long lddx, int dx_dtype, const void* gelu_pre, long ldpre, void* stream) {
  IVIT_CHECK_ARG(N % 8 == 0 && K % 8 == 0 && lddy % 8 == 0, "ivit_linear_dgrad: N, K, lddy must be multiples of 8");
  hipStream_t st = ivit_stream(stream);
  int rc;
  if (dtype == IVIT_BF16)
    rc = dx_dtype == IVIT_BF16 ? linear_dgrad_t<bf16, bf16>(dY, lddy, W, M, N, K, dX, lddx, gelu_pre, ldpre, st)
                               : linear_dgrad_t<bf16, float>(dY, lddy, W, M, N, K, dX, lddx, gelu_pre, ldpre, st);
  else
    rc = linear_dgrad_t<float, float>(dY, lddy, W, M, N, K, dX, lddx, gelu_pre, ldpre, st);
  if (rc) return rc;
  IVIT_LAUNCH_CHECK();
  return 0;
}

static long wgrad_splits(long Mo, long No, long Kr, bool bf) {
  const long tiles = (long)ivit_cdiv(Mo, GBM) * ivit_cdiv(No, GBN);
  return splitk_choice(tiles, Kr, bf ? GBK16 : GBK32);
}

extern "C" long ivit_linear_wgrad_workspace(long M, long N, long K) {
  const long s = wgrad_splits(N, K, M, true) > wgrad_splits(N, K, M, false) ? wgrad_splits(N, K, M, true)
                                                                             : wgrad_splits(N, K, M, false);
  const long cw = ivit_colsum_workspace(M, N);
  return s * N * K * 4 + (s * N * 4 > cw ? s * N * 4 : cw);
}

template <typename S>
static int linear_wgrad_t(const void* dY, long lddy, const void* X, long ldx, long M, long N, long K, float* slab,
                          float* bslab, int splits, hipStream_t st) {
  const bool bf = sizeof(S) == 2;
  LdDense<S> la{(const S*)dY, lddy, (int)M, (int)N, 0, 0, 0, {}};  // A[n][m] (MN-contig), rows = m
  LdDense<S> lb{(const S*)X, ldx, (int)M, (int)K, 0, 0, 0, {}};    // B[m][k] (MN-contig)
  EpiSlab e{slab, N, K, bslab};
  return launch_gemm<false, false>(bf, la, lb, e, N, K, M, 1, splits, st);
}

extern "C" int ivit_linear_wgrad(int dtype, const void* dY, long lddy, const void* X, long ldx, long M, long N,
                                 long K, float* dW, float* dbias, int accumulate, void* work, long work_bytes,
                                 void* stream) {
  IVIT_CHECK_ARG(N % 8 == 0 && K % 8 == 0 && lddy % 8 == 0 && ldx % 8 == 0,
                 "ivit_linear_wgrad: N, K, lddy, ldx must be multiples of 8");
  IVIT_CHECK_ARG(work_bytes >= ivit_linear_wgrad_workspace(M, N, K), "ivit_linear_wgrad: workspace too small");
  hipStream_t st = ivit_stream(stream);
  const bool bf = dtype == IVIT_BF16;
  const int splits = (int)wgrad_splits(N, K, M, bf);
  float* slab = (float*)work;
  float* bslab = (bf && dbias) ? slab + (long)splits * N * K : nullptr;  // bias fused into the bf16 GEMM
  int rc = bf ? linear_wgrad_t<bf16>(dY, lddy, X, ldx, M, N, K, slab, bslab, splits, st)
              : linear_wgrad_t<float>(dY, lddy, X, ldx, M, N, K, slab, nullptr, splits, st);
  if (rc) return rc;
  rc = reduce_wgrad(st, slab, N * K, dW, bslab, N, dbias, splits, accumulate);
  if (rc) return rc;
  if (dbias && !bslab) {
    char* cw = (char*)work + (long)splits * N * K * 4;
    rc = ivit_colsum(dY, dtype, lddy, 0, 0, 0, M, N, dbias, accumulate, cw, ivit_colsum_workspace(M, N), stream);
    if (rc) return rc;
  }
  return 0;
}

// ----------------------------------------------------------------------------- patch embedding
__global__ void cls_rows_kernel(float* out, long B, long Ntok, long D, const float* cls, const float* pos) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * D) return;
  const long b = i / D, d = i - b * D;
  out[b * Ntok * D + d] = cls[d] + pos[d];
}

template <typename S>
static int patch_fwd_t(const float* img, long B, long C, long H, long W, const void* Wt, const float* bias,
                       const float* pos, long D, float* out, hipStream_t st) {
  const bool bf = sizeof(S) == 2;
  const int Wp = (int)(W / 8), Np = (int)((H / 8) * (W / 8));
  LdPatch<float> la{img, (int)B, (int)C, (int)H, (int)W, Wp, Np, (int)(B * Np), (int)(C * 64)};
  LdDense<S> lb{(const S*)Wt, C * 64, (int)D, (int)(C * 64), 0, 0, 0, {}};
  EpiPatch e{out, Np, (int)D, bias, pos};
  return launch_gemm<true, true>(bf, la, lb, e, (int)(B * Np), (int)D, (int)(C * 64), 1, 1, st);
}

extern "C" int ivit_patch_embed_fwd(int dtype, const float* img, long B, long C, long H, long W, const void* Wt,
                                    const float* bias, const float* pos, const float* cls, long D, float* out,
                                    void* stream) {
  IVIT_CHECK_ARG(H % 8 == 0 && W % 8 == 0, "ivit_patch_embed_fwd: H, W must be multiples of the patch (8)");
  hipStream_t st = ivit_stream(stream);
  int rc = dtype == IVIT_BF16 ? patch_fwd_t<bf16>(img, B, C, H, W, Wt, bias, pos, D, out, st)
                              : patch_fwd_t<float>(img, B, C, H, W, Wt, bias, pos, D, out, st);
  if (rc) return rc;
  const long Ntok = (H / 8) * (W / 8) + 1;
  hipLaunchKernelGGL(cls_rows_kernel, dim3(ivit_cdiv(B * D, 256)), dim3(256), 0, st, out, B, Ntok, D, cls, pos);
  IVIT_LAUNCH_CHECK();
  return 0;
}

// dpos[t][d] (+)= sum_b dtok[b][t][d]; dcls = dpos[0] (before accumulation semantics: (+)=)
template <typename S>
__global__ void pos_grad_kernel(const S* __restrict__ dtok, long B, long Ntok, long D, float* dpos, float* dcls,
                                int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Ntok * D) return;
  float s = 0.f;
  for (long b = 0; b < B; ++b) s += to_f32(dtok[b * Ntok * D + i]);
  dpos[i] = accumulate ? dpos[i] + s : s;
  if (i < D && dcls) dcls[i] = accumulate ? dcls[i] + s : s;
}

// dpos[t][d] (+)= sum_b dtok[b][t][d] (dcls = row 0) and dbias[d] (+)= sum over t >= 1 of those sums,
// in ONE pass over dtok: 8 columns per thread (16-B loads), 4 row phases, RB rows per block; the
// block's partial bias row goes to `part` (reduced by colreduce_kernel). Replaces pos_grad_kernel's
// 2-B loads plus a separate column-sum pass over the same token gradient.
template <typename S>
__global__ __launch_bounds__(1024) void pos_bias_grad_kernel(const S* __restrict__ dtok, int B, int Ntok, int D,
                                                            int RB, int NPH, float* dpos, float* dcls, float* part,
                                                            int accumulate) {
  __shared__ float red[16 * 512];
  const int nc = D / 8, cc = threadIdx.x % nc, ph = threadIdx.x / nc;
  const int t0 = blockIdx.x * RB, t1 = min(Ntok, t0 + RB);
  float ps[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ps[j] = 0.f;
  for (int t = t0 + ph; t < t1; t += NPH) {
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = 0.f;
    int b = 0;
    for (; b + 4 <= B; b += 4) {  // four images' rows in flight, summed in image order
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) load8f(dtok + ((long)(b + u) * Ntok + t) * D + 8 * cc, v[u], 8);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += v[u][j];
    }
    for (; b < B; ++b) {
      const S* q = dtok + ((long)b * Ntok + t) * D + 8 * cc;
      float v[8];
      load8f(q, v, 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += v[j];
    }
    float* o = dpos + (long)t * D + 8 * cc;
    float x[8];
    if (accumulate) {
      load8f(o, x, 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] += s[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = s[j];
    }
    store8(o, x, 8);
    if (t == 0) {
      if (dcls) {
        float* oc = dcls + 8 * cc;
        float y[8];
        if (accumulate) {
          load8f(oc, y, 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) y[j] += s[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) y[j] = s[j];
        }
        store8(oc, y, 8);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) ps[j] += s[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[ph * D + 8 * cc + j] = ps[j];
  __syncthreads();
  if (ph == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 8 * cc + j;
      float v = red[c];
      for (int q = 1; q < NPH; ++q) v += red[q * D + c];
      part[(long)blockIdx.x * D + c] = v;
    }
  }
}

// pos / cls / bias gradients of the patch embedding from the token gradient (see pos_bias_grad_kernel);
// falls back to pos_grad_kernel + ivit_colsum for widths it does not take.
static int patch_pos_bias_grad(int dtype, const void* dtok, long B, long Np, long D, float* dbias, float* dpos,
                               float* dcls, int accumulate, void* cw, long cw_bytes, void* stream) {
  hipStream_t st = ivit_stream(stream);
  const long Ntok = Np + 1;
  const long nb0 = ivit_cdiv(B * Np, CS_ROWS);  // the column-sum workspace's partial rows
  int RB = (int)((Ntok + nb0 - 1) / nb0);
  RB = ((RB < 32 ? 32 : RB) + 3) / 4 * 4;
  const int nb = ivit_cdiv(Ntok, RB);
  const bool al = ((uintptr_t)dtok & 15) == 0 && ((uintptr_t)dpos & 15) == 0 && (!dcls || ((uintptr_t)dcls & 15) == 0);
  if (D % 8 == 0 && D <= 512 && al && (long)nb * D * 4 <= cw_bytes && dbias) {
    // row phases per block: as many as fit 1024 threads, at most 16 (the LDS partial rows)
    int nph = 1024 / (int)(D / 8);
    if (nph > 16) nph = 16;
    if (dtype == IVIT_BF16)
      hipLaunchKernelGGL(pos_bias_grad_kernel<bf16>, dim3(nb), dim3(nph * D / 8), 0, st, (const bf16*)dtok, (int)B,
                         (int)Ntok, (int)D, RB, nph, dpos, dcls, (float*)cw, accumulate);
    else
      hipLaunchKernelGGL(pos_bias_grad_kernel<float>, dim3(nb), dim3(nph * D / 8), 0, st, (const float*)dtok, (int)B,
                         (int)Ntok, (int)D, RB, nph, dpos, dcls, (float*)cw, accumulate);
    IVIT_LAUNCH_CHECK();
    launch_colreduce(st, (const float*)cw, nb, D, (int)D, dbias, (int)D, nullptr, accumulate);
    IVIT_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == IVIT_BF16)
    hipLaunchKernelGGL(pos_grad_kernel<bf16>, dim3(ivit_cdiv(Ntok * D, 256)), dim3(256), 0, st, (const bf16*)dtok, B,
                       Ntok, D, dpos, dcls, accumulate);
  else
    hipLaunchKernelGGL(pos_grad_kernel<float>, dim3(ivit_cdiv(Ntok * D, 256)), dim3(256), 0, st, (const float*)dtok,
                       B, Ntok, D, dpos, dcls, accumulate);
  IVIT_LAUNCH_CHECK();
  return ivit_colsum(dtok, dtype, D, Np, Ntok, 1, B * Np, D, dbias, accumulate, cw, ivit_colsum_workspace(B * Np, D),
                     stream);
}

extern "C" long ivit_patch_embed_wgrad_workspace(long B, long C, long H, long W, long D) {
  const long Np = (H / 8) * (W / 8);
  long s = wgrad_splits(D, C * 64, B * Np, false);
  const long s2 = wgrad_splits(D, C * 64, B * Np, true);
  if (s2 > s) s = s2;
  long main = s * D * C * 64 * 4;
  if (patch_wgrad_raster_ok(B, C, H, W, D) && patch_wgrad_raster_workspace2(B, C, H, W, D) > main)
    main = patch_wgrad_raster_workspace2(B, C, H, W, D);
  return main + ivit_colsum_workspace(B * Np, D);
}

template <typename S>
static int patch_wgrad_t(const void* dtok, const float* img, long B, long C, long H, long W, long D, float* slab,
                         int splits, hipStream_t st) {
  const bool bf = sizeof(S) == 2;
  const int Wp = (int)(W / 8), Np = (int)((H / 8) * (W / 8));
  const long Ntok = Np + 1;
  LdDense<S> la{(const S*)dtok, D, (int)(B * Np), (int)D, Np, Ntok, 1, {}};  // A[d][m] rows m -> token rows
  LdPatch<float> lb{img, (int)B, (int)C, (int)H, (int)W, Wp, Np, (int)(B * Np), (int)(C * 64)};
  EpiSlab e{slab, D, C * 64};
  return launch_gemm<false, false>(bf, la, lb, e, (int)D, (int)(C * 64), (int)(B * Np), 1, splits, st);
}

extern "C" int ivit_patch_embed_wgrad(int dtype, const void* dtok, const float* img, long B, long C, long H, long W,
                                      long D, float* dW, float* dbias, float* dpos, float* dcls, int accumulate,
                                      void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(B > 0 && C > 0 && H >= 8 && W >= 8 && D > 0, "patch wgrad: bad sizes (B %ld, C %ld, H %ld, W %ld, D %ld)",
                 B, C, H, W, D);
  IVIT_CHECK_ARG(work_bytes >= ivit_patch_embed_wgrad_workspace(B, C, H, W, D), "patch wgrad: workspace too small");
  hipStream_t st = ivit_stream(stream);
  const bool bf = dtype == IVIT_BF16;
  const long Np = (H / 8) * (W / 8);
  const long n = D * C * 64;
  const int splits = (int)wgrad_splits(D, C * 64, B * Np, bf);
  const bool raster = bf && patch_wgrad_raster_ok(B, C, H, W, D);  // raster read once (patch_embed.hip)
  const long cw_off = raster ? patch_wgrad_raster_workspace2(B, C, H, W, D) : (long)splits * n * 4;  // after the slab
  // the pos / cls / bias gradients first: they are short, and after the weight gradient (whose
  // persistent workgroups hold every CU's LDS) they waited for it and ran at the step's tail
  // (54.6 us for the LiDAR stream in profiles/r05_j_bench_kernel_stats.csv's trace)
  char* cw = (char*)work + cw_off;
  int rc = patch_pos_bias_grad(dtype, dtok, B, Np, D, dbias, dpos, dcls, accumulate, cw,
                               ivit_colsum_workspace(B * Np, D), stream);
  if (rc) return rc;
  if (raster) {
    rc = patch_wgrad_raster((const bf16*)dtok, img, B, C, H, W, D, dW, accumulate, work, st);
    if (rc) return rc;
    IVIT_LAUNCH_CHECK();
  } else {
    float* slab = (float*)work;
    rc = bf ? patch_wgrad_t<bf16>(dtok, img, B, C, H, W, D, slab, splits, st)
            : patch_wgrad_t<float>(dtok, img, B, C, H, W, D, slab, splits, st);
    if (rc) return rc;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, slab, n, splits, dW,
                       accumulate);
    IVIT_LAUNCH_CHECK();
  }
  return 0;
}

// bf16 patch matrix. One workgroup per (b, c, gy) = 8 consecutive raster rows (8*W floats,
// contiguous in NCHW); unit u = gx*8 + ky reads one 32-B run (kx = 0..7) and writes it as one
// 16-B bf16 chunk, so 8 consecutive lanes fill the full 128-B row segment of patch (b, gy, gx),
// channel c: coalesced reads, whole-line writes.
__global__ __launch_bounds__(256) void patch_im2col_kernel(const float* __restrict__ img, int C, int H, int W,
                                                           bf16* __restrict__ cols) {
  const int Hp = H / 8, Wp = W / 8;
  const long blk = blockIdx.x;  // (b * C + c) * Hp + gy
  const int gy = (int)(blk % Hp);
  const long bc = blk / Hp;
  const int c = (int)(bc % C);
  const long b = bc / C;
  const float* src = img + (bc * H + (long)gy * 8) * W;
  const long K = (long)C * 64;
  bf16* dst = cols + (b * Hp * Wp + (long)gy * Wp) * K + c * 64;
  for (int u = threadIdx.x; u < Wp * 8; u += 256) {
    const int gx = u >> 3, ky = u & 7;
    const float* p = src + (long)ky * W + gx * 8;
    const float4 a = *(const float4*)p, q = *(const float4*)(p + 4);
    *(uint4*)(dst + (long)gx * K + ky * 8) = f32x8_to_bf16x8(a, q);
  }
}

extern "C" int ivit_patch_im2col(const float* img, long B, long C, long H, long W, void* cols, void* stream) {
  IVIT_CHECK_ARG(H % 8 == 0 && W % 8 == 0, "ivit_patch_im2col: H, W must be multiples of the patch (8)");
  if (B * C * H * W == 0) return 0;
  hipStream_t st = ivit_stream(stream);
  hipLaunchKernelGGL(patch_im2col_kernel, dim3((unsigned)(B * C * (H / 8))), dim3(256), 0, st, img, (int)C, (int)H,
                     (int)W, (bf16*)cols);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_patch_embed_fwd_cols(const void* cols, long B, long C, long H, long W, const void* Wt,
                                         const float* bias, const float* pos, const float* cls, long D, float* out,
                                         void* stream) {
  IVIT_CHECK_ARG(H % 8 == 0 && W % 8 == 0, "ivit_patch_embed_fwd_cols: H, W must be multiples of the patch (8)");
  hipStream_t st = ivit_stream(stream);
  const int Np = (int)((H / 8) * (W / 8));
  const long K = C * 64;
  LdDense<bf16> la{(const bf16*)cols, K, (int)(B * Np), (int)K, 0, 0, 0, {}};
  LdDense<bf16> lb{(const bf16*)Wt, K, (int)D, (int)K, 0, 0, 0, {}};
  EpiPatch e{out, Np, (int)D, bias, pos};
  int rc = launch_gemm<true, true>(true, la, lb, e, (int)(B * Np), (int)D, (int)K, 1, 1, st);
  if (rc) return rc;
  const long Ntok = Np + 1;
  hipLaunchKernelGGL(cls_rows_kernel, dim3(ivit_cdiv(B * D, 256)), dim3(256), 0, st, out, B, Ntok, D, cls, pos);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_patch_embed_wgrad_cols(const void* dtok, const void* cols, long B, long C, long H, long W, long D,
                                           float* dW, float* dbias, float* dpos, float* dcls, int accumulate,
                                           void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(work_bytes >= ivit_patch_embed_wgrad_workspace(B, C, H, W, D), "patch wgrad: workspace too small");
  hipStream_t st = ivit_stream(stream);
  const long Np = (H / 8) * (W / 8), Ntok = Np + 1, K = C * 64;
  const int splits = (int)wgrad_splits(D, K, B * Np, true);
  float* slab = (float*)work;
  LdDense<bf16> la{(const bf16*)dtok, D, (int)(B * Np), (int)D, (int)Np, Ntok, 1, {}};  // A[d][m], token rows
  LdDense<bf16> lb{(const bf16*)cols, K, (int)(B * Np), (int)K, 0, 0, 0, {}};          // B[m][k]
  EpiSlab e{slab, D, K};
  int rc = launch_gemm<false, false>(true, la, lb, e, (int)D, (int)K, (int)(B * Np), 1, splits, st);
  if (rc) return rc;
  const long n = D * K;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, slab, n, splits, dW, accumulate);
  hipLaunchKernelGGL(pos_grad_kernel<bf16>, dim3(ivit_cdiv(Ntok * D, 256)), dim3(256), 0, st, (const bf16*)dtok, B,
                     Ntok, D, dpos, dcls, accumulate);
  IVIT_LAUNCH_CHECK();
  char* cw = (char*)work + (long)splits * n * 4;
  return ivit_colsum(dtok, IVIT_BF16, D, Np, Ntok, 1, B * Np, D, dbias, accumulate, cw,
                     ivit_colsum_workspace(B * Np, D), stream);
}

// ----------------------------------------------------------------------------- NHWC convolution
template <typename S, typename O>
static int conv_fwd_t(const void* X, long B, long H, long W, long Cin, const void* Wp, const float* bias, long Cout,
                      long ks, void* Y, long ldy, hipStream_t st) {
  const bool bf = sizeof(S) == 2;
  const int M = (int)(B * H * W), Kc = (int)(ks * ks * Cin);
  if constexpr (sizeof(S) == 2) {  // 288 x 256 panel tiles (conv_panel.hip) where the shape allows
    if (conv_panel_enabled() && conv_panel_ok(M, Cout, Cin, Cin, ks) && ldy % 4 == 0)
      return conv_panel_launch((const bf16*)X, Cin, (int)B, (int)H, (int)W, (int)Cin, (int)ks, (const bf16*)Wp,
                               (int)Cout, bias, Y, ldy, sizeof(O) == 2, st);
  }
  LdConv<S> la{(const S*)X, (int)H, (int)W, (int)Cin, (int)ks, M, Kc, Cin};
  LdDense<S> lb{(const S*)Wp, Kc, (int)Cout, Kc, 0, 0, 0, {}};
  EpiStore<O> e{(O*)Y, ldy, {}, bias, IVIT_ACT_NONE, nullptr, 1.f};
  return launch_gemm<true, true>(bf, la, lb, e, M, (int)Cout, Kc, 1, 1, st);
}

extern "C" int ivit_conv_fwd(int dtype, const void* X, long B, long H, long W, long Cin, const void* Wp,
                             const float* bias, long Cout, long ks, void* Y, long ldy, int y_dtype, void* stream) {
  IVIT_CHECK_ARG(Cin % 8 == 0 && (ks == 1 || ks == 3 || ks == 5), "ivit_conv_fwd: Cin %% 8 and ks in {1,3,5}");
  hipStream_t st = ivit_stream(stream);
  int rc;
  if (dtype == IVIT_BF16)
    rc = y_dtype == IVIT_BF16 ? conv_fwd_t<bf16, bf16>(X, B, H, W, Cin, Wp, bias, Cout, ks, Y, ldy, st)
                              : conv_fwd_t<bf16, float>(X, B, H, W, Cin, Wp, bias, Cout, ks, Y, ldy, st);
  else
    rc = conv_fwd_t<float, float>(X, B, H, W, Cin, Wp, bias, Cout, ks, Y, ldy, st);
  if (rc) return rc;
  IVIT_LAUNCH_CHECK();
  return 0;
}

template <typename S, typename O>
static int conv_dgrad_t(const void* dY, long lddy, long B, long H, long W, long Cout, const void* Wp, long Cin,
                        long ks, void* dX, hipStream_t st) {
  const bool bf = sizeof(S) == 2;
  const int M = (int)(B * H * W), Kc = (int)(ks * ks * Cout);
  LdConv<S> la{(const S*)dY, (int)H, (int)W, (int)Cout, (int)ks, M, Kc, lddy};
  LdConvWFlip<S> lb{(const S*)Wp, (int)Cout, (int)Cin, (int)ks, Kc, (int)Cin};
  EpiStore<O> e{(O*)dX, Cin, {}, nullptr, IVIT_ACT_NONE, nullptr, 1.f};
  return launch_gemm<true, false>(bf, la, lb, e, M, (int)Cin, Kc, 1, 1, st);
}

extern "C" int ivit_conv_dgrad(int dtype, const void* dY, long lddy, long B, long H, long W, long Cout, const void* Wp,
                               long Cin, long ks, void* dX, int dx_dtype, void* stream) {
  IVIT_CHECK_ARG(Cout % 8 == 0 && Cin % 8 == 0 && lddy % 8 == 0, "ivit_conv_dgrad: channel counts %% 8");
  hipStream_t st = ivit_stream(stream);
  int rc;
  if (dtype == IVIT_BF16)
    rc = dx_dtype == IVIT_BF16 ? conv_dgrad_t<bf16, bf16>(dY, lddy, B, H, W, Cout, Wp, Cin, ks, dX, st)
                               : conv_dgrad_t<bf16, float>(dY, lddy, B, H, W, Cout, Wp, Cin, ks, dX, st);
  else
    rc = conv_dgrad_t<float, float>(dY, lddy, B, H, W, Cout, Wp, Cin, ks, dX, st);
  if (rc) return rc;
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" long ivit_conv_wgrad_workspace(long B, long H, long W, long Cin, long Cout, long ks) {
  if (B <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || ks <= 0) return 0;
  const long M = B * H * W, Kc = ks * ks * Cin;
  long s = wgrad_splits(Cout, Kc, M, false);
  const long s2 = wgrad_splits(Cout, Kc, M, true);
  if (s2 > s) s = s2;
  const long s3 = conv_wgrad_panel_splits(M, Cout, Kc);
  if (s3 > s) s = s3;
  const long cw = ivit_colsum_workspace(M, Cout);
  return s * Cout * Kc * 4 + (s * Cout * 4 > cw ? s * Cout * 4 : cw);
}

template <typename S>
static int conv_wgrad_t(const void* dY, long lddy, const void* X, long B, long H, long W, long Cin, long Cout,
                        long ks, float* slab, float* bslab, int splits, hipStream_t st) {
  const bool bf = sizeof(S) == 2;
  const int M = (int)(B * H * W), Kc = (int)(ks * ks * Cin);
  LdDense<S> la{(const S*)dY, lddy, M, (int)Cout, 0, 0, 0, {}};                 // A[co][m]
  LdConv<S> lb{(const S*)X, (int)H, (int)W, (int)Cin, (int)ks, M, Kc, Cin};    // B[m][kk]
  EpiSlab e{slab, Cout, Kc, bslab};
  return launch_gemm<false, false>(bf, la, lb, e, (int)Cout, Kc, M, 1, splits, st);
}

extern "C" int ivit_conv_wgrad(int dtype, const void* dY, long lddy, const void* X, long B, long H, long W, long Cin,
                               long Cout, long ks, float* dWp, float* dbias, int accumulate, void* work,
                               long work_bytes, void* stream) {
  IVIT_CHECK_ARG(B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && ks > 0 && lddy >= Cout,
                 "ivit_conv_wgrad: bad sizes (B %ld, H %ld, W %ld, Cin %ld, Cout %ld, k %ld, lddy %ld)", B, H, W, Cin,
                 Cout, ks, lddy);
  IVIT_CHECK_ARG(Cout % 8 == 0 && Cin % 8 == 0 && lddy % 8 == 0, "ivit_conv_wgrad: channel counts %% 8");
  IVIT_CHECK_ARG(work_bytes >= ivit_conv_wgrad_workspace(B, H, W, Cin, Cout, ks), "conv wgrad: workspace too small");
  hipStream_t st = ivit_stream(stream);
  const bool bf = dtype == IVIT_BF16;
  const long M = B * H * W, Kc = ks * ks * Cin;
  const bool panel = bf && conv_panel_enabled() && conv_wgrad_panel_ok(M, Cout, Cin, ks, lddy);
  const int splits = panel ? conv_wgrad_panel_splits(M, Cout, Kc) : (int)wgrad_splits(Cout, Kc, M, bf);
  float* slab = (float*)work;
  const long n = Cout * Kc;
  float* bslab = (bf && dbias && !panel) ? slab + (long)splits * n : nullptr;
  int rc = panel ? conv_wgrad_panel_launch((const bf16*)dY, lddy, (const bf16*)X, (int)B, (int)H, (int)W, (int)Cin,
                                           (int)Cout, (int)ks, slab, splits, st)
           : bf  ? conv_wgrad_t<bf16>(dY, lddy, X, B, H, W, Cin, Cout, ks, slab, bslab, splits, st)
                 : conv_wgrad_t<float>(dY, lddy, X, B, H, W, Cin, Cout, ks, slab, nullptr, splits, st);
  if (rc) return rc;
  rc = reduce_wgrad(st, slab, n, dWp, bslab, Cout, dbias, splits, accumulate);
  if (rc) return rc;
  if (dbias && !bslab) {
    char* cw = (char*)work + (long)splits * n * 4;
    return ivit_colsum(dY, dtype, lddy, 0, 0, 0, M, Cout, dbias, accumulate, cw, ivit_colsum_workspace(M, Cout),
                       stream);
  }
  return 0;
}

template <typename O>
__global__ void pack_conv_kernel(const float* __restrict__ w, long Cout, long Cin, long ks, long Cpad, O* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = Cpad * ks * ks * Cin;
  if (i >= n) return;
  const long ci = i % Cin, t = i / Cin, kx = t % ks, t2 = t / ks, ky = t2 % ks, co = t2 / ks;
  const float v = co < Cout ? w[((co * Cin + ci) * ks + ky) * ks + kx] : 0.f;
  out[i] = from_f32<O>(v);
}

extern "C" int ivit_pack_conv_weight(int dtype, const float* w, long Cout, long Cin, long ks, long Cout_pad, void* out,
                                     void* stream) {
  hipStream_t st = ivit_stream(stream);
  const long n = Cout_pad * ks * ks * Cin;
  if (dtype == IVIT_BF16)
    hipLaunchKernelGGL(pack_conv_kernel<bf16>, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, w, Cout, Cin, ks, Cout_pad,
                       (bf16*)out);
  else
    hipLaunchKernelGGL(pack_conv_kernel<float>, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, w, Cout, Cin, ks, Cout_pad,
                       (float*)out);
  IVIT_LAUNCH_CHECK();
  return 0;
}

__global__ void unpack_conv_grad_kernel(const float* __restrict__ gp, long Cout, long Cin, long ks, float* out,
                                        int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = Cout * Cin * ks * ks;
  if (i >= n) return;
  const long kx = i % ks, t = i / ks, ky = t % ks, t2 = t / ks, ci = t2 % Cin, co = t2 / Cin;
  const float v = gp[((co * ks + ky) * ks + kx) * Cin + ci];
  out[i] = accumulate ? out[i] + v : v;
}

extern "C" int ivit_unpack_conv_grad(const float* gp, long Cout, long Cin, long ks, float* out, int accumulate,
                                     void* stream) {
  hipStream_t st = ivit_stream(stream);
  const long n = Cout * Cin * ks * ks;
  hipLaunchKernelGGL(unpack_conv_grad_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, gp, Cout, Cin, ks, out,
                     accumulate);
  IVIT_LAUNCH_CHECK();
  return 0;
}
