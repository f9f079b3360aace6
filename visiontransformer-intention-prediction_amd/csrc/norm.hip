// LayerNorm (timm Block norm1/norm2/norm, eps 1e-6; adapter LN eps 1e-5, model_vit.py:82-83)
// and BatchNorm2d in training mode (BasicBlock bn1/bn2/downsample, model_vit.py:24-31) on
// NHWC maps. All statistics in f32; column reductions are two-pass and deterministic.
#include "ivit_common.h"

namespace {

IVIT_DEV float ldv(const void* p, int dt, long i) {
  return dt == IVIT_BF16 ? bf2f(((const bf16*)p)[i]) : ((const float*)p)[i];
}
IVIT_DEV void stv(void* p, int dt, long i, float v) {
  if (dt == IVIT_BF16) ((bf16*)p)[i] = f2bf(v);
  else ((float*)p)[i] = v;
}
IVIT_DEV long rowmap(long r, long rpb, long rstride, long roff) {
  return rpb ? (r / rpb) * rstride + roff + r % rpb : r;
}

constexpr int LN_MAXV = 8;  // D <= 512

// one wave per row, D % 64 == 0
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ X, long ldx, long rpb, long rstride,
                                                     long roff, long M, int D, const float* __restrict__ g,
                                                     const float* __restrict__ bta, float eps, void* Y, long ldy,
                                                     int ydt, float* __restrict__ mean, float* __restrict__ rstd) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* x = X + rowmap(row, rpb, rstride, roff) * ldx;
  const int nv = D >> 6;
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i)
    if (i < nv) { v[i] = x[lane + 64 * i]; s += v[i]; }
  const float mu = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i)
    if (i < nv) { const float d = v[i] - mu; q += d * d; }
  const float var = wave_sum(q) / (float)D;
  const float rs = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i)
    if (i < nv) {
      const int c = lane + 64 * i;
      stv(Y, ydt, row * ldy + c, (v[i] - mu) * rs * g[c] + bta[c]);
    }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

constexpr int LNB_ROWS = 8;  // rows per wave; a block (4 waves) covers 32 rows

__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ X, long ldx, long rpb, long rstride,
                                                     long roff, long M, int D, const float* __restrict__ g,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const void* dY, long lddy, int dydt, const float* dres,
                                                     float* dX, long lddx, void* dXs, int dxsdt,
                                                     const float* __restrict__ rscale, long rps,
                                                     float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nv = D >> 6;
  float pg[LN_MAXV], pb[LN_MAXV];
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  const long r0 = ((long)blockIdx.x * 4 + wv) * LNB_ROWS;
  for (long row = r0; row < min(M, r0 + LNB_ROWS); ++row) {
    const float* x = X + rowmap(row, rpb, rstride, roff) * ldx;
    const float mu = mean[row], rs = rstd[row];
    float xh[LN_MAXV], gy[LN_MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i)
      if (i < nv) {
        const int c = lane + 64 * i;
        const float dy = ldv(dY, dydt, row * lddy + c);
        xh[i] = (x[c] - mu) * rs;
        gy[i] = dy * g[c];
        s1 += gy[i];
        s2 += gy[i] * xh[i];
        pg[i] += dy * xh[i];
        pb[i] += dy;
      }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
    const float sc = rscale ? rscale[row / rps] : 1.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i)
      if (i < nv) {
        const int c = lane + 64 * i;
        float d = rs * (gy[i] - s1 - xh[i] * s2);
        const long xr = rowmap(row, rpb, rstride, roff) * lddx + c;
        if (dres) d += dres[xr];
        dX[xr] = d;
        if (dXs) stv(dXs, dxsdt, row * D + c, d * sc);
      }
  }
  __shared__ float red[2][4][512];
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i)
    if (i < nv) { red[0][wv][lane + 64 * i] = pg[i]; red[1][wv][lane + 64 * i] = pb[i]; }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    part[((long)blockIdx.x * 2 + 0) * D + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    part[((long)blockIdx.x * 2 + 1) * D + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}


// ---------------------------------------------------------------- BatchNorm (NHWC [M, C])
constexpr int BN_ROWS = 128;

// mode 0: partial column sums of x; mode 1: sums of (x - mean)^2; mode 2: bwd sums of dz, dz*xhat
__global__ __launch_bounds__(256) void bn_partial_kernel(int mode, const void* X, int xdt, const void* Y, int ydt,
                                                         const void* dY, int dydt, long M, int C,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd, int relu,
                                                         float* __restrict__ part) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.y * BN_ROWS;
  float s = 0.f, t = 0.f;
  if (col < C) {
    const float mu = mode ? mean[col] : 0.f;
    const float is = mode == 2 ? invstd[col] : 0.f;
    for (long r = r0 + ph; r < min(M, r0 + BN_ROWS); r += 4) {
      const long i = r * C + col;
      const float x = ldv(X, xdt, i);
      if (mode == 0) s += x;
      else if (mode == 1) { const float d = x - mu; s += d * d; }
      else {
        float dz = ldv(dY, dydt, i);
        if (relu && ldv(Y, ydt, i) <= 0.f) dz = 0.f;
        s += dz;
        t += dz * (x - mu) * is;
      }
    }
  }
  __shared__ float red[2][4][64];
  red[0][ph][threadIdx.x & 63] = s;
  red[1][ph][threadIdx.x & 63] = t;
  __syncthreads();
  if (ph == 0 && col < C) {
    const int k = threadIdx.x;
    part[((long)blockIdx.y * 2 + 0) * C + col] = red[0][0][k] + red[0][1][k] + red[0][2][k] + red[0][3][k];
    part[((long)blockIdx.y * 2 + 1) * C + col] = red[1][0][k] + red[1][1][k] + red[1][2][k] + red[1][3][k];
  }
}

__global__ void bn_mean_kernel(const float* __restrict__ part, int nb, long M, int C, float* mean) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int k = 0; k < nb; ++k) s += part[(k * 2) * C + c];
  mean[c] = s / (float)M;
}

__global__ void bn_var_kernel(const float* __restrict__ part, int nb, long M, int C, const float* mean, float* invstd,
                              float* run_mean, float* run_var, float mom, float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int k = 0; k < nb; ++k) s += part[(k * 2) * C + c];
  const float var = s / (float)M;
  invstd[c] = 1.0f / sqrtf(var + eps);
  if (run_mean) run_mean[c] = (1.f - mom) * run_mean[c] + mom * mean[c];
  if (run_var) run_var[c] = (1.f - mom) * run_var[c] + mom * (M > 1 ? s / (float)(M - 1) : var);
}

__global__ void bn_apply_kernel(const void* X, int xdt, long M, int C, const float* __restrict__ mean,
                                const float* __restrict__ invstd, const float* __restrict__ g,
                                const float* __restrict__ b, const void* R, int relu, void* Y, int ydt, int rdt) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int c = (int)(i % C);
  float v = (ldv(X, xdt, i) - mean[c]) * invstd[c] * g[c] + b[c];
  if (R) v += ldv(R, rdt, i);
  if (relu) v = fmaxf(v, 0.f);
  stv(Y, ydt, i, v);
}

__global__ void bn_bwd_apply_kernel(const void* X, int xdt, const void* Y, int ydt, const void* dY, int dydt, long M,
                                    int C, const float* __restrict__ mean, const float* __restrict__ invstd,
                                    const float* __restrict__ g, const float* __restrict__ sums, int relu, void* dX,
                                    int dxdt, void* dR) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int c = (int)(i % C);
  float dz = ldv(dY, dydt, i);
  if (relu && ldv(Y, ydt, i) <= 0.f) dz = 0.f;
  if (dR) stv(dR, dxdt, i, dz);
  const float is = invstd[c];
  const float xh = (ldv(X, xdt, i) - mean[c]) * is;
  const float m1 = sums[c] / (float)M, m2 = sums[C + c] / (float)M;
  stv(dX, dxdt, i, is * g[c] * (dz - m1 - xh * m2));
}

__global__ void bn_bwd_final_kernel(const float* __restrict__ part, int nb, int C, float* sums, float* dg, float* db,
                                    int acc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f, t = 0.f;
  for (int k = 0; k < nb; ++k) { s += part[(k * 2) * C + c]; t += part[(k * 2 + 1) * C + c]; }
  sums[c] = s;
  sums[C + c] = t;
  if (db) db[c] = acc ? db[c] + s : s;
  if (dg) dg[c] = acc ? dg[c] + t : t;
}

}  // namespace

extern "C" int ivit_layernorm_fwd(const float* X, long ldx, long rpb, long rstride, long roff, long M, long D,
                                  const float* gamma, const float* beta, float eps, void* Y, long ldy, int y_dtype,
                                  float* mean, float* rstd, void* stream) {
  IVIT_CHECK_ARG(D % 64 == 0 && D <= 64 * LN_MAXV, "ivit_layernorm_fwd: D must be a multiple of 64, <= 512");
  if (M <= 0) return 0;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3(ivit_cdiv(M, 4)), dim3(256), 0, ivit_stream(stream), X, ldx, rpb, rstride,
                     roff, M, (int)D, gamma, beta, eps, Y, ldy, y_dtype, mean, rstd);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" long ivit_layernorm_bwd_workspace(long M, long D) {
  return (long)ivit_cdiv(M, 4 * LNB_ROWS) * 2 * D * 4 + 16;
}

extern "C" int ivit_layernorm_bwd(const float* X, long ldx, long rpb, long rstride, long roff, long M, long D,
                                  const float* gamma, const float* mean, const float* rstd, const void* dY, long lddy,
                                  int dy_dtype, const float* dres, float* dX, long lddx, void* dXs, int dxs_dtype,
                                  const float* row_scale, long rows_per_scale, float* dgamma, float* dbeta,
                                  int accumulate, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(D % 64 == 0 && D <= 64 * LN_MAXV, "ivit_layernorm_bwd: D must be a multiple of 64, <= 512");
  IVIT_CHECK_ARG(work_bytes >= ivit_layernorm_bwd_workspace(M, D), "ivit_layernorm_bwd: workspace too small");
  if (M <= 0) return 0;
  hipStream_t st = ivit_stream(stream);
  const int nb = ivit_cdiv(M, 4 * LNB_ROWS);
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(nb), dim3(256), 0, st, X, ldx, rpb, rstride, roff, M, (int)D, gamma, mean,
                     rstd, dY, lddy, dy_dtype, dres, dX, lddx, dXs, dxs_dtype, row_scale,
                     rows_per_scale > 0 ? rows_per_scale : 1, (float*)work);
  launch_colreduce(st, (const float*)work, nb, 2 * D, (int)(2 * D), dgamma, (int)D, dbeta, accumulate);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" long ivit_bn_workspace(long M, long C) { return ((long)ivit_cdiv(M, BN_ROWS) * 2 + 2) * C * 4; }

extern "C" int ivit_bn_stats(const void* X, int x_dtype, long M, long C, float* mean, float* invstd, float* run_mean,
                             float* run_var, float momentum, float eps, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(work_bytes >= ivit_bn_workspace(M, C), "ivit_bn_stats: workspace too small");
  hipStream_t st = ivit_stream(stream);
  const int nb = ivit_cdiv(M, BN_ROWS);
  dim3 g(ivit_cdiv(C, 64), nb);
  float* part = (float*)work;
  hipLaunchKernelGGL(bn_partial_kernel, g, dim3(256), 0, st, 0, X, x_dtype, nullptr, 0, nullptr, 0, M, (int)C,
                     nullptr, nullptr, 0, part);
  hipLaunchKernelGGL(bn_mean_kernel, dim3(ivit_cdiv(C, 256)), dim3(256), 0, st, part, nb, M, (int)C, mean);
  hipLaunchKernelGGL(bn_partial_kernel, g, dim3(256), 0, st, 1, X, x_dtype, nullptr, 0, nullptr, 0, M, (int)C, mean,
                     nullptr, 0, part);
  hipLaunchKernelGGL(bn_var_kernel, dim3(ivit_cdiv(C, 256)), dim3(256), 0, st, part, nb, M, (int)C, mean, invstd,
                     run_mean, run_var, momentum, eps);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_bn_apply(const void* X, int x_dtype, long M, long C, const float* mean, const float* invstd,
                             const float* g, const float* b, const void* R, int relu, void* Y, int y_dtype,
                             void* stream) {
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ivit_cdiv(M * C, 256)), dim3(256), 0, ivit_stream(stream), X, x_dtype, M,
                     (int)C, mean, invstd, g, b, R, relu, Y, y_dtype, y_dtype);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_bn_bwd(const void* X, int x_dtype, const void* Y, int y_dtype, const void* dY, int dy_dtype,
                           long M, long C, const float* mean, const float* invstd, const float* g, int relu, void* dX,
                           int dx_dtype, void* dR, float* dg, float* db, int accumulate, void* work, long work_bytes,
                           void* stream) {
  IVIT_CHECK_ARG(work_bytes >= ivit_bn_workspace(M, C), "ivit_bn_bwd: workspace too small");
  hipStream_t st = ivit_stream(stream);
  const int nb = ivit_cdiv(M, BN_ROWS);
  float* part = (float*)work;
  float* sums = part + (long)nb * 2 * C;
  hipLaunchKernelGGL(bn_partial_kernel, dim3(ivit_cdiv(C, 64), nb), dim3(256), 0, st, 2, X, x_dtype, Y, y_dtype, dY,
                     dy_dtype, M, (int)C, mean, invstd, relu, part);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(ivit_cdiv(C, 256)), dim3(256), 0, st, part, nb, (int)C, sums, dg, db,
                     accumulate);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ivit_cdiv(M * C, 256)), dim3(256), 0, st, X, x_dtype, Y, y_dtype, dY,
                     dy_dtype, M, (int)C, mean, invstd, g, sums, relu, dX, dx_dtype, dR);
  IVIT_LAUNCH_CHECK();
  return 0;
}
