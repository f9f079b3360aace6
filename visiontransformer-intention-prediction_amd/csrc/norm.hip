// LayerNorm (timm Block norm1/norm2/norm, eps 1e-6; adapter LN eps 1e-5, model_vit.py:82-83)
// and BatchNorm2d in training mode (BasicBlock bn1/bn2/downsample, model_vit.py:24-31) on
// NHWC maps. All statistics in f32; column reductions are two-pass and deterministic.
#include <stdlib.h>

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

// ---- vectorised LayerNorm: one half-wave (32 lanes) per row, 16 B per lane per access,
// 4 rows per half-wave in flight (a 256-thread block covers 32 rows). D % 128 == 0, D <= 512;
// all row strides multiples of 4 and base pointers 16-B aligned (checked on the host).
static inline bool al16h(const void* p) { return ((uintptr_t)p & 15) == 0; }
IVIT_DEV long rowmap32(int r, int rpb, int rstride, int roff) {
  return rpb ? (long)(r / rpb) * rstride + roff + r % rpb : (long)r;
}
IVIT_DEV float half_sum(float v) {
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 32);
  return v;
}
template <typename T> IVIT_DEV float4 ld4(const T* p);
template <> IVIT_DEV float4 ld4<float>(const float* p) { return *(const float4*)p; }
template <> IVIT_DEV float4 ld4<bf16>(const bf16* p) {
  Pack4 t;
  t.u = *(const uint2*)p;
  return make_float4(bf2f(t.h[0]), bf2f(t.h[1]), bf2f(t.h[2]), bf2f(t.h[3]));
}
template <typename T> IVIT_DEV void st4(T* p, float4 v);
template <> IVIT_DEV void st4<float>(float* p, float4 v) { *(float4*)p = v; }
template <> IVIT_DEV void st4<bf16>(bf16* p, float4 v) {
  Pack4 t;
  t.h[0] = f2bf(v.x); t.h[1] = f2bf(v.y); t.h[2] = f2bf(v.z); t.h[3] = f2bf(v.w);
  *(uint2*)p = t.u;
}
constexpr int LNV_ROWS = 4;  // rows per half-wave

template <typename TO, int NC>
__global__ __launch_bounds__(256) void ln_fwd_vec_kernel(const float* __restrict__ X, long ldx, int rpb, int rstride,
                                                         int roff, int M, const float* __restrict__ g,
                                                         const float* __restrict__ bta, float eps, TO* __restrict__ Y,
                                                         long ldy, float* __restrict__ mean,
                                                         float* __restrict__ rstd) {
  constexpr int D = NC * 128;
  const int hw = threadIdx.x >> 5, hl = threadIdx.x & 31;
  float4 gg[NC], bb[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    gg[i] = *(const float4*)(g + 4 * (hl + 32 * i));
    bb[i] = *(const float4*)(bta + 4 * (hl + 32 * i));
  }
  const int r0 = (blockIdx.x * 8 + hw) * LNV_ROWS;
#pragma unroll
  for (int k = 0; k < LNV_ROWS; ++k) {
    const int row = r0 + k;
    if (row < M) {
      const float* x = X + rowmap32(row, rpb, rstride, roff) * ldx;
      float4 v[NC];
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        v[i] = *(const float4*)(x + 4 * (hl + 32 * i));
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
      }
      const float mu = half_sum(s) * (1.0f / D);
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        const float a = v[i].x - mu, b = v[i].y - mu, c = v[i].z - mu, d = v[i].w - mu;
        q += (a * a + b * b) + (c * c + d * d);
      }
      const float rs = 1.0f / sqrtf(half_sum(q) * (1.0f / D) + eps);
      TO* y = Y + (long)row * ldy;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        float4 o;
        o.x = (v[i].x - mu) * rs * gg[i].x + bb[i].x;
        o.y = (v[i].y - mu) * rs * gg[i].y + bb[i].y;
        o.z = (v[i].z - mu) * rs * gg[i].z + bb[i].z;
        o.w = (v[i].w - mu) * rs * gg[i].w + bb[i].w;
        st4<TO>(y + 4 * (hl + 32 * i), o);
      }
      if (hl == 0) { mean[row] = mu; rstd[row] = rs; }
    }
  }
}

// dX(f32) = dres + rs*(g*dy - mean(g*dy) - xhat*mean(g*dy*xhat)); dXs = TS(dX * scale);
// per-block partial column sums of dy*xhat and dy -> part[blk][2][D]
template <typename TY, typename TS, int NC>
__global__ __launch_bounds__(256) void ln_bwd_vec_kernel(const float* __restrict__ X, long ldx, int rpb, int rstride,
                                                         int roff, int M, const float* __restrict__ g,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, const TY* __restrict__ dY,
                                                         long lddy, const float* dres, float* dX, long lddx,
                                                         TS* __restrict__ dXs, const float* __restrict__ rscale,
                                                         int rps, float* __restrict__ part) {
  constexpr int D = NC * 128;
  const int hw = threadIdx.x >> 5, hl = threadIdx.x & 31;
  float4 gg[NC], pg[NC], pb[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    gg[i] = *(const float4*)(g + 4 * (hl + 32 * i));
    pg[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    pb[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int r0 = (blockIdx.x * 8 + hw) * LNV_ROWS;
#pragma unroll
  for (int k = 0; k < LNV_ROWS; ++k) {
    const int row = r0 + k;
    if (row < M) {
      const long xr = rowmap32(row, rpb, rstride, roff);
      const float* x = X + xr * ldx;
      const TY* dy = dY + (long)row * lddy;
      const float mu = mean[row], rs = rstd[row];
      float4 xh[NC], gy[NC];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        const int c = 4 * (hl + 32 * i);
        const float4 xv = *(const float4*)(x + c);
        const float4 d = ld4<TY>(dy + c);
        xh[i] = make_float4((xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs);
        gy[i] = make_float4(d.x * gg[i].x, d.y * gg[i].y, d.z * gg[i].z, d.w * gg[i].w);
        s1 += (gy[i].x + gy[i].y) + (gy[i].z + gy[i].w);
        s2 += (gy[i].x * xh[i].x + gy[i].y * xh[i].y) + (gy[i].z * xh[i].z + gy[i].w * xh[i].w);
        pg[i].x += d.x * xh[i].x; pg[i].y += d.y * xh[i].y; pg[i].z += d.z * xh[i].z; pg[i].w += d.w * xh[i].w;
        pb[i].x += d.x; pb[i].y += d.y; pb[i].z += d.z; pb[i].w += d.w;
      }
      s1 = half_sum(s1) * (1.0f / D);
      s2 = half_sum(s2) * (1.0f / D);
      const float sc = rscale ? rscale[row / rps] : 1.f;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        const int c = 4 * (hl + 32 * i);
        float4 o;
        o.x = rs * (gy[i].x - s1 - xh[i].x * s2);
        o.y = rs * (gy[i].y - s1 - xh[i].y * s2);
        o.z = rs * (gy[i].z - s1 - xh[i].z * s2);
        o.w = rs * (gy[i].w - s1 - xh[i].w * s2);
        if (dres) {
          const float4 r = *(const float4*)(dres + xr * lddx + c);
          o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
        }
        *(float4*)(dX + xr * lddx + c) = o;
        if (dXs) st4<TS>(dXs + (long)row * D + c, make_float4(o.x * sc, o.y * sc, o.z * sc, o.w * sc));
      }
    }
  }
  __shared__ float4 red[2][8][NC * 32];
#pragma unroll
  for (int i = 0; i < NC; ++i) { red[0][hw][hl + 32 * i] = pg[i]; red[1][hw][hl + 32 * i] = pb[i]; }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * NC * 32; t += 256) {
    const int w = t / (NC * 32), c4 = t - w * (NC * 32);
    float4 a = red[w][0][c4];
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      const float4 b = red[w][j][c4];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    *(float4*)(part + ((long)blockIdx.x * 2 + w) * D + 4 * c4) = a;
  }
}

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
// Rows per partial block: 32 (1125 workgroups for the neck's 36 000 x 512 maps; 128-row blocks gave
// 282, ~4 waves per CU, latency-bound: mode-2 partials 50.4 -> 41.0 us, profiles/r06_m_*), doubled
// until the blocks fit the grid's y dimension (a B = 8 full-grid CNN map has 2.3 M rows)
static int bn_rows(long M) {
  long r = 32;
  while ((M + r - 1) / r > 65535) r *= 2;
  return (int)r;
}

// mode 0: partial column sums of x; mode 1: sums of (x - mean)^2; mode 2: bwd sums of dz, dz*xhat
__global__ __launch_bounds__(256) void bn_partial_kernel(int mode, const void* X, int xdt, const void* Y, int ydt,
                                                         const void* dY, int dydt, long M, int C,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd, int relu,
                                                         float* __restrict__ part, int rows) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.y * rows;
  float s = 0.f, t = 0.f;
  if (col < C) {
    const float mu = mode ? mean[col] : 0.f;
    const float is = mode == 2 ? invstd[col] : 0.f;
    for (long r = r0 + ph; r < min(M, r0 + rows); r += 4) {
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

// The same partials with 8 consecutive columns per thread (16-B bf16 / 2 x 16-B f32 loads) and
// the row loop unrolled, so several rows' loads are in flight per thread (the scalar form issued
// one 2-B load per lane per dependent add: latency-bound). Same per-column summation order as
// bn_partial_kernel (rows r0 + ph + 4k in sequence, then phases 0..3), so identical results.
// C % 8 == 0; 512 columns x 4 row phases per 256-thread block.
IVIT_DEV void ld8v(const void* p, int dt, long i, float (&x)[8]) {
  if (dt == IVIT_BF16) load8f<bf16>((const bf16*)p + i, x, 8);
  else load8f<float>((const float*)p + i, x, 8);
}
__global__ __launch_bounds__(256) void bn_partial8_kernel(int mode, const void* X, int xdt, const void* Y, int ydt,
                                                          const void* dY, int dydt, long M, int C,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, int relu,
                                                          float* __restrict__ part, int rows) {
  const int lc = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int col = (blockIdx.x * 64 + lc) * 8;
  const long r0 = (long)blockIdx.y * rows;
  float s[8], t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = t[e] = 0.f;
  if (col < C) {
    float mu[8], is[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = mode ? mean[col + e] : 0.f;
      is[e] = mode == 2 ? invstd[col + e] : 0.f;
    }
    const long rend = min(M, r0 + rows);
#pragma unroll 4
    for (long r = r0 + ph; r < rend; r += 4) {
      const long i = r * C + col;
      float x[8];
      ld8v(X, xdt, i, x);
      if (mode == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += x[e];
      } else if (mode == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = x[e] - mu[e];
          s[e] += d * d;
        }
      } else {
        float dz[8];
        ld8v(dY, dydt, i, dz);
        if (relu) {
          float y[8];
          ld8v(Y, ydt, i, y);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (y[e] <= 0.f) dz[e] = 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s[e] += dz[e];
          t[e] += dz[e] * (x[e] - mu[e]) * is[e];
        }
      }
    }
  }
  __shared__ float red[2][4][512];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][ph][lc * 8 + e] = s[e];
    red[1][ph][lc * 8 + e] = t[e];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 512; k += 256) {
    const int c = blockIdx.x * 512 + k;
    if (c < C) {
      part[((long)blockIdx.y * 2 + 0) * C + c] = red[0][0][k] + red[0][1][k] + red[0][2][k] + red[0][3][k];
      part[((long)blockIdx.y * 2 + 1) * C + c] = red[1][0][k] + red[1][1][k] + red[1][2][k] + red[1][3][k];
    }
  }
}

// partial-sum launch: the 8-column form when C % 8 == 0
static void launch_bn_partial(hipStream_t st, int mode, const void* X, int xdt, const void* Y, int ydt,
                              const void* dY, int dydt, long M, long C, const float* mean, const float* invstd,
                              int relu, float* part) {
  const int rows = bn_rows(M), nb = ivit_cdiv(M, rows);
  if (C % 8 == 0)
    hipLaunchKernelGGL(bn_partial8_kernel, dim3(ivit_cdiv(C, 512), nb), dim3(256), 0, st, mode, X, xdt, Y, ydt, dY,
                       dydt, M, (int)C, mean, invstd, relu, part, rows);
  else
    hipLaunchKernelGGL(bn_partial_kernel, dim3(ivit_cdiv(C, 64), nb), dim3(256), 0, st, mode, X, xdt, Y, ydt, dY,
                       dydt, M, (int)C, mean, invstd, relu, part, rows);
}

// Column sums of the per-block partials, BN_NC columns x BN_PH row phases per 1024-thread block
// (the partial lists are hundreds of rows long: one thread per column left them latency-bound);
// each phase's rows with eight loads in flight, summed in row order, then the phases in order.
constexpr int BN_PH = 64, BN_NC = 1024 / BN_PH;  // 16 columns x 64 phases: C / 16 workgroups
IVIT_DEV float bn_colsum(const float* __restrict__ part, int nb, long pstride, long off, int c, bool valid,
                         float (*red)[BN_NC]) {
  const int ph = threadIdx.x / BN_NC, lc = threadIdx.x % BN_NC;
  float s = 0.f;
  if (valid) {
    for (int k0 = ph; k0 < nb; k0 += 8 * BN_PH) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = k0 + i * BN_PH < nb ? part[(long)(k0 + i * BN_PH) * pstride + off + c] : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (k0 + i * BN_PH < nb) s += v[i];
    }
  }
  red[ph][lc] = s;
  __syncthreads();
  float t = 0.f;
  if (ph == 0) {
#pragma unroll 8
    for (int k = 0; k < BN_PH; ++k) t += red[k][lc];
  }
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(1024) void bn_mean_kernel(const float* __restrict__ part, int nb, long M, int C,
                                                       float* mean) {
  __shared__ float red[BN_PH][BN_NC];
  const int c = blockIdx.x * BN_NC + (threadIdx.x % BN_NC);
  const float s = bn_colsum(part, nb, 2L * C, 0, c, c < C, red);
  if (threadIdx.x < BN_NC && c < C) mean[c] = s / (float)M;
}

__global__ __launch_bounds__(1024) void bn_var_kernel(const float* __restrict__ part, int nb, long M, int C,
                                                      const float* mean, float* invstd, float* run_mean,
                                                      float* run_var, float mom, float eps) {
  __shared__ float red[BN_PH][BN_NC];
  const int c = blockIdx.x * BN_NC + (threadIdx.x % BN_NC);
  const float s = bn_colsum(part, nb, 2L * C, 0, c, c < C, red);
  if (threadIdx.x < BN_NC && c < C) {
    const float var = s / (float)M;
    invstd[c] = 1.0f / sqrtf(var + eps);
    if (run_mean) run_mean[c] = (1.f - mom) * run_mean[c] + mom * mean[c];
    if (run_var) run_var[c] = (1.f - mom) * run_var[c] + mom * (M > 1 ? s / (float)(M - 1) : var);
  }
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

// 8 consecutive channels x BN8_R rows per thread (C % 8 == 0, 16-B aligned operands): the channel
// parameters are loaded once per thread (per element they were 4x the bytes of the data), rows
// strided by C; the same per-element arithmetic as bn_apply_kernel / bn_bwd_apply_kernel (bitwise
// the same results), 16-B accesses. Thread t: chunk t % (C / 8), rows (t / (C / 8)) * BN8_R + 0..
constexpr int BN8_R = 2;  // (8 rows per thread: 4.4 workgroups per CU on the neck's maps)
__global__ __launch_bounds__(256) void bn_apply8_kernel(const void* X, int xdt, long M, int C,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ g, const float* __restrict__ b,
                                                       const void* R, int relu, void* Y, int ydt, int rdt) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nc = C / 8;
  const int c = (int)(t % nc) * 8;
  const long r0 = (t / nc) * BN8_R;
  if (r0 >= M) return;
  float mu[8], is[8], gg[8], bb[8];
  load8f(mean + c, mu, 8);
  load8f(invstd + c, is, 8);
  load8f(g + c, gg, 8);
  load8f(b + c, bb, 8);
  const long r1 = min(M, r0 + BN8_R);
  for (long r = r0; r < r1; ++r) {
    const long i = r * C + c;
    float x[8], q[8];
    ld8dt(X, xdt, i, x);
    if (R) ld8dt(R, rdt, i, q);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = (x[e] - mu[e]) * is[e] * gg[e] + bb[e];
      if (R) v += q[e];
      if (relu) v = fmaxf(v, 0.f);
      x[e] = v;
    }
    st8dt(Y, ydt, i, x);
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply8_kernel(const void* X, int xdt, const void* Y, int ydt,
                                                           const void* dY, int dydt, long M, int C,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ g,
                                                           const float* __restrict__ sums, int relu, void* dX,
                                                           int dxdt, void* dR) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nc = C / 8;
  const int c = (int)(t % nc) * 8;
  const long r0 = (t / nc) * BN8_R;
  if (r0 >= M) return;
  float mu[8], is[8], gg[8], m1[8], m2[8];
  load8f(mean + c, mu, 8);
  load8f(invstd + c, is, 8);
  load8f(g + c, gg, 8);
  load8f(sums + c, m1, 8);
  load8f(sums + C + c, m2, 8);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    m1[e] = m1[e] / (float)M;
    m2[e] = m2[e] / (float)M;
  }
  const long r1 = min(M, r0 + BN8_R);
  for (long r = r0; r < r1; ++r) {
    const long i = r * C + c;
    float dz[8], y[8], x[8];
    ld8dt(dY, dydt, i, dz);
    if (relu) ld8dt(Y, ydt, i, y);
    ld8dt(X, xdt, i, x);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (relu && y[e] <= 0.f) dz[e] = 0.f;
    if (dR) st8dt(dR, dxdt, i, dz);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (x[e] - mu[e]) * is[e];
      x[e] = is[e] * gg[e] * (dz[e] - m1[e] - xh * m2[e]);
    }
    st8dt(dX, dxdt, i, x);
  }
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

__global__ __launch_bounds__(1024) void bn_bwd_final_kernel(const float* __restrict__ part, int nb, int C,
                                                            float* sums, float* dg, float* db, int acc) {
  __shared__ float red[BN_PH][BN_NC];
  const int c = blockIdx.x * BN_NC + (threadIdx.x % BN_NC);
  const float s = bn_colsum(part, nb, 2L * C, 0, c, c < C, red);
  const float t = bn_colsum(part, nb, 2L * C, C, c, c < C, red);
  if (threadIdx.x < BN_NC && c < C) {
    sums[c] = s;
    sums[C + c] = t;
    if (db) db[c] = acc ? db[c] + s : s;
    if (dg) dg[c] = acc ? dg[c] + t : t;
  }
}

}  // namespace

extern "C" int ivit_layernorm_fwd(const float* X, long ldx, long rpb, long rstride, long roff, long M, long D,
                                  const float* gamma, const float* beta, float eps, void* Y, long ldy, int y_dtype,
                                  float* mean, float* rstd, void* stream) {
  IVIT_CHECK_ARG(D % 64 == 0 && D <= 64 * LN_MAXV, "ivit_layernorm_fwd: D must be a multiple of 64, <= 512");
  if (M <= 0) return 0;
  hipStream_t st = ivit_stream(stream);
  const bool vec = D % 128 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && al16h(X) && al16h(Y) && al16h(gamma) &&
                   al16h(beta) && M < (1L << 30) && rstride < (1L << 30) && roff < (1L << 30) && rpb < (1L << 30);
  if (vec) {
    const dim3 grid(ivit_cdiv(M, 8 * LNV_ROWS));
#define LNF(NC)                                                                                                   \
  if (D == NC * 128) {                                                                                            \
    if (y_dtype == IVIT_BF16)                                                                                     \
      hipLaunchKernelGGL((ln_fwd_vec_kernel<bf16, NC>), grid, dim3(256), 0, st, X, ldx, (int)rpb, (int)rstride,    \
                         (int)roff, (int)M, gamma, beta, eps, (bf16*)Y, ldy, mean, rstd);                         \
    else                                                                                                          \
      hipLaunchKernelGGL((ln_fwd_vec_kernel<float, NC>), grid, dim3(256), 0, st, X, ldx, (int)rpb, (int)rstride,   \
                         (int)roff, (int)M, gamma, beta, eps, (float*)Y, ldy, mean, rstd);                        \
  }
    LNF(1) LNF(2) LNF(3) LNF(4)
#undef LNF
  } else {
    hipLaunchKernelGGL(ln_fwd_kernel, dim3(ivit_cdiv(M, 4)), dim3(256), 0, st, X, ldx, rpb, rstride, roff, M, (int)D,
                       gamma, beta, eps, Y, ldy, y_dtype, mean, rstd);
  }
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
  const int nb = ivit_cdiv(M, 4 * LNB_ROWS);  // = cdiv(M, 8 * LNV_ROWS): both kernels cover 32 rows per block
  const int rps = (int)(rows_per_scale > 0 ? rows_per_scale : 1);
  const bool vec = D % 128 == 0 && ldx % 4 == 0 && lddy % 4 == 0 && lddx % 4 == 0 && al16h(X) && al16h(dY) &&
                   al16h(dX) && al16h(gamma) && (!dres || al16h(dres)) && (!dXs || al16h(dXs)) && M < (1L << 30) &&
                   rstride < (1L << 30) && roff < (1L << 30) && rpb < (1L << 30);
  if (vec) {
#define LNB(NC, TY, TS)                                                                                              \
  hipLaunchKernelGGL((ln_bwd_vec_kernel<TY, TS, NC>), dim3(nb), dim3(256), 0, st, X, ldx, (int)rpb, (int)rstride,     \
                     (int)roff, (int)M, gamma, mean, rstd, (const TY*)dY, lddy, dres, dX, lddx, (TS*)dXs, row_scale, \
                     rps, (float*)work)
#define LNB_D(NC)                                                                                                    \
  if (D == NC * 128) {                                                                                               \
    if (dy_dtype == IVIT_BF16) {                                                                                     \
      if (dxs_dtype == IVIT_BF16) LNB(NC, bf16, bf16); else LNB(NC, bf16, float);                                    \
    } else {                                                                                                         \
      if (dxs_dtype == IVIT_BF16) LNB(NC, float, bf16); else LNB(NC, float, float);                                  \
    }                                                                                                                \
  }
    LNB_D(1) LNB_D(2) LNB_D(3) LNB_D(4)
#undef LNB_D
#undef LNB
  } else {
    hipLaunchKernelGGL(ln_bwd_kernel, dim3(nb), dim3(256), 0, st, X, ldx, rpb, rstride, roff, M, (int)D, gamma, mean,
                       rstd, dY, lddy, dy_dtype, dres, dX, lddx, dXs, dxs_dtype, row_scale, (long)rps, (float*)work);
  }
  launch_colreduce(st, (const float*)work, nb, 2 * D, (int)(2 * D), dgamma, (int)D, dbeta, accumulate);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" long ivit_bn_workspace(long M, long C) { return ((long)ivit_cdiv(M, bn_rows(M)) * 2 + 2) * C * 4; }

extern "C" int ivit_bn_stats(const void* X, int x_dtype, long M, long C, float* mean, float* invstd, float* run_mean,
                             float* run_var, float momentum, float eps, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(work_bytes >= ivit_bn_workspace(M, C), "ivit_bn_stats: workspace too small");
  hipStream_t st = ivit_stream(stream);
  const int nb = ivit_cdiv(M, bn_rows(M));
  float* part = (float*)work;
  launch_bn_partial(st, 0, X, x_dtype, nullptr, 0, nullptr, 0, M, C, nullptr, nullptr, 0, part);
  hipLaunchKernelGGL(bn_mean_kernel, dim3(ivit_cdiv(C, BN_NC)), dim3(1024), 0, st, part, nb, M, (int)C, mean);
  launch_bn_partial(st, 1, X, x_dtype, nullptr, 0, nullptr, 0, M, C, mean, nullptr, 0, part);
  hipLaunchKernelGGL(bn_var_kernel, dim3(ivit_cdiv(C, BN_NC)), dim3(1024), 0, st, part, nb, M, (int)C, mean, invstd,
                     run_mean, run_var, momentum, eps);
  IVIT_LAUNCH_CHECK();
  return 0;
}

namespace {
// eval-mode BatchNorm statistics from the running buffers: mean = running_mean, invstd =
// rsqrtf(running_var + eps) — the values torch.rsqrt(rvar + eps) gives on the device
__global__ void bn_eval_stats_kernel(const float* __restrict__ rmean, const float* __restrict__ rvar, int C, float eps,
                                     float* __restrict__ mean, float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rmean[c];
  invstd[c] = rsqrtf(rvar[c] + eps);
}
}  // namespace

extern "C" int ivit_bn_eval_stats(const float* run_mean, const float* run_var, long C, float eps, float* mean,
                                  float* invstd, void* stream) {
  IVIT_CHECK_ARG(C >= 0 && C < (1L << 30), "ivit_bn_eval_stats: bad channel count %ld", C);
  if (C == 0) return 0;
  hipLaunchKernelGGL(bn_eval_stats_kernel, dim3(ivit_cdiv(C, 256)), dim3(256), 0, ivit_stream(stream), run_mean,
                     run_var, (int)C, eps, mean, invstd);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_bn_apply(const void* X, int x_dtype, long M, long C, const float* mean, const float* invstd,
                             const float* g, const float* b, const void* R, int relu, void* Y, int y_dtype,
                             void* stream) {
  const bool v8 = C % 8 == 0 && hal16(X) && hal16(Y) && (!R || hal16(R)) && hal16(mean) && hal16(invstd) && hal16(g) &&
                  hal16(b);
  if (v8)
    hipLaunchKernelGGL(bn_apply8_kernel, dim3(ivit_cdiv(ivit_cdiv(M, BN8_R) * (C / 8), 256)), dim3(256), 0,
                       ivit_stream(stream), X, x_dtype,
                       M, (int)C, mean, invstd, g, b, R, relu, Y, y_dtype, y_dtype);
  else
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
  const int nb = ivit_cdiv(M, bn_rows(M));
  float* part = (float*)work;
  float* sums = part + (long)nb * 2 * C;
  launch_bn_partial(st, 2, X, x_dtype, Y, y_dtype, dY, dy_dtype, M, C, mean, invstd, relu, part);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(ivit_cdiv(C, BN_NC)), dim3(1024), 0, st, part, nb, (int)C, sums, dg, db,
                     accumulate);
  const bool v8 = C % 8 == 0 && hal16(X) && (!relu || hal16(Y)) && hal16(dY) && hal16(dX) && (!dR || hal16(dR)) &&
                  hal16(mean) && hal16(invstd) && hal16(g) && hal16(sums);
  if (v8)
    hipLaunchKernelGGL(bn_bwd_apply8_kernel, dim3(ivit_cdiv(ivit_cdiv(M, BN8_R) * (C / 8), 256)), dim3(256), 0, st, X,
                       x_dtype, Y, y_dtype,
                       dY, dy_dtype, M, (int)C, mean, invstd, g, sums, relu, dX, dx_dtype, dR);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ivit_cdiv(M * C, 256)), dim3(256), 0, st, X, x_dtype, Y, y_dtype, dY,
                       dy_dtype, M, (int)C, mean, invstd, g, sums, relu, dX, dx_dtype, dR);
  IVIT_LAUNCH_CHECK();
  return 0;
}
