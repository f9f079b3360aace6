// Strided k x k convolutions of the IntentNetCNN variant (model_cnn.py:7-12, 14-33, 86-100;
// SURVEY.md §8f rank 4): stride-2 5x5 / 3x3 / 1x1 convs and stride-1 5x5 convs, run as
// im2col + the dense MFMA GEMMs (ivit_linear_fwd / _dgrad / _wgrad) on NHWC maps.
//   cols[(b, oy, ox)][(ky, kx, c)] = X[b, oy*s - p + ky, ox*s - p + kx, c]   (0 outside; 0 in
//   the pad columns K .. ldc-1), the [Cout][k][k][Cin] order of ivit_pack_conv_weight, so the
//   packed weight viewed [Cout, k*k*Cin] is the GEMM's W.
// col2im is the adjoint as a gather (no atomics, deterministic): dX[b, y, x, c] sums, over
// ky then kx ascending, the dcols entries of the output pixels whose window covers (y, x).
// Both are HBM-bound copies; the channel index is innermost, so a wave reads / writes
// contiguous channel runs.
#include "ivit_common.h"

#include <algorithm>

namespace {

// One wave per (output pixel, tap): the tap's source pixel is a contiguous run of C channels and
// so is its destination, so lanes stride over channels (coalesced, f32 -> bf16 in flight); the
// pixel / tap decomposition is done once per wave in 32-bit arithmetic. The last tap's wave also
// zeroes the pad columns K .. ldc-1.
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void im2col_kernel(const TI* __restrict__ X, int B, int H, int W, int C, int k,
                                                     int s, int p, int Ho, int Wo, TO* __restrict__ cols, long ldc,
                                                     int pairs) {
  const int lane = threadIdx.x & 63;
  const int taps = k * k;
  for (int pr = blockIdx.x * 4 + (threadIdx.x >> 6); pr < pairs; pr += gridDim.x * 4) {
    const int row = pr / taps, tap = pr - (pr / taps) * taps;
    const int ox = row % Wo, t = row / Wo, oy = t % Ho, b = t / Ho;
    const int ky = tap / k, kx = tap - (tap / k) * k;
    const int y = oy * s - p + ky, x = ox * s - p + kx;
    TO* dst = cols + (long)row * ldc + (long)tap * C;
    if (y >= 0 && y < H && x >= 0 && x < W) {
      const TI* src = X + (((long)b * H + y) * W + x) * C;
      for (int c = lane; c < C; c += 64) dst[c] = from_f32<TO>(to_f32(src[c]));
    } else {
      for (int c = lane; c < C; c += 64) dst[c] = from_f32<TO>(0.f);
    }
    if (tap == taps - 1)
      for (long c = (long)taps * C + lane; c < ldc; c += 64) cols[(long)row * ldc + c] = from_f32<TO>(0.f);
  }
}

// One wave per input pixel: lanes hold up to 8 x 64 channel sums (C <= 512) and the wave walks
// the taps whose output pixel exists (ky then kx ascending: the summation order is fixed).
__global__ __launch_bounds__(256) void col2im_kernel(const float* __restrict__ dcols, long ldc, int B, int H, int W,
                                                     int C, int k, int s, int p, int Ho, int Wo,
                                                     float* __restrict__ dX) {
  const int lane = threadIdx.x & 63;
  const int npix = B * H * W;
  for (int px = blockIdx.x * 4 + (threadIdx.x >> 6); px < npix; px += gridDim.x * 4) {
    const int x = px % W, t = px / W, y = t % H, b = t / H;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int ky = 0; ky < k; ++ky) {
      const int ny = y + p - ky;
      if (ny < 0 || ny % s) continue;
      const int oy = ny / s;
      if (oy >= Ho) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int nx = x + p - kx;
        if (nx < 0 || nx % s) continue;
        const int ox = nx / s;
        if (ox >= Wo) continue;
        const float* src = dcols + (((long)b * Ho + oy) * Wo + ox) * ldc + (long)(ky * k + kx) * C;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = lane + 64 * j;
          if (c < C) acc[j] += src[c];
        }
      }
    }
    float* dst = dX + (long)px * C;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = lane + 64 * j;
      if (c < C) dst[c] = acc[j];
    }
  }
}

}  // namespace

extern "C" int ivit_im2col(int x_dtype, const void* X, long B, long H, long W, long C, long k, long stride, long pad,
                           long Ho, long Wo, void* cols, long ldc, int cols_dtype, void* stream) {
  IVIT_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0 && k > 0 && stride > 0 && pad >= 0, "ivit_im2col: bad shape");
  IVIT_CHECK_ARG(Ho == (H + 2 * pad - k) / stride + 1 && Wo == (W + 2 * pad - k) / stride + 1 && Ho > 0 && Wo > 0,
                 "ivit_im2col: output size %ldx%ld does not match the conv geometry", Ho, Wo);
  IVIT_CHECK_ARG(ldc >= k * k * C, "ivit_im2col: ldc %ld < k*k*C", ldc);
  IVIT_CHECK_ARG(B * H * W * C < (1L << 40) && H < (1 << 30) && W < (1 << 30), "ivit_im2col: too large");
  IVIT_CHECK_ARG(B * Ho * Wo * k * k < (1L << 31) && B * H * W < (1L << 31), "ivit_im2col: too many pixel-taps");
  const long pairs = B * Ho * Wo * k * k;
  const int g = (int)std::min<long>((pairs + 3) / 4, 256L * 8 * 16);
  hipStream_t st = ivit_stream(stream);
#define IVIT_I2C(TI, TO)                                                                                       \
  hipLaunchKernelGGL((im2col_kernel<TI, TO>), dim3(g), dim3(256), 0, st, (const TI*)X, (int)B, (int)H, (int)W, \
                     (int)C, (int)k, (int)stride, (int)pad, (int)Ho, (int)Wo, (TO*)cols, ldc, (int)pairs)
  if (x_dtype == IVIT_F32 && cols_dtype == IVIT_BF16) IVIT_I2C(float, bf16);
  else if (x_dtype == IVIT_F32 && cols_dtype == IVIT_F32) IVIT_I2C(float, float);
  else if (x_dtype == IVIT_BF16 && cols_dtype == IVIT_BF16) IVIT_I2C(bf16, bf16);
  else IVIT_CHECK_ARG(false, "ivit_im2col: unsupported dtype pair (%d -> %d)", x_dtype, cols_dtype);
#undef IVIT_I2C
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_col2im(const float* dcols, long ldc, long B, long H, long W, long C, long k, long stride,
                           long pad, long Ho, long Wo, float* dX, void* stream) {
  IVIT_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0 && k > 0 && stride > 0 && pad >= 0, "ivit_col2im: bad shape");
  IVIT_CHECK_ARG(Ho == (H + 2 * pad - k) / stride + 1 && Wo == (W + 2 * pad - k) / stride + 1,
                 "ivit_col2im: output size does not match the conv geometry");
  IVIT_CHECK_ARG(ldc >= k * k * C, "ivit_col2im: ldc %ld < k*k*C", ldc);
  IVIT_CHECK_ARG(C <= 512 && B * H * W < (1L << 31), "ivit_col2im: C <= 512 channels");
  const long npix = B * H * W;
  hipLaunchKernelGGL(col2im_kernel, dim3((unsigned)std::min<long>((npix + 3) / 4, 256L * 8 * 16)), dim3(256), 0, ivit_stream(stream), dcols, ldc, (int)B,
                     (int)H, (int)W, (int)C, (int)k, (int)stride, (int)pad, (int)Ho, (int)Wo, dX);
  IVIT_LAUNCH_CHECK();
  return 0;
}
