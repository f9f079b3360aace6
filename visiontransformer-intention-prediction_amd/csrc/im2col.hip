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

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void im2col_kernel(const TI* __restrict__ X, int B, int H, int W, int C, int k,
                                                     int s, int p, int Ho, int Wo, TO* __restrict__ cols, long ldc) {
  const long K = (long)k * k * C, total = (long)B * Ho * Wo * ldc;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long row = i / ldc, col = i - row * ldc;
    float v = 0.f;
    if (col < K) {
      const int c = (int)(col % C), kk = (int)(col / C), kx = kk % k, ky = kk / k;
      const int ox = (int)(row % Wo);
      const long t = row / Wo;
      const int oy = (int)(t % Ho), b = (int)(t / Ho);
      const int y = oy * s - p + ky, x = ox * s - p + kx;
      if (y >= 0 && y < H && x >= 0 && x < W) v = to_f32(X[(((long)b * H + y) * W + x) * C + c]);
    }
    cols[i] = from_f32<TO>(v);
  }
}

__global__ __launch_bounds__(256) void col2im_kernel(const float* __restrict__ dcols, long ldc, int B, int H, int W,
                                                     int C, int k, int s, int p, int Ho, int Wo,
                                                     float* __restrict__ dX) {
  const long total = (long)B * H * W * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H), b = (int)(t / H);
    float acc = 0.f;
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
        acc += dcols[(((long)b * Ho + oy) * Wo + ox) * ldc + ((long)ky * k + kx) * C + c];
      }
    }
    dX[i] = acc;
  }
}

int grid_for(long n) { return (int)std::min<long>((n + 255) / 256, 256L * 8 * 16); }

}  // namespace

extern "C" int ivit_im2col(int x_dtype, const void* X, long B, long H, long W, long C, long k, long stride, long pad,
                           long Ho, long Wo, void* cols, long ldc, int cols_dtype, void* stream) {
  IVIT_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0 && k > 0 && stride > 0 && pad >= 0, "ivit_im2col: bad shape");
  IVIT_CHECK_ARG(Ho == (H + 2 * pad - k) / stride + 1 && Wo == (W + 2 * pad - k) / stride + 1 && Ho > 0 && Wo > 0,
                 "ivit_im2col: output size %ldx%ld does not match the conv geometry", Ho, Wo);
  IVIT_CHECK_ARG(ldc >= k * k * C, "ivit_im2col: ldc %ld < k*k*C", ldc);
  IVIT_CHECK_ARG(B * H * W * C < (1L << 40) && H < (1 << 30) && W < (1 << 30), "ivit_im2col: too large");
  const long n = B * Ho * Wo * ldc;
  const int g = grid_for(n);
  hipStream_t st = ivit_stream(stream);
#define IVIT_I2C(TI, TO)                                                                                       \
  hipLaunchKernelGGL((im2col_kernel<TI, TO>), dim3(g), dim3(256), 0, st, (const TI*)X, (int)B, (int)H, (int)W, \
                     (int)C, (int)k, (int)stride, (int)pad, (int)Ho, (int)Wo, (TO*)cols, ldc)
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
  const long n = B * H * W * C;
  hipLaunchKernelGGL(col2im_kernel, dim3(grid_for(n)), dim3(256), 0, ivit_stream(stream), dcols, ldc, (int)B,
                     (int)H, (int)W, (int)C, (int)k, (int)stride, (int)pad, (int)Ho, (int)Wo, dX);
  IVIT_LAUNCH_CHECK();
  return 0;
}
