// Differing LiDAR / map patch grids (model_vit.py:64,71 with a patch-16 vit_model_name, :139):
//   * PatchEmbed for patch sizes P != 8 (timm vit_*_patch16_224): a patch matrix + the linear
//     GEMM, then the CLS / pos_embed token assembly; backward: the assembly's adjoint (compact
//     patch-row gradient, pos / CLS gradients) + the linear weight gradient.
//   * F.interpolate(mode='bilinear', align_corners=False) of the map features onto the LiDAR
//     grid, forward and its adjoint (a deterministic gather: no atomics).
// All HBM-bound element-wise passes: one thread per output element, coalesced along the
// fastest output axis.
#include "ivit_common.h"

namespace {

// cols[b*Np + gy*Wp + gx][(c*P + ky)*P + kx] = img[b][c][gy*P + ky][gx*P + kx]; thread per
// output element, consecutive threads = consecutive columns (kx fastest: P-float runs of a row).
template <typename O>
__global__ __launch_bounds__(256) void patch_im2col_p_kernel(const float* __restrict__ img, int C, int H, int W, int P,
                                                             long total, O* __restrict__ cols) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int Hp = H / P, Wp = W / P;
  const long K = (long)C * P * P;
  const long row = i / K;
  const int col = (int)(i - row * K);
  const int kx = col % P, ky = (col / P) % P, c = col / (P * P);
  const long b = row / ((long)Hp * Wp);
  const int p = (int)(row - b * Hp * Wp), gy = p / Wp, gx = p - gy * Wp;
  cols[i] = from_f32<O>(img[((b * C + c) * H + (long)gy * P + ky) * W + (long)gx * P + kx]);
}

// out[b][0] = cls + pos[0]; out[b][1 + p] = Y[b*Np + p] + pos[1 + p]   (timm _pos_embed, f32)
__global__ __launch_bounds__(256) void patch_tokens_kernel(const float* __restrict__ Y, long B, long Np, long D,
                                                           const float* __restrict__ pos,
                                                           const float* __restrict__ cls, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long Ntok = Np + 1;
  if (i >= B * Ntok * D) return;
  const long d = i % D, t = (i / D) % Ntok, b = i / (D * Ntok);
  out[i] = (t == 0 ? cls[d] : Y[(b * Np + t - 1) * D + d]) + pos[t * D + d];
}

// dY[b*Np + p] = dtok[b][1 + p] (dtype O); dpos[t] (+)= sum_b dtok[b][t]; dcls (+)= dpos[0] part.
template <typename S, typename O>
__global__ __launch_bounds__(256) void patch_tokens_bwd_kernel(const S* __restrict__ dtok, long B, long Np, long D,
                                                               O* __restrict__ dY, float* __restrict__ dpos,
                                                               float* __restrict__ dcls, int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over Ntok * D
  const long Ntok = Np + 1;
  if (i >= Ntok * D) return;
  const long t = i / D;
  float s = 0.f;
  for (long b = 0; b < B; ++b) {
    const float g = to_f32(dtok[b * Ntok * D + i]);
    s += g;
    if (t > 0) dY[(b * Np + t - 1) * D + (i - t * D)] = from_f32<O>(g);
  }
  dpos[i] = accumulate ? dpos[i] + s : s;
  if (t == 0 && dcls) dcls[i] = accumulate ? dcls[i] + s : s;
}

// ATen's linear-interpolation taps (UpSampleKernel.cpp compute_indices_weights_linear,
// align_corners = false, no explicit scale): real = max(scale*(o + 0.5) - 0.5, 0) with
// scale = (float)in / out; i0 = (int)real; l1 = clamp(real - i0, 0, 1); l0 = 1 - l1;
// the second tap is i0 + 1, or i0 itself at the last input index.
struct Tap {
  int i0, i1;
  float l0, l1;
};
IVIT_DEV Tap lin_tap(int o, float scale, int n_in) {
  float real = scale * ((float)o + 0.5f) - 0.5f;
  real = real < 0.f ? 0.f : real;
  Tap t;
  t.i0 = (int)real;
  if (t.i0 > n_in - 1) t.i0 = n_in - 1;
  float l1 = real - (float)t.i0;
  l1 = l1 < 0.f ? 0.f : (l1 > 1.f ? 1.f : l1);
  t.l1 = l1;
  t.l0 = 1.f - l1;
  t.i1 = t.i0 < n_in - 1 ? t.i0 + 1 : t.i0;
  return t;
}

// Y[z][oh][ow] = h0*(w0*X[i0][j0] + w1*X[i0][j1]) + h1*(w0*X[i1][j0] + w1*X[i1][j1])
__global__ __launch_bounds__(256) void bilinear_fwd_kernel(const float* __restrict__ X, long Z, int Hi, int Wi,
                                                           float* __restrict__ Y, int Ho, int Wo, float sh, float sw) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Z * Ho * Wo) return;
  const int ow = (int)(i % Wo), oh = (int)((i / Wo) % Ho);
  const long z = i / ((long)Ho * Wo);
  const Tap h = lin_tap(oh, sh, Hi), w = lin_tap(ow, sw, Wi);
  const float* x = X + z * Hi * Wi;
  const float r0 = w.l0 * x[(long)h.i0 * Wi + w.i0] + w.l1 * x[(long)h.i0 * Wi + w.i1];
  const float r1 = w.l0 * x[(long)h.i1 * Wi + w.i0] + w.l1 * x[(long)h.i1 * Wi + w.i1];
  Y[i] = h.l0 * r0 + h.l1 * r1;
}

// Weight of input index `in` in output o's taps (both taps when they coincide at the edge).
IVIT_DEV float tap_weight(const Tap& t, int in) {
  return (t.i0 == in ? t.l0 : 0.f) + (t.i1 == in ? t.l1 : 0.f);
}

// Output range [lo, hi) whose taps can reach input index `in` (real in (in - 1, in + 1]),
// widened by 2 and clamped; tap_weight() decides exactly.
IVIT_DEV void out_range(int in, float scale, int n_out, int& lo, int& hi) {
  lo = (int)floorf(((float)in - 1.f + 0.5f) / scale - 0.5f) - 2;
  hi = (int)ceilf(((float)in + 1.f + 0.5f) / scale - 0.5f) + 3;
  lo = lo < 0 ? 0 : lo;
  hi = hi > n_out ? n_out : hi;
}

// dX[z][ih][iw] = sum_{oh, ow} wh(oh, ih) ww(ow, iw) dY[z][oh][ow]   (gather, deterministic)
__global__ __launch_bounds__(256) void bilinear_bwd_kernel(const float* __restrict__ dY, long Z, int Hi, int Wi,
                                                           int Ho, int Wo, float sh, float sw,
                                                           float* __restrict__ dX) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Z * Hi * Wi) return;
  const int iw = (int)(i % Wi), ih = (int)((i / Wi) % Hi);
  const long z = i / ((long)Hi * Wi);
  int h_lo, h_hi, w_lo, w_hi;
  out_range(ih, sh, Ho, h_lo, h_hi);
  out_range(iw, sw, Wo, w_lo, w_hi);
  const float* g = dY + z * Ho * Wo;
  float s = 0.f;
  for (int oh = h_lo; oh < h_hi; ++oh) {
    const float wh = tap_weight(lin_tap(oh, sh, Hi), ih);
    if (wh == 0.f) continue;
    float r = 0.f;
    for (int ow = w_lo; ow < w_hi; ++ow) {
      const float ww = tap_weight(lin_tap(ow, sw, Wi), iw);
      if (ww != 0.f) r += ww * g[(long)oh * Wo + ow];
    }
    s += wh * r;
  }
  dX[i] = s;
}

}  // namespace

extern "C" int ivit_patch_im2col_p(const float* img, long B, long C, long H, long W, long P, void* cols,
                                   int cols_dtype, void* stream) {
  IVIT_CHECK_ARG(P > 0 && H % P == 0 && W % P == 0, "ivit_patch_im2col_p: H, W must be multiples of the patch %ld", P);
  const long total = B * (H / P) * (W / P) * C * P * P;
  if (total == 0) return 0;
  hipStream_t st = ivit_stream(stream);
  if (cols_dtype == IVIT_BF16)
    hipLaunchKernelGGL(patch_im2col_p_kernel<bf16>, dim3(ivit_cdiv(total, 256)), dim3(256), 0, st, img, (int)C, (int)H,
                       (int)W, (int)P, total, (bf16*)cols);
  else
    hipLaunchKernelGGL(patch_im2col_p_kernel<float>, dim3(ivit_cdiv(total, 256)), dim3(256), 0, st, img, (int)C,
                       (int)H, (int)W, (int)P, total, (float*)cols);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_patch_tokens(const float* Y, long B, long Np, long D, const float* pos, const float* cls,
                                 float* out, void* stream) {
  const long total = B * (Np + 1) * D;
  if (total == 0) return 0;
  hipLaunchKernelGGL(patch_tokens_kernel, dim3(ivit_cdiv(total, 256)), dim3(256), 0, ivit_stream(stream), Y, B, Np, D,
                     pos, cls, out);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_patch_tokens_bwd(const void* dtok, int dtok_dtype, long B, long Np, long D, void* dY, int dy_dtype,
                                     float* dpos, float* dcls, int accumulate, void* stream) {
  const long n = (Np + 1) * D;
  if (n == 0) return 0;
  hipStream_t st = ivit_stream(stream);
  const dim3 g(ivit_cdiv(n, 256));
  if (dtok_dtype == IVIT_BF16) {
    if (dy_dtype == IVIT_BF16)
      hipLaunchKernelGGL((patch_tokens_bwd_kernel<bf16, bf16>), g, dim3(256), 0, st, (const bf16*)dtok, B, Np, D,
                         (bf16*)dY, dpos, dcls, accumulate);
    else
      hipLaunchKernelGGL((patch_tokens_bwd_kernel<bf16, float>), g, dim3(256), 0, st, (const bf16*)dtok, B, Np, D,
                         (float*)dY, dpos, dcls, accumulate);
  } else {
    if (dy_dtype == IVIT_BF16)
      hipLaunchKernelGGL((patch_tokens_bwd_kernel<float, bf16>), g, dim3(256), 0, st, (const float*)dtok, B, Np, D,
                         (bf16*)dY, dpos, dcls, accumulate);
    else
      hipLaunchKernelGGL((patch_tokens_bwd_kernel<float, float>), g, dim3(256), 0, st, (const float*)dtok, B, Np, D,
                         (float*)dY, dpos, dcls, accumulate);
  }
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_bilinear_fwd(const float* X, long Z, long Hi, long Wi, float* Y, long Ho, long Wo, void* stream) {
  IVIT_CHECK_ARG(Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "ivit_bilinear_fwd: empty spatial size");
  const long total = Z * Ho * Wo;
  if (total == 0) return 0;
  hipLaunchKernelGGL(bilinear_fwd_kernel, dim3(ivit_cdiv(total, 256)), dim3(256), 0, ivit_stream(stream), X, Z,
                     (int)Hi, (int)Wi, Y, (int)Ho, (int)Wo, (float)Hi / (float)Ho, (float)Wi / (float)Wo);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_bilinear_bwd(const float* dY, long Z, long Hi, long Wi, long Ho, long Wo, float* dX, void* stream) {
  IVIT_CHECK_ARG(Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "ivit_bilinear_bwd: empty spatial size");
  const long total = Z * Hi * Wi;
  if (total == 0) return 0;
  hipLaunchKernelGGL(bilinear_bwd_kernel, dim3(ivit_cdiv(total, 256)), dim3(256), 0, ivit_stream(stream), dY, Z,
                     (int)Hi, (int)Wi, (int)Ho, (int)Wo, (float)Hi / (float)Ho, (float)Wi / (float)Wo, dX);
  IVIT_LAUNCH_CHECK();
  return 0;
}
