// Internal interface of patch_embed.hip used by gemm_ops.hip (not part of the C ABI).
#pragma once
#include "ivit_common.h"

namespace ivit {
// Weight gradient of the patch embedding straight from the f32 raster (bf16 products, f32 sums):
// dW [D][C*64] (+)= sum over patches of dtok (token rows, CLS skipped) x patch(raster).
bool patch_wgrad_raster_ok(long B, long C, long H, long W, long D);
long patch_wgrad_raster_workspace(long D);
long patch_wgrad_raster_workspace2(long B, long C, long H, long W, long D);  // every schedule of the shape
int patch_wgrad_raster(const bf16* dtok, const float* img, long B, long C, long H, long W, long D, float* dW,
                       int accumulate, void* work, hipStream_t st);
}  // namespace ivit
