// Panel implicit-GEMM convolution (conv_panel.hip): the fusion-block 3x3 / 1x1 convolutions' forward
// and data gradient (model_vit.py:12-43 BasicBlock, reached from model_vit.py:141).
#pragma once
#include "ivit_common.h"

namespace ivit {

// C[m][n] = bias[n] + sum_{tap, c} A[pixel m shifted by tap][c] * Bk[n][tap * Cin + c]
//   A: NHWC bf16 map, pixel stride lda elements, Cin channels (Cin % 64 == 0), k x k "same" taps;
//   Bk: bf16 [N][ks * ks * Cin] (K-contiguous packed weights); C: f32 or bf16, row stride ldy.
// Returns false (nothing launched) when the shape is not one the kernel takes.
bool conv_panel_ok(long M, long N, long Cin, long lda, long ks);
// stats != nullptr: also the per-tile BatchNorm partials ([ceil(M / 288)][2][N]: channel sum, sum of
// squares about the tile mean; conv_panel_stats_floats floats).
int conv_panel_launch(const bf16* A, long lda, int Bn, int H, int W, int Cin, int ks, const bf16* Bk, int N,
                      const float* bias, void* Y, long ldy, bool y_bf16, hipStream_t st, float* stats = nullptr);
long conv_panel_stats_floats(long M, long N);
// Weight gradient on 256 x 256 panel tiles, the pixel reduction split `splits` ways into an f32 slab
// [splits][Cout][ks*ks*Cin] (the engine's EpiSlab layout; reduced by the caller).
bool conv_wgrad_panel_ok(long M, long Cout, long Cin, long ks, long lddy);
int conv_wgrad_panel_splits(long M, long Cout, long N);
int conv_wgrad_panel_launch(const bf16* dY, long lddy, const bf16* X, int Bn, int H, int W, int Cin, int Cout, int ks,
                            float* slab, int splits, hipStream_t st);
// ivit_set_knob(IVIT_KNOB_CONV_PANEL, 0) turns the panel kernels off (the 128x128 engine instead: the
// tests compare the two); default on.
bool conv_panel_enabled();

}  // namespace ivit
