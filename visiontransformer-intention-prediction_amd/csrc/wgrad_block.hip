// Weight + bias gradients of one timm Block's four linears in ONE launch (model_vit.py:64,71 ->
// timm Block: Mlp.fc2, Mlp.fc1, Attention.proj, Attention.qkv), bf16 operands, f32 results:
//
//   dW_g[n][k] = sum_t dY_g[t][n] X_g[t][k],   db_g[n] = sum_t dY_g[t][n]     (t over B*N tokens)
//
// The four GEMMs share the long token reduction (M = 36 008 at the bench shape) and have small
// outputs (0.15-0.59 M elements each), so each one alone is a split-K GEMM whose partial-slab
// round trip and short grid dominate (the four engine launches took ~265 us per block). Here the
// four are one grid of 128 x 384 output tiles (fc2 12, fc1 12, proj 3, qkv 9 = 36 tiles) times
// S token splits (S = 7 at the bench shape: 252 workgroups, one per CU), reduced by one launch:
// the partial traffic is paid once per block instead of once per GEMM, and every CU streams.
//
// Workgroup: 8 compute waves (2 along rows x 4 along columns, each 64 x 96 = 2 x 3 blocks of
// v_mfma_f32_32x32x16_bf16) + 4 loader waves, K step 32 tokens, 4 LDS stages (32 KiB each: the
// dY block's 128 columns and the X block's 384 columns as token-major 256-B-row images), three
// steps in flight by LDS-DMA, one barrier per step. Both operands are read by transposing LDS
// reads (frag_mn).
// Bias: row sums of the dY block on the matrix pipe against a ones operand (tiles with tn == 0;
// each wave adds one MFMA per step: its row block wn & 1 on substep wn >> 1).
#include "gemm_engine.h"
#include "panel_common.h"

using namespace ivit;

namespace {

constexpr int WB_BK = 32;                   // tokens per K step
constexpr int WB_NS = 4;                    // LDS stages (5 measured: no faster)
constexpr int WB_IMG = WB_BK * 256;         // one token-major image: 32 rows x 128 bf16 columns
constexpr int WB_STAGE = 4 * WB_IMG;        // dY block (1 image) + X block (3 images)
constexpr int WB_TM = 128, WB_TN = 384;     // output tile
constexpr int WB_SMAX = 7;                  // token splits (workspace bound)

struct WbGemm {
  const bf16* dy;  // [M][N] token-major
  const bf16* x;   // [M][K]
  int N, K;        // dW is [N][K]
  int tiles_m, tiles_n;
  long slab_off;   // element offset of this GEMM's [N][K] block inside one split's slab
  long bias_off;   // element offset of its [N] bias block inside one (split, half) bias slab
};
struct WbArgs {
  WbGemm g[4];
  int tile_base[5];  // prefix sums of tiles_m * tiles_n
  int M, splits, kchunk;
  long slab_n, bias_n;  // elements per split (weights) / per (split, half) (biases)
  float* slab;
  float* bslab;
};

// Roles: waves 0..7 compute (2 along rows x 4 along columns, each 64 x 96), waves 8..11 only
// issue the LDS-DMA (8 pieces each per step): an LDS-DMA piece costs its issuing wave ~100-185
// cycles beside MFMAs (MI355X_MICROARCH.md cycle constants), and with every wave issuing its own
// pieces the DMA and MFMA phases ran nearly serialised (anatomy: DMA skeleton 112 us + MFMA-only
// 105 us -> 206 us together). Both roles pass exactly one barrier per step.
// MODE (anatomy builds: -DIVIT_WB_ANATOMY=MODE via tools/ab_build.sh): 0 product, 1 no MFMAs (the DMA / barrier
// skeleton), 2 no DMA after the prologue (MFMAs on stale stages), 3 the product kernel without the
// reduce launch.
constexpr int WB_CW = 8, WB_LW = 4;  // compute / loader waves
#ifndef IVIT_WB_ANATOMY
#define IVIT_WB_ANATOMY 0
#endif
template <int MODE>
__global__ __launch_bounds__(64 * (WB_CW + WB_LW), 1) void wgrad_block_kernel(const WbArgs args) {
  __shared__ __attribute__((aligned(16))) char smem[WB_NS * WB_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = args.tile_base[4];
  // consecutive flat ids (same split, neighbouring tiles) on one XCD: the split's token panels
  // are fetched into one L2 and shared by its tiles
  const int flat = xcd_remap(blockIdx.x, gridDim.x);
  const int split = flat / ntiles, tile = flat - split * ntiles;
  int gi = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q) gi += tile >= args.tile_base[q] ? 1 : 0;
  const WbGemm g = args.g[gi];
  const int lt = tile - args.tile_base[gi];
  const int tm = lt / g.tiles_n, tn = lt - tm * g.tiles_n;
  const int kbeg = split * args.kchunk, kend = min(args.M, kbeg + args.kchunk);
  const int nk = (kend - kbeg + WB_BK - 1) / WB_BK;

  if (wv >= WB_CW) {  // ---------------------------------------------------------------- loader
    const bf16* Abase = g.dy + tm * WB_TM;  // the dY block's first column
    const bf16* Bbase = g.x + tn * WB_TN;   // the X block's first column
    const int lda = g.N, ldb = g.K;
    const int lw = wv - WB_CW;
    // 32 pieces of 1 KiB per stage, 8 per loader wave: piece p < 8 -> dY image rows 4p.., else X
    // image (p - 8) / 8; a piece is 4 token rows x 16 chunks, chunk c of row r at c ^ 4(r & 3)
    unsigned voff[8];
    int prow[8], pcol[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int p = lw * 8 + i;
      const int img = p >> 3, row = (p & 7) * 4 + (lane >> 4);
      const int c = (lane & 15) ^ ((row & 3) << 2);
      const int col = (img == 0 ? 0 : (img - 1) * 128) + c * 8;
      prow[i] = row;
      pcol[i] = col;
      voff[i] = 2u * (unsigned)(row * (img == 0 ? lda : ldb) + col);
    }
    const bool isa = lw == 0;  // wave-uniform: loader 0 fills the dY image, 1..3 the X images
    auto issue = [&](int stage, int k0) {
      char* st = smem + stage * WB_STAGE + lw * 8192;
      if (k0 + WB_BK <= kend) {
        const char* sb = isa ? uniform_ptr(Abase + (long)k0 * lda) : uniform_ptr(Bbase + (long)k0 * ldb);
#pragma unroll
        for (int i = 0; i < 8; ++i) glds_s<false>(voff[i], sb, st + i * 1024);
      } else {  // the ragged last step: token rows >= kend read the zero page
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int t = k0 + prow[i];
          const void* src = t < kend ? (const void*)((isa ? Abase + (long)t * lda : Bbase + (long)t * ldb) + pcol[i])
                                     : (const void*)g_zero16;
          glds<16>(src, st + i * 1024);
        }
      }
    };
#pragma unroll
    for (int s = 0; s < WB_NS - 1; ++s)
      if (s < nk) issue(s, kbeg + s * WB_BK);
    for (int kt = 0; kt < nk; ++kt) {
      // this step's pieces have landed (later steps stay in flight) ...
      static_assert(WB_NS == 4, "counted waits below assume three steps in flight");
      if (MODE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // ... published by the barrier, which also tells that the compute waves are done with the
      // stage refilled next (read in step kt-1)
      __builtin_amdgcn_s_barrier();
      if (MODE != 2 && kt + WB_NS - 1 < nk) issue((kt + WB_NS - 1) % WB_NS, kbeg + (kt + WB_NS - 1) * WB_BK);
    }
    return;
  }

  // ------------------------------------------------------------------------------------ compute
  const int wm = wv >> 2, wn = wv & 3;
  f32x16 acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  f32x16 accb;
#pragma unroll
  for (int r = 0; r < 16; ++r) accb[r] = 0.f;
  const bool dob = tn == 0 && args.bslab != nullptr;
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;

  for (int kt = 0; kt < nk; ++kt) {
    __builtin_amdgcn_s_barrier();
    const char* st = smem + (kt % WB_NS) * WB_STAGE;
#pragma unroll
    for (int t = 0; t < (MODE == 1 ? 0 : 2); ++t) {
      bf16x8 fa[2], fb[3];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = frag_mn(st, 16 * t, 64 * wm + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int cb = 96 * wn + 32 * j;
        fb[j] = frag_mn(st + WB_IMG * (1 + (cb >> 7)), 16 * t, cb & 127, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if (dob && t == (wn >> 1)) {  // uniform branches: a runtime index into fa is lowered to
        if (wn & 1)                 // per-element select chains (240 VALU per step)
          accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], ones, accb, 0, 0, 0);
        else
          accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], ones, accb, 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // my reads of this stage are done
  }

  // partial tile -> this split's slab, in dW's own [N][K] layout (the reduce is a plain sum)
  float* slab = args.slab + (long)split * args.slab_n + g.slab_off;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int col = tn * WB_TN + 96 * wn + 32 * j + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tm * WB_TM + 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
        slab[(long)row * g.K + col] = acc[i][j][r];
      }
    }
  if (dob && (lane & 31) == 0) {  // every column of accb holds the row sum
    float* bs = args.bslab + ((long)split * 2 + (wn >> 1)) * args.bias_n + g.bias_off;
#pragma unroll
    for (int r = 0; r < 16; ++r) bs[tm * WB_TM + 64 * wm + 32 * (wn & 1) + (r & 3) + 8 * (r >> 2) + 4 * hl] = accb[r];
  }
}

struct WbOut {
  float* dw[4];
  float* db[4];
  long off[5];   // weight element offsets in one split's slab (prefix), off[4] = slab_n
  long boff[5];  // bias offsets, boff[4] = bias_n
};

// out = sum over splits (and the two bias halves) in a fixed order: deterministic. Four outputs
// per thread (16-B accesses; every size is a multiple of 4).
__global__ void wgrad_block_reduce_kernel(const float* __restrict__ slab, const float* __restrict__ bslab,
                                          const WbOut o, int splits) {
  const long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long nw = o.off[4];
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < nw) {
    int gi = 0;
#pragma unroll
    for (int q = 1; q < 4; ++q) gi += i4 >= o.off[q] ? 1 : 0;
#pragma unroll 7
    for (int k = 0; k < splits; ++k) {
      const float4 v = *(const float4*)(slab + (long)k * nw + i4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    *(float4*)(o.dw[gi] + (i4 - o.off[gi])) = s;
    return;
  }
  const long j4 = i4 - nw, nb = o.boff[4];
  if (j4 >= nb) return;
  int gi = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q) gi += j4 >= o.boff[q] ? 1 : 0;
  for (int k = 0; k < 2 * splits; ++k) {
    const float4 v = *(const float4*)(bslab + (long)k * nb + j4);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  if (o.db[gi] != nullptr) *(float4*)(o.db[gi] + (j4 - o.boff[gi])) = s;
}

int wb_splits(long M) {
  const long steps = (M + WB_BK - 1) / WB_BK;
  return (int)(steps < WB_SMAX ? (steps > 0 ? steps : 1) : WB_SMAX);
}

}  // namespace

extern "C" long ivit_vit_block_wgrad_workspace(long M, long D, long Hd) {
  const long S = wb_splits(M);
  const long nw = 2 * D * Hd + D * D + 3 * D * D;  // fc2 [D][Hd], fc1 [Hd][D], proj [D][D], qkv [3D][D]
  const long nb = D + Hd + D + 3 * D;
  return S * (nw + 2 * nb) * 4 + 256;
}

extern "C" int ivit_vit_block_wgrad(long M, long D, long Hd, const void* dy2, const void* a, const void* dh,
                                    const void* x2, const void* dyp, const void* o, const void* dyq, const void* x1,
                                    float* dw2, float* db2, float* dw1, float* db1, float* dwp, float* dbp,
                                    float* dwq, float* dbq, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(D == 384 && Hd % 384 == 0 && Hd > 0, "ivit_vit_block_wgrad: D must be 384, Hd a multiple of 384");
  IVIT_CHECK_ARG(M > 0 && M < (1L << 31) / (3 * D), "ivit_vit_block_wgrad: bad token count %ld", M);
  IVIT_CHECK_ARG(dy2 && a && dh && x2 && dyp && o && dyq && x1 && dw2 && dw1 && dwp && dwq,
                 "ivit_vit_block_wgrad: null operand");
  IVIT_CHECK_ARG(work_bytes >= ivit_vit_block_wgrad_workspace(M, D, Hd), "ivit_vit_block_wgrad: workspace too small");
  const void* ops[8] = {dy2, a, dh, x2, dyp, o, dyq, x1};
  for (int i = 0; i < 8; ++i) IVIT_CHECK_ARG(((uintptr_t)ops[i] & 15) == 0, "ivit_vit_block_wgrad: operand not 16-B aligned");
  // the reduce stores 16 B per thread into every output (ddp.GradBuckets aligns its views)
  const void* outs[8] = {dw2, db2, dw1, db1, dwp, dbp, dwq, dbq};
  for (int i = 0; i < 8; ++i)
    IVIT_CHECK_ARG(((uintptr_t)outs[i] & 15) == 0, "ivit_vit_block_wgrad: output %d not 16-B aligned", i);
  const int S = wb_splits(M);
  const long steps = (M + WB_BK - 1) / WB_BK;
  const int kchunk = (int)((steps + S - 1) / S) * WB_BK;
  WbArgs args;
  // (dY, X, N, K): fc2 dY = dx2s [M][D], X = gelu output [M][Hd]; fc1 dY = dh [M][Hd], X = ln2;
  // proj dY = dx1s, X = attention output; qkv dY = dqkv [M][3D], X = ln1
  const struct { const void* dy; const void* x; long N, K; } gs[4] = {
      {dy2, a, D, Hd}, {dh, x2, Hd, D}, {dyp, o, D, D}, {dyq, x1, 3 * D, D}};
  WbOut out;
  float* dws[4] = {dw2, dw1, dwp, dwq};
  float* dbs[4] = {db2, db1, dbp, dbq};
  long off = 0, boff = 0;
  args.tile_base[0] = 0;
  for (int q = 0; q < 4; ++q) {
    WbGemm& g = args.g[q];
    g.dy = (const bf16*)gs[q].dy;
    g.x = (const bf16*)gs[q].x;
    g.N = (int)gs[q].N;
    g.K = (int)gs[q].K;
    g.tiles_m = (int)(gs[q].N / WB_TM);
    g.tiles_n = (int)(gs[q].K / WB_TN);
    g.slab_off = off;
    g.bias_off = boff;
    out.dw[q] = dws[q];
    out.db[q] = dbs[q];
    out.off[q] = off;
    out.boff[q] = boff;
    off += gs[q].N * gs[q].K;
    boff += gs[q].N;
    args.tile_base[q + 1] = args.tile_base[q] + g.tiles_m * g.tiles_n;
  }
  out.off[4] = off;
  out.boff[4] = boff;
  args.M = (int)M;
  args.splits = S;
  args.kchunk = kchunk;
  args.slab_n = off;
  args.bias_n = boff;
  char* w = (char*)(((uintptr_t)work + 255) & ~(uintptr_t)255);
  args.slab = (float*)w;
  args.bslab = args.slab + (long)S * off;
  hipStream_t st = ivit_stream(stream);
  // anatomy builds (tools/ab_build.sh -DIVIT_WB_ANATOMY=1 / 2) compile a diagnostic body instead
  hipLaunchKernelGGL(wgrad_block_kernel<IVIT_WB_ANATOMY>, dim3(args.tile_base[4] * S), dim3(64 * (WB_CW + WB_LW)), 0,
                     st, args);
  IVIT_LAUNCH_CHECK();
  if (IVIT_WB_ANATOMY == 3) return 0;  // anatomy 3: the product kernel without its reduce (timing only)
  hipLaunchKernelGGL(wgrad_block_reduce_kernel, dim3(ivit_cdiv((off + boff) / 4, 256)), dim3(256), 0, st, args.slab,
                     args.bslab, out, S);
  IVIT_LAUNCH_CHECK();
  return 0;
}
