// Panel implicit-GEMM convolution for the fusion block (BasicBlock conv3x3 / conv1x1, model_vit.py:12-43,
// reached from model_vit.py:141): forward Y = conv(X, W) and the data gradient dX = conv(dY, flip(W)^T).
//
// The 128 x 128 engine tile (gemm_engine.h) streams one LDS fragment read per MFMA and, at two
// workgroups per CU, keeps the LDS array as busy as the matrix pipe; and 36 000 output pixels of a
// B = 8 fusion map cut into 282 x 4 such tiles fill the 512 workgroup slots 2.2 times (the third
// round a fifth full). Here a workgroup of 8 waves owns 288 pixels x 256 output channels:
//   * 36 000 = 125 x 288, so a 512-channel convolution is 250 tiles, one round over the 256 CUs;
//   * each wave computes 144 pixels x 64 channels with v_mfma_f32_16x16x32_bf16 (9 x 4 blocks),
//     13 fragment reads per 36 MFMAs (a third of the engine's LDS read traffic per flop);
//   * both operands stream by LDS-DMA into a double-buffered [rows][64 k] image (68 KiB per
//     stage): the map through per-lane tap addresses (a padding tap reads a zero page), the packed
//     weights [N][k*k*Cin] by the saddr form;
//   * the weights are the MFMA's A operand, so each lane's accumulators are 4 consecutive output
//     channels of one pixel and the epilogue stores 16 B (f32) / 8 B (bf16) per lane directly.
// Same sums as the engine (f32 accumulation of bf16 products), K in the same tap-major order.
#include "conv_panel.h"

#include <stdlib.h>

#include "gemm_engine.h"
#include "panel_common.h"

namespace ivit {
namespace {

constexpr int CP_BM = 288, CP_BN = 256, CP_W = 8;
constexpr int CP_WM = 144, CP_WN = 64;                      // wave tile: 2 (M) x 4 (N) waves
constexpr int CP_MB = CP_WM / 16, CP_NB = CP_WN / 16;       // 9 x 4 MFMA blocks per wave
constexpr int CP_SA = CP_BM * 128, CP_SB = CP_BN * 128;     // [rows][64 k] bf16 images
constexpr int CP_STAGE = CP_SA + CP_SB;                     // 68 KiB
constexpr int CP_PA = CP_BM / 8, CP_PB = CP_BN / 8;         // 1-KiB DMA pieces (8 rows) per image
constexpr int CP_PAW = (CP_PA + CP_W - 1) / CP_W;           // 5: waves 0-3 take 5 A pieces, 4-7 four
constexpr int CP_PAX = CP_PA - (CP_PAW - 1) * CP_W;         // waves with CP_PAW pieces
constexpr int CP_PBW = CP_PB / CP_W;                        // 4 B pieces per wave
static_assert(CP_PB % CP_W == 0 && CP_PAX > 0, "piece split");

__device__ __attribute__((aligned(16))) uint4 cp_zero16[4];
// anatomy builds (tools/ab_build.sh -DCP_ANAT=1 / 2; timing only, wrong results): 1 no fragment reads
// or MFMAs (the DMA / barrier skeleton), 2 no DMA after the first K tile (MFMAs on stale stages)
#ifndef CP_ANAT
#define CP_ANAT 0
#endif

// 128-B image rows (64 k), 16-B chunk c of row r at chunk c ^ ((r >> 1) & 7): the 16x16x32 operand
// reads (rows r0 .. r0+15, chunks 4t .. 4t+3) hit 16 distinct bank quads per ds_read_b128 lane group.
IVIT_DEV int cp_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

struct CpArgs {
  const bf16* A;
  long lda;
  int H, W, Cin, ks, M;
  const bf16* Bk;
  int N, K;
  const float* bias;
  void* Y;
  long ldy;
  int tilesN;
  float* stats;  // STATS: [tilesM][2][N] per-tile channel sum and centred sum of squares
};

template <typename O, bool STATS>
__global__ __launch_bounds__(512, 1) void conv_panel_kernel(CpArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * CP_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), wm = wv >> 2, wn = wv & 3;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);  // the N tiles of one pixel panel share an XCD
  const int tm = lin / p.tilesN, tn = lin - tm * p.tilesN;
  const int m0 = tm * CP_BM, n0 = tn * CP_BN;
  const int pad = p.ks >> 1;
  const int npa = wv < CP_PAX ? CP_PAW : CP_PAW - 1;

  // per-lane DMA state (k-invariant): the map pixel (flat offset + y, x) of each A piece row, the
  // weight row offset of each B piece row; rows past M / N are clamped (computed, never stored)
  int abase[CP_PAW], ayx[CP_PAW];
#pragma unroll
  for (int i = 0; i < CP_PAW; ++i) {
    const int piece = min(wv + CP_W * i, CP_PA - 1);
    const int row = piece * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
    const int m = min(m0 + row, p.M - 1);
    const int x = m % p.W, y = (m / p.W) % p.H;
    abase[i] = m * (int)p.lda + c * 8;
    ayx[i] = (y << 16) | x;
  }
  unsigned boff[CP_PBW];
#pragma unroll
  for (int i = 0; i < CP_PBW; ++i) {
    const int row = (wv + CP_W * i) * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
    const int n = min(n0 + row, p.N - 1);
    boff[i] = 2u * (unsigned)(n * p.K + c * 8);
  }
  // K order: channel tile major, the k*k taps inside it (Cin % 64 == 0: a K tile is one tap), so
  // the k*k shifted reads of a 64-channel slab of the pixel panel follow each other and all but
  // the first hit the XCD's L2 (tap-major order streamed the whole panel once per tap: 9x the
  // Infinity-Cache traffic for a 3x3 conv)
  struct Tile { long shift; const char* bsb; int dy, dx; };
  auto tile_of = [&](int kt) {
    const int nt = p.ks * p.ks, ct = kt / nt, tap = kt - ct * nt, ci0 = ct * 64;
    const int k0 = tap * p.Cin + ci0;  // the weight's K offset ([N][k][k][Cin] packing)
    const int ky = tap / p.ks, kx = tap - ky * p.ks;
    Tile t;
    t.dy = ky - pad;
    t.dx = kx - pad;
    t.shift = (long)(t.dy * p.W + t.dx) * p.lda + ci0;
    t.bsb = uniform_ptr(p.Bk + k0);
    return t;
  };
  // the zero page's address once, in SGPRs (re-deriving it per piece is a GOT scalar load whose
  // lgkmcnt(0) wait would also drain the fragment reads in flight)
  const char* zpage = (const char*)cp_zero16;
  asm volatile("" : "+s"(zpage));
  // piece q of a K tile: q < CP_PAW the wave's A (map) piece q, else its B (weight) piece q - CP_PAW
  auto issue_piece = [&](const Tile& t, int s, int q) {
    char* sa = smem + s * CP_STAGE;
    if (q < CP_PAW) {
      if (q < npa) {
        const int yy = (ayx[q] >> 16) + t.dy, xx = (ayx[q] & 0xffff) + t.dx;
        const bool ok = (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
        const void* src = ok ? (const void*)(p.A + (t.shift + abase[q])) : (const void*)zpage;
        glds_v<false>(src, sa + (wv + CP_W * q) * 1024);
      }
    } else {
      glds_s<false>(boff[q - CP_PAW], t.bsb, sa + CP_SA + (wv + CP_W * (q - CP_PAW)) * 1024);
    }
  };
  auto issue = [&](int kt, int s) {
    const Tile t = tile_of(kt);
#pragma unroll
    for (int q = 0; q < CP_PAW + CP_PBW; ++q) issue_piece(t, s, q);
  };

  f32x4 acc[CP_MB][CP_NB];
#pragma unroll
  for (int i = 0; i < CP_MB; ++i)
#pragma unroll
    for (int j = 0; j < CP_NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / 64;
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // one barrier per K tile: it publishes tile kt (every wave's pieces landed) and tells that every
    // wave is done reading stage cur ^ 1 (tile kt-1), which tile kt+1 then refills
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // (the pieces issued one per MFMA group instead of this burst: 136-137 vs 138-139 us at
    // 512 -> 512, not kept)
    if (kt + 1 < nk && CP_ANAT != 2) issue(kt + 1, cur ^ 1);
    if (CP_ANAT == 1) continue;
    const char* ia = smem + cur * CP_STAGE;
    const char* ib = ia + CP_SA;
    bf16x8 bfr[2][CP_NB];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < CP_NB; ++j)
        bfr[t][j] = *(const bf16x8*)(ib + cp_off(wn * CP_WN + 16 * j + (lane & 15), 4 * t + (lane >> 4)));
    // A fragment f = (t = f / 9: 32-k half, mb = f % 9), read three ahead of its MFMAs
    auto rdf = [&](int f) {
      const int t = f / CP_MB, mb = f % CP_MB;
      return *(const bf16x8*)(ia + cp_off(wm * CP_WM + 16 * mb + (lane & 15), 4 * t + (lane >> 4)));
    };
    bf16x8 fr[4];
    fr[0] = rdf(0);
    fr[1] = rdf(1);
    fr[2] = rdf(2);
#pragma unroll
    for (int f = 0; f < 2 * CP_MB; ++f) {
      const int t = f / CP_MB, mb = f % CP_MB;
      if (f + 3 < 2 * CP_MB) fr[(f + 3) % 4] = rdf(f + 3);
#pragma unroll
      for (int j = 0; j < CP_NB; ++j)
        acc[mb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[t][j], fr[f % 4], acc[mb][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // my reads of this stage are done
  }

  // epilogue: acc[mb][j] lane l = channels n .. n+3 (n = n0 + 64 wn + 16 j + 4 (l >> 4)) of pixel
  // m0 + 144 wm + 16 mb + (l & 15)
  O* Y = (O*)p.Y;
  // every bias value before the first store (a load under the store branches makes the compiler
  // wait vmcnt(0), i.e. for all earlier stores too, before each one)
  float4 bv[CP_NB];
#pragma unroll
  for (int j = 0; j < CP_NB; ++j) {
    const int n = min(n0 + wn * CP_WN + 16 * j + 4 * (lane >> 4), p.N - 4);
    bv[j] = p.bias ? *(const float4*)(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < CP_NB; ++j)
#pragma unroll
    for (int mb = 0; mb < CP_MB; ++mb) {
      acc[mb][j] += f32x4{bv[j].x, bv[j].y, bv[j].z, bv[j].w};
      asm volatile("" : "+v"(acc[mb][j]));  // the adds stay out of the store branches
    }
  if constexpr (STATS) {
    // BatchNorm statistics of this tile's stored values (the next BatchNorm2d's training-mode batch
    // statistics, model_vit.py:24-27): per channel the sum and the sum of squares about the TILE
    // mean (two passes over the registers), merged across tiles by bn_merge_kernel (Chan et al.).
    // Channel c = 64 wn + 16 j + 4 (lane >> 4) + e of the tile sits in the 16 lanes of one lane
    // group and the 9 blocks mb of both row waves wm.
    float* red = (float*)smem;  // [2 passes][2 wm][256]
    __builtin_amdgcn_s_barrier();  // every wave is past its last fragment read of the stages
    const int nv = min(CP_BM, p.M - m0);
    float sm[CP_NB][4];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int j = 0; j < CP_NB; ++j) {
        float mu[4];
        if (pass) {
          const int c = wn * CP_WN + 16 * j + 4 * (lane >> 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) mu[e] = (red[c + e] + red[256 + c + e]) / (float)nv;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = 0.f;
#pragma unroll
          for (int mb = 0; mb < CP_MB; ++mb) {
            const int m = m0 + wm * CP_WM + 16 * mb + (lane & 15);
            const float v = acc[mb][j][e];
            const float d = pass ? v - mu[e] : v;
            t += m < p.M ? (pass ? d * d : d) : 0.f;
          }
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) t += __shfl_xor(t, o, 64);
          sm[j][e] = t;
        }
      }
      if (pass) __builtin_amdgcn_s_barrier();  // pass 0's sums read by every wave before reuse
      if ((lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < CP_NB; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) red[wm * 256 + wn * CP_WN + 16 * j + 4 * (lane >> 4) + e] = sm[j][e];
      }
      lds_barrier();
      if (threadIdx.x < 256 && n0 + (int)threadIdx.x < p.N)  // pass 0: tile sums, pass 1: centred squares
        p.stats[((long)tm * 2 + pass) * p.N + n0 + threadIdx.x] = red[threadIdx.x] + red[256 + threadIdx.x];
    }
  }
#pragma unroll
  for (int j = 0; j < CP_NB; ++j) {
    const int n = n0 + wn * CP_WN + 16 * j + 4 * (lane >> 4);
#pragma unroll
    for (int mb = 0; mb < CP_MB; ++mb) {
      const int m = m0 + wm * CP_WM + 16 * mb + (lane & 15);
      const f32x4 a = acc[mb][j];
      O* y = Y + (long)m * p.ldy + n;
      if (m < p.M && n < p.N) {
        if constexpr (sizeof(O) == 4) *(float4*)y = make_float4(a[0], a[1], a[2], a[3]);
        else *(uint2*)y = make_uint2(pk_bf16(a[0], a[1]), pk_bf16(a[2], a[3]));
      }
    }
  }
}

// ----------------------------------------------------------------------------- weight gradient
// dW[co][tap * Cin + ci] = sum_p dY[p][co] X[p shifted by tap][ci]  (f32 partial slab per split)
//
// Output tiles of 256 co x 256 (tap, ci), the pixel reduction split S ways so that tiles x S
// fills the 256 CUs once (512 -> 512 3x3: 36 tiles x 7). Both operands are pixel-major, so the
// K-step images are [64 pixels][256 columns] (two 128-column halves in the engine's MN layout,
// gemm_engine.h mn_off) read by transposing LDS reads (frag_mn) as 32x32x16 operands; 8 waves of
// 128 co x 64 columns (4 x 2 blocks). The map operand's columns are (tap, ci) chunks: each lane
// owns one chunk (its tap's shift) and four pixel rows, whose (y, x) advance by 64 pixels a step
// without divisions; padding taps and pixels past the split read the zero page.
constexpr int CW_BK = 64, CW_IMG = CW_BK * 256, CW_STAGE = 4 * CW_IMG;  // A halves | B halves: 64 KiB

struct CwArgs {
  const bf16* dy;
  long lddy;
  const bf16* x;
  long ldx;
  int H, W, Cin, ks, M, Cout, N;
  int tilesM, tilesN, kchunk;
  int qW, rW;  // 64 = qW * W + rW
  float* slab;
};

__global__ __launch_bounds__(512, 1) void conv_wgrad_panel_kernel(CwArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * CW_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), wm = wv >> 2, wn = wv & 3;
  const int tiles = p.tilesM * p.tilesN;
  const int flat = xcd_remap(blockIdx.x, gridDim.x);  // a split's tiles on one XCD: its pixel panels shared in L2
  const int split = flat / tiles, tile = flat - split * tiles;
  const int tm = tile / p.tilesN, tn = tile - tm * p.tilesN;
  const int m0 = tm * 256, n0 = tn * 256;
  const int kbeg = split * p.kchunk, kend = min(p.M, kbeg + p.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + CW_BK - 1) / CW_BK : 0;
  const int pad = p.ks >> 1;

  // this wave's 4 pieces of each image: half h = wv >> 2, rows r_i = 16 (wv & 3) + 4 i + (lane >> 4),
  // source chunk c (the same for the four rows: (r_i & 3) = (lane >> 4) & 3)
  const int h = wv >> 2;
  const int c = (lane & 15) ^ (((lane >> 4) & 3) << 2);
  const int co = min(m0 + h * 128 + c * 8, p.Cout - 8);
  const int n = min(n0 + h * 128 + c * 8, p.N - 8);
  const int tap = n / p.Cin, ci = n - tap * p.Cin;
  const int ky = tap / p.ks;
  const int dy = ky - pad, dx = tap - ky * p.ks - pad;
  const long xshift = (long)(dy * p.W + dx) * p.ldx + ci;
  unsigned voffa[4];
  int py[4], px[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 16 * (wv & 3) + 4 * i + (lane >> 4);
    voffa[i] = 2u * (unsigned)(r * (int)p.lddy + co);
    const int pp = min(kbeg + r, p.M - 1);
    px[i] = pp % p.W;
    py[i] = (pp / p.W) % p.H;
  }
  auto issue = [&](int kt, int s) {
    char* sa = smem + s * CW_STAGE + h * CW_IMG + (wv & 3) * 4096;
    char* sb = sa + 2 * CW_IMG;
    const int k0 = kbeg + kt * CW_BK;
    if (k0 + CW_BK <= kend) {
      const char* ab = uniform_ptr(p.dy + (long)k0 * p.lddy);
#pragma unroll
      for (int i = 0; i < 4; ++i) glds_s<false>(voffa[i], ab, sa + i * 1024);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pix = k0 + 16 * (wv & 3) + 4 * i + (lane >> 4);
        const void* src = pix < kend ? (const void*)(p.dy + (long)pix * p.lddy + co) : (const void*)cp_zero16;
        glds_v<false>(src, sa + i * 1024);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pix = k0 + 16 * (wv & 3) + 4 * i + (lane >> 4);
      const bool ok = pix < kend && (unsigned)(py[i] + dy) < (unsigned)p.H && (unsigned)(px[i] + dx) < (unsigned)p.W;
      const void* src = ok ? (const void*)(p.x + ((long)pix * p.ldx + xshift)) : (const void*)cp_zero16;
      glds_v<false>(src, sb + i * 1024);
      // advance the row's pixel by one K step (64 = qW * W + rW)
      int xx = px[i] + p.rW, yy = py[i] + p.qW;
      if (xx >= p.W) { xx -= p.W; ++yy; }
      while (yy >= p.H) yy -= p.H;
      px[i] = xx;
      py[i] = yy;
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // one barrier per K tile (as conv_panel_kernel)
    __builtin_amdgcn_s_barrier();
    if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
    const char* ia = smem + cur * CW_STAGE + wm * CW_IMG;             // this wave's 128 co
    const char* ib = smem + cur * CW_STAGE + (2 + (wn >> 1)) * CW_IMG; // its 64 columns' half
    const int cb = (wn & 1) * 64;
    bf16x8 fa[2][4], fb[2][2];
    auto ldf = [&](int t, bf16x8 (&xa)[4], bf16x8 (&xb)[2]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) xa[i] = frag_mn(ia, 16 * t, 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) xb[j] = frag_mn(ib, 16 * t, cb + 32 * j, lane);
    };
    ldf(0, fa[0], fb[0]);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < 3) ldf(t + 1, fa[(t + 1) & 1], fb[(t + 1) & 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[t & 1][i], fb[t & 1][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // partial tile -> slab[split][co][n]: col = lane & 31 (n), row = (r & 3) + 8 (r >> 2) + 4 hl (co)
  float* slab = p.slab + (long)split * p.Cout * p.N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 128 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (row < p.Cout && col < p.N) slab[(long)row * p.N + col] = acc[i][j][r];
      }
    }
}

// BatchNorm batch statistics from the per-tile (sum, centred sum of squares) of conv_panel_kernel:
// Chan et al.'s pairwise update, 16 phases per channel (tiles t = ph, ph + 16, ...) then the 16 phase
// results in order — a fixed order (deterministic). Then as bn_var_kernel: invstd = 1/sqrt(var + eps)
// (biased variance), running mean / unbiased running variance with the momentum.
__global__ __launch_bounds__(1024) void bn_merge_kernel(const float* __restrict__ stats, int T, long M, int C,
                                                       float* mean, float* invstd, float* run_mean, float* run_var,
                                                       float mom, float eps) {
  __shared__ float sn[16][64], smu[16][64], sm2[16][64];
  const int lc = threadIdx.x & 63, ph = threadIdx.x >> 6, c = blockIdx.x * 64 + lc;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (c < C) {
    for (int t = ph; t < T; t += 16) {
      const float nb = (float)min((long)CP_BM, M - (long)t * CP_BM);
      const float mb = stats[(long)t * 2 * C + c] / nb, q = stats[((long)t * 2 + 1) * C + c];
      const float nn = n + nb, d = mb - mu;
      mu += d * (nb / nn);
      m2 += q + d * d * (n * nb / nn);
      n = nn;
    }
  }
  sn[ph][lc] = n;
  smu[ph][lc] = mu;
  sm2[ph][lc] = m2;
  __syncthreads();
  if (ph == 0 && c < C) {
    n = sn[0][lc];
    mu = smu[0][lc];
    m2 = sm2[0][lc];
    for (int k = 1; k < 16; ++k) {
      const float nb = sn[k][lc];
      if (nb <= 0.f) continue;
      const float nn = n + nb, d = smu[k][lc] - mu;
      mu += d * (nb / nn);
      m2 += sm2[k][lc] + d * d * (n * nb / nn);
      n = nn;
    }
    const float var = m2 / (float)M;
    mean[c] = mu;
    invstd[c] = 1.0f / sqrtf(var + eps);
    if (run_mean) run_mean[c] = (1.f - mom) * run_mean[c] + mom * mu;
    if (run_var) run_var[c] = (1.f - mom) * run_var[c] + mom * (M > 1 ? m2 / (float)(M - 1) : var);
  }
}

// dgrad weights: Bt[ci][(ky', kx'), co] = w[co][ci][ks-1-ky'][ks-1-kx']  (torch f32 layout in); Cpad >= Cout
// channels per row, zero for co >= Cout (the pack of a gradient zero-padded to Cpad channels)
template <typename O>
__global__ void pack_conv_t_kernel(const float* __restrict__ w, long Cout, long Cin, long ks, long Cpad, O* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = Cin * ks * ks * Cpad;
  if (i >= n) return;
  const long co = i % Cpad, t = i / Cpad, tap = t % (ks * ks), ci = t / (ks * ks);
  const long ky = ks - 1 - tap / ks, kx = ks - 1 - tap % ks;
  out[i] = co < Cout ? from_f32<O>(w[((co * Cin + ci) * ks + ky) * ks + kx]) : from_f32<O>(0.f);
}

}  // namespace

bool conv_panel_enabled() { return ivit_knob(IVIT_KNOB_CONV_PANEL) != 0; }

bool conv_panel_ok(long M, long N, long Cin, long lda, long ks) {
  return M >= CP_BM && N >= 128 && N % 8 == 0 && Cin % 64 == 0 && lda % 8 == 0 && (ks == 1 || ks == 3 || ks == 5) &&
         M * lda + 64 < 0x7fffffffL && N * ks * ks * Cin < 0x3fffffffL;
}

int conv_wgrad_panel_splits(long M, long Cout, long N) {
  if (M <= 0 || Cout <= 0 || N <= 0) return 1;
  const long tiles = (long)ivit_cdiv(Cout, 256) * ivit_cdiv(N, 256);
  long s = 256 / tiles;
  const long steps = (M + CW_BK - 1) / CW_BK;
  if (s > steps / 4) s = steps / 4;  // at least ~4 K steps per workgroup
  return s < 1 ? 1 : (int)s;
}

bool conv_wgrad_panel_ok(long M, long Cout, long Cin, long ks, long lddy) {
  return M >= 256 && Cout >= 128 && Cout % 8 == 0 && Cin % 8 == 0 && lddy % 8 == 0 && (ks == 1 || ks == 3 || ks == 5) &&
         ks * ks * Cin >= 128 && M * lddy < 0x7fffffffL && M * Cin < 0x7fffffffL;
}

int conv_wgrad_panel_launch(const bf16* dY, long lddy, const bf16* X, int Bn, int H, int W, int Cin, int Cout, int ks,
                            float* slab, int splits, hipStream_t st) {
  const int M = Bn * H * W, N = ks * ks * Cin;
  const long steps = (M + CW_BK - 1) / CW_BK;
  CwArgs p{dY, lddy, X, Cin, H, W, Cin, ks, M, Cout, N, ivit_cdiv(Cout, 256), ivit_cdiv(N, 256),
           (int)((steps + splits - 1) / splits) * CW_BK, 64 / W, 64 % W, slab};
  hipLaunchKernelGGL(conv_wgrad_panel_kernel, dim3(p.tilesM * p.tilesN * splits), dim3(512), 0, st, p);
  return 0;
}

int conv_panel_launch(const bf16* A, long lda, int Bn, int H, int W, int Cin, int ks, const bf16* Bk, int N,
                      const float* bias, void* Y, long ldy, bool y_bf16, hipStream_t st, float* stats) {
  const int M = Bn * H * W;
  CpArgs p{A, lda, H, W, Cin, ks, M, Bk, N, ks * ks * Cin, bias, Y, ldy, ivit_cdiv(N, CP_BN), stats};
  const dim3 grid(ivit_cdiv(M, CP_BM) * p.tilesN);
  if (stats) {
    if (y_bf16)
      hipLaunchKernelGGL((conv_panel_kernel<bf16, true>), grid, dim3(512), 0, st, p);
    else
      hipLaunchKernelGGL((conv_panel_kernel<float, true>), grid, dim3(512), 0, st, p);
  } else if (y_bf16) {
    hipLaunchKernelGGL((conv_panel_kernel<bf16, false>), grid, dim3(512), 0, st, p);
  } else {
    hipLaunchKernelGGL((conv_panel_kernel<float, false>), grid, dim3(512), 0, st, p);
  }
  return 0;
}

long conv_panel_stats_floats(long M, long N) { return (long)ivit_cdiv(M, CP_BM) * 2 * N; }

}  // namespace ivit

using namespace ivit;

extern "C" int ivit_pack_conv_weight_t(int dtype, const float* w, long Cout, long Cin, long ks, long Cout_pad, void* out,
                                       void* stream) {
  IVIT_CHECK_ARG(Cout_pad >= Cout && Cout > 0, "ivit_pack_conv_weight_t: Cout_pad < Cout");
  hipStream_t st = ivit_stream(stream);
  const long n = Cin * ks * ks * Cout_pad;
  if (dtype == IVIT_BF16)
    hipLaunchKernelGGL(pack_conv_t_kernel<bf16>, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, w, Cout, Cin, ks, Cout_pad,
                       (bf16*)out);
  else
    hipLaunchKernelGGL(pack_conv_t_kernel<float>, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, w, Cout, Cin, ks, Cout_pad,
                       (float*)out);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_conv_dgrad_t(int dtype, const void* dY, long lddy, long B, long H, long W, long Cout,
                                 const void* WpT, long Cin, long ks, void* dX, int dx_dtype, void* stream) {
  IVIT_CHECK_ARG(dtype == IVIT_BF16, "ivit_conv_dgrad_t: bf16 only");
  IVIT_CHECK_ARG(conv_panel_ok(B * H * W, Cin, Cout, lddy, ks), "ivit_conv_dgrad_t: shape not supported");
  hipStream_t st = ivit_stream(stream);
  conv_panel_launch((const bf16*)dY, lddy, (int)B, (int)H, (int)W, (int)Cout, (int)ks, (const bf16*)WpT, (int)Cin,
                    nullptr, dX, Cin, dx_dtype == IVIT_BF16, st);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" long ivit_conv_bn_fwd_workspace(long B, long H, long W, long Cout) {
  const long M = B * H * W;
  const long a = conv_panel_stats_floats(M, Cout) * 4, b = ivit_bn_workspace(M, Cout);
  return a > b ? a : b;
}

extern "C" int ivit_conv_bn_fwd(int dtype, const void* X, long B, long H, long W, long Cin, const void* Wp, long Cout,
                                long ks, void* Y, long ldy, int y_dtype, float* mean, float* invstd, float* run_mean,
                                float* run_var, float momentum, float eps, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(work_bytes >= ivit_conv_bn_fwd_workspace(B, H, W, Cout), "ivit_conv_bn_fwd: workspace too small");
  IVIT_CHECK_ARG(ldy == Cout, "ivit_conv_bn_fwd: the output must be dense (ldy == Cout)");
  hipStream_t st = ivit_stream(stream);
  const long M = B * H * W;
  if (dtype == IVIT_BF16 && conv_panel_enabled() && conv_panel_ok(M, Cout, Cin, Cin, ks) && ldy % 4 == 0) {
    float* stats = (float*)work;
    conv_panel_launch((const bf16*)X, Cin, (int)B, (int)H, (int)W, (int)Cin, (int)ks, (const bf16*)Wp, (int)Cout,
                      nullptr, Y, ldy, y_dtype == IVIT_BF16, st, stats);
    IVIT_LAUNCH_CHECK();
    hipLaunchKernelGGL(bn_merge_kernel, dim3(ivit_cdiv(Cout, 64)), dim3(1024), 0, st, stats, ivit_cdiv(M, CP_BM), M,
                       (int)Cout, mean, invstd, run_mean, run_var, momentum, eps);
    IVIT_LAUNCH_CHECK();
    return 0;
  }
  int rc = ivit_conv_fwd(dtype, X, B, H, W, Cin, Wp, nullptr, Cout, ks, Y, ldy, y_dtype, stream);
  if (rc) return rc;
  return ivit_bn_stats(Y, y_dtype, M, Cout, mean, invstd, run_mean, run_var, momentum, eps, work, work_bytes, stream);
}
