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
// Workgroup: 4 compute waves + 4 loader waves (below), K step 32 tokens, 4 LDS stages (32 KiB
// each: the dY block's 128 columns and the X block's 384 columns as token-major 256-B-row images),
// three steps in flight by LDS-DMA, one barrier per step. Both operands are read by transposing
// LDS reads. Rounds 3-4 ran 8 compute waves (64 x 96 each, two per SIMD in lock step, the bias as
// an extra MFMA against a ones operand) + 4 loaders: 175-176 us isolated vs 158-169 us for this
// form (profiles/r05_l_*); the dedicated loader waves themselves came from the round-3 anatomy
// (every wave issuing its own pieces: DMA skeleton 112 us + MFMA-only 105 us -> 206 us together,
// an LDS-DMA piece costing its wave ~100-185 cycles beside MFMAs).
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

// MODE (anatomy builds: -DIVIT_WB_ANATOMY=MODE via tools/ab_build.sh; timing only): 0 product, 1 no
// MFMAs (the DMA / barrier skeleton), 2 no DMA after the prologue (MFMAs on stale stages), 3 the
// product kernel without the reduce launch.
#ifndef IVIT_WB_ANATOMY
#define IVIT_WB_ANATOMY 0
#endif
// Wave-specialised form (round 5): waves 0-3 compute, one per SIMD, each the tile's 128 rows x 96
// columns (4 x 3 blocks of v_mfma_f32_32x32x16_bf16, 192 accumulator VGPRs); waves 4-7 load (the
// same 32 LDS-DMA pieces per step) and also sum the dY block's columns for the bias (VALU on the
// landed image; those waves idle otherwise), so the compute waves hold no bias accumulator.
// Fragment reads run one substep ahead of the MFMAs across the step boundary: the step's barrier
// sits between its two substeps' MFMA groups, after the compute waves' reads of the stage are
// complete, so the next stage's first fragments are read while the current stage's second MFMA
// group runs. wgrad_block_kernel's anatomy (MFMA side alone 144 us against a 64-us floor) was
// the read latency exposed after each step's barrier, at 2 waves per SIMD in lock step.
// Barriers: B_0 publishes step 0; B_j (j = 1 .. nk) publishes step j and certifies that every
// compute wave has read stage j - 1 completely, which the loaders then refill with step j + 3.
template <int MODE>
__global__ __launch_bounds__(512, 1) void wgrad_block_kernel(const WbArgs args) {
  __shared__ __attribute__((aligned(16))) char smem[WB_NS * WB_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = args.tile_base[4];
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
  const bool dob = tn == 0 && args.bslab != nullptr;

  if (wv >= 4) {  // ---------------------------------------------------------------- loader
    const bf16* Abase = g.dy + tm * WB_TM;
    const bf16* Bbase = g.x + tn * WB_TN;
    const int lda = g.N, ldb = g.K;
    const int lw = wv - 4;
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
    const bool isa = lw == 0;
    auto issue = [&](int stage, int k0) {
      char* st = smem + stage * WB_STAGE + lw * 8192;
      if (k0 + WB_BK <= kend) {
        const char* sb = isa ? uniform_ptr(Abase + (long)k0 * lda) : uniform_ptr(Bbase + (long)k0 * ldb);
#pragma unroll
        for (int i = 0; i < 8; ++i) glds_s<false>(voff[i], sb, st + i * 1024);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int t = k0 + prow[i];
          const void* src = t < kend ? (const void*)((isa ? Abase + (long)t * lda : Bbase + (long)t * ldb) + pcol[i])
                                     : (const void*)g_zero16;
          glds<16>(src, st + i * 1024);
        }
      }
    };
    // bias: column 32 lw + (lane & 31) of the dY block, tokens 16 hl .. 16 hl + 15 of each step
    const int bcol = 32 * lw + (lane & 31);
    int boff[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 16 * hl + r;
      boff[r] = row * 256 + (((bcol >> 3) ^ ((row & 3) << 2)) << 4) + (bcol & 7) * 2;
    }
    float bsum = 0.f;
    auto bias = [&](int stage) {
      const char* im = smem + stage * WB_STAGE;
#pragma unroll
      for (int r = 0; r < 16; ++r) bsum += __uint_as_float((unsigned)*(const unsigned short*)(im + boff[r]) << 16);
    };
    auto wait_step = [&](int j) {  // step j landed; steps j+1, j+2 (those issued) stay in flight
      const int after = (j + 1 < nk ? 8 : 0) + (j + 2 < nk ? 8 : 0);
      if (after == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (after == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
#pragma unroll
    for (int s = 0; s < WB_NS - 1; ++s)
      if (s < nk) issue(s, kbeg + s * WB_BK);
    wait_step(0);
    __builtin_amdgcn_s_barrier();  // B_0
    if (3 < nk) issue(3, kbeg + 3 * WB_BK);
    if (dob) bias(0);
    for (int j = 1; j <= nk; ++j) {
      if (j < nk) wait_step(j);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // my bias reads of stage j - 1 are done
      __builtin_amdgcn_s_barrier();  // B_j
      if (MODE != 2 && j + 3 < nk) issue((j + 3) % WB_NS, kbeg + (j + 3) * WB_BK);
      if (dob && j < nk) bias(j % WB_NS);
    }
    if (dob) {
      float* bs = args.bslab + ((long)split * 2 + hl) * args.bias_n + g.bias_off;
      bs[tm * WB_TM + bcol] = bsum;
    }
    return;
  }

  // ------------------------------------------------------------------------------------ compute
  const int cw = wv;  // columns 96 cw .. 96 cw + 95 of the X block
  f32x16 acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  struct Frags { bf16x8 a[4], b[3]; };
  // frag_mn's addresses, factored: the 32-column block m of an image is at lane offset
  // lc + 64 (m ^ q) (the row swizzle 4 (r & 3) only touches the chunk bits m covers); lc and q are
  // laundered per load set so the compiler forms the 7 offsets there instead of holding them
  // (at 192 accumulators + two fragment sets the held offsets spilled)
  const int fq = (lane >> 2) & 3;
  const int flc = (8 * (lane >> 5) + fq) * 256 + 32 * ((lane >> 4) & 1) + 16 * ((lane & 3) >> 1) + (lane & 1) * 8;
  auto load = [&](Frags& f, int stage, int t) {
    int q = fq, lc = flc;
    asm volatile("" : "+v"(q), "+v"(lc));
    const char* st = smem + stage * WB_STAGE + 4096 * t;
    auto rd = [&](const char* img, int m) {
      const char* a = img + lc + 64 * (m ^ q);
      union { s16x4 s[2]; bf16x8 v; } u;
      u.s[0] = ds_tr(a);
      u.s[1] = ds_tr(a + 1024);
      return u.v;
    };
#pragma unroll
    for (int i = 0; i < 4; ++i) f.a[i] = rd(st, i);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int cb = 96 * cw + 32 * j;
      f.b[j] = rd(st + WB_IMG * (1 + (cb >> 7)), (cb & 127) >> 5);
    }
  };
  auto mma = [&](const Frags& f) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (MODE != 1) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[i], f.b[j], acc[i][j], 0, 0, 0);
  };
  Frags f0, f1;
  __builtin_amdgcn_s_barrier();  // B_0
  load(f0, 0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    load(f1, kt % WB_NS, 1);
    mma(f0);
    // the scheduler must not move MFMAs across the barrier (it sank 9 of mma(f0)'s 12 below it,
    // which left f1's reads 3 MFMAs to land before the lgkmcnt(0))
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // stage kt fully read
    __builtin_amdgcn_s_barrier();                        // B_{kt+1}
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) load(f0, (kt + 1) % WB_NS, 0);
    mma(f1);
    __builtin_amdgcn_sched_barrier(0);
  }

  // the lane's slab offset laundered here, so that the store addresses are formed after the loop
  int lo = 4 * hl * g.K + (lane & 31);
  asm volatile("" : "+v"(lo));
  float* slab = args.slab + (long)split * args.slab_n + g.slab_off + (long)(tm * WB_TM) * g.K + tn * WB_TN + 96 * cw + lo;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) slab[(long)(32 * i + (r & 3) + 8 * (r >> 2)) * g.K + 32 * j] = acc[i][j][r];
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
  hipLaunchKernelGGL(wgrad_block_kernel<IVIT_WB_ANATOMY>, dim3(args.tile_base[4] * S), dim3(512), 0, st, args);
  IVIT_LAUNCH_CHECK();
  if (IVIT_WB_ANATOMY == 3) return 0;  // anatomy 3: the product kernel without its reduce (timing only)
  hipLaunchKernelGGL(wgrad_block_reduce_kernel, dim3(ivit_cdiv((off + boff) / 4, 256)), dim3(256), 0, st, args.slab,
                     args.bslab, out, S);
  IVIT_LAUNCH_CHECK();
  return 0;
}
