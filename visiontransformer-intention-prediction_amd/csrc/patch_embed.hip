// Fused bf16 patch embedding (timm PatchEmbed, Conv2d k = s = 8) over an f32 NCHW BEV raster:
//
//   x[b, 1 + p, n] = sum_{c, ky, kx} img[b, c, 8 gy + ky, 8 gx + kx] * W[n, c, ky, kx] + bias[n] + pos[1 + p, n]
//
// one pass, no im2col buffer (north_star: "a fused Conv2d patch-embed with coalesced HBM reads of
// the multi-channel BEV grid into LDS tiles"). The raster is the only large operand (LiDAR:
// 8 x 290 x 400 x 720 f32 = 2.67 GB, read once); the weight (D x 64C bf16, 14 MB) is re-read by
// every workgroup from L2.
//
// Workgroup = 144 consecutive patches (9 MFMA row blocks of 16; 36 000 LiDAR patches = 250
// workgroups, one per CU) x ALL D output columns, so each raster byte is fetched exactly once.
// K loop = one input channel (8 x 8 taps = 64 k) per stage:
//   * A (raster): LDS-DMA of raw f32 into a 3-stage ring, 36 KiB per stage, two stages in flight
//     (72 KiB of HBM reads per CU, the depth the guide measures for ~6 TB/s streaming). A stage is
//     [ky][patch][8 kx] — 32-byte records, consecutive lanes fetch consecutive 16-B halves so each
//     DMA wave-instruction reads one contiguous 1 KiB run of raster rows; the two halves of a
//     record swap places on every other 8-record group, which makes the MFMA operand reads
//     (16 patches x 16 B per lane group) bank-conflict-free. f32 -> bf16 happens in the operand
//     read (4 v_cvt_pk_bf16_f32 per fragment).
//   * B (weight): pre-packed in MFMA fragment order (ivit_patch_weight_pack), loaded straight into
//     VGPRs one stage ahead — 1 KiB contiguous per wave-instruction.
//   * 4 waves, wave w owns output columns [w D/4, (w+1) D/4): 9 x (D/64) accumulators of
//     v_mfma_f32_16x16x32_bf16 (216 AGPRs at D = 384).
// Every memory operation of the loop is inline asm retired by counted vmcnt waits: the compiler's
// waitcnt pass cannot see the DMAs, and a compiler-placed wait on a register load would drain the
// in-flight raster stages (the counter retires in issue order). Issue order per stage kt-1 ->
// kt: B(kt), then A(kt+1), so waiting for B(kt) leaves A(kt+1) in flight (vmcnt(9)).
#include "patch_embed.h"
#include "panel_common.h"

#include <type_traits>

namespace ivit {
namespace {

constexpr int PE_MT = 144;                    // patches per workgroup
constexpr int PE_MB = PE_MT / 16;             // 16-row MFMA blocks
constexpr int PE_STAGE = PE_MT * 8 * 32;      // bytes per LDS stage: [ky 8][patch][32 B]
constexpr int PE_NS = 3;                      // f32 LDS stages (raster DMA ring)
constexpr int PE_BSTAGE = PE_MT * 8 * 16;     // bf16 operand stage: [ky 8][patch][16 B]
constexpr int PE_PIECES = PE_STAGE / 1024;    // 1-KiB DMA pieces per stage (36)

IVIT_DEV bf16x8 cvt8(const float4 a, const float4 b) {
  Pack8 p;
  p.u = f32x8_to_bf16x8(a, b);
  return p.v;
}

// NW waves = D / 48 (8 at D = 384: two per SIMD; 4 at D = 192).
//
// Pipeline, iteration kt (one input channel): the raster of channels kt+1 .. kt+3 and the weight
// fragments of kt+1 .. kt+2 are in flight or landed. Each wave converts ITS OWN landed f32
// pieces of channel kt+1 to bf16 (its own DMA data needs no barrier), which frees its f32 region
// for channel kt+4 at once — three raster stages (108 KiB per CU) stay in flight while the
// MFMAs of channel kt read the bf16 image the whole workgroup converted one iteration earlier.
// vmcnt retires in issue order, so weights are issued two channels ahead, between the raster
// stages they must not drain: ... A(kt+1) B(kt) A(kt+2) B(kt+1) A(kt+3) | B(kt+2) A(kt+4).
template <int NW>
__global__ __launch_bounds__(64 * NW, 1) void patch_fwd_kernel(const float* __restrict__ img, int C, int H, int W,
                                                           int Wp, int Np, int M, const u32x4* __restrict__ wpack,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ pos, int D,
                                                           float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char smem[PE_NS * PE_STAGE + 2 * PE_BSTAGE];
  char* const bimg = smem + PE_NS * PE_STAGE;  // two bf16 stages [ky][patch][8 kx]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * PE_MT;
  const long HW = (long)H * W;

  // pieces of a stage per wave: 36 / NW, the first 36 % NW waves one more
  constexpr int PW = (PE_PIECES + NW - 1) / NW, PREM = PE_PIECES % NW;
  const int npc = (PREM == 0 || wv < PREM) ? PW : PW - 1;
  const int pc0 = (PREM == 0 || wv < PREM) ? wv * PW : PREM * PW + (wv - PREM) * (PW - 1);
  // per-lane DMA sources: piece q covers records 32q .. 32q+31 (record = (ky, patch)); byte
  // offsets from the first image of the tile at channel c (the host checks they fit 32 bits)
  const int b0 = m0 / Np;
  unsigned voff[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int rec = min(pc0 + i, PE_PIECES - 1) * 32 + (lane >> 1);
    const int ky = rec / PE_MT, p = rec - ky * PE_MT;
    const int half = (lane & 1) ^ ((rec >> 3) & 1);  // stored position (lane & 1) holds this half
    const int m = min(m0 + p, M - 1);                // rows past M are computed, never stored
    const int b = m / Np, pi = m - b * Np, gy = pi / Wp, gx = pi - gy * Wp;
    voff[i] = (unsigned)((((long)(b - b0) * C * H + gy * 8 + ky) * W + gx * 8 + half * 4) * 4);
  }
  const float* img0 = img + (long)b0 * C * HW;
  char* const freg = smem + pc0 * 1024;  // this wave's pieces inside each f32 stage
  auto issue_a = [&](int c) {
    char* st = freg + (c % PE_NS) * PE_STAGE;
    const char* sb = uniform_ptr(img0 + c * HW);
#pragma unroll
    for (int i = 0; i < PW; ++i)
      if (i < npc) glds_s(voff[i], sb, st + i * 1024);
  };
  // own pieces of channel c (landed) -> bf16 stage (c & 1): lane l of piece q holds half h of
  // record 32q + (l >> 1); it writes those 4 kx as 8 bytes of the 16-B bf16 record
  auto convert = [&](int c) {
    const char* fs = freg + (c % PE_NS) * PE_STAGE + lane * 16;
    char* bs = bimg + (c & 1) * PE_BSTAGE;
    float4 v[PW];
#pragma unroll
    for (int i = 0; i < PW; ++i)
      if (i < npc) v[i] = *(const float4*)(fs + i * 1024);
#pragma unroll
    for (int i = 0; i < PW; ++i)
      if (i < npc) {
        const int rec = (pc0 + i) * 32 + (lane >> 1);
        const int half = (lane & 1) ^ ((rec >> 3) & 1);
        *(uint2*)(bs + rec * 16 + half * 8) = make_uint2(pk_bf16(v[i].x, v[i].y), pk_bf16(v[i].z, v[i].w));
      }
  };
  // weight fragments: wpack[s][nb][lane] (16 B), s = 32-k step, nb = 16-column block; the wave's
  // NBW blocks of a step are NBW contiguous KiB
  const int NB16 = D / 16;
  const unsigned vb = lane * 16;
  auto issue_b = [&](int c, u32x4 (&r)[2 * NBW]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const char* sb = uniform_ptr(wpack + ((long)(2 * c + t) * NB16 + wv * NBW) * 64);
      gload_b128<0>(r[t * NBW + 0], vb, sb);
      gload_b128<1024>(r[t * NBW + 1], vb, sb);
      gload_b128<2048>(r[t * NBW + 2], vb, sb);
    }
  };

  f32x4 acc[PE_MB][NBW];
#pragma unroll
  for (int i = 0; i < PE_MB; ++i)
#pragma unroll
    for (int j = 0; j < NBW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 breg[3][2 * NBW];
  // operand read: lane group g = lane >> 4 takes ky = 4t + g, patches 16 mb + (lane & 15)
  const int rl = ((lane >> 4) * PE_MT + (lane & 15)) * 16;

  auto stage = [&](int kt, u32x4 (&cur)[2 * NBW], u32x4 (&nb2)[2 * NBW]) {
    // outstanding after A(kt+1), B(kt): A(kt+2), B(kt+1), A(kt+3) (those that exist)
    const bool a2 = kt + 2 < C, a3 = kt + 3 < C, b1 = kt + 1 < C;
    wait_vm((a2 ? npc : 0) + (b1 ? 2 * NBW : 0) + (a3 ? npc : 0));
    tie(cur);
    __builtin_amdgcn_s_barrier();  // bf16 stage kt&1 complete; bf16 stage (kt+1)&1 free
    if (kt + 2 < C) issue_b(kt + 2, nb2);
    // operand fragments f = 0..17 (t = f / 9: 32-k step, mb = f % 9: row block) are read three
    // ahead of their MFMAs; sched barriers pin that distance (the scheduler otherwise sinks each
    // read next to its use and every pair of fragments waits out the LDS latency). The wave's
    // own raster pieces of channel kt+1 are converted after the first fragments' MFMAs are
    // queued, then its f32 region is refilled with channel kt+4.
    const char* ia = bimg + (kt & 1) * PE_BSTAGE + rl;
    auto rdf = [&](int f) { return *(const bf16x8*)(ia + (4 * (f / PE_MB) * PE_MT + 16 * (f % PE_MB)) * 16); };
    bf16x8 fr[4];
    fr[0] = rdf(0);
    fr[1] = rdf(1);
    fr[2] = rdf(2);
#pragma unroll
    for (int f = 0; f < 2 * PE_MB; ++f) {
      const int t = f / PE_MB, mb = f % PE_MB;
      if (f + 3 < 2 * PE_MB) fr[(f + 3) % 4] = rdf(f + 3);
#pragma unroll
      for (int j = 0; j < NBW; ++j) {
        union { u32x4 u; bf16x8 v; } bw;
        bw.u = cur[t * NBW + j];
        acc[mb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[f % 4], bw.v, acc[mb][j], 0, 0, 0);
      }
      if (f == 1 && kt + 1 < C) {
        convert(kt + 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // f32 region read before it is refilled
        if (kt + 4 < C) issue_a(kt + 4);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // my reads of bf16 stage kt are done
  };

  // prologue: A(0) landed and converted; then A(1) B(0) A(2) B(1) A(3) in flight (the invariant)
  issue_a(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  convert(0);
  if (C > 1) issue_a(1);
  issue_b(0, breg[0]);
  if (C > 2) issue_a(2);
  if (C > 1) issue_b(1, breg[1]);
  if (C > 3) issue_a(3);
  for (int kt = 0; kt < C; kt += 3) {
    stage(kt, breg[0], breg[2]);
    if (kt + 1 < C) stage(kt + 1, breg[1], breg[0]);
    if (kt + 2 < C) stage(kt + 2, breg[2], breg[1]);
  }

  // epilogue: lane holds rows 4(lane>>4) + i of each 16-row block, column 16 nb + (lane & 15)
  float bv[NBW];
#pragma unroll
  for (int j = 0; j < NBW; ++j) bv[j] = bias[(wv * NBW + j) * 16 + (lane & 15)];
#pragma unroll
  for (int mb = 0; mb < PE_MB; ++mb) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + 16 * mb + 4 * (lane >> 4) + i;
      if (m >= M) continue;
      const int b = m / Np, p = m - b * Np;
      const float* pr = pos + (long)(1 + p) * D;
      float* orow = out + ((long)b * (Np + 1) + 1 + p) * D;
#pragma unroll
      for (int j = 0; j < NBW; ++j) {
        const int n = (wv * NBW + j) * 16 + (lane & 15);
        orow[n] = acc[mb][j][i] + bv[j] + pr[n];
      }
    }
  }
}

// W [D][K] f32 (K = 64 C) -> wpack[s][nb][lane][8] bf16: lane l of 16-column block nb at 32-k
// step s holds W[16 nb + (l & 15)][32 s + 8 (l >> 4) + 0..7] (the 16x16x32 B operand).
__global__ __launch_bounds__(256) void patch_pack_kernel(const float* __restrict__ w, long D, long K,
                                                         uint4* __restrict__ wp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long NB16 = D / 16, total = (K / 32) * NB16 * 64;
  if (i >= total) return;
  const int lane = (int)(i & 63);
  const long snb = i >> 6, s = snb / NB16, nb = snb - s * NB16;
  const float* q = w + (nb * 16 + (lane & 15)) * K + s * 32 + 8 * (lane >> 4);
  wp[i] = f32x8_to_bf16x8(*(const float4*)q, *(const float4*)(q + 4));
}

// W [K][N] f32 (a dgrad operand, e.g. fc1.weight [1536][384]) packed as its transpose [N][K].
__global__ __launch_bounds__(256) void pack_t_kernel(const float* __restrict__ w, long K, long N, uint4* __restrict__ wp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long NB16 = N / 16, total = (K / 32) * NB16 * 64;
  if (i >= total) return;
  const int lane = (int)(i & 63);
  const long snb = i >> 6, s = snb / NB16, nb = snb - s * NB16;
  const long n = nb * 16 + (lane & 15), k0 = s * 32 + 8 * (lane >> 4);
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = w[(k0 + e) * N + n];
  wp[i] = make_uint4(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]), pk_bf16(v[4], v[5]), pk_bf16(v[6], v[7]));
}

// Every pack of a list in one launch (FusedAdamW's refresh after the update): blockIdx.y = pack;
// tr = 0: W [rows][cols] -> the patch_pack_kernel layout, 1: W [rows = K][cols = N] -> the
// pack_t_kernel layout of W^T.
struct PackJob {
  const float* w;
  uint4* wp;
  long rows, cols;
  int tr;
};
__global__ __launch_bounds__(256) void multi_pack_kernel(const PackJob* __restrict__ jobs) {
  const PackJob j = jobs[blockIdx.y];
  const long total = j.rows * j.cols / 8;  // uint4 outputs
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int lane = (int)(i & 63);
    const long snb = i >> 6;
    if (!j.tr) {  // D = rows, K = cols
      const long NB16 = j.rows / 16, s = snb / NB16, nb = snb - s * NB16;
      const float* q = j.w + (nb * 16 + (lane & 15)) * j.cols + s * 32 + 8 * (lane >> 4);
      j.wp[i] = f32x8_to_bf16x8(*(const float4*)q, *(const float4*)(q + 4));
    } else {  // K = rows, N = cols
      const long NB16 = j.cols / 16, s = snb / NB16, nb = snb - s * NB16;
      const long n = nb * 16 + (lane & 15), k0 = s * 32 + 8 * (lane >> 4);
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = j.w[(k0 + e) * j.cols + n];
      j.wp[i] = make_uint4(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]), pk_bf16(v[4], v[5]), pk_bf16(v[6], v[7]));
    }
  }
}

__global__ void patch_cls_kernel(float* out, long B, long Ntok, long D, const float* cls, const float* pos) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * D) return;
  const long b = i / D, d = i - b * D;
  out[b * Ntok * D + d] = cls[d] + pos[d];
}

}  // namespace
}  // namespace ivit

using namespace ivit;

extern "C" long ivit_patch_weight_pack_bytes(long D, long C) { return D * C * 64 * 2; }

extern "C" int ivit_patch_weight_pack(const float* w, long D, long C, void* wpack, void* stream) {
  IVIT_CHECK_ARG(D > 0 && D % 16 == 0 && C > 0, "ivit_patch_weight_pack: D must be a positive multiple of 16");
  const long K = C * 64, n = (K / 32) * (D / 16) * 64;
  hipLaunchKernelGGL(patch_pack_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, ivit_stream(stream), w, D, K,
                     (uint4*)wpack);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_weight_pack_multi(long n, const void* jobs, long max_rows_cols, void* stream) {
  if (n <= 0) return 0;
  IVIT_CHECK_ARG(n < 65536 && jobs != nullptr, "ivit_weight_pack_multi: bad job table");
  // x blocks per job: a grid of 1024 x jobs left most blocks of the ~150 small packs (<= 288 blocks
  // of work each) empty; the large ones (the patch embedding's) grid-stride instead
  int gx = ivit_cdiv(max_rows_cols / 8, 256);
  if (gx > 288) gx = 288;
  hipLaunchKernelGGL(multi_pack_kernel, dim3(gx, n), dim3(256), 0, ivit_stream(stream), (const PackJob*)jobs);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_weight_pack_t(const float* w, long K, long N, void* wpack, void* stream) {
  IVIT_CHECK_ARG(N > 0 && N % 16 == 0 && K > 0 && K % 32 == 0, "ivit_weight_pack_t: N % 16, K % 32 must be 0");
  const long n = (K / 32) * (N / 16) * 64;
  hipLaunchKernelGGL(pack_t_kernel, dim3(ivit_cdiv(n, 256)), dim3(256), 0, ivit_stream(stream), w, K, N, (uint4*)wpack);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_patch_embed_fwd_packed(const float* img, long B, long C, long H, long W, const void* wpack,
                                           const float* bias, const float* pos, const float* cls, long D,
                                           float* out, void* stream) {
  IVIT_CHECK_ARG(H % 8 == 0 && W % 8 == 0 && H > 0 && W > 0 && B > 0 && C > 0,
                 "ivit_patch_embed_fwd_packed: H, W must be positive multiples of the patch (8)");
  IVIT_CHECK_ARG(D == 384 || D == 192, "ivit_patch_embed_fwd_packed: D must be 384 or 192 (got %ld)", D);
  // a 144-patch tile spans at most 1 + ceil(143 / Np) images; per-lane DMA offsets are 32-bit
  const long span = 1 + (PE_MT - 1 + (H / 8) * (W / 8) - 1) / ((H / 8) * (W / 8));
  IVIT_CHECK_ARG((H / 8) * (W / 8) * B < (1L << 31) && span * C * H * W * 4 < (1L << 32),
                 "ivit_patch_embed_fwd_packed: raster too large");
  IVIT_CHECK_ARG(((uintptr_t)img & 15) == 0 && ((uintptr_t)wpack & 15) == 0,
                 "ivit_patch_embed_fwd_packed: raster and packed weight must be 16-byte aligned");
  hipStream_t st = ivit_stream(stream);
  const int Wp = (int)(W / 8), Np = (int)((H / 8) * Wp), M = (int)(B * Np);
  const dim3 grid(ivit_cdiv(M, PE_MT));
  if (D == 384)
    hipLaunchKernelGGL(patch_fwd_kernel<8>, grid, dim3(512), 0, st, img, (int)C, (int)H, (int)W, Wp, Np, M,
                       (const u32x4*)wpack, bias, pos, (int)D, out);
  else
    hipLaunchKernelGGL(patch_fwd_kernel<4>, grid, dim3(256), 0, st, img, (int)C, (int)H, (int)W, Wp, Np, M,
                       (const u32x4*)wpack, bias, pos, (int)D, out);
  IVIT_LAUNCH_CHECK();
  const long Ntok = (long)Np + 1;
  hipLaunchKernelGGL(patch_cls_kernel, dim3(ivit_cdiv(B * D, 256)), dim3(256), 0, st, out, B, Ntok, D, cls, pos);
  IVIT_LAUNCH_CHECK();
  return 0;
}

// ============================================================================= weight gradient
// dW[n][k] = sum_m dtok[token(m)][n] * X[m][k],  X[m][c*64 + ky*8 + kx] = bf16(img[b][c][8gy+ky][8gx+kx])
// straight from the f32 raster (no patch matrix). The raster must again be read once, so a
// workgroup owns ALL D rows of its output tile; the tile spans one channel pair (128 k) and the
// reduction runs over patches. Work = (channel pair g, 32-patch chunk j) units, g-major, split
// evenly over 256 persistent workgroups (a range of <= J units meets at most two channel pairs;
// patch_wgrad_raster_ok checks it); each
// workgroup writes its per-pair partial tile to a slab and a reduction kernel sums the partials
// of every pair in a fixed order (deterministic). Per unit: raster 2 ch x 8 ky x 32 patches
// (16 KiB f32 by LDS-DMA, converted per wave like the forward), dtok 32 token rows x D (bf16 by
// LDS-DMA); both operands are MN-contiguous images read with ds_read_b64_tr_b16;
// v_mfma_f32_32x32x16_bf16, 8 waves, a wave = 3 n-blocks x NBK k-blocks of 32 x 32.
namespace ivit {
namespace {

constexpr int WG_NWG = 256;                   // persistent workgroups
constexpr int WG_MU = 32;                     // patches per unit
constexpr int WG_RST = 2 * 8 * WG_MU * 32;    // raster f32 region per unit: 16 KiB (16 pieces)
constexpr int WG_XST = WG_MU * 256;           // X bf16 image [32 m][128 k]: 8 KiB
constexpr int WG_TIMG = WG_MU * 256;          // one 128-column dtok image [32 m][128 n]: 8 KiB

IVIT_DEV int wg_mn_off(int r, int c) { return r * 256 + ((c ^ ((r & 3) << 2)) << 4); }

IVIT_DEV s16x4 wg_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
// 32x32x16 operand from an MN-contiguous [k rows][128 cols] image, rows kbase .. kbase+15:
// lane l gets column colbase + (l & 31)'s k = kbase + 8 (l >> 5) + 0..7 (two transposing reads)
IVIT_DEV bf16x8 wg_frag(const char* img, int kbase, int colbase, int lane) {
  const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = colbase + 16 * (G & 1) + 4 * p;
  const int r0 = kbase + 8 * (G >> 1) + q;
  const int c = col >> 3, e = (col & 7) * 2;
  union { s16x4 s[2]; bf16x8 v; } u;
  u.s[0] = wg_tr(img + wg_mn_off(r0, c) + e);
  u.s[1] = wg_tr(img + wg_mn_off(r0 + 4, c) + e);
  return u.v;
}

IVIT_DEV long wg_unit_start(int w, long U) { return (long)w * U / WG_NWG; }


// NT = D / 128 dtok images; NBK = k-blocks (of 32) per wave (D = 384: NT = 3, NBK = 2).
// 256 persistent workgroups over the g-major (pair, chunk) units (a range meets at most two pairs;
// slab [w][2][D][128]).
template <int NT, int NBK>
__global__ __launch_bounds__(512, 1) void patch_wgrad_kernel(const bf16* __restrict__ dtok,
                                                            const float* __restrict__ img, int C, int H, int W,
                                                            int Wp, int Np, int M, int J, float* __restrict__ slab) {
  constexpr int D = NT * 128, NBN = 3;
  constexpr int TPW = NT;                            // dtok pieces (4 rows x 256 B) per wave per unit
  constexpr int RPW = 2;                             // raster pieces per wave per unit
  constexpr int TST = NT * WG_TIMG;                  // dtok stage bytes
  constexpr int NGRP = D / 32 / NBN;                 // wave groups along n (4 or 2)
  static_assert(NGRP * (4 / NBK) == 8, "8 waves");
  constexpr int RN = 4;                              // raster ring (three units in flight)
  __shared__ __attribute__((aligned(16))) char smem[RN * WG_RST + 3 * TST + 2 * WG_XST];
  char* const rreg = smem;
  char* const treg = smem + RN * WG_RST;
  char* const ximg = treg + 3 * TST;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ng = wv % NGRP, kg = wv / NGRP;
  const long U = (long)((C + 1) / 2) * J;
  const int w = blockIdx.x;
  const long u0 = wg_unit_start(w, U), u1 = wg_unit_start(w + 1, U);
  const int nu = (int)(u1 - u0);
  const int g0 = (int)(u0 / J);
  const int j0 = (int)(u0 - (long)g0 * J);
  slab += (long)w * 2 * D * 128;
  if (nu <= 0) return;
  const int Hp = H / 8, Bn = M / Np;

  // Per-unit addressing is incremental (no integer division in the loop: a runtime-divisor
  // division is a ~40-instruction VALU sequence, and the loop would be VALU-bound on it).
  // A cursor = (g, j) of one unit, advanced by one unit per iteration; the lane positions of
  // its 32-patch chunk advance by 32 patches with carries.
  struct Cur { int g, j; };
  auto cnext = [&](Cur& c) { if (++c.j == J) { c.j = 0; ++c.g; } };
  // raster lane position: patch (lane >> 1) of the chunk as (b, gy, gx)
  struct RPos { int b, gy, gx; };
  auto rpos_at = [&](int m) { RPos r; r.b = m / Np; const int pi = m - r.b * Np; r.gy = pi / Wp; r.gx = pi - r.gy * Wp; return r; };
  auto radv = [&](RPos& r) {
    r.gx += WG_MU;
    while (r.gx >= Wp) { r.gx -= Wp; if (++r.gy == Hp) { r.gy = 0; ++r.b; } }
  };
  // dtok lane rows: patches row_i of the chunk as (b, p), i = the wave's pieces
  struct TPos { int b, p; };
  auto tadv = [&](TPos& t) { t.p += WG_MU; while (t.p >= Np) { t.p -= Np; ++t.b; } };
  const RPos r_first = rpos_at(min(lane >> 1, M - 1));
  TPos t_first[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int row = ((wv * TPW + i) & 7) * 4 + (lane >> 4), m = min(row, M - 1);
    t_first[i].b = m / Np; t_first[i].p = m - t_first[i].b * Np;
  }
  // cursors: raster issue (runs 4 ahead of compute), dtok issue (2 ahead), convert (1 ahead), compute
  Cur cr{g0, j0}, ct{g0, j0}, cc{g0, j0}, cm{g0, j0};
  RPos rp = rpos_at(min(j0 * WG_MU + (lane >> 1), M - 1));
  TPos tp[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int row = ((wv * TPW + i) & 7) * 4 + (lane >> 4), m = min(j0 * WG_MU + row, M - 1);
    tp[i].b = m / Np; tp[i].p = m - tp[i].b * Np;
  }
  const long HWl = (long)H * W;

  // raster pieces of the raster cursor's unit into ring region k % RN: piece q = (channel of the
  // pair cl, ky); lane = (patch l >> 1, 16-B half l & 1); then advance the cursor
  auto issue_r = [&](int k) {
    const bool mok = cr.j * WG_MU + (lane >> 1) < M;
    const int b = mok ? rp.b : Bn - 1, gy = mok ? rp.gy : Hp - 1, gx = mok ? rp.gx : Wp - 1;
    char* st = rreg + (k % RN) * WG_RST;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int q = wv * RPW + i, cl = q >> 3, ky = q & 7;
      const int c = min(2 * cr.g + cl, C - 1);  // a missing odd channel is zeroed in convert
      const float* src = img + ((long)b * C + c) * HWl + (long)(gy * 8 + ky) * W + gx * 8 + (lane & 1) * 4;
      glds_v<true>(src, st + q * 1024);
    }
    cnext(cr);
    if (cr.j == 0) rp = r_first; else radv(rp);
  };
  // dtok rows of the dtok cursor's unit: piece = (image ti = 128-column block, 4-row group)
  auto issue_t = [&](int k) {
    char* st = treg + (k % 3) * TST;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int piece = wv * TPW + i, ti = piece >> 3, row = (piece & 7) * 4 + (lane >> 4);
      const int c = (lane & 15) ^ ((row & 3) << 2);
      const bool mok = ct.j * WG_MU + row < M;
      const int b = mok ? tp[i].b : Bn - 1, p = mok ? tp[i].p : Np - 1;
      const bf16* src = dtok + ((long)b * (Np + 1) + 1 + p) * D + ti * 128 + c * 8;
      glds_v<false>(src, st + ti * WG_TIMG + (piece & 7) * 1024);
    }
    cnext(ct);
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (ct.j == 0) tp[i] = t_first[i];
      else tadv(tp[i]);
    }
  };
  // own raster pieces of the convert cursor's unit (landed) -> X image k & 1 in MN-contiguous
  // layout: lane's 4 kx of (cl, ky, patch) -> 8 bytes of chunk cl*8 + ky of row = patch; zero
  // past M / C
  auto convert = [&](int k) {
    const char* st = rreg + (k % RN) * WG_RST + lane * 16;
    char* xi = ximg + (k & 1) * WG_XST;
    float4 v[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) v[i] = *(const float4*)(st + (wv * RPW + i) * 1024);
    const int p = lane >> 1;
    const bool pok = cc.j * WG_MU + p < M;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int q = wv * RPW + i, cl = q >> 3, ky = q & 7;
      const bool ok = pok && 2 * cc.g + cl < C;
      const uint2 val = ok ? make_uint2(pk_bf16(v[i].x, v[i].y), pk_bf16(v[i].z, v[i].w)) : make_uint2(0u, 0u);
      *(uint2*)(xi + wg_mn_off(p, cl * 8 + ky) + (lane & 1) * 8) = val;
    }
    cnext(cc);
  };

  f32x16 acc[NBN][NBK];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < NBN; ++i)
#pragma unroll
      for (int j = 0; j < NBK; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  };
  // partial tile of pair g -> slab[w][g - g0][n][128]: C layout col = lane & 31 (k),
  // row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) (n); 32 lanes store one 128-B row segment
  auto flush = [&](int g) {
    float* o = slab + (long)(g - g0) * D * 128;
#pragma unroll
    for (int i = 0; i < NBN; ++i)
#pragma unroll
      for (int j = 0; j < NBK; ++j) {
        const int n0 = (ng * NBN + i) * 32, k0 = (kg * NBK + j) * 32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int n = n0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          o[(long)n * 128 + k0 + (lane & 31)] = acc[i][j][r];
        }
      }
  };
  zero();

  // Pipeline (unit index i = u - u0). vmcnt retires in issue order, so the dtok stage T(i) is
  // issued between raster units: entering iteration i the order is
  //   R(i+1) ... T(i) R(i+2) | T(i+1) R(i+3)
  // and T(i), R(i+1) must land (vmcnt = pieces of R(i+2), T(i+1), R(i+3)). Iteration i issues
  // T(i+2) R(i+4): R(i+4) reuses R(i)'s region (converted in iteration i-1, own pieces), T(i+2)
  // reuses T(i-1)'s stage (read by iteration i-1's MFMAs, before this iteration's barrier).
  issue_t(0);
  issue_r(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  convert(0);
  if (nu > 1) issue_r(1);
  if (nu > 2) issue_r(2);
  if (nu > 1) issue_t(1);
  if (nu > 3) issue_r(3);
  for (int i = 0; i < nu; ++i) {
    wait_vm((i + 2 < nu ? RPW : 0) + (i + 1 < nu ? TPW : 0) + (i + 3 < nu ? RPW : 0));
    __builtin_amdgcn_s_barrier();
    if (i + 2 < nu) issue_t(i + 2);
    const char* ti = treg + (i % 3) * TST;
    const char* xi = ximg + (i & 1) * WG_XST;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16x8 fa[NBN], fb[NBK];
#pragma unroll
      for (int a = 0; a < NBN; ++a) {
        const int nb = ng * NBN + a;  // 32-column block of D
        fa[a] = wg_frag(ti + (nb >> 2) * WG_TIMG, 16 * t, (nb & 3) * 32, lane);
      }
#pragma unroll
      for (int j = 0; j < NBK; ++j) fb[j] = wg_frag(xi, 16 * t, (kg * NBK + j) * 32, lane);
#pragma unroll
      for (int a = 0; a < NBN; ++a)
#pragma unroll
        for (int j = 0; j < NBK; ++j)
          acc[a][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[j], acc[a][j], 0, 0, 0);
    }
    // the next unit's raster converts while these MFMAs drain; then its region is refilled
    if (i + 1 < nu) convert(i + 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + 4 < nu) issue_r(i + 4);
    const int g = cm.g;
    cnext(cm);
    if (i + 1 == nu || cm.g != g) {
      flush(g);
      zero();
    }
  }
}

// The wave-specialised form of patch_wgrad_kernel (same units, slab layout and sums): waves 0-3
// only compute, waves 4-7 only load. patch_wgrad_kernel's eight waves each issue their unit's
// LDS-DMA pieces, convert their raster pieces and compute, behind one barrier per unit, and the
// unit cadence (~1.6 us per 40 KiB unit per CU, 25 GB/s of intake) was its bound, not either
// operand's source. Here:
//   * a compute wave owns 96 output rows (n) x the pair's 128 columns (k): 3 x 4 blocks of
//     v_mfma_f32_32x32x16_bf16 (192 accumulator VGPRs), one wave per SIMD, 7 fragment reads
//     (14 transposing LDS reads) per 12 MFMAs;
//   * a loader wave fetches its share of a unit's token-gradient rows by LDS-DMA (6 of the 24
//     1-KiB pieces) three units ahead, and its raster pieces (one channel of the pair, 4 of the 8
//     ky rows: 4 x 16 B per lane) into VGPRs four units ahead, converts them to bf16 and writes
//     the unit's X image itself just before the barrier that publishes the unit — the f32 raster
//     never passes through LDS;
//   * LDS: 4 token-gradient stages (24 KiB) + 2 X images (8 KiB) = 112 KiB.
// Issue order per loader wave (vmcnt retires in issue order): R(0) T(0) R(1) T(1) R(2) T(2) R(3),
// then iteration k issues T(k+3) R(k+4); before the barrier of unit i, R(i) and T(i) must have
// landed: vmcnt = the ops issued after T(i) (R(i+1) and iterations i-2, i-1).
// anatomy builds (tools/ab_build.sh -DPW_ANAT=n; timing only, wrong results): 1 no MFMAs, 2 no raster
// loads, 3 no token-gradient DMA, 4 neither load, 5 every unit's token-gradient rows from chunk 0
#ifndef PW_ANAT
#define PW_ANAT 0
#endif
constexpr int PW_NT = 4;  // token-gradient LDS stages
constexpr int PW_RR = 4;  // raster register sets (units in flight)
template <int SLOT>
using pw_slot = std::integral_constant<int, SLOT>;

// Schedules. P == 0, linear: as patch_wgrad_kernel (workgroup w takes the g-major unit range
// [u0, u1), at most two pairs; slab [w][2][D][128]). P > 0, XCD-sharded: workgroup b runs on XCD
// x = b % 8 (round-robin dispatch) as its s = b / 8-th workgroup, and takes pairs s, s + P, ... over
// the XCD's chunk range [x J / 8, (x+1) J / 8); the P workgroups of an XCD move through the same
// chunks together, so each token-gradient chunk comes from HBM / Infinity Cache once per XCD and
// from its L2 for the other pairs (the full-grid token gradient re-read per pair was 4 GB of the
// 6.9 GB a LiDAR launch fetched; with every unit reading one L2-resident chunk the kernel took
// 0.66 vs 0.95 ms). Slab [x][G][D][128], reduced over x by patch_wgrad_xreduce_kernel.
__global__ __launch_bounds__(512, 1) void patch_wgrad_ws_kernel(const bf16* __restrict__ dtok,
                                                              const float* __restrict__ img, int C, int H, int W,
                                                              int Wp, int Np, int M, int J, int P,
                                                              float* __restrict__ slab) {
  constexpr int D = 384, NT = 3;
  constexpr int TST = NT * WG_TIMG;  // 24 KiB
  __shared__ __attribute__((aligned(16))) char smem[PW_NT * TST + 2 * WG_XST];
  char* const treg = smem;
  char* const ximg = smem + PW_NT * TST;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = (C + 1) / 2;
  const int w = blockIdx.x;
  int g0, j0, nu, jb, je, gstep;
  long slot0;  // slab slot (of D x 128 floats) of pair g0; pair g's is slot0 + (g - g0) / gstep
  if (P == 0) {
    const long U = (long)G * J;
    const long u0 = wg_unit_start(w, U), u1 = wg_unit_start(w + 1, U);
    nu = (int)(u1 - u0);
    g0 = (int)(u0 / J);
    j0 = (int)(u0 - (long)g0 * J);
    jb = 0;
    je = J;
    gstep = 1;
    slot0 = (long)w * 2;
  } else {
    const int x = w & 7, sx = w >> 3;
    jb = x * J / 8;
    je = (x + 1) * J / 8;
    g0 = sx;
    j0 = jb;
    gstep = P;
    nu = (g0 < G ? (G - 1 - g0) / P + 1 : 0) * (je - jb);
    slot0 = (long)x * G + g0;
  }
  if (nu <= 0) return;
  const int Hp = H / 8;
  struct Cur { int g, j; };
  auto cnext = [&](Cur& c) { if (++c.j == je) { c.j = jb; c.g += gstep; } };
  // slab slot of pair g: w * 2 + (g - g0) (linear), x * G + g (sharded)
  auto slot_of = [&](int g) { return slot0 + (g - g0); };

  if (wv >= 4) {  // ------------------------------------------------------------------- loader
    // Addressing is wave-uniform chunk cursors (scalar) + per-lane constants: a 32-patch chunk
    // meets at most two images and two patch rows (the host launches this form for Wp >= 32 only),
    // so a lane's position is the chunk's plus one conditional wrap.
    const int lw = wv - 4;
    const int cl = lw >> 1, ky0 = (lw & 1) * 4;  // raster: channel cl of the pair, ky rows ky0 .. +3
    const int pl = lane >> 1, half = lane & 1;   // raster lane: patch pl of the chunk, 16-B half
    const long HWl = (long)H * W;
    const unsigned chw4 = (unsigned)(C * HWl * 4);  // one image of the raster, bytes (host: < 2^32)
    const unsigned row4 = (unsigned)W * 4;
    // token-gradient pieces 6 lw .. 6 lw + 5 (image ti = piece >> 3, rows 4 (piece & 7) + lane >> 4);
    // a lane's 16-B chunk of its 256-B row segment is the same in every piece
    constexpr int TPL = 6;
    const unsigned tcol = (unsigned)(((lane & 15) ^ ((lane >> 4) << 2)) * 16);
    const int tok_last = (M - 1) + (M - 1) / Np + 1;  // token row of patch M - 1 (rows past M clamp)
    const char* dsb = uniform_ptr(dtok);
    // X image byte offsets of the lane's four (cl, ky0 + i) chunks in row pl
    int xoff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xoff[i] = wg_mn_off(pl, cl * 8 + ky0 + i) + half * 8;
    u32x4 rr[PW_RR][4];

    // chunk cursors (all wave-uniform): unit (g, j); its first patch at image b, in-image patch p,
    // patch row gy, column gx
    struct Ch { int g, j, b, p, gy, gx; };
    auto ch_at = [&](int g, int j) {
      Ch c;
      c.g = g;
      c.j = j;
      const int m = j * WG_MU;
      c.b = m / Np;
      c.p = m - c.b * Np;
      c.gy = c.p / Wp;
      c.gx = c.p - c.gy * Wp;
      return c;
    };
    auto ch_next = [&](Ch& c) {
      if (++c.j == je) {
        c = ch_at(c.g + gstep, jb);
        return;
      }
      c.p += WG_MU;
      if (c.p >= Np) { c.p -= Np; ++c.b; }
      c.gx += WG_MU;
      if (c.gx >= Wp) { c.gx -= Wp; if (++c.gy == Hp) { c.gy = 0; } }
    };
    Ch cr = ch_at(g0, j0), ct = cr;
    Cur cc{g0, j0};

    auto issue_t = [&](int k) {
      char* st = treg + (k % PW_NT) * TST;
      const int tbase = ct.b * (Np + 1) + 1;
#pragma unroll
      for (int i = 0; i < TPL; ++i) {
        const int piece = lw * TPL + i, ti = piece >> 3, row = (piece & 7) * 4 + (lane >> 4);
        const int p = ct.p + row;
        int tok = tbase + p + (p >= Np ? 1 : 0);
        tok = ct.j * WG_MU + row < M ? tok : tok_last;
        if (PW_ANAT == 5) tok = 1 + row;  // diagnostic: every unit reads chunk 0 (L2-resident)
        if (PW_ANAT != 3 && PW_ANAT != 4)
          glds_s<false>((unsigned)tok * (unsigned)(D * 2) + (unsigned)(ti * 256) + tcol, dsb,
                        st + ti * WG_TIMG + (piece & 7) * 1024);
      }
      ch_next(ct);
    };
    // the raster cursor's unit into register set SLOT (4 x 16 B per lane, streamed: nt)
    auto issue_r = [&](auto slot) {
      constexpr int S = decltype(slot)::value;
      const int c = min(2 * cr.g + cl, C - 1);  // a missing odd channel is zeroed in convert
      const char* sb = uniform_ptr(img + ((long)cr.b * C + c) * HWl + (long)ky0 * W);
      int gx = cr.gx + pl, gy = cr.gy;
      unsigned ib = 0;
      if (gx >= Wp) {
        gx -= Wp;
        if (++gy == Hp) { gy = 0; ib = chw4; }
      }
      unsigned vo = ib + (unsigned)(gy * 8) * row4 + (unsigned)(gx * 32 + half * 16);
      vo = cr.j * WG_MU + pl < M ? vo : 0u;  // past M: any valid address (zeroed in convert)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (PW_ANAT != 2 && PW_ANAT != 4)
          asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=v"(rr[S][i]) : "v"(vo), "s"(sb) : "memory");
        vo += row4;
      }
      ch_next(cr);
    };
    // register set SLOT (landed) -> X image k & 1: lane's 4 kx of (cl, ky, patch) -> 8 bytes of
    // chunk cl * 8 + ky of row = patch; zero past M / C
    auto convert = [&](auto slot, int k) {
      constexpr int S = decltype(slot)::value;
      char* xi = ximg + (k & 1) * WG_XST;
      const bool ok = cc.j * WG_MU + pl < M && 2 * cc.g + cl < C;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        asm volatile("" : "+v"(rr[S][i]));  // after the counted wait
        const float4 v = __builtin_bit_cast(float4, rr[S][i]);
        const uint2 val = ok ? make_uint2(pk_bf16(v.x, v.y), pk_bf16(v.z, v.w)) : make_uint2(0u, 0u);
        *(uint2*)(xi + xoff[i]) = val;
      }
      cnext(cc);
    };
    // prologue: R(0) T(0) R(1) T(1) R(2) T(2) R(3)
    issue_r(pw_slot<0>{});
    issue_t(0);
    if (nu > 1) issue_r(pw_slot<1>{});
    if (nu > 1) issue_t(1);
    if (nu > 2) issue_r(pw_slot<2>{});
    if (nu > 2) issue_t(2);
    if (nu > 3) issue_r(pw_slot<3>{});
    // one unit of the loader's loop with register set SLOT = i % 4
    auto step = [&](auto slot, int i) {
      if (i >= 2 && i + 4 < nu) {  // steady state: R(i+1) and iterations i-2, i-1 issued after T(i)
        asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      } else {
        int after = i + 1 < nu ? 4 : 0;
#pragma unroll
        for (int k = i - 2; k < i; ++k) after += (k + 3 < nu ? 6 : 0) + (k + 4 < nu ? 4 : 0);
        wait_vm(after);
      }
      convert(slot, i);
      lds_barrier();  // publishes X(i) (own ds_writes) and, with every loader's wait, T(i)
      if (i + 3 < nu) issue_t(i + 3);
      if (i + 4 < nu) issue_r(slot);  // (i + 4) % 4 == i % 4: the set converted just now
    };
    for (int i = 0; i < nu; i += 4) {
      step(pw_slot<0>{}, i);
      if (i + 1 < nu) step(pw_slot<1>{}, i + 1);
      if (i + 2 < nu) step(pw_slot<2>{}, i + 2);
      if (i + 3 < nu) step(pw_slot<3>{}, i + 3);
    }
    return;
  }

  // ------------------------------------------------------------------------------------ compute
  const int nb0 = wv * 3;  // 32-row n blocks nb0 .. nb0 + 2
  f32x16 acc[3][4];
  auto zero = [&]() {
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][j][r] = 0.f;
  };
  auto flush = [&](int g) {
    // the lane's offset laundered here, so that the 192 store addresses are formed at the flush
    // and not hoisted out of the unit loop (they spilled: 272 B of scratch)
    int lo = 4 * (lane >> 5) * 128 + (lane & 31);
    asm volatile("" : "+v"(lo));
    float* o = slab + slot_of(g) * D * 128 + nb0 * 32 * 128 + lo;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[(a * 32 + (r & 3) + 8 * (r >> 2)) * 128 + j * 32] = acc[a][j][r];
  };
  zero();
  Cur cm{g0, j0};
  for (int i = 0; i < nu; ++i) {
    __builtin_amdgcn_s_barrier();
    const char* ti = treg + (i % PW_NT) * TST;
    const char* xi = ximg + (i & 1) * WG_XST;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16x8 fa[3], fb[4];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int nb = nb0 + a;
        fa[a] = wg_frag(ti + (nb >> 2) * WG_TIMG, 16 * t, (nb & 3) * 32, lane);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = wg_frag(xi, 16 * t, j * 32, lane);
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (PW_ANAT != 1) acc[a][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[j], acc[a][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // my reads of this unit are done
    const int g = cm.g;
    cnext(cm);
    if (i + 1 == nu || cm.g != g) {
      flush(g);
      zero();
    }
  }
}

// dW[n][g*128 + k] (+)= sum of the partial tiles of pair g (workgroups whose unit range meets it).
// D * 128 is a multiple of the block's 256 V elements, so a block's pair g, and the range of
// workgroups whose unit range meets it, are block-uniform (scalar; one 64-bit division per block,
// not per element). V = 4: four consecutive k per thread with 16-B accesses (the V = 1 form's
// 27 840 one-element-per-thread blocks at the LiDAR shape were launch-latency-bound: 58 us for 50 MB).
// Every element is summed in the same order either way.
template <int V>
__global__ __launch_bounds__(256) void patch_wgrad_reduce_kernel(const float* __restrict__ slab, int C, int J, int D,
                                                                 float* __restrict__ dW, int accumulate) {
  using VT = typename std::conditional<V == 4, float4, float>::type;
  const int G = (C + 1) / 2;
  const long per = (long)D * 128, i0 = (long)blockIdx.x * 256 * V;
  const int g = (int)(i0 / per);
  if (g >= G) return;
  const int e = (int)(i0 - (long)g * per) + threadIdx.x * V, n = e >> 7, k = e & 127;
  const long U = (long)G * J, ga = (long)g * J, gb = ga + J;
  // the contiguous workgroup range [w0, w1) whose unit ranges meet pair g (block-uniform); only w0
  // can have begun in the previous pair (its partial tile of g is then its second slab slot)
  int w0 = (int)(ga * WG_NWG / U);
  while (w0 > 0 && wg_unit_start(w0, U) > ga) --w0;
  while (w0 < WG_NWG && wg_unit_start(w0 + 1, U) <= ga) ++w0;
  int w1 = w0;
  while (w1 < WG_NWG && wg_unit_start(w1, U) < gb) ++w1;
  const int slot0 = wg_unit_start(w0, U) < ga ? 1 : 0;
  auto ld = [&](long off) { return *(const VT*)(slab + off); };
  auto add = [](VT& s, const VT& v) {
    if constexpr (V == 4) { s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w; }
    else s += v;
  };
  VT s{};
  const long estride = 2L * D * 128;  // one workgroup's two slab slots
  const long base = ((long)w0 * 2 * D + n) * 128 + k;
  if (U < WG_NWG) {  // tiny grids: some workgroups own no units (and wrote no slab): skip them
    for (int w = w0; w < w1; ++w) {
      const long a = wg_unit_start(w, U), b = wg_unit_start(w + 1, U);
      if (b <= a) continue;
      add(s, ld((((long)w * 2 + (a < ga ? 1 : 0)) * D + n) * 128 + k));
    }
  } else if (w0 < w1) {
    s = ld(base + (long)slot0 * D * 128);
    // the rest start in pair g (slot 0): independent loads, eight in flight, summed in order
    int w = w0 + 1;
    for (; w + 8 <= w1; w += 8) {
      VT v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = ld(base + (long)(w - w0 + q) * estride);
#pragma unroll
      for (int q = 0; q < 8; ++q) add(s, v[q]);
    }
    for (; w < w1; ++w) add(s, ld(base + (long)(w - w0) * estride));
  }
  if (2 * g + (k >> 6) >= C) return;
  VT* o = (VT*)(dW + (long)n * C * 64 + (long)g * 128 + k);
  if (accumulate) {
    VT t = *o;
    add(t, s);
    *o = t;
  } else {
    *o = s;
  }
}

// dW[n][g*128 + k] (+)= sum over the XCDs x (in order; those with a non-empty chunk range) of
// slab[x][g][n][k] (the sharded schedule's partials), four consecutive k per thread.
__global__ __launch_bounds__(256) void patch_wgrad_xreduce_kernel(const float* __restrict__ slab, int C, int J, int D,
                                                                  float* __restrict__ dW, int accumulate) {
  const int G = (C + 1) / 2;
  const long per = (long)D * 128, e = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (e >= (long)G * per) return;
  const int g = (int)(e / per), r = (int)(e - (long)g * per), n = r >> 7, k = r & 127;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    if ((x + 1) * J / 8 == x * J / 8) continue;
    const float4 v = *(const float4*)(slab + ((long)x * G + g) * per + r);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  if (2 * g + (k >> 6) >= C) return;
  float4* o = (float4*)(dW + (long)n * C * 64 + (long)g * 128 + k);
  if (accumulate) {
    const float4 t = *o;
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  *o = s;
}

}  // namespace

long patch_wgrad_raster_workspace(long D) { return (long)WG_NWG * 2 * D * 128 * 4; }
// the XCD-sharded schedule's workgroups per XCD (0: the linear schedule)
int pw_shard_p(long C, long Wp, long J) {
  const long G = (C + 1) / 2;
  if (Wp < WG_MU || G < 32 || J < 64) return 0;
  const long R = (G + 31) / 32;  // pairs per workgroup
  return (int)((G + R - 1) / R);
}
long patch_wgrad_raster_workspace2(long B, long C, long H, long W, long D) {
  const long Np = (H / 8) * (W / 8), J = (B * Np + WG_MU - 1) / WG_MU;
  const long lin = patch_wgrad_raster_workspace(D);
  const long sh = pw_shard_p(C, W / 8, J) ? 8 * ((C + 1) / 2) * D * 128 * 4 : 0;
  return lin > sh ? lin : sh;
}

bool patch_wgrad_raster_ok(long B, long C, long H, long W, long D) {
  if (D != 384 || H % 8 || W % 8 || B <= 0 || C <= 0) return false;
  const long Np = (H / 8) * (W / 8), M = B * Np, J = (M + WG_MU - 1) / WG_MU, U = (C + 1) / 2 * J;
  // every workgroup's unit range (<= ceil(U / 256) units) must meet at most two channel pairs
  if ((U + WG_NWG - 1) / WG_NWG > J) return false;
  const long span = 1 + (WG_MU - 1 + Np - 1) / Np;  // images a 32-patch chunk can touch
  return M < (1L << 31) && span * C * H * W * 4 < (1L << 32) && span * (Np + 1) * D * 2 < (1L << 32);
}

int patch_wgrad_raster(const bf16* dtok, const float* img, long B, long C, long H, long W, long D, float* dW,
                       int accumulate, void* work, hipStream_t st) {
  const int Wp = (int)(W / 8), Np = (int)((H / 8) * Wp), M = (int)(B * Np), J = ivit_cdiv(M, WG_MU);
  float* slab = (float*)work;
  const long n = (long)((C + 1) / 2) * D * 128;
  // Dispatch: P > 0 (at least 32 channel pairs, patch rows >= 32 wide: the LiDAR raster) runs the
  // wave-specialised kernel on the XCD-sharded schedule (each XCD's P workgroups walk the same
  // chunk range over different channel pairs, so the token-gradient rows come from that XCD's L2)
  // + the 8-way partial reduce; patch rows >= 32 wide otherwise (the map raster) run the
  // wave-specialised kernel on the linear schedule + its reduce; narrower grids patch_wgrad_kernel.
  // (Round 4 measured and removed an older all-waves XCD-sharded form, 1.387 vs 1.116 ms; the
  // history is in DESIGN.md §8.)
  if ((D * 128) % 256) return IVIT_ERR_UNSUPPORTED;  // the reduce's block-uniform pair
  const int P = pw_shard_p(C, Wp, J);
  if (P > 0 && (D * 128) % 4 == 0 && ((uintptr_t)dW & 15) == 0 && (C * 64) % 4 == 0) {
    hipLaunchKernelGGL(patch_wgrad_ws_kernel, dim3(8 * P), dim3(512), 0, st, dtok, img, (int)C, (int)H, (int)W, Wp, Np,
                       M, J, P, slab);
    const long tot = (long)((C + 1) / 2) * D * 128;
    hipLaunchKernelGGL(patch_wgrad_xreduce_kernel, dim3(ivit_cdiv(tot, 1024)), dim3(256), 0, st, slab, (int)C, J,
                       (int)D, dW, accumulate);
    return 0;
  }
  if (Wp >= WG_MU)  // the wave-specialised form's lane positions need Wp >= 32
    hipLaunchKernelGGL(patch_wgrad_ws_kernel, dim3(WG_NWG), dim3(512), 0, st, dtok, img, (int)C, (int)H, (int)W, Wp, Np,
                       M, J, 0, slab);
  else
    hipLaunchKernelGGL((patch_wgrad_kernel<3, 2>), dim3(WG_NWG), dim3(512), 0, st, dtok, img, (int)C, (int)H, (int)W,
                       Wp, Np, M, J, slab);
  if ((D * 128) % 1024 == 0 && ((uintptr_t)dW & 15) == 0 && (C * 64) % 4 == 0)
    hipLaunchKernelGGL(patch_wgrad_reduce_kernel<4>, dim3(ivit_cdiv(n, 1024)), dim3(256), 0, st, slab, (int)C, J,
                       (int)D, dW, accumulate);
  else
    hipLaunchKernelGGL(patch_wgrad_reduce_kernel<1>, dim3(ivit_cdiv(n, 256)), dim3(256), 0, st, slab, (int)C, J,
                       (int)D, dW, accumulate);
  return 0;
}

}  // namespace ivit
