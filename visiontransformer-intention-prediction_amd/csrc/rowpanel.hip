// Residual GEMM with the following LayerNorm fused into its epilogue (timm Block: x1 = x +
// dp1(proj(attn)); then norm2(x1) — model_vit.py:64,71 -> timm Block.forward):
//
//   X[m][n] = R[m][n] + scale[m / rps] * (sum_k A[m][k] W[n][k] + bias[n])           f32, N = 384
//   Y[m][n] = bf16((X[m][n] - mean_m) * rstd_m * gamma[n] + beta[n]),  mean_m, rstd_m   (eps)
//
// LayerNorm needs whole rows, so a workgroup owns a panel of 144 rows x ALL 384 columns (the
// patch-embedding kernel's tiling: 250 workgroups for the 36 008 token rows of a B = 8 ViT
// stream, one per CU). A (bf16 activations, K-contiguous) streams through a 4-stage LDS ring by
// LDS-DMA; the weight, packed in MFMA fragment order (ivit_patch_weight_pack layout), goes to
// VGPRs two K-stages ahead; 8 waves x (144 rows x 48 columns) of v_mfma_f32_16x16x32_bf16.
// Epilogue per 16-row block: acc + bias through LDS into row-major order, then 32 lanes per row
// add the residual (coalesced), store X, reduce the row mean and the centred variance by
// cross-lane shuffles (two passes, as torch's LayerNorm) and store Y, mean, rstd. This replaces
// the EpiResid GEMM + ln_fwd_vec_kernel pair (the LayerNorm re-read X from HBM).
#include "panel_common.h"

namespace ivit {
namespace {

constexpr int RP_MT = 144;                 // rows per workgroup
constexpr int RP_MB = RP_MT / 16;          // 16-row MFMA blocks
constexpr int RP_N = 384;                  // output columns (8 waves x 3 x 16)
constexpr int RP_STAGE = RP_MT * 128;      // A stage: [144 rows][64 k] bf16, 16-B chunks swizzled
constexpr int RP_NS = 4;                   // A ring (three stages in flight)
constexpr int RP_PIECES = RP_STAGE / 1024; // 18 DMA pieces of 8 rows
constexpr int RP_TLD = RP_N + 4;           // epilogue row stride (floats)

IVIT_DEV int rp_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// The streamed operand's per-lane LDS-DMA sources (row-panel-invariant): 18 pieces of 8 rows per
// stage over W waves (W = 8: the first two waves take three, the rest two; W = 4: five / four).
constexpr int RP_PWMAX = 5;
struct PanelA {
  const bf16* A0;
  unsigned voff[RP_PWMAX];
  int npc, pc0;
};

template <int W = 8>
IVIT_DEV PanelA panel_a_setup(const bf16* A, long lda, int M, int m0, int wv, int lane) {
  constexpr int PW = (RP_PIECES + W - 1) / W, PREM = RP_PIECES % W;
  static_assert(PREM != 0 && PW <= RP_PWMAX, "piece split");
  PanelA p;
  p.npc = wv < PREM ? PW : PW - 1;
  p.pc0 = wv < PREM ? wv * PW : PREM * PW + (wv - PREM) * (PW - 1);
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int row = min(p.pc0 + i, RP_PIECES - 1) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);  // stored chunk (lane & 7) holds source chunk c
    const int m = min(m0 + row, M - 1) - m0;      // rows past M are computed, never stored
    p.voff[i] = (unsigned)(((long)m * lda + c * 8) * 2);
  }
  p.A0 = A + (long)m0 * lda;
  return p;
}

// acc[9][3] = rows m0 .. m0+143 of A (K = 64 KT) times the 48 columns of 16-column blocks
// nb0 .. nb0+2 of a packed weight with NB16 blocks in total.
// TR: the MFMA operands swapped (weights as A, the panel as B), so acc holds the output
// transposed: lane l has columns 4 (l >> 4) + i, i < 4, of row l & 15 of each 16 x 16 block.
template <int W = 8, bool TR = false>
IVIT_DEV void panel_mainloop(f32x4 (&acc)[RP_MB][NBW], char* smem, const PanelA& pa, const u32x4* wpack, int NB16,
                             int nb0, int KT, int wv, int lane, u64* t_first = nullptr) {
  constexpr int PW = (RP_PIECES + W - 1) / W;
  auto issue_a = [&](int kt) {
    char* st = smem + (kt % RP_NS) * RP_STAGE + pa.pc0 * 1024;
    const char* sb = uniform_ptr(pa.A0 + kt * 64);
#pragma unroll
    for (int i = 0; i < PW; ++i)
      if (i < pa.npc) glds_s<false>(pa.voff[i], sb, st + i * 1024);
  };
  const unsigned vb = lane * 16;
  auto issue_b = [&](int kt, u32x4 (&r)[2 * NBW]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) load_wfrag(r, t, uniform_ptr(wpack + ((long)(2 * kt + t) * NB16 + nb0) * 64), vb);
  };
#pragma unroll
  for (int i = 0; i < RP_MB; ++i)
#pragma unroll
    for (int j = 0; j < NBW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 breg[3][2 * NBW];
  const int npc = pa.npc;
  // Issue order: A(kt) B(kt) ... with B(kt) between A(kt) and A(kt+1); iteration kt issues
  // B(kt+2) A(kt+3), and waits for A(kt), B(kt) with A(kt+1) B(kt+1) A(kt+2) still in flight.
  auto stage = [&](int kt, u32x4 (&cur)[2 * NBW], u32x4 (&nb2)[2 * NBW]) {
    wait_vm((kt + 1 < KT ? npc + 2 * NBW : 0) + (kt + 2 < KT ? npc : 0));
    tie(cur);
    __builtin_amdgcn_s_barrier();  // every wave's pieces of A(kt); stage (kt-1) % 4 free
    if (t_first && kt == 0) *t_first = clk_now();
    if (kt + 2 < KT) issue_b(kt + 2, nb2);
    if (kt + 3 < KT) issue_a(kt + 3);
    const char* ia = smem + (kt % RP_NS) * RP_STAGE;
    // fragment f = (t = f / 9: 32-k half, mb = f % 9): rows 16 mb + (lane & 15), chunk 4t + lane/16;
    // read three ahead of their MFMAs (sched barriers pin the distance)
    auto rdf = [&](int f) {
      const int row = 16 * (f % RP_MB) + (lane & 15), ch = 4 * (f / RP_MB) + (lane >> 4);
      return *(const bf16x8*)(ia + rp_off(row, ch));
    };
    bf16x8 fr[4];
    fr[0] = rdf(0);
    fr[1] = rdf(1);
    fr[2] = rdf(2);
#pragma unroll
    for (int f = 0; f < 2 * RP_MB; ++f) {
      const int t = f / RP_MB, mb = f % RP_MB;
      if (f + 3 < 2 * RP_MB) fr[(f + 3) % 4] = rdf(f + 3);
#pragma unroll
      for (int j = 0; j < NBW; ++j) {
        union { u32x4 u; bf16x8 v; } bw;
        bw.u = cur[t * NBW + j];
        if constexpr (TR)
          acc[mb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw.v, fr[f % 4], acc[mb][j], 0, 0, 0);
        else
          acc[mb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[f % 4], bw.v, acc[mb][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // my reads of stage kt are done
  };

  issue_a(0);
  issue_b(0, breg[0]);
  if (KT > 1) issue_a(1);
  if (KT > 1) issue_b(1, breg[1]);
  if (KT > 2) issue_a(2);
  for (int kt = 0; kt < KT; kt += 3) {
    stage(kt, breg[0], breg[2]);
    if (kt + 1 < KT) stage(kt + 1, breg[1], breg[0]);
    if (kt + 2 < KT) stage(kt + 2, breg[2], breg[1]);
  }
}

// Backward form (BWD = true): the GEMM is the LayerNorm input's dgrad, dY[m][n] = sum_k A[m][k] W[k][n]
// (W packed transposed), and the epilogue is the LayerNorm backward of timm's norm:
//   xh = (X - mean) rstd,  g = dY gamma,  dX = dres + rstd (g - mean_n(g) - xh mean_n(g xh)),
//   dXs = bf16(dX * scale[m / rps]) (optional), per-workgroup partial column sums of dY xh / dY.
// Pointer roles in BWD: R = dres (nullable), X = X (read), Y = dXs, mean / rstd read, bias unused,
// part = [gridDim.x][2][384] partials (reduced by colreduce_kernel).
#ifndef RP_WPF
#define RP_WPF 1
#endif
#ifndef RP_PF_FWD
#define RP_PF_FWD 1
#endif
#ifndef RP_PF_BWD
#define RP_PF_BWD 1
#endif
#ifndef RP_PFB_BWD
#define RP_PFB_BWD 1
#endif
template <bool BWD, bool ST = false>
__global__ __launch_bounds__(512, 1) void rowpanel_ln_kernel(
    const bf16* __restrict__ A, long lda, int M, int K, const u32x4* __restrict__ wpack,
    const float* __restrict__ bias, const float* R, long ldr, const float* __restrict__ scale, int rps,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float* X, long ldx,
    bf16* __restrict__ Y, long ldy, float* mean, float* rstd, float* dX, long lddx, float* __restrict__ part,
    u64* stamps) {
  __shared__ __attribute__((aligned(16))) char smem[RP_NS * RP_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * RP_MT;
  Stamps stp;
  if constexpr (ST) stp.begin();

  PanelA pa = panel_a_setup(A, lda, M, m0, wv, lane);
  f32x4 acc[RP_MB][NBW];
  panel_mainloop(acc, smem, pa, wpack, RP_N / 16, wv * NBW, K / 64, wv, lane, ST ? &stp.t1 : nullptr);
  if constexpr (ST) stp.t2 = clk_now();

  // ---- epilogue, one 16-row block at a time through LDS
  __builtin_amdgcn_s_barrier();  // every wave is done with the A ring
  float* T = (float*)smem;       // [16][RP_TLD]
  float bv[NBW];
#pragma unroll
  for (int j = 0; j < NBW; ++j) bv[j] = (!BWD && bias) ? bias[(wv * NBW + j) * 16 + (lane & 15)] : 0.f;
  const int r = tid >> 5, c0 = (tid & 31) * 12;  // row phase: 32 lanes per row, 12 columns each
  float gm[12], bt[12];
#pragma unroll
  for (int e = 0; e < 12; ++e) { gm[e] = gamma[c0 + e]; bt[e] = BWD ? 0.f : beta[c0 + e]; }
  // row operands of block mb + 1 (residual; or X and dres) are loaded while block mb is reduced
  struct RowIn { float4 a[3]; float s, mu, rs; };
  struct RowB { float4 b[3]; };  // BWD: dres
  auto load_row = [&](int mb, RowIn& in) {
    const int m = min(m0 + 16 * mb + r, M - 1);
    in.s = scale ? scale[m / rps] : 1.f;
    if constexpr (!BWD) {
      const float* rrow = R + (long)m * ldr + c0;
#pragma unroll
      for (int e = 0; e < 3; ++e) in.a[e] = *(const float4*)(rrow + 4 * e);
    } else {
      const float* xrow = X + (long)m * ldx + c0;
#pragma unroll
      for (int e = 0; e < 3; ++e) in.a[e] = *(const float4*)(xrow + 4 * e);
      in.mu = mean[m];
      in.rs = rstd[m];
    }
  };
  auto load_b = [&](int mb, RowB& in) {
    const int m = min(m0 + 16 * mb + r, M - 1);
    if (R) {
      const float* drow = R + (long)m * ldr + c0;
#pragma unroll
      for (int e = 0; e < 3; ++e) in.b[e] = *(const float4*)(drow + 4 * e);
    } else {
#pragma unroll
      for (int e = 0; e < 3; ++e) in.b[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  float pg[12], pb[12];  // BWD: this thread's partial column sums of dY xh, dY
#pragma unroll
  for (int e = 0; e < 12; ++e) { pg[e] = 0.f; pb[e] = 0.f; }
  // The row operands are prefetched PF blocks ahead (a ring of register sets; the loop is
  // unrolled, so the compiler's counted waits stay exact): one block in flight per CU is 24 KiB
  // (48 with BWD's two operands), which pulls the residual at ~10 GB/s per CU — the epilogue was
  // bound by that latency, not by HBM bandwidth (r03 stamps: 23 us for 0.55 MB per workgroup).
  constexpr int PF = BWD ? RP_PF_BWD : RP_PF_FWD, PFB = BWD ? RP_PFB_BWD : 1;
  RowIn ring[PF];
  RowB ringb[PFB];
#pragma unroll
  for (int i = 0; i < PF; ++i)
    if (i < RP_MB) load_row(i, ring[i]);
  if constexpr (BWD) {
#pragma unroll
    for (int i = 0; i < PFB; ++i)
      if (i < RP_MB) load_b(i, ringb[i]);
  }
#pragma unroll
  for (int mb = 0; mb < RP_MB; ++mb) {
    RowIn& in = ring[mb % PF];
    RowB& inb = ringb[mb % PFB];
#pragma unroll
    for (int j = 0; j < NBW; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        T[(4 * (lane >> 4) + i) * RP_TLD + (wv * NBW + j) * 16 + (lane & 15)] = acc[mb][j][i] + bv[j];
    lds_barrier();
    const int m = m0 + 16 * mb + r;
    const bool ok = m < M;
    float t[12], u[12];
#pragma unroll
    for (int e = 0; e < 12; e += 4) {
      const float4 tv = *(const float4*)(T + r * RP_TLD + c0 + e);
      t[e] = tv.x; t[e + 1] = tv.y; t[e + 2] = tv.z; t[e + 3] = tv.w;
      const float4 q = in.a[e / 4];
      u[e] = q.x; u[e + 1] = q.y; u[e + 2] = q.z; u[e + 3] = q.w;
    }
    if constexpr (!BWD) {
      const float sc = in.s;
      float x[12];
#pragma unroll
      for (int e = 0; e < 12; ++e) x[e] = u[e] + sc * t[e];
      if (mb + PF < RP_MB) load_row(mb + PF, in);
      float sum = 0.f;
#pragma unroll
      for (int e = 0; e < 12; ++e) sum += x[e];
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
      const float mu = sum * (1.f / RP_N);
      float sq = 0.f;
#pragma unroll
      for (int e = 0; e < 12; ++e) { const float d = x[e] - mu; sq += d * d; }
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) sq += __shfl_xor(sq, o, 64);
      const float rs = rsqrtf(sq * (1.f / RP_N) + eps);
      if (ok) {
        float* xrow = X + (long)m * ldx + c0;
#pragma unroll
        for (int e = 0; e < 12; e += 4) *(float4*)(xrow + e) = make_float4(x[e], x[e + 1], x[e + 2], x[e + 3]);
        unsigned pk[6];
#pragma unroll
        for (int e = 0; e < 12; e += 2)
          pk[e / 2] = pk_bf16((x[e] - mu) * rs * gm[e] + bt[e], (x[e + 1] - mu) * rs * gm[e + 1] + bt[e + 1]);
        bf16* yrow = Y + (long)m * ldy + c0;
        *(uint2*)yrow = make_uint2(pk[0], pk[1]);
        *(uint2*)(yrow + 4) = make_uint2(pk[2], pk[3]);
        *(uint2*)(yrow + 8) = make_uint2(pk[4], pk[5]);
        if ((tid & 31) == 0) { mean[m] = mu; rstd[m] = rs; }
      }
    } else {
      const float mu = in.mu, rs = in.rs, sc = in.s;
      float dr[12];
#pragma unroll
      for (int e = 0; e < 12; e += 4) {
        const float4 q = inb.b[e / 4];
        dr[e] = q.x; dr[e + 1] = q.y; dr[e + 2] = q.z; dr[e + 3] = q.w;
      }
      if (mb + PFB < RP_MB) load_b(mb + PFB, inb);
      if (mb + PF < RP_MB) load_row(mb + PF, in);
      float xh[12], gy[12], s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 12; ++e) {
        xh[e] = (u[e] - mu) * rs;
        gy[e] = t[e] * gm[e];
        s1 += gy[e];
        s2 += gy[e] * xh[e];
      }
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
      s1 *= 1.f / RP_N;
      s2 *= 1.f / RP_N;
      if (ok) {
        float o[12];
#pragma unroll
        for (int e = 0; e < 12; ++e) {
          o[e] = rs * (gy[e] - s1 - xh[e] * s2) + dr[e];
          pg[e] += t[e] * xh[e];
          pb[e] += t[e];
        }
        float* drow = dX + (long)m * lddx + c0;
#pragma unroll
        for (int e = 0; e < 12; e += 4) *(float4*)(drow + e) = make_float4(o[e], o[e + 1], o[e + 2], o[e + 3]);
        if (Y) {
          unsigned pk[6];
#pragma unroll
          for (int e = 0; e < 12; e += 2) pk[e / 2] = pk_bf16(o[e] * sc, o[e + 1] * sc);
          bf16* yrow = Y + (long)m * ldy + c0;
          *(uint2*)yrow = make_uint2(pk[0], pk[1]);
          *(uint2*)(yrow + 4) = make_uint2(pk[2], pk[3]);
          *(uint2*)(yrow + 8) = make_uint2(pk[4], pk[5]);
        }
      }
    }
    __builtin_amdgcn_s_barrier();  // T is rewritten by the next block
  }
  if constexpr (BWD) {
    // column partials of the 16 row slots -> one [2][384] partial row per workgroup
    float* red = (float*)smem;  // [16][2][384]
#pragma unroll
    for (int e = 0; e < 12; ++e) {
      red[(r * 2 + 0) * RP_N + c0 + e] = pg[e];
      red[(r * 2 + 1) * RP_N + c0 + e] = pb[e];
    }
    lds_barrier();
    for (int c = tid; c < 2 * RP_N; c += 512) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) a += red[k * 2 * RP_N + c];
      part[(long)blockIdx.x * 2 * RP_N + c] = a;
    }
  }
  if constexpr (ST) stp.end(stamps);
}

// ============================================================================= wide outputs
// The same row panel for outputs wider than 384 columns (qkv 1152, fc1 1536, fc2's dgrad 1536)
// and the plain proj dgrad: the A panel of 144 rows is streamed once per 192- (or 384-) column
// chunk (from L2 for all but the first), and each chunk's row segments are written whole.
//   EPI_QS:     Y = bf16((acc + bias[n]) * (n < qcols ? qscale : 1))        (qkv, Q block prescaled)
//   EPI_GELU:   P = bf16(acc + bias[n]), Y = bf16(gelu(acc + bias[n]))       (fc1 + pre-activation)
//   EPI_DGELU:  Y = bf16(acc * gelu'(P[m][n]))                                (fc2 dgrad, W packed transposed)
//   EPI_GELUD:  P = bf16(gelu'(acc + bias[n])), Y = bf16(gelu(acc + bias[n]))    (fc1, training)
//   EPI_DMUL:   Y = bf16(acc * P[m][n])   (fc2 dgrad, P = the GELU' EPI_GELUD wrote)
constexpr int EPI_QS = 0, EPI_GELU = 1, EPI_DGELU = 2, EPI_GELUD = 3, EPI_DMUL = 4;
constexpr bool epi_reads_p(int e) { return e == EPI_DGELU || e == EPI_DMUL; }
constexpr bool epi_writes_p(int e) { return e == EPI_GELU || e == EPI_GELUD; }

// Transposed-accumulator epilogue of the wide kernels (EV = 1): acc[mb][j][i] is column
// nw + 16 j + 4 (lane >> 4) + i of row m0 + 16 mb + (lane & 15).
template <int EPI>
IVIT_DEV void wide_epilogue_tr(const f32x4 (&acc)[RP_MB][NBW], int nw, int m0, int M, const float* __restrict__ bias,
                               int qcols, float qscale, bf16* __restrict__ Y, long ldy, bf16* __restrict__ P,
                               long ldp, int lane) {
  const int g = lane >> 4, tl = lane & 15;
  const bool odd = g & 1;
  const int cb = nw + 4 * g;  // + 16 j: this lane's first column in block j
  float bv[NBW][4];
#pragma unroll
  for (int j = 0; j < NBW; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[j][i] = (!epi_reads_p(EPI) && bias) ? bias[cb + 16 * j + i] : 0.f;
  const float qs = (EPI == EPI_QS && nw < qcols) ? qscale : 1.f;  // qcols is a multiple of 384 (of the chunk)
  // packed Y (and P) words of block (mb, j); DGELU: h = the 4 pre-activations
  auto compute = [&](int mb, int j, uint2 h, uint2& y, uint2& p) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = acc[mb][j][i] + bv[j][i];
    if constexpr (EPI == EPI_QS) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] *= qs;
    } else if constexpr (EPI == EPI_GELU) {
      p = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = gelu_t<bf16>(v[i]);
    } else if constexpr (EPI == EPI_GELUD) {
      float d[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) gelu_fast2(v[i], v[i], d[i]);
      p = make_uint2(pk_bf16(d[0], d[1]), pk_bf16(d[2], d[3]));
    } else {
      Pack4 q;
      q.u = h;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] *= EPI == EPI_DMUL ? (float)q.h[i] : gelu_grad_t<bf16>((float)q.h[i]);
    }
    y = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
  };
  auto load_h = [&](int mb, uint2 (&h)[NBW]) {
    const bf16* pr = P + (long)min(m0 + 16 * mb + tl, M - 1) * ldp + cb;
#pragma unroll
    for (int j = 0; j < NBW; ++j) h[j] = *(const uint2*)(pr + 16 * j);
  };
  uint2 h0[NBW], h1[NBW];
#pragma unroll
  for (int j = 0; j < NBW; ++j) h0[j] = h1[j] = make_uint2(0, 0);
#pragma unroll
  for (int q = 0; q < RP_MB / 2; ++q) {
    const int mb0 = 2 * q, mb1 = 2 * q + 1;
    if constexpr (epi_reads_p(EPI)) {
      load_h(mb0, h0);
      load_h(mb1, h1);
    }
    const int m = m0 + 16 * (odd ? mb1 : mb0) + tl;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      uint2 y0, y1, p0, p1;
      compute(mb0, j, h0[j], y0, p0);
      compute(mb1, j, h1[j], y1, p1);
      // odd rows of (block mb0's words) <-> even rows of (block mb1's words)
      const auto s0 = __builtin_amdgcn_permlane16_swap(y0.x, y1.x, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(y0.y, y1.y, false, false);
      const uint4 out = odd ? make_uint4(s0[0], s1[0], y1.x, y1.y) : make_uint4(y0.x, y0.y, s0[1], s1[1]);
      const int c = cb + 16 * j - (odd ? 4 : 0);
      if (m < M) *(uint4*)(Y + (long)m * ldy + c) = out;
      if constexpr (epi_writes_p(EPI)) {
        if (P) {
          const auto t0 = __builtin_amdgcn_permlane16_swap(p0.x, p1.x, false, false);
          const auto t1 = __builtin_amdgcn_permlane16_swap(p0.y, p1.y, false, false);
          const uint4 po = odd ? make_uint4(t0[0], t1[0], p1.x, p1.y) : make_uint4(p0.x, p0.y, t0[1], t1[1]);
          if (m < M) *(uint4*)(P + (long)m * ldp + c) = po;
        }
      }
    }
  }
  if constexpr (RP_MB % 2 == 1) {  // the last block alone: 8-B stores
    constexpr int mb = RP_MB - 1;
    if constexpr (epi_reads_p(EPI)) load_h(mb, h0);
    const int m = m0 + 16 * mb + tl;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      uint2 y, p;
      compute(mb, j, h0[j], y, p);
      if (m < M) {
        *(uint2*)(Y + (long)m * ldy + cb + 16 * j) = y;
        if constexpr (epi_writes_p(EPI)) {
          if (P) *(uint2*)(P + (long)m * ldp + cb + 16 * j) = p;
        }
      }
    }
  }
}

// W = 8: one 512-thread workgroup per 144-row panel walks the N / 384 column chunks (one per CU).
// W = 4: a 256-thread workgroup per (panel, 192-column chunk), two per CU (2 x 74 KiB LDS): the
// epilogue of one (VALU + stores) runs beside the other's MFMA main loop instead of after it.
// EV = 1 (Y, and P when written, 16-B aligned with ldy, ldp multiples of 8): the transposed
// accumulators (panel_mainloop<W, true>) go out straight from registers — each lane holds 4
// consecutive columns of one row per block; one v_permlane16_swap per word pairs lane l's row
// of block mb with lane l ^ 16's of block mb + 1, so every lane stores 8 consecutive columns
// (16 B, 32 contiguous bytes per row per instruction): no LDS round trip, no barriers. The
// round-2 form (EV = 0: through an f32 LDS tile, 8-B stores, two barriers per 16-row block)
// measured 4.2 us of a 12.5-us workgroup on the qkv projection (tools/panel_stamps.py).
template <int EPI, int W, bool ST = false, int EV = 0>
__global__ __launch_bounds__(64 * W, 8 / W) void rowpanel_wide_kernel(const bf16* __restrict__ A, long lda, int M,
                                                                      int K, const u32x4* __restrict__ wpack, int N,
                                                                      const float* __restrict__ bias, int qcols,
                                                                      float qscale, bf16* __restrict__ Y, long ldy,
                                                                      bf16* __restrict__ P, long ldp, u64* stamps) {
  Stamps stp;
  if constexpr (ST) stp.begin();
  constexpr int CW = 48 * W, TLD = CW + 4, LPR = CW / 12;  // chunk width, T row stride, lanes per row
  __shared__ __attribute__((aligned(16))) char smem[RP_NS * RP_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nch = N / CW;
  int rp, nc_begin, nc_end;
  if constexpr (W == 8) {
    rp = xcd_remap(blockIdx.x, gridDim.x);
    nc_begin = 0;
    nc_end = nch;
  } else {  // (panel, chunk) with the chunks of a panel adjacent: one XCD, the A panel in one L2
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    rp = id / nch;
    nc_begin = id - rp * nch;
    nc_end = nc_begin + 1;
  }
  const int m0 = rp * RP_MT;
  const PanelA pa = panel_a_setup<W>(A, lda, M, m0, wv, lane);
  const int r = tid / LPR, c0 = (tid % LPR) * 12;  // row phase: LPR lanes per row, 12 columns each
  float* T = (float*)smem;                          // [16][TLD] after the main loop
#pragma unroll 1
  for (int nc = nc_begin; nc < nc_end; ++nc) {
    f32x4 acc[RP_MB][NBW];
    panel_mainloop<W, EV == 1>(acc, smem, pa, wpack, N / 16, nc * (CW / 16) + wv * NBW, K / 64, wv, lane,
                               ST && nc == nc_begin ? &stp.t1 : nullptr);
    if constexpr (ST) stp.t2 = clk_now();
    if constexpr (EV == 1) {
      if (nc + 1 < nc_end) __builtin_amdgcn_s_barrier();  // the next chunk's prologue rewrites the A ring
      wide_epilogue_tr<EPI>(acc, nc * CW + wv * NBW * 16, m0, M, bias, qcols, qscale, Y, ldy, P, ldp, lane);
      continue;
    }
    __builtin_amdgcn_s_barrier();  // every wave is done with the A ring
    const int n0 = nc * CW;
    float bv[NBW];
#pragma unroll
    for (int j = 0; j < NBW; ++j)
      bv[j] = (!epi_reads_p(EPI) && bias) ? bias[n0 + (wv * NBW + j) * 16 + (lane & 15)] : 0.f;
    const float qs = (EPI == EPI_QS && n0 < qcols) ? qscale : 1.f;  // qcols is a multiple of 384 (of CW)
    // P rows prefetched WPF blocks ahead (one block of a 192-column chunk is only 6 KiB: at one
    // block in flight the epilogue waited on the read latency, ~11 us of an 18-us workgroup)
    constexpr int WPF = RP_WPF;
    uint2 pvr[WPF][3];
    auto load_pre = [&](int mb) {
      const int m = min(m0 + 16 * mb + r, M - 1);
      const bf16* prow = P + (long)m * ldp + n0 + c0;
#pragma unroll
      for (int e = 0; e < 3; ++e) pvr[mb % WPF][e] = *(const uint2*)(prow + 4 * e);
    };
    if constexpr (epi_reads_p(EPI)) {
#pragma unroll
      for (int i = 0; i < WPF; ++i)
        if (i < RP_MB) load_pre(i);
    }
#pragma unroll
    for (int mb = 0; mb < RP_MB; ++mb) {
      uint2 (&pv)[3] = pvr[mb % WPF];
#pragma unroll
      for (int j = 0; j < NBW; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          T[(4 * (lane >> 4) + i) * TLD + (wv * NBW + j) * 16 + (lane & 15)] = acc[mb][j][i] + bv[j];
      lds_barrier();
      const int m = m0 + 16 * mb + r;
      float v[12];
#pragma unroll
      for (int e = 0; e < 12; e += 4) {
        const float4 tv = *(const float4*)(T + r * TLD + c0 + e);
        v[e] = tv.x; v[e + 1] = tv.y; v[e + 2] = tv.z; v[e + 3] = tv.w;
      }
      float h[12];
      if constexpr (epi_reads_p(EPI)) {
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          Pack4 q;
          q.u = pv[e];
#pragma unroll
          for (int k = 0; k < 4; ++k) h[4 * e + k] = (float)q.h[k];
        }
        if (mb + WPF < RP_MB) load_pre(mb + WPF);
      }
      if (m < M) {
        unsigned y[6], p[6];
#pragma unroll
        for (int e = 0; e < 12; e += 2) {
          float a = v[e], b = v[e + 1];
          if constexpr (EPI == EPI_QS) {
            a *= qs; b *= qs;
          } else if constexpr (EPI == EPI_GELU) {
            p[e / 2] = pk_bf16(a, b);
            a = gelu_t<bf16>(a); b = gelu_t<bf16>(b);
          } else if constexpr (EPI == EPI_GELUD) {
            float da, db;
            gelu_fast2(a, a, da);
            gelu_fast2(b, b, db);
            p[e / 2] = pk_bf16(da, db);
          } else if constexpr (EPI == EPI_DMUL) {
            a *= h[e]; b *= h[e + 1];
          } else {
            a *= gelu_grad_t<bf16>(h[e]); b *= gelu_grad_t<bf16>(h[e + 1]);
          }
          y[e / 2] = pk_bf16(a, b);
        }
        bf16* yrow = Y + (long)m * ldy + n0 + c0;
#pragma unroll
        for (int e = 0; e < 3; ++e) *(uint2*)(yrow + 4 * e) = make_uint2(y[2 * e], y[2 * e + 1]);
        if constexpr (epi_writes_p(EPI)) {
          if (P) {
            bf16* prow = P + (long)m * ldp + n0 + c0;
#pragma unroll
            for (int e = 0; e < 3; ++e) *(uint2*)(prow + 4 * e) = make_uint2(p[2 * e], p[2 * e + 1]);
          }
        }
      }
      __builtin_amdgcn_s_barrier();  // T is rewritten by the next block (or the next chunk's ring)
    }
  }
  if constexpr (ST) stp.end(stamps);
}

}  // namespace
}  // namespace ivit

using namespace ivit;

namespace {
template <bool BWD>
auto ln_kernel(bool st) {
  return st ? rowpanel_ln_kernel<BWD, true> : rowpanel_ln_kernel<BWD, false>;
}
// The wide kernel build for (EPI, stamps, epilogue form): EV = 1 needs 16-B aligned rows of Y
// (and of P when the kernel writes it). wide_epi: 0 (default) the LDS-tile form for every
// epilogue — in the bench step, beside the other ViT stream's attention, it beat the transposed
// form for QS / GELUD in 6 of 7 same-call pairs (43.67-43.87 vs 43.80-44.17 ms), though alone the
// transposed one is faster (GELUD 89.5 -> 85.8 us) and DMUL's LDS-tile form is faster either way
// (76.2 vs 83.6 us); 1: transposed for QS / GELUD; 2: transposed for all. Set by
// ivit_set_knob(IVIT_KNOB_WIDE_EPI) (the tests cover every form).
template <int EPI>
void launch_wide(dim3 g, hipStream_t st, bool ev1, u64* sb, const bf16* A, long lda, int M, int K, const u32x4* wp,
                 int N, const float* bias, int qcols, float qscale, bf16* Y, long ldy, bf16* P, long ldp) {
  const int mode = ivit_knob(IVIT_KNOB_WIDE_EPI);
  ev1 = ev1 && mode != 0 && (EPI == EPI_QS || EPI == EPI_GELUD || mode == 2);
  auto k = ev1 ? (sb ? rowpanel_wide_kernel<EPI, 4, true, 1> : rowpanel_wide_kernel<EPI, 4, false, 1>)
               : (sb ? rowpanel_wide_kernel<EPI, 4, true, 0> : rowpanel_wide_kernel<EPI, 4, false, 0>);
  hipLaunchKernelGGL(k, g, dim3(256), 0, st, A, lda, M, K, wp, N, bias, qcols, qscale, Y, ldy, P, ldp, sb);
}
bool al16_rows(const void* p, long ld) { return p == nullptr || (((uintptr_t)p & 15) == 0 && ld % 8 == 0); }
}  // namespace

extern "C" int ivit_linear_resid_ln_fwd(const void* A, long lda, long M, long N, long K, const void* wpack,
                                        const float* bias, const float* R, long ldr, const float* scale, long rps,
                                        const float* gamma, const float* beta, float eps, float* X, long ldx, void* Y,
                                        long ldy, float* mean, float* rstd, void* stream) {
  IVIT_CHECK_ARG(N == RP_N, "ivit_linear_resid_ln_fwd: N must be %d (got %ld)", RP_N, N);
  IVIT_CHECK_ARG(M > 0 && K > 0 && K % 64 == 0, "ivit_linear_resid_ln_fwd: K must be a positive multiple of 64");
  IVIT_CHECK_ARG(lda >= K && lda % 8 == 0 && ldr >= N && ldr % 4 == 0 && ldx >= N && ldx % 4 == 0 && ldy >= N &&
                     ldy % 4 == 0 && rps > 0,
                 "ivit_linear_resid_ln_fwd: bad leading dimensions");
  IVIT_CHECK_ARG(RP_MT * lda * 2 < (1L << 32) && M < (1L << 31), "ivit_linear_resid_ln_fwd: too large");
  IVIT_CHECK_ARG(((uintptr_t)A & 15) == 0 && ((uintptr_t)wpack & 15) == 0 && ((uintptr_t)R & 15) == 0 &&
                     ((uintptr_t)X & 15) == 0 && ((uintptr_t)Y & 7) == 0,
                 "ivit_linear_resid_ln_fwd: misaligned operand");
  u64* sb = ivit_stamp_buffer(ivit_cdiv(M, RP_MT));
  hipLaunchKernelGGL(ln_kernel<false>(sb != nullptr), dim3(ivit_cdiv(M, RP_MT)),
                     dim3(512), 0, ivit_stream(stream), (const bf16*)A, lda, (int)M, (int)K, (const u32x4*)wpack,
                     bias, R, ldr, scale, (int)rps, gamma, beta, eps, X, ldx, (bf16*)Y, ldy, mean, rstd, nullptr, 0L,
                     nullptr, sb);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" long ivit_linear_dgrad_ln_bwd_workspace(long M, long N) { return (long)ivit_cdiv(M, RP_MT) * 2 * N * 4; }

extern "C" int ivit_linear_dgrad_ln_bwd(const void* dY, long lddy, long M, long N, long K, const void* wpack_t,
                                        const float* X, long ldx, const float* gamma, const float* mean,
                                        const float* rstd, const float* dres, long ldr, float* dX, long lddx,
                                        void* dXs, const float* scale, long rps, float* dgamma, float* dbeta,
                                        int accumulate, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(N == RP_N, "ivit_linear_dgrad_ln_bwd: N must be %d (got %ld)", RP_N, N);
  IVIT_CHECK_ARG(M > 0 && K > 0 && K % 64 == 0, "ivit_linear_dgrad_ln_bwd: K must be a positive multiple of 64");
  IVIT_CHECK_ARG(lddy >= K && lddy % 8 == 0 && ldx >= N && ldx % 4 == 0 && lddx >= N && lddx % 4 == 0 &&
                     (!dres || (ldr >= N && ldr % 4 == 0)) && rps > 0,
                 "ivit_linear_dgrad_ln_bwd: bad leading dimensions");
  IVIT_CHECK_ARG(RP_MT * lddy * 2 < (1L << 32) && M < (1L << 31), "ivit_linear_dgrad_ln_bwd: too large");
  IVIT_CHECK_ARG(work_bytes >= ivit_linear_dgrad_ln_bwd_workspace(M, N), "ivit_linear_dgrad_ln_bwd: workspace too small");
  IVIT_CHECK_ARG(((uintptr_t)dY & 15) == 0 && ((uintptr_t)wpack_t & 15) == 0 && ((uintptr_t)X & 15) == 0 &&
                     ((uintptr_t)dX & 15) == 0 && ((uintptr_t)dres & 15) == 0 && ((uintptr_t)dXs & 7) == 0,
                 "ivit_linear_dgrad_ln_bwd: misaligned operand");
  hipStream_t st = ivit_stream(stream);
  const int nb = ivit_cdiv(M, RP_MT);
  u64* sb = ivit_stamp_buffer(nb);
  hipLaunchKernelGGL(ln_kernel<true>(sb != nullptr), dim3(nb), dim3(512), 0, st,
                     (const bf16*)dY, lddy, (int)M, (int)K, (const u32x4*)wpack_t, nullptr, dres, ldr, scale,
                     (int)rps, gamma, nullptr, 0.f, (float*)X, ldx, (bf16*)dXs, (long)RP_N, (float*)mean,
                     (float*)rstd, dX, lddx, (float*)work, sb);
  IVIT_LAUNCH_CHECK();
  launch_colreduce(st, (const float*)work, nb, 2 * N, (int)(2 * N), dgamma, (int)N, dbeta, accumulate);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_linear_fwd_panel(const void* A, long lda, long M, long N, long K, const void* wpack,
                                     const float* bias, int act, long qcols, float qscale, void* Y, long ldy,
                                     void* Ypre, long ldpre, void* stream) {
  IVIT_CHECK_ARG(M > 0 && N > 0 && N % RP_N == 0 && K > 0 && K % 64 == 0 && qcols % RP_N == 0,
                 "ivit_linear_fwd_panel: N and qcols must be multiples of %d, K of 64", RP_N);
  IVIT_CHECK_ARG(act == IVIT_ACT_NONE || ((act == IVIT_ACT_GELU || act == IVIT_ACT_GELU_D) && qcols == 0),
                 "ivit_linear_fwd_panel: bad act");
  IVIT_CHECK_ARG(lda >= K && lda % 8 == 0 && ldy >= N && ldy % 4 == 0 && (!Ypre || (ldpre >= N && ldpre % 4 == 0)),
                 "ivit_linear_fwd_panel: bad leading dimensions");
  IVIT_CHECK_ARG(RP_MT * lda * 2 < (1L << 32) && M < (1L << 31), "ivit_linear_fwd_panel: too large");
  IVIT_CHECK_ARG(((uintptr_t)A & 15) == 0 && ((uintptr_t)wpack & 15) == 0 && ((uintptr_t)Y & 7) == 0 &&
                     ((uintptr_t)Ypre & 7) == 0,
                 "ivit_linear_fwd_panel: misaligned operand");
  const dim3 g(ivit_cdiv(M, RP_MT) * (N / 192));
  hipStream_t st = ivit_stream(stream);
  u64* sb = ivit_stamp_buffer(g.x);
  if (act == IVIT_ACT_GELU_D)
    launch_wide<EPI_GELUD>(g, st, al16_rows(Y, ldy) && al16_rows(Ypre, ldpre), sb, (const bf16*)A, lda, (int)M,
                           (int)K, (const u32x4*)wpack, (int)N, bias, 0, 1.f, (bf16*)Y, ldy, (bf16*)Ypre, ldpre);
  else if (act == IVIT_ACT_GELU)
    launch_wide<EPI_GELU>(g, st, al16_rows(Y, ldy) && al16_rows(Ypre, ldpre), sb, (const bf16*)A, lda, (int)M,
                          (int)K, (const u32x4*)wpack, (int)N, bias, 0, 1.f, (bf16*)Y, ldy, (bf16*)Ypre, ldpre);
  else
    launch_wide<EPI_QS>(g, st, al16_rows(Y, ldy), sb, (const bf16*)A, lda, (int)M, (int)K, (const u32x4*)wpack,
                        (int)N, bias, (int)qcols, qscale, (bf16*)Y, ldy, nullptr, 0L);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_linear_dgrad_gelu_panel(const void* dY, long lddy, long M, long N, long K, const void* wpack_t,
                                            const void* pre, long ldpre, void* dX, long lddx, void* stream) {
  IVIT_CHECK_ARG(M > 0 && N > 0 && N % RP_N == 0 && K > 0 && K % 64 == 0,
                 "ivit_linear_dgrad_gelu_panel: N must be a multiple of %d, K of 64", RP_N);
  IVIT_CHECK_ARG(lddy >= K && lddy % 8 == 0 && lddx >= N && lddx % 4 == 0 && ldpre >= N && ldpre % 4 == 0,
                 "ivit_linear_dgrad_gelu_panel: bad leading dimensions");
  IVIT_CHECK_ARG(RP_MT * lddy * 2 < (1L << 32) && M < (1L << 31), "ivit_linear_dgrad_gelu_panel: too large");
  IVIT_CHECK_ARG(((uintptr_t)dY & 15) == 0 && ((uintptr_t)wpack_t & 15) == 0 && ((uintptr_t)dX & 7) == 0 &&
                     ((uintptr_t)pre & 7) == 0,
                 "ivit_linear_dgrad_gelu_panel: misaligned operand");
  const dim3 g(ivit_cdiv(M, RP_MT) * (N / 192));
  u64* sb = ivit_stamp_buffer(g.x);
  launch_wide<EPI_DGELU>(g, ivit_stream(stream), al16_rows(dX, lddx), sb, (const bf16*)dY, lddy, (int)M, (int)K,
                         (const u32x4*)wpack_t, (int)N, nullptr, 0, 1.f, (bf16*)dX, lddx, (bf16*)pre, ldpre);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_linear_dgrad_mul_panel(const void* dY, long lddy, long M, long N, long K, const void* wpack_t,
                                           const void* G, long ldg, void* dX, long lddx, void* stream) {
  IVIT_CHECK_ARG(M > 0 && N > 0 && N % RP_N == 0 && K > 0 && K % 64 == 0,
                 "ivit_linear_dgrad_mul_panel: N must be a multiple of %d, K of 64", RP_N);
  IVIT_CHECK_ARG(lddy >= K && lddy % 8 == 0 && lddx >= N && lddx % 4 == 0 && ldg >= N && ldg % 4 == 0,
                 "ivit_linear_dgrad_mul_panel: bad leading dimensions");
  IVIT_CHECK_ARG(RP_MT * lddy * 2 < (1L << 32) && M < (1L << 31), "ivit_linear_dgrad_mul_panel: too large");
  IVIT_CHECK_ARG(((uintptr_t)dY & 15) == 0 && ((uintptr_t)wpack_t & 15) == 0 && ((uintptr_t)dX & 7) == 0 &&
                     ((uintptr_t)G & 7) == 0,
                 "ivit_linear_dgrad_mul_panel: misaligned operand");
  const dim3 g(ivit_cdiv(M, RP_MT) * (N / 192));
  u64* sb = ivit_stamp_buffer(g.x);
  launch_wide<EPI_DMUL>(g, ivit_stream(stream), al16_rows(dX, lddx), sb, (const bf16*)dY, lddy, (int)M, (int)K,
                        (const u32x4*)wpack_t, (int)N, nullptr, 0, 1.f, (bf16*)dX, lddx, (bf16*)G, ldg);
  IVIT_LAUNCH_CHECK();
  return 0;
}
