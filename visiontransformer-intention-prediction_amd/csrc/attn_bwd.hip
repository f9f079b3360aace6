// Fused flash-attention backward (bf16) for the ViT blocks: timm Attention ->
// F.scaled_dot_product_attention backward, reached from model_vit.py:64,71,119.
// Compiled with -mllvm -amdgpu-mfma-vgpr-form (Makefile): with one wave per SIMD the dK / dV
// accumulators fill the AGPR half of the 512-register file and every other MFMA result must
// stay in VGPRs; the default AGPR-form allocation spills 52-168 VGPRs here.
#include <stdlib.h>

#include "attn_common.h"

namespace {

// ------------------------------------------------------------------------- backward (bf16, fused)
// One pass per (key block, batch, head) computes all five products of the flash backward
// (cdna_hip_programming.md, Appendix B "Attention backward"):
//   S = Q K^T - lse2 (row constant as the initial accumulator), dP = dO V^T - delta,
//   P = exp2(S), dS = P dP, dV += P^T dO, dK += dS^T Q, dQ += dS K.
// instead of the two-kernel form (dQ kernel: S, dP, dQ; dK/dV kernel: S, dP, dV, dK), which
// computed S, dP, P and dS twice (7 products, twice the exp / multiply / convert VALU).
// Layout: 4 waves, one per SIMD (512 registers each); a wave owns 96 keys (3 key tiles of 32:
// dK^T / dV^T accumulators 192 registers, V fragments 48; at 128 keys per wave the 320 resident
// registers left too few for the working set and the compiler parked V in AGPRs, re-reading it
// before every dP MFMA); the workgroup owns 384 keys
// (their K image in LDS: the B operand of S by rows and of dQ by transposed reads) and sweeps the
// queries in slices of 32 (Q / dO tiles and their row constants by LDS-DMA, double-buffered).
// Keys sit on the MFMA lane, so the accumulators of P and dS are already the operands of dV and
// dK (accumulator-as-operand); dS crosses LDS once, as a [key][q] image, for dQ.
// dQ: each slice's 32 x 64 dQ tile over the workgroup's 512 keys is split into eight 16x16
// tiles (two per wave, 16x16x32 MFMAs, A = dS and B = K by ds_read_b64_tr_b16) and stored as an
// f32 partial per key block; attn_dq_reduce_kernel sums the ceil(N/384) partials in a fixed order
// (deterministic, no atomics) and writes bf16 dQ.
constexpr int BKW = 96;        // keys per wave
constexpr int BKB = 4 * BKW;   // keys per workgroup (6 K tiles of 64)
constexpr int NKT = BKW / 32;  // key tiles per wave
constexpr int BQS = 64;        // queries per slice (two 32-row subtiles)

// Negated row constants for the fused backward, [z][NP] with NP = round64(N) + 64:
// nl = -lse * lmul (lmul = log2(e) for prescaled Q, 1/scale otherwise), -1e30 on padding rows
// (probabilities exactly 0), nd = -rowsum(dO * O) (0 on padding).
__global__ void attn_rows_neg_kernel(const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                     const float* __restrict__ lse, int B, int N, int NP, int H, float lmul,
                                     float* __restrict__ nlp, float* __restrict__ ndp) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long i = t >> 3;
  const int part = (int)(t & 7);
  if (i >= (long)B * H * NP) return;
  const int z = (int)(i / NP), n = (int)(i - (long)z * NP);
  float s = 0.f;
  if (n < N) {
    const int b = z / H, h = z - b * H, D = H * 64;
    const long off = ((long)b * N + n) * D + h * 64 + part * 8;
    Pack8 x, y;
    x.u = *(const uint4*)(o + off);
    y.u = *(const uint4*)(dout + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) s = fmaf(bf2f(x.h[j]), bf2f(y.h[j]), s);
  }
  s += __shfl_xor(s, 1, 8);
  s += __shfl_xor(s, 2, 8);
  s += __shfl_xor(s, 4, 8);
  if (part == 0) {
    ndp[i] = -s;
    nlp[i] = n < N ? -lse[(long)z * N + n] * lmul : -1e30f;
  }
}

// 32x32x16 operand with natural k order (element j of lane l <-> row rbase + 8(l>>5) + j, column
// l&31 of the 32-column block) from a t_off image (128-B rows, swz128 chunk swizzle): two
// transposing reads of 4 rows. `off` is the per-lane byte offset for rbase = 0 (lo half) —
// rows rbase + 16m keep the swizzle bits, so a k-step adds m * 2048 bytes.
IVIT_DEV int trn_off(int lane, int cbase, int hi) {
  const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = cbase + 16 * (G & 1) + 4 * p;
  return t_off(8 * (G >> 1) + 4 * hi + q, col >> 3) + (col & 7) * 2;
}
IVIT_DEV bf16x8 trn_read(const char* img, const int (&off)[2], int step) {
  union { s16x4 s[2]; bf16x8 v; } u;
  u.s[0] = ds_tr(img + off[0] + step * 2048);
  u.s[1] = ds_tr(img + off[1] + step * 2048);
  return u.v;
}

template <bool Q2>
__global__ __launch_bounds__(256, 1) void attn_bwd_fused_kernel(const bf16* __restrict__ qkv,
                                                                const bf16* __restrict__ dout,
                                                                const float* __restrict__ nlp,
                                                                const float* __restrict__ ndp, int N, int NP, int H,
                                                                bf16* __restrict__ dqkv, float* __restrict__ part,
                                                                float c2, float kscale) {
  __shared__ __attribute__((aligned(16))) char kimg[BKB * 128];   // the block's keys [key][d], t_off rows
  __shared__ __attribute__((aligned(16))) char dsimg[BKB * 128];  // dS of one slice [key][q], t_off rows
  __shared__ __attribute__((aligned(16))) char qimg[2][8192];     // Q slice, t_off image
  __shared__ __attribute__((aligned(16))) char gimg[2][8192];     // dO slice
  __shared__ __attribute__((aligned(16))) float srow[2][2][64];   // [stage][nl | nd][row]
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int2 bid = attn_block_id();
  const int kb = bid.x, z = bid.y, b = z / H, h = z - b * H;
  const int Z = gridDim.y;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16* Qb = qkv + (long)b * N * ld + h * 64;
  const bf16* Kb = Qb + D;
  const bf16* Vb = Qb + 2 * D;
  const bf16* Gb = dout + (long)b * N * D + h * 64;
  const float* NL = nlp + (long)z * NP;
  const float* ND = ndp + (long)z * NP;
  const int key0 = kb * BKB;
  const int ns = (N + BQS - 1) / BQS;

#pragma unroll
  for (int t = 0; t < BKB / 64; ++t) tile_glds_w<4>(Kb, ld, key0 + 64 * t, N, kimg + 8192 * t, wv, lane);
  auto issue = [&](int s, int st) {  // Q and dO slice tiles (64 rows): 2 pieces per wave each
    tile_glds_w<4>(Qb, ld, s * BQS, N, qimg[st], wv, lane);
    tile_glds_w<4>(Gb, D, s * BQS, N, gimg[st], wv, lane);
    if (wv == 0) {
      glds<4>((NL + s * BQS + lane), &srow[st][0][0]);
      glds<4>((ND + s * BQS + lane), &srow[st][1][0]);
    }
  };
  issue(0, 0);
  bf16x8 vf[NKT][4];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const int key = key0 + wv * BKW + 32 * kt + (lane & 31);
    load_row_frags(Vb + (long)key * ld, key < N, lane, vf[kt]);
  }
  retire_loads(vf[0], vf[1]);
  retire_loads(vf[NKT - 1], vf[NKT - 2]);
  f32x16 dk[NKT][2], dv[NKT][2];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int dd = 0; dd < 2; ++dd) {
      dk[kt][dd] = zero16();
      dv[kt][dd] = zero16();
    }
  const bool ragged = key0 + BKB > N;  // keys past N only in the last block
  // dQ tile of this wave: queries 32 qt.. of the slice, columns 32 dt..
  const int qt = wv & 1, dt = wv >> 1;
  int aoff[2], boff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    aoff[i] = trn_off(lane, 32 * qt, i);
    boff[i] = trn_off(lane, 32 * dt, i);
  }
  float* P0 = part + ((long)kb * Z + z) * N * 64;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int s = 0; s < ns; ++s) {
    const int st = s & 1;
    // slice s landed (the dQ partial stores of slice s - 1 may still be in flight)
    if (s > 0) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // B1: slice s visible; every wave is done with slice s - 1
    if (s + 1 < ns) issue(s + 1, st ^ 1);
    const char* qi = qimg[st];
    const char* gi = gimg[st];
#pragma unroll
    for (int t = 0; t < 2; ++t) {  // 32-query subtiles
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 qa[4], ga[4], qb[2][2], gb[2][2];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        qa[ks] = *(const bf16x8*)(qi + t_off(32 * t + (lane & 31), 2 * ks + hl));
        ga[ks] = *(const bf16x8*)(gi + t_off(32 * t + (lane & 31), 2 * ks + hl));
      }
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int dd = 0; dd < 2; ++dd) {
          qb[ss][dd] = tr_acc_order(qi, 32 * t + 16 * ss, 32 * dd, lane);
          gb[ss][dd] = tr_acc_order(gi, 32 * t + 16 * ss, 32 * dd, lane);
        }
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const int kw = wv * BKW + 32 * kt;  // first key of this tile within the block
        f32x16 sc, dp;  // row constants (-lse2, -delta) as the initial accumulators
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 a = *(const float4*)&srow[st][0][32 * t + 8 * g + 4 * hl];
          const float4 d = *(const float4*)&srow[st][1][32 * t + 8 * g + 4 * hl];
          sc[4 * g] = a.x; sc[4 * g + 1] = a.y; sc[4 * g + 2] = a.z; sc[4 * g + 3] = a.w;
          dp[4 * g] = d.x; dp[4 * g + 1] = d.y; dp[4 * g + 2] = d.z; dp[4 * g + 3] = d.w;
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const bf16x8 kf = *(const bf16x8*)(kimg + t_off(kw + (lane & 31), 2 * ks + hl));
          sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa[ks], kf, sc, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[ks], vf[kt][ks], dp, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = fast_exp2(Q2 ? sc[r] : sc[r] * c2);  // P[q][key]
        if (ragged) {  // wave-uniform: only the last key block has keys past N
          if (key0 + kw + (lane & 31) >= N) {
#pragma unroll
            for (int r = 0; r < 16; ++r) sc[r] = 0.f;
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) dp[r] *= sc[r];  // dS[q][key]
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const bf16x8 pa = pack_acc(sc, ss);
          const bf16x8 da = pack_acc(dp, ss);
          dv[kt][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, gb[ss][0], dv[kt][0], 0, 0, 0);
          dv[kt][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, gb[ss][1], dv[kt][1], 0, 0, 0);
          dk[kt][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, qb[ss][0], dk[kt][0], 0, 0, 0);
          dk[kt][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, qb[ss][1], dk[kt][1], 0, 0, 0);
          // dS (the same bf16 values) into the [key][q] image: q = 32t + 16ss + 8g2 + 4hl + 0..3
#pragma unroll
          for (int g2 = 0; g2 < 2; ++g2) {
            Pack4 w;
#pragma unroll
            for (int e = 0; e < 4; ++e) w.h[e] = da[4 * g2 + e];
            const int q = 32 * t + 16 * ss + 8 * g2 + 4 * hl;
            *(uint2*)(dsimg + t_off(kw + (lane & 31), q >> 3) + (q & 7) * 2) = w.u;
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // B2: dS of the slice complete for all the block's keys
    // dQ partial: dS[32 q][384 keys] . K[384 keys][32 d], 24 k-steps of 16 keys
    f32x16 dq = zero16();
#pragma unroll
    for (int k = 0; k < BKB / 16; ++k)
      dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trn_read(dsimg, aoff, k), trn_read(kimg, boff, k), dq, 0, 0, 0);
    // rows q = 32 qt + (r&3) + 8(r>>2) + 4hl, column 32 dt + (lane&31)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = s * BQS + 32 * qt + (r & 3) + 8 * (r >> 2) + 4 * hl;
      if (q < N) P0[(long)q * 64 + 32 * dt + (lane & 31)] = dq[r];
    }
  }
  // dK = kscale dS^T Q, dV = P^T dO: rows = keys (registers), columns = d (lanes)
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = key0 + wv * BKW + 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hl;
      if (key < N) {
        bf16* row = dqkv + ((long)b * N + key) * ld + h * 64 + (lane & 31);
        row[D] = (bf16)(dk[kt][0][r] * kscale);
        row[D + 32] = (bf16)(dk[kt][1][r] * kscale);
        row[2 * D] = (bf16)dv[kt][0][r];
        row[2 * D + 32] = (bf16)dv[kt][1][r];
      }
    }
}

// dQ = scale * sum over key blocks of the f32 partials (fixed order), bf16 into dqkv's Q block.
// One thread per (z, query, 8 columns): 16-B bf16 stores, float4 partial loads.
__global__ void attn_dq_reduce_kernel(const float* __restrict__ part, int nkb, int Z, int N, int H, float scale,
                                      bf16* __restrict__ dqkv) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)Z * N * 8) return;
  const int c = (int)(t & 7);
  const long zq = t >> 3;  // z * N + q
  const int z = (int)(zq / N), q = (int)(zq - (long)z * N);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const long plane = (long)Z * N * 64;
  const float* p = part + zq * 64 + 8 * c;
  for (int k = 0; k < nkb; ++k, p += plane) {
    const float4 x = *(const float4*)p, y = *(const float4*)(p + 4);
    a[0] += x.x; a[1] += x.y; a[2] += x.z; a[3] += x.w;
    a[4] += y.x; a[5] += y.y; a[6] += y.z; a[7] += y.w;
  }
  const int b = z / H, h = z - b * H;
  Pack8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o.h[j] = (bf16)(a[j] * scale);
  *(uint4*)(dqkv + ((long)b * N + q) * (3L * H * 64) + h * 64 + 8 * c) = o.u;
}



}  // namespace

namespace ivit {

// TEMPORARY development A/B switch (removed once the fused kernel is measured): IVIT_ATTN_BWD_OLD=1
bool bwd_old() {
  const char* v = getenv("IVIT_ATTN_BWD_OLD");
  return v && v[0] == '1';
}

long fused_np(long N) { return (N + 63) / 64 * 64 + 64; }
long fused_nkb(long N) { return (N + BKB - 1) / BKB; }
long attn_bwd_fused_ws(long B, long N, long H) {
  return 2 * B * H * fused_np(N) * 4 + fused_nkb(N) * B * H * N * 64 * 4;
}

int attn_bwd_fused(bool q2, const bf16* qkv, const bf16* out, const bf16* dout, const float* lse, long B, long N,
                   long H, bf16* dqkv, void* work, hipStream_t st) {
  const long Z = B * H, NP = fused_np(N), nkb = fused_nkb(N);
  const float scale = 0.125f;  // 1/sqrt(64)
  float* nlp = (float*)work;
  float* ndp = nlp + Z * NP;
  float* part = ndp + Z * NP;
  hipLaunchKernelGGL(attn_rows_neg_kernel, dim3(ivit_cdiv(Z * NP * 8, 256)), dim3(256), 0, st, out, dout, lse, (int)B,
                     (int)N, (int)NP, (int)H, q2 ? LOG2E : 1.0f / scale, nlp, ndp);
  if (q2)
    hipLaunchKernelGGL(attn_bwd_fused_kernel<true>, dim3(nkb, Z), dim3(256), 0, st, qkv, dout, nlp, ndp, (int)N,
                       (int)NP, (int)H, dqkv, part, 1.0f, 0.69314718055994531f);
  else
    hipLaunchKernelGGL(attn_bwd_fused_kernel<false>, dim3(nkb, Z), dim3(256), 0, st, qkv, dout, nlp, ndp, (int)N,
                       (int)NP, (int)H, dqkv, part, scale * LOG2E, scale);
  hipLaunchKernelGGL(attn_dq_reduce_kernel, dim3(ivit_cdiv(Z * N * 8, 256)), dim3(256), 0, st, part, (int)nkb, (int)Z,
                     (int)N, (int)H, scale, dqkv);
  return 0;
}

}  // namespace ivit
