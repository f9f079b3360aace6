
// Multi-head self-attention core (timm Attention -> F.scaled_dot_product_attention,
// reached from model_vit.py:64,71,119): O = softmax(Q K^T * Dh^-0.5) V per (batch, head).
//
// bf16 path: flash-style kernels, never materialising N x N.
//   forward : S^T = K Q^T (keys in registers, query on the lane) so the online-softmax
//             max/sum of a query are lane-local (+1 cross-half swap); O^T += V^T P^T takes
//             P^T straight from the S^T accumulator (no LDS round trip) and V^T by the
//             CDNA4 transposing LDS read.
//   backward: dQ kernel (query block, sweep keys) and dK/dV kernel (key block, sweep
//             queries); both recompute P from the saved LSE. No atomics. Both bf16 entry points
//             run the software-pipelined 16x16x32 v4 kernels: the ViT block path with Q prescaled
//             in qkv (ivit_attn_bwd_q2), the plain one (ivit_attn_bwd) on a prescaled Q copy.
// f32 path (parity): exact-f32 MFMA GEMMs through the generic engine with the score
//             matrix materialised in the workspace, plus row-softmax kernels.
#include "attn_common.h"

#include <hip/hip_ext.h>

#include <mutex>
#include <vector>

namespace {

// ------------------------------------------------------------------------- forward (bf16)
// Software-pipelined across key tiles, so the matrix pipe and the softmax VALU of ONE wave
// overlap (at head dim 64 the softmax is as long as the two products of a tile):
//   step j:  S_{j+1} = K_{j+1} Q^T  (8 MFMA)   ||  P_j = exp2(c2 S_j - m), cvt     (VALU)
//            O^T += V_j^T P_j^T, l += 1^T P_j^T  (8 + 4 MFMA) ||  rowmax(S_{j+1})  (VALU)
// One barrier per key tile: K runs two tiles ahead and V one (both double-buffered: K_j is dead
// once S_j exists, V_j once P_j V_j is issued). Lazy rescale: the running max m only moves when
// a tile's max exceeds it by more than TAU (log2 units), so P <= 2^TAU (exact in f32 / bf16
// range) and the O rescale branch is rare; O / l and lse = m + log2 l are unchanged by it.
constexpr float TAU = 8.0f;

// One v_max3_f32 (fmaxf on MFMA outputs makes the compiler canonicalise each operand with an
// extra v_max first: 3 instructions for what one does; scores are never NaN here).
IVIT_DEV float vmax3(float a, float b, float c) {
  float d;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// Per-lane LDS byte offsets of the forward's fragment reads, computed once per kernel: the 128-B-row
// chunk swizzle makes each read's address an XOR of lane bits with the k step (not base +
// immediate), and the compiler re-derived them inside the tile loop (~40 VALU per 64-key tile of
// a VALU-issue-bound loop). With these in registers every read is base + immediate (the stage and
// the row block differences are multiples that leave the swizzle bits unchanged).
//   k[ks]     : K fragment, row lane & 31, chunk 2 ks + hl        (+ 4096 per 32-key block)
//   v[cb][h]  : V^T transposing read, column block cb (0 / 32), row half h (+ 2048 per 16 keys)
struct FwdLdsOff {
  unsigned k[4], v[2][2];
};
IVIT_DEV FwdLdsOff fwd_lds_off(int lane) {
  FwdLdsOff o;
  const int hl = lane >> 5;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) o.k[ks] = (unsigned)t_off(lane & 31, 2 * ks + hl);
  const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int col = 32 * cb + 16 * (G & 1) + 4 * p;
    const int r0 = 4 * (G >> 1) + q, c = col >> 3, e = (col & 7) * 2;
    o.v[cb][0] = (unsigned)(t_off(r0, c) + e);
    o.v[cb][1] = (unsigned)(t_off(r0 + 8, c) + e);
  }
  // opaque: kept in registers, not re-derived from the lane id at every use
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(o.k[ks]));
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) asm volatile("" : "+v"(o.v[cb][0]), "+v"(o.v[cb][1]));
  return o;
}

template <bool MASK>
IVIT_DEV float tile_rowmax(f32x16 (&s)[2], int kbase, int N, int lane) {
  const int hl = lane >> 5;
  float a = NEG_BIG, b = NEG_BIG;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (MASK) {
        const int key = kbase + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (key >= N) s[t][r] = NEG_BIG;
      }
      if (r & 1) b = fmaxf(b, s[t][r]);  // two chains: v_max3-friendly and half the latency
      else a = fmaxf(a, s[t][r]);
    }
  return half_swap_max(fmaxf(a, b));
}

// ------------------------------------------------------------------------- forward v6 (bf16)
// v5 with the softmax scale and the running max folded into the matrix pipe: Q is prescaled by
// c2 = log2(e)/sqrt(Dh) once (in f32, rounded to bf16 — one more bf16 rounding of Q, the
// same size as the one the QKV GEMM output already carries), and every S chain starts from
// the accumulator -m (a persistent register block), so the MFMA returns S' - m directly and
// p = exp2(acc): the 32 v_fma_f32 per wave-tile (4 issue cycles each, of a VALU-issue-bound
// step: tools/pmc_anatomy.py) disappear. When the lazy rescale moves m, the already computed
// next tile is shifted by the same amount (rare).
IVIT_DEV void qk_tile_c(const char* kimg, const bf16x8 (&qf)[4], const f32x16& init, f32x16 (&s)[2], int lane) {
  const int hl = lane >> 5;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 ka = *(const bf16x8*)(kimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[ks], ks == 0 ? init : s[t], 0, 0, 0);
    }
  }
}

// kbase = the next tile's first key; when it is the ragged last tile (or past the end) its keys
// >= N are set to NEG_BIG before the row max (a uniform branch), so their P = exp2(.) is 0 in the
// next step.
IVIT_DEV float fwd_step_fenced6(const char* kimg, const char* vimg, const bf16x8 (&qf)[4], const f32x16 (&cur)[2],
                                f32x16 (&nxt)[2], f32x16& o0, f32x16& o1, f32x16& lacc, const bf16x8& ones,
                                const f32x16& negm, int lane, int kbase, int N, const FwdLdsOff& lo) {
  const int hl = lane >> 5;
  auto kfrag = [&](int i) { return *(const bf16x8*)(kimg + lo.k[i & 3] + 4096 * (i >> 2)); };
  // P of this tile as 16 packed words (word w = elements 2w, 2w + 1: two exp2 + one cvt_pk, ~21 issue
  // cycles, inside one 32x32x16 gap's 24 free), each pinned in the gap it is computed in: left to
  // the compiler, the exps of later words were sunk to their conversions and piled up in a few gaps
  unsigned pw[16];
  auto exw = [&](int w) {
    pw[w] = pk_bf16(fast_exp2(cur[(2 * w) >> 4][(2 * w) & 15]), fast_exp2(cur[(2 * w + 1) >> 4][(2 * w + 1) & 15]));
    asm volatile("" : "+v"(pw[w]));
  };
  auto pfrag = [&](int g) {
    return __builtin_bit_cast(bf16x8, make_uint4(pw[4 * g], pw[4 * g + 1], pw[4 * g + 2], pw[4 * g + 3]));
  };
  bf16x8 ka[8];
  ka[0] = kfrag(0);
  ka[1] = kfrag(1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i + 2 < 8) ka[i + 2] = kfrag(i + 2);
    const int t = i >> 2, ks = i & 3;
    nxt[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[i], qf[ks], ks == 0 ? negm : nxt[t], 0, 0, 0);
    exw(i);
    __builtin_amdgcn_sched_barrier(0);
  }
  bf16x8 vf[8];
  auto vread = [&](int f) {
    union { s16x4 s[2]; bf16x8 v; } u;
    u.s[0] = ds_tr(vimg + lo.v[f & 1][0] + 2048 * (f >> 1));
    u.s[1] = ds_tr(vimg + lo.v[f & 1][1] + 2048 * (f >> 1));
    vf[f] = u.v;
  };
  vread(0);
  vread(1);
  __builtin_amdgcn_sched_barrier(0);
  // words 8 .. 13 beside the first six P.V / row-sum MFMAs (words 8-11 are P[2], needed at k = 6),
  // words 14, 15 beside the next two (P[3], needed at k = 9)
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int g = k / 3, which = k % 3;
    if (k == 0) vread(2);
    if (k == 1) vread(3);
    if (k == 3) vread(4);
    if (k == 4) vread(5);
    if (which == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g], pfrag(g), o0, 0, 0, 0);
    else if (which == 1) o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g + 1], pfrag(g), o1, 0, 0, 0);
    else lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pfrag(g), lacc, 0, 0, 0);
    exw(8 + k);
    __builtin_amdgcn_sched_barrier(0);
  }
  float a = NEG_BIG, bm = NEG_BIG;
  if (kbase + AK > N) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kbase + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;
        nxt[t][r] = key >= N ? NEG_BIG : nxt[t][r];
      }
  }
#pragma unroll
  for (int k = 6; k < 12; ++k) {
    const int g = k / 3, which = k % 3;
    if (k == 6) vread(6);
    if (k == 7) vread(7);
    if (which == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g], pfrag(g), o0, 0, 0, 0);
    else if (which == 1) o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g + 1], pfrag(g), o1, 0, 0, 0);
    else lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pfrag(g), lacc, 0, 0, 0);
    if (k == 6) exw(14);
    if (k == 7) exw(15);
    const int v0 = 6 * (k - 6);
#pragma unroll
    for (int v = v0; v < v0 + 6 && v < 32; v += 2) {
      if ((v >> 1) & 1) bm = vmax3(bm, nxt[v >> 4][v & 15], nxt[v >> 4][(v & 15) + 1]);
      else a = vmax3(a, nxt[v >> 4][v & 15], nxt[v >> 4][(v & 15) + 1]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return half_swap_max(fmaxf(a, bm));  // max of S'_{j+1} - m
}

// PRE: prescale Q by c2 in the kernel (ivit_attn_fwd, plain qkv); otherwise the Q block of qkv
// already holds q * c2 (ivit_attn_fwd_q2).
template <int W, bool PRE>
__global__ __launch_bounds__(64 * W, 8 / W) void attn_fwd_bf16_v6_kernel(const bf16* __restrict__ qkv, int N, int H,
                                                                        bf16* __restrict__ out,
                                                                        float* __restrict__ lse, float c2) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][8192];  // [stage][K|V]
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int2 bid = attn_block_id();
  const int z = bid.y, b = z / H, h = z - b * H;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16* Qb = qkv + (long)b * N * ld + h * 64;
  const bf16* Kb = Qb + D;
  const bf16* Vb = Qb + 2 * D;
  const int q = bid.x * (32 * W) + wv * 32 + (lane & 31);
  bf16x8 qf[4];
  load_row_frags(Qb + (long)q * ld, q < N, lane, qf);
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[i][e] = (bf16)((float)qf[i][e] * c2);
  }
  const int nt = (N + AK - 1) / AK, nfull = N / AK;
  // saddr LDS-DMA (tile base in SGPRs, k-invariant 32-bit byte offsets); keys past N are clamped
  // to row N-1 (finite V rows; their scores are masked to P = 0)
  unsigned off[8 / W];
#pragma unroll
  for (int i = 0; i < 8 / W; ++i) off[i] = 2u * dma_off<W>(i, wv, lane, ld);
  auto issue1 = [&](const bf16* base, int kt, char* img) {
    const char* sb = uniform_ptr(base + (long)kt * AK * ld);
#pragma unroll
    for (int i = 0; i < 8 / W; ++i) {
      const int piece = wv * (8 / W) + i;
      unsigned o = off[i];
      if (kt >= nfull) {
        const int row = piece * 8 + (lane >> 3), c = (lane & 7) ^ swz128(row);
        o = 2u * (unsigned)((min(kt * AK + row, N - 1) - kt * AK) * ld + c * 8);
      }
      glds_s<false>(o, sb, img + piece * 1024);
    }
  };
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;

  // prologue: S'_0 (from a zero accumulator), m = its row max, then S'_0 - m; K_1 in flight
  issue1(Kb, 0, smem[0][0]);
  issue1(Vb, 0, smem[0][1]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (nt > 1) issue1(Kb, 1, smem[1][0]);
  if (bid.x * (32 * W) + wv * 32 >= N) {
    // a wave whose 32 queries are all past N (the ragged last row tile: at N = 4501 three of its four
    // waves) only keeps the workgroup's DMA / barrier cadence
    for (int j = 0; j < nt; ++j) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (j + 2 < nt) issue1(Kb, j + 2, smem[j & 1][0]);
      if (j + 1 < nt) issue1(Vb, j + 1, smem[(j & 1) ^ 1][1]);
    }
    return;
  }
  f32x16 sc[2], sn[2];
  qk_tile_c(smem[0][0], qf, zero16(), sc, lane);
  float m = nfull > 0 ? tile_rowmax<false>(sc, 0, N, lane) : tile_rowmax<true>(sc, 0, N, lane);
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[t][r] -= m;
  f32x16 negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) negm[r] = -m;
  f32x16 o0 = zero16(), o1 = zero16(), lacc = zero16();
  const FwdLdsOff lo = fwd_lds_off(lane);

  // after S'_{j+1} - m and its row max mt: move m lazily; the next tile is shifted with it
  auto rescale = [&](float mt, f32x16(&nxt)[2]) {
    const bool moved = mt > TAU;
    if (__any(moved)) {
      const float d = moved ? mt : 0.f;  // new m = m + d
      const float alpha = fast_exp2(-d);
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
      lacc[0] *= alpha;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) nxt[t][r] -= d;
      m += d;
      // in place (tied asm operands): negm keeps ONE register home across the rare branch, so
      // the common path needs no phi copies of its 16 registers
#pragma unroll
      for (int r = 0; r < 16; ++r) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(negm[r]) : "v"(d));
    }
  };
  // One key tile per body, all through the one fenced step; the next tile's keys past N are
  // masked inside it (the S' of a tile past the end is computed from the stale K stage and
  // discarded). A separate unfenced tail body (round 2) raised the kernel's register demand past
  // 256: 68 VGPRs spilled in the prologue (PMC: ~100 MB of scratch writes per launch).
  auto body = [&](auto stage, int j, f32x16(&cur)[2], f32x16(&nxt)[2]) {
    constexpr int S = decltype(stage)::value;  // V_j in smem[S][1], K_{j+1} in smem[S^1][0]
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (j + 2 < nt) issue1(Kb, j + 2, smem[S][0]);
    if (j + 1 < nt) issue1(Vb, j + 1, smem[S ^ 1][1]);
    rescale(fwd_step_fenced6(smem[S ^ 1][0], smem[S][1], qf, cur, nxt, o0, o1, lacc, ones, negm, lane,
                               (j + 1) * AK, N, lo),
              nxt);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  int j = 0;
  for (; j + 1 < nt; j += 2) {
    body(I0{}, j, sc, sn);
    body(I1{}, j + 1, sn, sc);
  }
  if (j < nt) body(I0{}, j, sc, sn);
  // epilogue: register 4g+e of o0 / o1 is dim 8g + 4hl + e (+32) of query q. One
  // v_permlane32_swap per word pairs lane q's half-block with lane q+32's, so each lane holds
  // 8 contiguous dims: lanes < 32 blocks g+1, lanes >= 32 blocks g (g even) — 16-B stores, 32
  // contiguous bytes per row per instruction (8-B stores left partial lines: PMC writes 4.7x)
  const float l = lacc[0];
  const float inv = 1.f / l;
  bf16* orow = out + ((long)b * N + (q < N ? q : 0)) * D + h * 64;
  auto emit = [&](const f32x16& o, int dbase) {
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
      const unsigned e0 = pk_bf16(o[4 * g] * inv, o[4 * g + 1] * inv);
      const unsigned e1 = pk_bf16(o[4 * g + 2] * inv, o[4 * g + 3] * inv);
      const unsigned d0 = pk_bf16(o[4 * g + 4] * inv, o[4 * g + 5] * inv);
      const unsigned d1 = pk_bf16(o[4 * g + 6] * inv, o[4 * g + 7] * inv);
      const auto s0 = __builtin_amdgcn_permlane32_swap(d0, e0, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(d1, e1, false, false);
      if (q < N) *(uint4*)(orow + dbase + 8 * (hl ? g : g + 1)) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
  };
  emit(o0, 0);
  emit(o1, 32);
  if (q < N && hl == 0) lse[(long)z * N + q] = (m + log2f(l)) * 0.69314718055994531f;
}

// ------------------------------------------------------------------------- Q prescale (plain entry)
// ivit_attn_bwd (bf16) on unscaled qkv: q' = bf16(q * c2), rounded as the forward's PRE path
// rounds its Q fragments, into a [B*N, D] workspace the v4 kernels read Q from (ldq = D).
__global__ void attn_prescale_q_kernel(const bf16* __restrict__ qkv, long rows, int D, float c2,
                                       bf16* __restrict__ q2) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;  // 8 columns per thread
  const int cpr = D / 8;
  if (t >= rows * cpr) return;
  const long r = t / cpr;
  const int c = (int)(t - r * cpr) * 8;
  Pack8 x;
  x.u = *(const uint4*)(qkv + r * 3 * D + c);
#pragma unroll
  for (int e = 0; e < 8; ++e) x.h[e] = (bf16)((float)x.h[e] * c2);
  *(uint4*)(q2 + r * D + c) = x.u;
}

// ------------------------------------------------------------------------- backward pipeline (prescaled Q)
// (The round-2 "v3" structure, kept by the 16x16x32 v4 kernels below.) The round-2 v2 loops were issue-bound: per 64x32 wave-tile of the dK/dV kernel ~140 VALU beside 32
// MFMAs (the element-wise bf16 packing re-shuffled by v_alignbit / v_perm, accumulator copies),
// and every S / dP chain MFMA waited (lgkmcnt) on the LDS read issued just before it. v3 keeps
// the same algorithm and data flow, software-pipelined over 32-row units u (half a 64-row tile):
//   body(u) = [ A(u): S / dP chains (8 MFMA)        || E(u-1): exp2, dS = P dP, cvt_pk (VALU),
//                                                       tr-reads for B(u-1)                  ]
//             [ B(u-1): the products fed by P / dS   || LDS reads of A(u+1)'s fragments and
//                       (dV/dK: 8 MFMA, dQ: 4 MFMA)       row constants                        ]
// so no MFMA waits on a read issued in its own gap and the softmax VALU of one unit runs under
// the matrix work of the next. 3 LDS stages: a tile's last reader (B of its second unit) runs in
// the first body of the following tile. One barrier per tile, in the middle of its second body:
// it publishes the next tile (DMA issued one tile ahead) and frees the stage of the tile before.

constexpr int BNS = 3;  // LDS stages of the pipelined backward kernels

// ------------------------------------------------------------------------- backward v4 (16x16x32)
// The dK/dV kernel with every product as v_mfma_f32_16x16x32_bf16 (MI355X_MICROARCH.md DVFS item 7:
// at equal cycles per flop the 16x16x32 loops held a higher clock than 32x32x16). Same algorithm,
// data flow, LDS stages and barrier cadence as v3; per wave 32 keys = 2 key blocks j of 16, per
// 32-row query unit 2 query blocks i of 16:
//   S_ij  = Q_i K_j^T  (C layout: lane (g = l >> 4, c = l & 15) holds rows 4g..4g+3 of q-block i,
//                       key 16j + c),  dP_ij = dO_i V_j^T  — 16 MFMA per unit, K_j / V_j in registers
//   dV_je += P_.j^T dO_.e,  dK_je += dS_.j^T Q_.e  (e = 16-column d block) — 16 MFMA per unit: the A
//     operand of key block j is (S_0j, S_1j) packed as they stand (k slot 8g + jj <-> query
//     4g + jj, jj < 4, else 16 + 4g + jj - 4), the B operand two transposing reads of 4 rows each.
// The row constants enter as the S / dP chains' initial accumulators (4 rows per lane instead of
// 16). Q / dO images: chunk c of row r at c ^ (r & 6) — conflict-free for the 16x16x32 row reads
// (16 rows x one chunk per 16-lane group) and for the transposed reads (8 rows x 2 chunks per
// half-wave); the 32x32 images' swz128 leaves the latter 2-way.
template <int W>
__global__ __launch_bounds__(64 * W, 8 / W) void attn_bwd_dkv_v4_kernel(const bf16* __restrict__ qkv,
                                                                 const bf16* __restrict__ dout,
                                                                 const float* __restrict__ nlse2p,
                                                                 const float* __restrict__ ndeltap, int N, int Npad,
                                                                 int H, bf16* __restrict__ dqkv, float scale,
                                                                 const bf16* __restrict__ qsrc, int ldq) {
  __shared__ __attribute__((aligned(16))) char smem[BNS][2][8192];  // [stage][Q|dO]
  __shared__ __attribute__((aligned(16))) float srow[BNS][2][AK];  // [stage][-lse2|-delta]
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = lane >> 4, c16 = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int2 bid = attn_block_id();
  const int z = bid.y, b = z / H, h = z - b * H;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16* Kb = qkv + (long)b * N * ld + D + h * 64;
  const bf16* Vb = Kb + D;
  const bf16* Qb = qsrc + (long)b * N * ldq + h * 64;  // q' (prescaled): in qkv, or the plain entry's copy
  const bf16* Gb = dout + (long)b * N * D + h * 64;
  const char* Ls = uniform_ptr(nlse2p + (long)z * Npad);
  const char* Ds = uniform_ptr(ndeltap + (long)z * Npad);
  constexpr int PW = 8 / W;
  const int kw = bid.x * (32 * W) + wv * 32;
  // B operands of S / dP: lane holds K[key 16j + c][dims 32s + 8g .. +7]
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = kw + 16 * j + c16;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Pack8 pk, pv;
      pk.u = key < N ? *(const uint4*)(Kb + (long)key * ld + 32 * s + 8 * g) : make_uint4(0, 0, 0, 0);
      pv.u = key < N ? *(const uint4*)(Vb + (long)key * ld + 32 * s + 8 * g) : make_uint4(0, 0, 0, 0);
      kf[j][s] = pk.v;
      vf[j][s] = pv.v;
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(kf[j][0]), "v"(kf[j][1]), "v"(vf[j][0]), "v"(vf[j][1]));
  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) dk[j][e] = dv[j][e] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nt = (N + AK - 1) / AK, nfull = N / AK;
  unsigned offq[PW], offg[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    offq[i] = 2u * dma_off16<W>(i, wv, lane, ldq);
    offg[i] = 2u * dma_off16<W>(i, wv, lane, D);
  }
  auto issue = [&](int qt, int S) {
    char* qimg = smem[S][0];
    char* gimg = smem[S][1];
    const char* qb = uniform_ptr(Qb + (long)qt * AK * ldq);
    const char* gb = uniform_ptr(Gb + (long)qt * AK * D);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int piece = wv * PW + i;
      unsigned oq = offq[i], og = offg[i];
      if (qt >= nfull) {
        const int row = piece * 8 + (lane >> 3), c = (lane & 7) ^ (row & 6);
        const int r = min(qt * AK + row, N - 1) - qt * AK;
        oq = 2u * (unsigned)(r * ldq + c * 8);
        og = 2u * (unsigned)(r * D + c * 8);
      }
      glds_s<false>(oq, qb, qimg + piece * 1024);
      glds_s<false>(og, gb, gimg + piece * 1024);
    }
    if (wv == 0) {
      glds4_s(4u * (lane + qt * AK), Ls, &srow[S][0][0]);
      glds4_s(4u * (lane + qt * AK), Ds, &srow[S][1][0]);
    }
  };
  // per-lane LDS offsets (the unit / block offsets 4096 t, 2048 i leave (r & 6) unchanged: immediates)
  unsigned ro[2], tro[4];
#pragma unroll
  for (int s = 0; s < 2; ++s) ro[s] = (unsigned)t16_off(c16, 4 * s + g);
  {
    const int q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
    for (int e = 0; e < 4; ++e) tro[e] = (unsigned)(t16_off(4 * g + q, 2 * e + (p >> 1)) + 8 * (p & 1));
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) asm volatile("" : "+v"(ro[s]));
#pragma unroll
  for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(tro[e]));

  bf16x8 qa[2][2], ga[2][2];   // A(u) fragments [i][s]
  f32x4 sn[2], dn[2];          // A(u+1)'s initial accumulators (-lse2 / -delta of its rows), [i]
  bf16x8 tg[4], tq[4];         // transposed dO / Q fragments of the pending B, [e]
  auto read_frag = [&](const char* qimg, const char* gimg, int t, int i, int s) {
    qa[i][s] = *(const bf16x8*)(qimg + ro[s] + 4096 * t + 2048 * i);
    ga[i][s] = *(const bf16x8*)(gimg + ro[s] + 4096 * t + 2048 * i);
  };
  auto read_rows = [&](const float* lr, const float* dr, int t, int i) {
    sn[i] = *(const f32x4*)(lr + 32 * t + 16 * i + 4 * g);
    dn[i] = *(const f32x4*)(dr + 32 * t + 16 * i + 4 * g);
  };
  auto word8 = [&](const unsigned (&w)[4]) { return __builtin_bit_cast(bf16x8, make_uint4(w[0], w[1], w[2], w[3])); };
  auto read_b = [&](const char* qimg, const char* gimg, int t, int e) {
    union { s16x4 s[2]; bf16x8 v; } a, c;
    a.s[0] = ds_tr(gimg + tro[e] + 4096 * t);
    a.s[1] = ds_tr(gimg + tro[e] + 4096 * t + 2048);
    c.s[0] = ds_tr(qimg + tro[e] + 4096 * t);
    c.s[1] = ds_tr(qimg + tro[e] + 4096 * t + 2048);
    tg[e] = a.v;
    tq[e] = c.v;
  };
  // E (exp2, dS = P dP, bf16 packing) of one unit is 8 pairs of elements — 16 exp, 16 mul, 16 cvt,
  // ~264 issue cycles against the 256 the unit's 32 MFMA gaps leave free — so it is spread over
  // BOTH halves of the body instead of the A half alone (where it took ~34 cycles per 2 MFMAs and
  // stalled the matrix pipe whenever the SIMD's other wave was in its A half too): the key-block-0
  // half of E(u) runs beside B(u-1)'s products, right after A(u), the key-block-1 half beside
  // A(u+1). One pair (i, hh) is four sub-steps, one per MFMA gap: exp, exp, two multiplies, two
  // conversions (8-9 issue cycles each).
  float ep0, ep1, et0, et1;
  // (each result is pinned where it is computed by an empty asm that "modifies" it: the pure
  // arithmetic would otherwise be sunk past the body's branches to its first use)
  auto e_sub = [&](const f32x4& S, const f32x4& DP, int hh, int ph, unsigned& wu, unsigned& wd) {
    if (ph == 0) {
      ep0 = fast_exp2(S[2 * hh]);
      asm volatile("" : "+v"(ep0));
    }
    if (ph == 1) {
      ep1 = fast_exp2(S[2 * hh + 1]);
      asm volatile("" : "+v"(ep1));
    }
    if (ph == 2) {
      et0 = ep0 * DP[2 * hh];
      et1 = ep1 * DP[2 * hh + 1];
      asm volatile("" : "+v"(et0), "+v"(et1));
    }
    if (ph == 3) {
      wu = pk_bf16(ep0, ep1);
      wd = pk_bf16(et0, et1);
      asm volatile("" : "+v"(wu), "+v"(wd));
    }
  };
  f32x4 sc1[2], dc1[2];        // A(u-1)'s key-block-1 results [i] (their E half runs beside A(u))
  unsigned upA[4], udA[4];     // key block 0 of the pending B: packed P / dS words
  unsigned up1[4], ud1[4];     // key block 1 of the pending B
  // body: A(u) on (SA, tA) || E(u-1) key block 1; B(u-1) on (SB, tB) || E(u) key block 0, reads of
  // A(u+1) on (SN, tN).
  auto body = [&](auto sa, auto ta, auto sb, auto tb, auto sn_, auto tn, auto bar, int jn, bool more) {
    constexpr int SA = decltype(sa)::value, TA = decltype(ta)::value, SB = decltype(sb)::value;
    constexpr int TB = decltype(tb)::value, SN = decltype(sn_)::value, TN = decltype(tn)::value;
    constexpr bool BAR = decltype(bar)::value;
    f32x4 s[2][2], dp[2][2];
    unsigned upN[4], udN[4];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int ks = m >> 3, i = (m >> 2) & 1, j = (m >> 1) & 1;
      if ((m & 1) == 0) s[i][j] = mfma16(qa[i][ks], kf[j][ks], ks == 0 ? sn[i] : s[i][j]);
      else dp[i][j] = mfma16(ga[i][ks], vf[j][ks], ks == 0 ? dn[i] : dp[i][j]);
      if (m == 0) read_frag(smem[SA][0], smem[SA][1], TA, 0, 1);
      if (m == 2) read_frag(smem[SA][0], smem[SA][1], TA, 1, 1);
      {  // E(u-1), key block 1: pair q = m / 4 (i = q >> 1, hh = q & 1), sub-step m % 4
        const int q = m >> 2, ie = q >> 1, hh = q & 1;
        e_sub(sc1[ie], dc1[ie], hh, m & 3, up1[2 * ie + hh], ud1[2 * ie + hh]);
      }
      if (m == 9) read_b(smem[SB][0], smem[SB][1], TB, 0);
      if (m == 12) read_b(smem[SB][0], smem[SB][1], TB, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (BAR) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (jn < nt) issue(jn, jn % BNS);
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int e = m >> 2, j = (m >> 1) & 1;
      if (m == 0) read_b(smem[SB][0], smem[SB][1], TB, 2);
      if (m == 2) read_b(smem[SB][0], smem[SB][1], TB, 3);
      if ((m & 1) == 0) dv[j][e] = mfma16(word8(j ? up1 : upA), tg[e], dv[j][e]);
      else dk[j][e] = mfma16(word8(j ? ud1 : udA), tq[e], dk[j][e]);
      {  // E(u), key block 0 (A(u)'s s[i][0] / dp[i][0], complete since its MFMA 13)
        const int q = m >> 2, ie = q >> 1, hh = q & 1;
        e_sub(s[ie][0], dp[ie][0], hh, m & 3, upN[2 * ie + hh], udN[2 * ie + hh]);
      }
      if (more) {
        if (m == 5) read_rows(srow[SN][0], srow[SN][1], TN, 0);
        if (m == 7) read_rows(srow[SN][0], srow[SN][1], TN, 1);
        if (m == 9) read_frag(smem[SN][0], smem[SN][1], TN, 0, 0);
        if (m == 11) read_frag(smem[SN][0], smem[SN][1], TN, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sc1[i] = s[i][1];
      dc1[i] = dp[i][1];
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      upA[w] = upN[w];
      udA[w] = udN[w];
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using F = std::false_type;
  using T = std::true_type;

  issue(0, 0);
  if (nt > 1) issue(1, 1);
  {
    uint4* z2 = (uint4*)&smem[2][0][0];  // B(-1)'s stage: finite zeros
    for (int i = tid; i < 2 * 8192 / 16; i += 64 * W) z2[i] = make_uint4(0, 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    read_rows(srow[0][0], srow[0][1], 0, i);
    read_frag(smem[0][0], smem[0][1], 0, i, 0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    sc1[i] = f32x4{NEG_BIG, NEG_BIG, NEG_BIG, NEG_BIG};  // exp2 -> 0: B(-1) adds zeros
    dc1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) upA[w] = udA[w] = 0u;
  if (kw >= N) {  // all 32 keys past N (ragged last key tile): the DMA / barrier cadence only
    for (int j = 0; j < nt; ++j) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (j + 2 < nt) issue(j + 2, (j + 2) % BNS);
    }
    __syncthreads();  // the store phase's barrier
    return;
  }
  auto tile = [&](auto st, int j) {
    constexpr int S = decltype(st)::value;
    using SP = std::integral_constant<int, (S + BNS - 1) % BNS>;
    using SNX = std::integral_constant<int, (S + 1) % BNS>;
    using SC = std::integral_constant<int, S>;
    body(SC{}, I0{}, SP{}, I1{}, SC{}, I1{}, F{}, 0, true);
    body(SC{}, I1{}, SC{}, I0{}, SNX{}, I0{}, T{}, j + 2, j + 1 < nt);
  };
  int j = 0;
  for (; j + 3 <= nt; j += 3) {
    tile(I0{}, j);
    tile(I1{}, j + 1);
    tile(I2{}, j + 2);
  }
  if (j < nt) tile(I0{}, j);
  if (j + 1 < nt) tile(I1{}, j + 1);
  {  // drain: the key-block-1 half of E and all of B for the last unit (tile nt-1, rows 32..63)
    const int S = (nt - 1) % BNS;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) e_sub(sc1[q >> 1], dc1[q >> 1], q & 1, ph, up1[q], ud1[q]);
#pragma unroll
    for (int e = 0; e < 4; ++e) read_b(smem[S][0], smem[S][1], 1, e);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      dv[0][e] = mfma16(word8(upA), tg[e], dv[0][e]);
      dk[0][e] = mfma16(word8(udA), tq[e], dk[0][e]);
      dv[1][e] = mfma16(word8(up1), tg[e], dv[1][e]);
      dk[1][e] = mfma16(word8(ud1), tq[e], dk[1][e]);
    }
  }
  // lane holds rows key 16j + 4g + r, column d = 16e + c16; stored through LDS as whole rows (2-byte
  // stores from the C layout: pair 0.7220-0.7222 vs 0.7187-0.7190 ms, profiles/r06_b_attn_epi_ab.txt)
  __syncthreads();  // every wave is past its last stage read: the stages become the store tiles
  char* tl = &smem[0][0][0] + wv * 2 * 4608;
  bf16* base = dqkv + (long)b * N * ld + h * 64;
  wave_tile_store(tl, dk, scale, base + D, ld, kw, N, lane);
  wave_tile_store(tl + 4608, dv, 1.0f, base + 2 * D, ld, kw, N, lane);
}

// ------------------------------------------------------------------------- dQ v4 (16x16x32)
// The dQ kernel in the 16x16x32 form of attn_bwd_dkv_v4_kernel: per wave 32 queries = 2 query
// blocks i of 16 (Q_i, dO_i as the B operands, in registers), per 32-key unit 2 key blocks j:
//   S^T_ji = K_j Q_i^T, dP^T_ji = V_j dO_i^T  (C layout: lane (g, c) holds keys 4g..4g+3 of block
//   j, query 16i + c; initial accumulators -lse2 / -delta of the lane's query)     16 MFMA per unit
//   dQ_ie += dS_i K_.e  (A operand (dS^T_0i, dS^T_1i) as they stand, B operand two transposing
//   reads of the K image: keys 4g.. and 16 + 4g.., columns 16e..)                    8 MFMA per unit
// The ragged last key tile (keys past N masked) runs through dq16_tile_masked afterwards.
IVIT_DEV void dq16_tile_masked(const char* kimg, const char* vimg, const bf16x8 (&qf)[2][2], const bf16x8 (&gf)[2][2],
                               const f32x4 (&nl)[2], const f32x4 (&nd)[2], f32x4 (&dq)[2][4], int kbase, int N,
                               int lane) {
  const int g = lane >> 4, c16 = lane & 15, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (kbase + 32 * t >= N) break;  // a 32-key unit wholly past N adds nothing (N = 4501: the second)
    f32x4 s[2][2], dp[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        s[j][i] = nl[i];
        dp[j][i] = nd[i];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 ka = *(const bf16x8*)(kimg + t16_off(32 * t + 16 * j + c16, 4 * ks + g));
          const bf16x8 va = *(const bf16x8*)(vimg + t16_off(32 * t + 16 * j + c16, 4 * ks + g));
          s[j][i] = mfma16(ka, qf[i][ks], s[j][i]);
          dp[j][i] = mfma16(va, gf[i][ks], dp[j][i]);
        }
      }
    unsigned w[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float d0 = fast_exp2(s[j][i][2 * hh]) * dp[j][i][2 * hh];
          float d1 = fast_exp2(s[j][i][2 * hh + 1]) * dp[j][i][2 * hh + 1];
          const int key = kbase + 32 * t + 16 * j + 4 * g + 2 * hh;
          if (key >= N) d0 = 0.f;
          if (key + 1 >= N) d1 = 0.f;
          w[i][2 * j + hh] = pk_bf16(d0, d1);
        }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int off = t16_off(32 * t + 4 * g + q, 2 * e + (p >> 1)) + 8 * (p & 1);
      union { s16x4 s[2]; bf16x8 v; } u;
      u.s[0] = ds_tr(kimg + off);
      u.s[1] = ds_tr(kimg + off + 2048);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        dq[i][e] = mfma16(__builtin_bit_cast(bf16x8, make_uint4(w[i][0], w[i][1], w[i][2], w[i][3])), u.v, dq[i][e]);
    }
  }
}

template <int W>
__global__ __launch_bounds__(64 * W, 8 / W) void attn_bwd_dq_v4_kernel(const bf16* __restrict__ qkv,
                                                                const bf16* __restrict__ dout,
                                                                float* __restrict__ nlse2p,
                                                                float* __restrict__ ndeltap, int N, int Npad, int H,
                                                                bf16* __restrict__ dqkv, float scale,
                                                                const bf16* __restrict__ out,
                                                                const float* __restrict__ lse,
                                                                const bf16* __restrict__ qsrc, int ldq) {
  __shared__ __attribute__((aligned(16))) char smem[BNS][2][8192];  // [stage][K|V]
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = lane >> 4, c16 = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int2 bid = attn_block_id();
  const int z = bid.y, b = z / H, h = z - b * H;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16* Kb = qkv + (long)b * N * ld + D + h * 64;
  const bf16* Vb = Kb + D;
  const bf16* Qb = qsrc + (long)b * N * ldq + h * 64;  // q' (prescaled)
  constexpr int PW = 8 / W;
  const int qw = bid.x * (32 * W) + wv * 32;
  // B operands: lane (g, c) holds Q / dO of query qw + 16i + c, dims 32s + 8g .. +7
  bf16x8 qf[2][2], gf[2][2];
  f32x4 nl[2], nd[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = qw + 16 * i + c16;
    const bool qv = q < N;
    bf16x8 of[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Pack8 pq, pg, po;
      const long orow = ((long)b * N + q) * D + h * 64 + 32 * s + 8 * g;
      pq.u = qv ? *(const uint4*)(Qb + (long)q * ldq + 32 * s + 8 * g) : make_uint4(0, 0, 0, 0);
      pg.u = qv ? *(const uint4*)(dout + orow) : make_uint4(0, 0, 0, 0);
      po.u = qv ? *(const uint4*)(out + orow) : make_uint4(0, 0, 0, 0);
      qf[i][s] = pq.v;
      gf[i][s] = pg.v;
      of[s] = po.v;
    }
    float d = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf((float)of[s][e], (float)gf[i][s][e], d);
    d += __shfl_xor(d, 16, 64);  // the query's 64 dims sit in lanes c, c + 16, c + 32, c + 48
    d += __shfl_xor(d, 32, 64);
    const float lse2 = qv ? lse[(long)z * N + q] * LOG2E : 1e30f;
    const float dlt = qv ? d : 0.f;
    if (g == 0 && q < Npad) {
      nlse2p[(long)z * Npad + q] = -lse2;
      ndeltap[(long)z * Npad + q] = -dlt;
    }
    nl[i] = f32x4{-lse2, -lse2, -lse2, -lse2};
    nd[i] = f32x4{-dlt, -dlt, -dlt, -dlt};
  }
  f32x4 dq[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) dq[i][e] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nt = (N + AK - 1) / AK, nfull = N / AK;
  unsigned off[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) off[i] = 2u * dma_off16<W>(i, wv, lane, ld);
  auto issue = [&](int kt, int S) {  // keys past N (ragged tile) are clamped to row N-1 and masked
    char* kimg = smem[S][0];
    char* vimg = smem[S][1];
    const char* kb = uniform_ptr(Kb + (long)kt * AK * ld);
    const char* vb = uniform_ptr(Vb + (long)kt * AK * ld);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int piece = wv * PW + i;
      unsigned o = off[i];
      if (kt >= nfull) {
        const int row = piece * 8 + (lane >> 3), c = (lane & 7) ^ (row & 6);
        o = 2u * (unsigned)((min(kt * AK + row, N - 1) - kt * AK) * ld + c * 8);
      }
      glds_s<false>(o, kb, kimg + piece * 1024);
      glds_s<false>(o, vb, vimg + piece * 1024);
    }
  };
  issue(0, 0);
  if (nt > 1) issue(1, 1);
  {
    uint4* z2 = (uint4*)&smem[2][0][0];
    for (int i = tid; i < 2 * 8192 / 16; i += 64 * W) z2[i] = make_uint4(0, 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  if (qw >= N) {  // all 32 queries past N (ragged last row tile): the DMA / barrier cadence only
    for (int j = 0; j < nfull; ++j) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (j + 2 < nt) issue(j + 2, (j + 2) % BNS);
    }
    if (nt > nfull) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    __syncthreads();  // the store phase's barrier
    return;
  }
  if (nfull > 0) {
    unsigned ro[2], tro[4];
#pragma unroll
    for (int s = 0; s < 2; ++s) ro[s] = (unsigned)t16_off(c16, 4 * s + g);
    {
      const int q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
      for (int e = 0; e < 4; ++e) tro[e] = (unsigned)(t16_off(4 * g + q, 2 * e + (p >> 1)) + 8 * (p & 1));
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) asm volatile("" : "+v"(ro[s]));
#pragma unroll
    for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(tro[e]));
    bf16x8 ka[2][2], va[2][2];  // A(u) fragments [j][ks]
    bf16x8 tk[4];               // transposed K fragments of the pending B, [e]
    auto read_a = [&](const char* kimg, const char* vimg, int t, int j, int ks) {
      ka[j][ks] = *(const bf16x8*)(kimg + ro[ks] + 4096 * t + 2048 * j);
      va[j][ks] = *(const bf16x8*)(vimg + ro[ks] + 4096 * t + 2048 * j);
    };
    auto read_b = [&](const char* kimg, int t, int e) {
      union { s16x4 s[2]; bf16x8 v; } u;
      u.s[0] = ds_tr(kimg + tro[e] + 4096 * t);
      u.s[1] = ds_tr(kimg + tro[e] + 4096 * t + 2048);
      tk[e] = u.v;
    };
    auto word8 = [&](const unsigned (&w)[4]) { return __builtin_bit_cast(bf16x8, make_uint4(w[0], w[1], w[2], w[3])); };
    // E (exp2, dS = P dP, bf16 packing) spread over both halves of the body as in the dK/dV kernel:
    // the query-block-0 half of E(u) beside B(u-1)'s 8 products (two sub-steps per gap), the
    // query-block-1 half beside A(u+1) (one per gap); results pinned where they are computed.
    float ep0, ep1, et0, et1;
    auto e_sub = [&](const f32x4& S, const f32x4& DP, int hh, int ph, unsigned& w) {
      if (ph == 0) {
        ep0 = fast_exp2(S[2 * hh]);
        asm volatile("" : "+v"(ep0));
      }
      if (ph == 1) {
        ep1 = fast_exp2(S[2 * hh + 1]);
        asm volatile("" : "+v"(ep1));
      }
      if (ph == 2) {
        et0 = ep0 * DP[2 * hh];
        et1 = ep1 * DP[2 * hh + 1];
        asm volatile("" : "+v"(et0), "+v"(et1));
      }
      if (ph == 3) {
        w = pk_bf16(et0, et1);
        asm volatile("" : "+v"(w));
      }
    };
    f32x4 sc1[2], dc1[2];  // A(u-1)'s query-block-1 results [j]
    unsigned pdqA[4];      // query block 0 of the pending B: packed dS words
    unsigned pdq1[4];      // query block 1 of the pending B
    auto body = [&](auto sa, auto ta, auto sb, auto tb, auto sn_, auto tn, auto bar, int jn, bool more) {
      constexpr int SA = decltype(sa)::value, TA = decltype(ta)::value, SB = decltype(sb)::value;
      constexpr int TB = decltype(tb)::value, SN = decltype(sn_)::value, TN = decltype(tn)::value;
      constexpr bool BAR = decltype(bar)::value;
      f32x4 s[2][2], dp[2][2];
      unsigned pdqN[4];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int ks = m >> 3, j = (m >> 2) & 1, i = (m >> 1) & 1;
        if ((m & 1) == 0) s[j][i] = mfma16(ka[j][ks], qf[i][ks], ks == 0 ? nl[i] : s[j][i]);
        else dp[j][i] = mfma16(va[j][ks], gf[i][ks], ks == 0 ? nd[i] : dp[j][i]);
        if (m == 0) read_a(smem[SA][0], smem[SA][1], TA, 0, 1);
        if (m == 2) read_a(smem[SA][0], smem[SA][1], TA, 1, 1);
        {  // E(u-1), query block 1: pair q = m / 4 (j = q >> 1, hh = q & 1), sub-step m % 4
          const int q = m >> 2, je = q >> 1, hh = q & 1;
          e_sub(sc1[je], dc1[je], hh, m & 3, pdq1[2 * je + hh]);
        }
        if (m == 8) read_b(smem[SB][0], TB, 0);
        if (m == 10) read_b(smem[SB][0], TB, 1);
        if (m == 12) read_b(smem[SB][0], TB, 2);
        if (m == 14) read_b(smem[SB][0], TB, 3);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (BAR) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (jn < nt) issue(jn, jn % BNS);
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int e = m >> 1, i = m & 1;
        dq[i][e] = mfma16(word8(i ? pdq1 : pdqA), tk[e], dq[i][e]);
        {  // E(u), query block 0 (A(u)'s s[j][0] / dp[j][0], complete since its MFMA 13): 2 sub-steps
          const int q = m >> 1, je = q >> 1, hh = q & 1;
          e_sub(s[je][0], dp[je][0], hh, 2 * (m & 1), pdqN[2 * je + hh]);
          e_sub(s[je][0], dp[je][0], hh, 2 * (m & 1) + 1, pdqN[2 * je + hh]);
        }
        if (more) {
          if (m == 1) read_a(smem[SN][0], smem[SN][1], TN, 0, 0);
          if (m == 3) read_a(smem[SN][0], smem[SN][1], TN, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        sc1[j] = s[j][1];
        dc1[j] = dp[j][1];
      }
#pragma unroll
      for (int w = 0; w < 4; ++w) pdqA[w] = pdqN[w];
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using F = std::false_type;
    using T = std::true_type;
#pragma unroll
    for (int j = 0; j < 2; ++j) read_a(smem[0][0], smem[0][1], 0, j, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      sc1[j] = f32x4{NEG_BIG, NEG_BIG, NEG_BIG, NEG_BIG};  // B(-1) adds zeros
      dc1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) pdqA[w] = 0u;
    auto tile = [&](auto st, int j) {
      constexpr int S = decltype(st)::value;
      using SP = std::integral_constant<int, (S + BNS - 1) % BNS>;
      using SNX = std::integral_constant<int, (S + 1) % BNS>;
      using SC = std::integral_constant<int, S>;
      body(SC{}, I0{}, SP{}, I1{}, SC{}, I1{}, F{}, 0, true);
      body(SC{}, I1{}, SC{}, I0{}, SNX{}, I0{}, T{}, j + 2, j + 1 < nfull);
    };
    int j = 0;
    for (; j + 3 <= nfull; j += 3) {
      tile(I0{}, j);
      tile(I1{}, j + 1);
      tile(I2{}, j + 2);
    }
    if (j < nfull) tile(I0{}, j);
    if (j + 1 < nfull) tile(I1{}, j + 1);
    {  // drain: the query-block-1 half of E and all of B for the last unit (tile nfull-1, keys 32..63)
      const int S = (nfull - 1) % BNS;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) e_sub(sc1[q >> 1], dc1[q >> 1], q & 1, ph, pdq1[q]);
#pragma unroll
      for (int e = 0; e < 4; ++e) read_b(smem[S][0], 1, e);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dq[0][e] = mfma16(word8(pdqA), tk[e], dq[0][e]);
        dq[1][e] = mfma16(word8(pdq1), tk[e], dq[1][e]);
      }
    }
  }
  if (nt > nfull) {  // ragged last key tile (DMA issued one tile ahead, or in the prologue)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int S = nfull % BNS;
    dq16_tile_masked(smem[S][0], smem[S][1], qf, gf, nl, nd, dq, nfull * AK, N, lane);
  }
  // lane holds rows q = qw + 16i + 4g + r, column d = 16e + c16 (stored through LDS as whole rows)
  __syncthreads();  // every wave is past its last stage read
  wave_tile_store(&smem[0][0][0] + wv * 4608, dq, scale, dqkv + (long)b * N * ld + h * 64, ld, qw, N, lane);
}

// ------------------------------------------------------------------------- f32 row kernels
// S rows (already scaled) -> P = softmax, zero padding columns; lse = max + log(sum).
__global__ void softmax_rows_kernel(float* __restrict__ S, long ldS, int N, float* __restrict__ lse) {
  const long row = blockIdx.x;  // z * N + q
  float* s = S + row * ldS;
  __shared__ float red[4];
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < N; i += 256) mx = fmaxf(mx, s[i]);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int i = threadIdx.x; i < N; i += 256) {
    const float e = expf(s[i] - mx);
    s[i] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  sum = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.f / sum;
  for (int i = threadIdx.x; i < ldS; i += 256) s[i] = i < N ? s[i] * inv : 0.f;
  if (threadIdx.x == 0) lse[row] = mx + logf(sum);
}

// P = exp(S - lse) (recompute in backward), zero padding.
__global__ void prob_rows_kernel(float* __restrict__ S, long ldS, int N, const float* __restrict__ lse) {
  const long row = blockIdx.x;
  float* s = S + row * ldS;
  const float l = lse[row];
  for (int i = threadIdx.x; i < ldS; i += 256) s[i] = i < N ? expf(s[i] - l) : 0.f;
}

// dS = P * (dP - rowsum(P * dP)) in place of dP.
__global__ void dsoftmax_rows_kernel(const float* __restrict__ P, float* __restrict__ dP, long ldS, int N) {
  const long row = blockIdx.x;
  const float* p = P + row * ldS;
  float* g = dP + row * ldS;
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < N; i += 256) s += p[i] * g[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  for (int i = threadIdx.x; i < ldS; i += 256) g[i] = i < N ? p[i] * (g[i] - s) : 0.f;
}

long ld_scores(long N) { return (N + 7) / 8 * 8; }

}  // namespace

// ------------------------------------------------------------------------- kernel timing
// ivit_ktime_arm / _read (ivit.h): while armed, the q2 entry points launch through
// hipExtLaunchKernel with an event pair bound to the kernel command, so the elapsed time is the
// kernel's own execution interval. Events are pooled across arm() calls.
namespace {
struct KtRec {
  int tag;
  hipEvent_t start, stop;
};
std::mutex kt_mu;
bool kt_on = false;
std::vector<KtRec> kt_recs;
std::vector<hipEvent_t> kt_pool;
size_t kt_used = 0;

hipEvent_t kt_event() {
  if (kt_used == kt_pool.size()) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    kt_pool.push_back(e);
  }
  return kt_pool[kt_used++];
}

// Launch through hipExtLaunchKernelGGL with a recorded event pair when armed, else plainly.
template <typename K, typename... Args>
void kt_launch(int tag, K kernel, dim3 g, dim3 b, hipStream_t st, Args... args) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  {
    std::lock_guard<std::mutex> lk(kt_mu);
    if (kt_on) {
      e0 = kt_event();
      e1 = e0 ? kt_event() : nullptr;
      if (e0 && e1) kt_recs.push_back({tag, e0, e1});
    }
  }
  if (e0 && e1)
    hipExtLaunchKernelGGL(kernel, g, b, 0, st, e0, e1, 0, args...);
  else
    hipLaunchKernelGGL(kernel, g, b, 0, st, args...);
}
}  // namespace


// The v4 backward pair; Q (prescaled by c2) is read from qsrc with row stride ldq: the Q block of
// qkv (ldq = 3D) on the q2 path, the plain entry's copy (ldq = D) otherwise.
namespace {
void attn_bwd_v4_launch(const void* qkv, const void* out, const void* dout, const float* lse, long B, long N, long H,
                        void* dqkv, float* nlse2p, const void* qsrc, int ldq, hipStream_t st) {
  const float scale = 0.125f;  // 1 / sqrt(64)
  const long Npad = (N + AK - 1) / AK * AK;
  float* ndeltap = nlse2p + B * H * Npad;
  // dQ also forms the row constants (-lse2, -delta) the dK/dV kernel reads: no rows kernel.
  // 4 waves per workgroup, two workgroups per CU: 8-wave workgroups (half the L2 -> LDS bytes,
  // one per CU) measured 0.875 vs 0.814 ms per pair (the 8-wave tile barrier, no second
  // independent workgroup to fill its gaps)
  constexpr int BW = 4;
  const dim3 gw(ivit_cdiv(N, 32 * BW), B * H);
  // the 16x16x32 forms (v4). Same-call A/B against the 32x32x16 v3 kernels they replaced (removed):
  // dK/dV 0.441-0.445 -> 0.406 ms, dQ 0.332-0.334 -> 0.316 ms isolated, step 44.07-44.14 -> 43.29 ms
  // with dK/dV alone (profiles/r05_b_attn_dkv16_ab.txt, r05_c_attn_dq16_ab.txt, r05_c_ab_dkv16_*.json)
  kt_launch(IVIT_KT_ATTN_BWD_DQ, attn_bwd_dq_v4_kernel<BW>, gw, dim3(64 * BW), st, (const bf16*)qkv,
            (const bf16*)dout, nlse2p, ndeltap, (int)N, (int)Npad, (int)H, (bf16*)dqkv, scale, (const bf16*)out, lse,
            (const bf16*)qsrc, ldq);
  kt_launch(IVIT_KT_ATTN_BWD_DKV, attn_bwd_dkv_v4_kernel<BW>, gw, dim3(64 * BW), st, (const bf16*)qkv,
            (const bf16*)dout, nlse2p, ndeltap, (int)N, (int)Npad, (int)H, (bf16*)dqkv, 0.69314718055994531f,
            (const bf16*)qsrc, ldq);
}
}  // namespace

// bf16 backward: the -lse2 and -delta rows (f32, padded to whole key tiles)
static long attn_rows_bytes(long B, long N, long H) { return 2 * B * H * ((N + AK - 1) / AK * AK) * 4; }

extern "C" long ivit_attn_workspace(int dtype, long B, long N, long H, long Dh, int backward) {
  // bf16 backward: the row constants + the prescaled Q copy of the plain entry (ivit_attn_bwd)
  if (dtype == IVIT_BF16) return backward ? attn_rows_bytes(B, N, H) + B * N * H * Dh * 2 : 0;
  const long one = B * H * N * ld_scores(N) * 4;
  return backward ? 2 * one : one;
}

extern "C" int ivit_attn_fwd(int dtype, const void* qkv, long B, long N, long H, long Dh, void* out, float* lse,
                             void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(Dh == 64, "ivit_attn_fwd: head dim must be 64 (got %ld)", Dh);
  IVIT_CHECK_ARG(work_bytes >= ivit_attn_workspace(dtype, B, N, H, Dh, 0), "ivit_attn_fwd: workspace too small");
  hipStream_t st = ivit_stream(stream);
  const float scale = 1.0f / sqrtf((float)Dh);
  if (B * N * H == 0) return 0;
  if (dtype == IVIT_BF16) {
    // prescaled-Q kernel with the c2 = log2(e)/sqrt(Dh) multiply done on the Q fragments
    dim3 g(ivit_cdiv(N, 128), B * H);
    hipLaunchKernelGGL((attn_fwd_bf16_v6_kernel<4, true>), g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H,
                       (bf16*)out, lse, scale * LOG2E);
    IVIT_LAUNCH_CHECK();
    return 0;
  }
  const long D = H * Dh, ldq = 3 * D, ldS = ld_scores(N);
  float* S = (float*)work;
  const float* Q = (const float*)qkv;
  // S = scale * Q K^T
  LdDense<float> la{Q, ldq, (int)N, (int)Dh, 0, 0, 0, {H, N * ldq, Dh}};
  LdDense<float> lb{Q + D, ldq, (int)N, (int)Dh, 0, 0, 0, {H, N * ldq, Dh}};
  EpiStore<float> es{S, ldS, {1, N * ldS, 0}, nullptr, IVIT_ACT_NONE, nullptr, scale};
  launch_gemm<true, true>(false, la, lb, es, (int)N, (int)N, (int)Dh, (int)(B * H), 1, st);
  hipLaunchKernelGGL(softmax_rows_kernel, dim3(B * H * N), dim3(256), 0, st, S, ldS, (int)N, lse);
  // O = P V
  LdDense<float> lp{S, ldS, (int)N, (int)ldS, 0, 0, 0, {1, N * ldS, 0}};
  LdDense<float> lv{Q + 2 * D, ldq, (int)N, (int)Dh, 0, 0, 0, {H, N * ldq, Dh}};
  EpiStore<float> eo{(float*)out, D, {H, N * D, Dh}, nullptr, IVIT_ACT_NONE, nullptr, 1.f};
  launch_gemm<true, false>(false, lp, lv, eo, (int)N, (int)Dh, (int)ldS, (int)(B * H), 1, st);
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_attn_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse, long B,
                             long N, long H, long Dh, void* dqkv, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(Dh == 64, "ivit_attn_bwd: head dim must be 64 (got %ld)", Dh);
  IVIT_CHECK_ARG(work_bytes >= ivit_attn_workspace(dtype, B, N, H, Dh, 1), "ivit_attn_bwd: workspace too small");
  hipStream_t st = ivit_stream(stream);
  const float scale = 1.0f / sqrtf((float)Dh);
  if (B * N * H == 0) return 0;
  const long D = H * Dh, ldq = 3 * D;
  if (dtype == IVIT_BF16) {
    // the product's v4 pair: Q prescaled by c2 = log2(e)/sqrt(Dh) into the workspace, as the
    // forward (ivit_attn_fwd) scales its fragments, then the q2 kernels reading Q from that copy
    float* nlse2p = (float*)work;
    bf16* q2 = (bf16*)((char*)work + attn_rows_bytes(B, N, H));
    hipLaunchKernelGGL(attn_prescale_q_kernel, dim3(ivit_cdiv(B * N * D / 8, 256)), dim3(256), 0, st,
                       (const bf16*)qkv, B * N, (int)D, scale * LOG2E, q2);
    attn_bwd_v4_launch(qkv, out, dout, lse, B, N, H, dqkv, nlse2p, q2, (int)D, st);
    IVIT_LAUNCH_CHECK();
    return 0;
  }
  const long ldS = ld_scores(N), zs = N * ldS;
  float* P = (float*)work;
  float* dP = P + B * H * zs;
  const float* Q = (const float*)qkv;
  float* dq = (float*)dqkv;
  const int Z = (int)(B * H);
  const BatchOff qoff{H, N * ldq, Dh}, soff{1, zs, 0}, ooff{H, N * D, Dh};
  // recompute P
  {
    LdDense<float> la{Q, ldq, (int)N, (int)Dh, 0, 0, 0, qoff};
    LdDense<float> lb{Q + D, ldq, (int)N, (int)Dh, 0, 0, 0, qoff};
    EpiStore<float> es{P, ldS, soff, nullptr, IVIT_ACT_NONE, nullptr, scale};
    launch_gemm<true, true>(false, la, lb, es, (int)N, (int)N, (int)Dh, Z, 1, st);
    hipLaunchKernelGGL(prob_rows_kernel, dim3(Z * N), dim3(256), 0, st, P, ldS, (int)N, lse);
  }
  // dV = P^T dO
  {
    LdDense<float> la{P, ldS, (int)N, (int)ldS, 0, 0, 0, soff};
    LdDense<float> lb{(const float*)dout, D, (int)N, (int)Dh, 0, 0, 0, ooff};
    EpiStore<float> e{dq + 2 * D, ldq, qoff, nullptr, IVIT_ACT_NONE, nullptr, 1.f};
    launch_gemm<false, false>(false, la, lb, e, (int)N, (int)Dh, (int)N, Z, 1, st);
  }
  // dP = dO V^T ; dS
  {
    LdDense<float> la{(const float*)dout, D, (int)N, (int)Dh, 0, 0, 0, ooff};
    LdDense<float> lb{Q + 2 * D, ldq, (int)N, (int)Dh, 0, 0, 0, qoff};
    EpiStore<float> e{dP, ldS, soff, nullptr, IVIT_ACT_NONE, nullptr, 1.f};
    launch_gemm<true, true>(false, la, lb, e, (int)N, (int)N, (int)Dh, Z, 1, st);
    hipLaunchKernelGGL(dsoftmax_rows_kernel, dim3(Z * N), dim3(256), 0, st, P, dP, ldS, (int)N);
  }
  // dQ = scale * dS K ; dK = scale * dS^T Q
  {
    LdDense<float> la{dP, ldS, (int)N, (int)ldS, 0, 0, 0, soff};
    LdDense<float> lb{Q + D, ldq, (int)N, (int)Dh, 0, 0, 0, qoff};
    EpiStore<float> e{dq, ldq, qoff, nullptr, IVIT_ACT_NONE, nullptr, scale};
    launch_gemm<true, false>(false, la, lb, e, (int)N, (int)Dh, (int)ldS, Z, 1, st);
  }
  {
    LdDense<float> la{dP, ldS, (int)N, (int)ldS, 0, 0, 0, soff};
    LdDense<float> lb{Q, ldq, (int)N, (int)Dh, 0, 0, 0, qoff};
    EpiStore<float> e{dq + D, ldq, qoff, nullptr, IVIT_ACT_NONE, nullptr, scale};
    launch_gemm<false, false>(false, la, lb, e, (int)N, (int)Dh, (int)N, Z, 1, st);
  }
  IVIT_LAUNCH_CHECK();
  return 0;
}

extern "C" int ivit_ktime_arm(int on) {
  std::lock_guard<std::mutex> lk(kt_mu);
  if (on) {
    kt_recs.clear();
    kt_used = 0;
  }
  kt_on = on != 0;
  return 0;
}

extern "C" int ivit_ktime_read(int tag, double* start_ms, double* stop_ms, long cap, long* count) {
  IVIT_CHECK_ARG(tag >= 0 && tag < IVIT_KT_NTAGS, "ivit_ktime_read: unknown tag %d", tag);
  IVIT_CHECK_ARG(count && (cap == 0 || (start_ms && stop_ms)), "ivit_ktime_read: null output");
  std::lock_guard<std::mutex> lk(kt_mu);
  long n = 0;
  for (const KtRec& r : kt_recs) {
    if (r.tag != tag) continue;
    // times relative to the first recorded launch's start event (all tags share it)
    float t0 = 0.f, t1 = 0.f;
    hipError_t e = hipEventSynchronize(r.stop);
    if (e == hipSuccess) e = hipEventElapsedTime(&t0, kt_recs[0].start, r.start);
    if (e == hipSuccess) e = hipEventElapsedTime(&t1, kt_recs[0].start, r.stop);
    if (e != hipSuccess) {
      ivit_set_error("ivit_ktime_read: %s", hipGetErrorString(e));
      return (int)e;
    }
    if (n < cap) {
      start_ms[n] = t0;
      stop_ms[n] = t1;
    }
    ++n;
  }
  *count = n;
  return 0;
}

// ------------------------------------------------------------------------- Q-prescaled bf16 path
extern "C" int ivit_attn_fwd_q2(const void* qkv, long B, long N, long H, long Dh, void* out, float* lse, void* work,
                                long work_bytes, void* stream) {
  IVIT_CHECK_ARG(Dh == 64, "ivit_attn_fwd_q2: head dim must be 64 (got %ld)", Dh);
  (void)work;
  (void)work_bytes;
  if (B * N * H == 0) return 0;
  dim3 g(ivit_cdiv(N, 128), B * H);
  // (a 16x16x32 form of this kernel measured slower: 0.295-0.302 vs 0.281-0.283 ms isolated, 43.65-43.88
  // vs 42.77-42.83 ms per step, profiles/r05_d_attn_fwd16_ab.txt; removed)
  kt_launch(IVIT_KT_ATTN_FWD, attn_fwd_bf16_v6_kernel<4, false>, g, dim3(256), ivit_stream(stream), (const bf16*)qkv,
            (int)N, (int)H, (bf16*)out, lse, 1.0f);
  IVIT_LAUNCH_CHECK();
  return 0;
}

// With q' = q c2 in qkv: P = exp2(q'k - lse2) (c2 = 1 in the kernels); dQ = scale dS K as before
// (the gradient w.r.t. the unscaled q); dK = ln2 dS^T q' = scale dS^T q.
// With q' = q c2 in qkv: P = exp2(q'k - lse2) (c2 = 1 in the kernels); dQ = scale dS K as before
// (the gradient w.r.t. the unscaled q); dK = ln2 dS^T q' = scale dS^T q.
extern "C" int ivit_attn_bwd_q2(const void* qkv, const void* out, const void* dout, const float* lse, long B, long N,
                                long H, long Dh, void* dqkv, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(Dh == 64, "ivit_attn_bwd_q2: head dim must be 64 (got %ld)", Dh);
  IVIT_CHECK_ARG(work_bytes >= attn_rows_bytes(B, N, H), "ivit_attn_bwd_q2: workspace too small");
  if (B * N * H == 0) return 0;
  attn_bwd_v4_launch(qkv, out, dout, lse, B, N, H, dqkv, (float*)work, qkv, (int)(3 * H * Dh), ivit_stream(stream));
  IVIT_LAUNCH_CHECK();
  return 0;
}
