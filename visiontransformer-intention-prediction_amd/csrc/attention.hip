// Multi-head self-attention core (timm Attention -> F.scaled_dot_product_attention,
// reached from model_vit.py:64,71,119): O = softmax(Q K^T * Dh^-0.5) V per (batch, head).
//
// bf16 path: flash-style kernels, never materialising N x N.
//   forward : S^T = K Q^T (keys in registers, query on the lane) so the online-softmax
//             max/sum of a query are lane-local (+1 cross-half swap); O^T += V^T P^T takes
//             P^T straight from the S^T accumulator (no LDS round trip) and V^T by the
//             CDNA4 transposing LDS read.
//   backward: dQ kernel (query block, sweep keys) and dK/dV kernel (key block, sweep
//             queries); both recompute P from the saved LSE. No atomics.
// f32 path (parity): exact-f32 MFMA GEMMs through the generic engine with the score
//             matrix materialised in the workspace, plus row-softmax kernels.
#include <stdlib.h>

#include <mutex>

#include "gemm_engine.h"

using namespace ivit;

namespace {

constexpr int AQ = 128;  // queries per workgroup (4 waves x 32)
constexpr int AK = 64;   // keys per tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float NEG_BIG = -1.0e30f;

// tile image: 64 rows x 64 bf16 (128-B rows), chunk swizzle swz128 (see gemm_engine.h)
IVIT_DEV int t_off(int r, int c) { return r * 128 + ((c ^ swz128(r)) << 4); }

// Load a 64 x 64 bf16 tile (rows r0.., cols c0.. of a row-major matrix with row stride ld)
// into registers: 512 16-B chunks, 2 per thread. Rows >= nrows are zero.
IVIT_DEV void tile_gload(const bf16* base, long ld, int r0, int nrows, int tid, uint4 (&r)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = tid + 256 * i, row = idx >> 3, ch = idx & 7;
    r[i] = (r0 + row < nrows) ? *(const uint4*)(base + (long)(r0 + row) * ld + ch * 8) : make_uint4(0, 0, 0, 0);
  }
}
// The same 64 x 64 tile by LDS-DMA: 8 lane-linear 1-KiB pieces (2 per wave), the chunk
// swizzle applied to the per-lane source address; rows >= nrows read the zero page.
IVIT_DEV void tile_glds(const bf16* base, long ld, int r0, int nrows, char* img, int wv, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wv * 2 + i;
    const int row = piece * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz128(row);
    const void* src = (r0 + row < nrows) ? (const void*)(base + (long)(r0 + row) * ld + c * 8) : (const void*)g_zero16;
    glds<16>(src, img + piece * 1024);
  }
}
IVIT_DEV void tile_sstore(char* img, int tid, const uint4 (&r)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = tid + 256 * i;
    *(uint4*)(img + t_off(idx >> 3, idx & 7)) = r[i];
  }
}

// 32x32x16 operand from a [row = reduction index][col] tile image by transposing reads,
// with the k order an f32 32x32 accumulator uses when fed back as an operand
// (element j of lane-half h <-> reduction row rb + 8(j>>2) + 4h + (j&3); cdna_hip_programming.md §3).
IVIT_DEV bf16x8 tr_acc_order(const char* img, int rb, int colbase, int lane) {
  const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = colbase + 16 * (G & 1) + 4 * p;
  const int r0 = rb + 4 * (G >> 1) + q;
  const int c = col >> 3, e = (col & 7) * 2;
  union { s16x4 s[2]; bf16x8 v; } u;
  u.s[0] = ds_tr(img + t_off(r0, c) + e);
  u.s[1] = ds_tr(img + t_off(r0 + 8, c) + e);
  return u.v;
}

// Pack accumulator registers 8s..8s+7 (f32) into a bf16x8 operand.
IVIT_DEV bf16x8 pack_acc(const f32x16& a, int s) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)a[8 * s + j];
  return v;
}

// Register operand: lane l holds row (l&31), k = 16s + 8(l>>5) .. +7 of a 64-wide row.
IVIT_DEV void load_row_frags(const bf16* rowp, bool valid, int lane, bf16x8 (&f)[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    Pack8 p;
    p.u = valid ? *(const uint4*)(rowp + 16 * s + 8 * (lane >> 5)) : make_uint4(0, 0, 0, 0);
    f[s] = p.v;
  }
}

IVIT_DEV f32x16 zero16() {
  f32x16 a;
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = 0.f;
  return a;
}

// ------------------------------------------------------------------------- forward (bf16)
// (query or key block, b*H + h) of this workgroup. Workgroups reach the 8 XCDs round-robin in
// flat dispatch order (x fastest); remapping the flat id gives each XCD a contiguous run of
// blocks, i.e. whole (b, h) pairs, so each pair's K/V (or Q/dO) panel is fetched into ONE L2
// and shared by its ~36 blocks. With blockIdx.y = (b, h) directly, a pair's blocks spread
// over all 8 XCDs and every attention launch read its operands ~5x from HBM (PMC FETCH_SIZE).
IVIT_DEV int2 attn_block_id() {
  const int nb = gridDim.x;
  const int flat = xcd_remap(blockIdx.x + blockIdx.y * nb, nb * gridDim.y);
  return make_int2(flat % nb, flat / nb);
}

__global__ __launch_bounds__(256, 2) void attn_fwd_bf16_kernel(const bf16* __restrict__ qkv, int N, int H,
                                                               bf16* __restrict__ out, float* __restrict__ lse,
                                                               float c2) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][8192];  // [stage][K|V]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hl = lane >> 5;
  const int2 bid = attn_block_id();
  const int z = bid.y, b = z / H, h = z - b * H;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16* Qb = qkv + (long)b * N * ld + h * 64;
  const bf16* Kb = Qb + D;
  const bf16* Vb = Qb + 2 * D;
  const int q = bid.x * AQ + wv * 32 + (lane & 31);

  bf16x8 qf[4];
  load_row_frags(Qb + (long)q * ld, q < N, lane, qf);

  f32x16 o0 = zero16(), o1 = zero16();
  float m = NEG_BIG, l = 0.f;
  const int nt = (N + AK - 1) / AK;
  uint4 rk[2], rv[2];
  tile_gload(Kb, ld, 0, N, tid, rk);
  tile_gload(Vb, ld, 0, N, tid, rv);
  tile_sstore(smem[0][0], tid, rk);
  tile_sstore(smem[0][1], tid, rv);
  __syncthreads();
  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nt) {
      tile_gload(Kb, ld, (kt + 1) * AK, N, tid, rk);
      tile_gload(Vb, ld, (kt + 1) * AK, N, tid, rv);
    }
    const char* kimg = smem[cur][0];
    const char* vimg = smem[cur][1];
    f32x16 s[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t] = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 ka = *(const bf16x8*)(kimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
        s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[ks], s[t], 0, 0, 0);
      }
    }
    // scale into the log2 domain, mask keys >= N, row max over this tile
    float mx = NEG_BIG;
    const int kbase = kt * AK;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kbase + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const float v = key < N ? s[t][r] * c2 : NEG_BIG;
        s[t][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = half_swap_max(mx);
    const float mn = fmaxf(m, mx);
    const float alpha = fast_exp2(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fast_exp2(s[t][r] - mn);
        s[t][r] = p;
        rs += p;
      }
    rs = half_swap_sum(rs);
    l = l * alpha + rs;
    m = mn;
#pragma unroll
    for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 pb = pack_acc(s[t], ss);
        const int rb = 32 * t + 16 * ss;
        const bf16x8 va0 = tr_acc_order(vimg, rb, 0, lane);
        const bf16x8 va1 = tr_acc_order(vimg, rb, 32, lane);
        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va0, pb, o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va1, pb, o1, 0, 0, 0);
      }
    if (kt + 1 < nt) {
      tile_sstore(smem[cur ^ 1][0], tid, rk);
      tile_sstore(smem[cur ^ 1][1], tid, rv);
    }
    __syncthreads();
  }
  if (q < N) {
    const float inv = 1.f / l;
    bf16* orow = out + ((long)b * N + q) * D + h * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      Pack4 a, c;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a.h[j] = (bf16)(o0[4 * g + j] * inv);
        c.h[j] = (bf16)(o1[4 * g + j] * inv);
      }
      const int d = 8 * g + 4 * hl;  // rows (r&3) + 8(r>>2) + 4h of O^T
      *(uint2*)(orow + d) = a.u;
      *(uint2*)(orow + 32 + d) = c.u;
    }
    if (hl == 0) lse[(long)z * N + q] = (m + log2f(l)) * 0.69314718055994531f;
  }
}

// ------------------------------------------------------------------------- forward v2 (bf16)
// 64 queries per wave (two 32-query groups share every K/V fragment read: half the LDS bytes
// per MFMA of v1), 256 queries per workgroup. Softmax per score: one FMA (scale folded in)
// + one exp2; key masking only on the last (partial) tile; the O rescale is skipped when no
// lane's running max moved (exact, wave-uniform test).
constexpr int AQ2 = 256;

template <bool MASK>
IVIT_DEV void fwd_tile2(const char* kimg, const char* vimg, const bf16x8 (&qf)[2][4], f32x16 (&o)[2][2],
                        float (&m)[2], float (&l)[2], int kbase, int N, float c2, int lane) {
  const int hl = lane >> 5;
  // one 32-key sub-tile at a time: scores for both query groups = 32 live f32 registers
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    f32x16 s[2] = {zero16(), zero16()};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 ka = *(const bf16x8*)(kimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[0][ks], s[0], 0, 0, 0);
      s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[1][ks], s[1], 0, 0, 0);
    }
    bool moved = false;
    float alpha[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      float mx = NEG_BIG;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (MASK) {
          const int key = kbase + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (key >= N) s[g][r] = NEG_BIG;
        }
        mx = fmaxf(mx, s[g][r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[g], mx * c2);
      alpha[g] = exp2f(m[g] - mn);
      moved |= mn != m[g];
      m[g] = mn;
      float rs = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = exp2f(fmaf(s[g][r], c2, -mn));
        s[g][r] = p;
        rs += p;
      }
      rs += __shfl_xor(rs, 32, 64);
      l[g] = l[g] * alpha[g] + rs;
    }
    if (__any(moved)) {
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) { o[g][0][r] *= alpha[g]; o[g][1][r] *= alpha[g]; }
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const int rb = 32 * t + 16 * ss;
      const bf16x8 va0 = tr_acc_order(vimg, rb, 0, lane);
      const bf16x8 va1 = tr_acc_order(vimg, rb, 32, lane);
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const bf16x8 pb = pack_acc(s[g], ss);
        o[g][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va0, pb, o[g][0], 0, 0, 0);
        o[g][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va1, pb, o[g][1], 0, 0, 0);
      }
    }
  }
}

__global__ __launch_bounds__(256, 2) void attn_fwd_bf16_v2_kernel(const bf16* __restrict__ qkv, int N, int H,
                                                                  bf16* __restrict__ out, float* __restrict__ lse,
                                                                  float c2) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][8192];  // [stage][K|V]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hl = lane >> 5;
  const int2 bid = attn_block_id();
  const int z = bid.y, b = z / H, h = z - b * H;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16* Qb = qkv + (long)b * N * ld + h * 64;
  const bf16* Kb = Qb + D;
  const bf16* Vb = Qb + 2 * D;
  const int qw = bid.x * AQ2 + wv * 64;
  bf16x8 qf[2][4];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int q = qw + 32 * g + (lane & 31);
    load_row_frags(Qb + (long)q * ld, q < N, lane, qf[g]);
  }
  f32x16 o[2][2];
  float m[2] = {NEG_BIG, NEG_BIG}, l[2] = {0.f, 0.f};
#pragma unroll
  for (int g = 0; g < 2; ++g) { o[g][0] = zero16(); o[g][1] = zero16(); }
  const int nt = (N + AK - 1) / AK;
  // K/V tiles stream HBM -> LDS by LDS-DMA, one tile ahead; raw barriers + explicit vmcnt
  tile_glds(Kb, ld, 0, N, smem[0][0], wv, lane);
  tile_glds(Vb, ld, 0, N, smem[0][1], wv, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nt) {
      tile_glds(Kb, ld, (kt + 1) * AK, N, smem[cur ^ 1][0], wv, lane);
      tile_glds(Vb, ld, (kt + 1) * AK, N, smem[cur ^ 1][1], wv, lane);
    }
    if ((kt + 1) * AK <= N)
      fwd_tile2<false>(smem[cur][0], smem[cur][1], qf, o, m, l, kt * AK, N, c2, lane);
    else
      fwd_tile2<true>(smem[cur][0], smem[cur][1], qf, o, m, l, kt * AK, N, c2, lane);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // next tile landed; my reads done
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int q = qw + 32 * g + (lane & 31);
    if (q >= N) continue;
    const float inv = 1.f / l[g];
    bf16* orow = out + ((long)b * N + q) * D + h * 64;
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      Pack4 a, c;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a.h[j] = (bf16)(o[g][0][4 * gg + j] * inv);
        c.h[j] = (bf16)(o[g][1][4 * gg + j] * inv);
      }
      const int d = 8 * gg + 4 * hl;
      *(uint2*)(orow + d) = a.u;
      *(uint2*)(orow + 32 + d) = c.u;
    }
    if (hl == 0) lse[(long)z * N + q] = (m[g] + log2f(l[g])) * 0.69314718055994531f;
  }
}

// ------------------------------------------------------------------------- forward v3 (bf16)
// v1's shape (32 queries per wave) with: K/V by LDS-DMA one tile ahead (no staging VGPRs),
// key masking only on the last tile, the scale folded into one FMA before exp2, and the O
// rescale skipped when no lane's max moved. WAVES = 4 or 8 waves per workgroup share a tile.
// MSUM: the row sums l come from the MFMA pipe (a ones operand beside P·V, kept in lacc) instead
// of 32 VALU adds per tile — the loop is VALU-issue-bound at head dim 64.
template <bool MASK, bool MSUM = false>
IVIT_DEV void fwd_tile3(const char* kimg, const char* vimg, const bf16x8 (&qf)[4], f32x16& o0, f32x16& o1,
                        float& m, float& l, int kbase, int N, float c2, int lane, f32x16* lacc = nullptr) {
  const int hl = lane >> 5;
  f32x16 s[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    s[t] = zero16();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 ka = *(const bf16x8*)(kimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[ks], s[t], 0, 0, 0);
    }
  }
  float mx = NEG_BIG;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (MASK) {
        const int key = kbase + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (key >= N) s[t][r] = NEG_BIG;
      }
      mx = fmaxf(mx, s[t][r]);
    }
  mx = half_swap_max(mx);
  const float mn = fmaxf(m, mx * c2);
  const float alpha = fast_exp2(m - mn);
  const bool moved = mn != m;
  m = mn;
  float rs = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = fast_exp2(fmaf(s[t][r], c2, -mn));
      s[t][r] = p;
      if (!MSUM) rs += p;
    }
  if (!MSUM) {
    rs = half_swap_sum(rs);
    l = l * alpha + rs;
  }
  if (__any(moved)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    if (MSUM) (*lacc)[0] *= alpha;  // only element 0 is read back
  }
  bf16x8 ones;
  if (MSUM) {
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 pb = pack_acc(s[t], ss);
      const int rb = 32 * t + 16 * ss;
      const bf16x8 va0 = tr_acc_order(vimg, rb, 0, lane);
      const bf16x8 va1 = tr_acc_order(vimg, rb, 32, lane);
      o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va0, pb, o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va1, pb, o1, 0, 0, 0);
      if (MSUM) *lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pb, *lacc, 0, 0, 0);
    }
}

// LDS-DMA of a 64x64 tile spread over W waves (8 pieces)
template <int W>
IVIT_DEV void tile_glds_w(const bf16* base, long ld, int r0, int nrows, char* img, int wv, int lane) {
#pragma unroll
  for (int i = 0; i < 8 / W; ++i) {
    const int piece = wv * (8 / W) + i;
    const int row = piece * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz128(row);
    const void* src = (r0 + row < nrows) ? (const void*)(base + (long)(r0 + row) * ld + c * 8) : (const void*)g_zero16;
    glds<16>(src, img + piece * 1024);
  }
}

template <int W>
__global__ __launch_bounds__(64 * W, 8 / W) void attn_fwd_bf16_v3_kernel(const bf16* __restrict__ qkv, int N, int H,
                                                                        bf16* __restrict__ out,
                                                                        float* __restrict__ lse, float c2) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][8192];  // [stage][K|V]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hl = lane >> 5;
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
  f32x16 o0 = zero16(), o1 = zero16();
  float m = NEG_BIG, l = 0.f;
  const int nt = (N + AK - 1) / AK;
  tile_glds_w<W>(Kb, ld, 0, N, smem[0][0], wv, lane);
  tile_glds_w<W>(Vb, ld, 0, N, smem[0][1], wv, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nt) {
      tile_glds_w<W>(Kb, ld, (kt + 1) * AK, N, smem[cur ^ 1][0], wv, lane);
      tile_glds_w<W>(Vb, ld, (kt + 1) * AK, N, smem[cur ^ 1][1], wv, lane);
    }
    if ((kt + 1) * AK <= N)
      fwd_tile3<false>(smem[cur][0], smem[cur][1], qf, o0, o1, m, l, kt * AK, N, c2, lane);
    else
      fwd_tile3<true>(smem[cur][0], smem[cur][1], qf, o0, o1, m, l, kt * AK, N, c2, lane);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  if (q < N) {
    const float inv = 1.f / l;
    bf16* orow = out + ((long)b * N + q) * D + h * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      Pack4 a, c;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a.h[j] = (bf16)(o0[4 * g + j] * inv);
        c.h[j] = (bf16)(o1[4 * g + j] * inv);
      }
      const int d = 8 * g + 4 * hl;
      *(uint2*)(orow + d) = a.u;
      *(uint2*)(orow + 32 + d) = c.u;
    }
    if (hl == 0) lse[(long)z * N + q] = (m + log2f(l)) * 0.69314718055994531f;
  }
}

// ------------------------------------------------------------------------- forward v4 (bf16)
// v3 with (a) k-invariant per-lane DMA source offsets (a full tile is base + r0*ld + off,
// the row guard only on the ragged last tile) and (b) the tile loop unrolled by two so the
// LDS stage is a compile-time constant: every fragment read is a per-lane base plus an
// immediate offset instead of fresh address arithmetic per tile.
template <int W>
IVIT_DEV int dma_off(int i, int wv, int lane, long ld) {
  const int piece = wv * (8 / W) + i;
  const int row = piece * 8 + (lane >> 3);
  const int c = (lane & 7) ^ swz128(row);
  return (int)(row * ld) + c * 8;
}

// Consume register-loaded fragments before a tile loop. Without a use ahead of the loop the
// compiler places the s_waitcnt for these loads at their first use INSIDE the loop, where it
// runs every iteration and (counting only its own loads) also drains the next tile's in-flight
// LDS DMA (tools/loop_waits.py lists such waits).
IVIT_DEV void retire_loads(bf16x8 (&a)[4], bf16x8 (&b)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(a[i]), "v"(b[i]));
}

template <int W, int MINB = 8 / W, bool MSUM = false>
__global__ __launch_bounds__(64 * W, MINB) void attn_fwd_bf16_v4_kernel(const bf16* __restrict__ qkv, int N, int H,
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
  f32x16 o0 = zero16(), o1 = zero16(), lacc = zero16();
  float m = NEG_BIG, l = 0.f;
  const int nt = (N + AK - 1) / AK, nfull = N / AK;
  int off[8 / W];
#pragma unroll
  for (int i = 0; i < 8 / W; ++i) off[i] = dma_off<W>(i, wv, lane, ld);
  auto issue = [&](int kt, char* kimg, char* vimg) {
    if (kt < nfull) {
      const bf16* kb = Kb + (long)kt * AK * ld;
      const bf16* vb = Vb + (long)kt * AK * ld;
#pragma unroll
      for (int i = 0; i < 8 / W; ++i) {
        const int piece = wv * (8 / W) + i;
        glds<16>((kb + off[i]), kimg + piece * 1024);
        glds<16>((vb + off[i]), vimg + piece * 1024);
      }
    } else {
      tile_glds_w<W>(Kb, ld, kt * AK, N, kimg, wv, lane);
      tile_glds_w<W>(Vb, ld, kt * AK, N, vimg, wv, lane);
    }
  };
  auto step = [&](auto stage, int kt) {
    constexpr int S = decltype(stage)::value;
    if (kt + 1 < nt) issue(kt + 1, smem[S ^ 1][0], smem[S ^ 1][1]);
    if (kt < nfull)
      fwd_tile3<false, MSUM>(smem[S][0], smem[S][1], qf, o0, o1, m, l, kt * AK, N, c2, lane, &lacc);
    else
      fwd_tile3<true, MSUM>(smem[S][0], smem[S][1], qf, o0, o1, m, l, kt * AK, N, c2, lane, &lacc);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  issue(0, smem[0][0], smem[0][1]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nt; kt += 2) {
    step(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < nt) step(std::integral_constant<int, 1>{}, kt + 1);
  }
  if (MSUM) l = lacc[0];
  if (q < N) {
    const float inv = 1.f / l;
    bf16* orow = out + ((long)b * N + q) * D + h * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      Pack4 a, c;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a.h[j] = (bf16)(o0[4 * g + j] * inv);
        c.h[j] = (bf16)(o1[4 * g + j] * inv);
      }
      const int d = 8 * g + 4 * hl;
      *(uint2*)(orow + d) = a.u;
      *(uint2*)(orow + 32 + d) = c.u;
    }
    if (hl == 0) lse[(long)z * N + q] = (m + log2f(l)) * 0.69314718055994531f;
  }
}

// ------------------------------------------------------------------------- forward v5 (bf16)
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

IVIT_DEV void qk_tile(const char* kimg, const bf16x8 (&qf)[4], f32x16 (&s)[2], int lane) {
  const int hl = lane >> 5;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    s[t] = zero16();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 ka = *(const bf16x8*)(kimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[ks], s[t], 0, 0, 0);
    }
  }
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

// One steady-state step of the pipelined forward in a hand-fixed instruction order: every chunk
// is closed by sched_barrier(0) and LDS operands are read two chunks ahead, so each MFMA gap
// carries about the VALU the gap can hide (cdna_hip_programming.md: <= ~24 issue cycles):
//   A : 8 x { K fragment read, 1 QK^T MFMA of S_{j+1}, exp + cvt of 2 scores of P_j (t = 0) }
//   B1: 6 x { V reads, 1 P.V / row-sum MFMA (t = 0), exp + cvt of 2-3 scores of P_j (t = 1) }
//   B2: 6 x { V reads, 1 P.V / row-sum MFMA (t = 1), ~6 values of rowmax(S_{j+1}) }
// Returns the scaled row max of S_{j+1}.
IVIT_DEV float fwd_step_fenced(const char* kimg, const char* vimg, const bf16x8 (&qf)[4], const f32x16 (&cur)[2],
                               f32x16 (&nxt)[2], f32x16& o0, f32x16& o1, f32x16& lacc, const bf16x8& ones, float m,
                               float c2, int lane) {
  const int hl = lane >> 5;
  auto kfrag = [&](int i) {
    return *(const bf16x8*)(kimg + t_off(32 * (i >> 2) + (lane & 31), 2 * (i & 3) + hl));
  };
  bf16x8 p[4];
  auto ex = [&](int i) {  // score i of P_j: t = i >> 4, register i & 15
    p[i >> 3][i & 7] = (bf16)fast_exp2(fmaf(cur[i >> 4][i & 15], c2, -m));
  };
  const f32x16 zero = zero16();
  bf16x8 ka[8];
  ka[0] = kfrag(0);
  ka[1] = kfrag(1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i + 2 < 8) ka[i + 2] = kfrag(i + 2);
    const int t = i >> 2, ks = i & 3;
    nxt[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[i], qf[ks], ks == 0 ? zero : nxt[t], 0, 0, 0);
    ex(2 * i);
    ex(2 * i + 1);
    __builtin_amdgcn_sched_barrier(0);
  }
  // V^T operands: vf[2 * (2t + ss) + half]
  bf16x8 vf[8];
  auto vread = [&](int f) { vf[f] = tr_acc_order(vimg, 16 * (f >> 1), 32 * (f & 1), lane); };
  vread(0);
  vread(1);
  __builtin_amdgcn_sched_barrier(0);
  // B1: P(t=0) . V, exp of t = 1 (scores 16..31: 3,3,3,3,2,2 per chunk)
  constexpr int e0[7] = {16, 19, 22, 25, 28, 30, 32};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int g = k / 3, which = k % 3;  // p[g]; which: o0 / o1 / row sum
    if (k == 0) vread(2);
    if (k == 1) vread(3);
    if (k == 3) vread(4);
    if (k == 4) vread(5);
    if (which == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g], p[g], o0, 0, 0, 0);
    else if (which == 1) o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g + 1], p[g], o1, 0, 0, 0);
    else lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, p[g], lacc, 0, 0, 0);
#pragma unroll
    for (int i = e0[k]; i < e0[k + 1]; ++i) ex(i);
    __builtin_amdgcn_sched_barrier(0);
  }
  // B2: P(t=1) . V, rowmax of S_{j+1} (32 values, 6 per chunk)
  float a = NEG_BIG, bm = NEG_BIG;
#pragma unroll
  for (int k = 6; k < 12; ++k) {
    const int g = k / 3, which = k % 3;
    if (k == 6) vread(6);
    if (k == 7) vread(7);
    if (which == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g], p[g], o0, 0, 0, 0);
    else if (which == 1) o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g + 1], p[g], o1, 0, 0, 0);
    else lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, p[g], lacc, 0, 0, 0);
    const int v0 = 6 * (k - 6);
#pragma unroll
    for (int v = v0; v < v0 + 6 && v < 32; v += 2) {
      if ((v >> 1) & 1) bm = vmax3(bm, nxt[v >> 4][v & 15], nxt[v >> 4][(v & 15) + 1]);
      else a = vmax3(a, nxt[v >> 4][v & 15], nxt[v >> 4][(v & 15) + 1]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return half_swap_max(fmaxf(a, bm)) * c2;
}

// SCHED: the steady-state step (next tile full) runs fwd_step_fenced.
template <int W, bool SCHED = false>
__global__ __launch_bounds__(64 * W, 8 / W) void attn_fwd_bf16_v5_kernel(const bf16* __restrict__ qkv, int N, int H,
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
  const int nt = (N + AK - 1) / AK, nfull = N / AK;
  int off[8 / W];
#pragma unroll
  for (int i = 0; i < 8 / W; ++i) off[i] = dma_off<W>(i, wv, lane, ld);
  auto issue1 = [&](const bf16* base, int kt, char* img) {  // one 64-key tile of K or V
    if (kt < nfull) {
      const bf16* src = base + (long)kt * AK * ld;
#pragma unroll
      for (int i = 0; i < 8 / W; ++i)
        glds<16>((src + off[i]), img + (wv * (8 / W) + i) * 1024);
    } else {
      tile_glds_w<W>(base, ld, kt * AK, N, img, wv, lane);
    }
  };
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;

  // prologue: S_0 and its max; K_1 in flight
  issue1(Kb, 0, smem[0][0]);
  issue1(Vb, 0, smem[0][1]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (nt > 1) issue1(Kb, 1, smem[1][0]);
  f32x16 sc[2], sn[2];
  qk_tile(smem[0][0], qf, sc, lane);
  float m = (nfull > 0 ? tile_rowmax<false>(sc, 0, N, lane) : tile_rowmax<true>(sc, 0, N, lane)) * c2;
  f32x16 o0 = zero16(), o1 = zero16(), lacc = zero16();

  // NX = 1: the next tile exists and is full (branch-free body); NX = 3: generic (tail steps)
  auto body = [&](auto stage, auto nxmode, int j, f32x16(&cur)[2], f32x16(&nxt)[2]) {
    constexpr int S = decltype(stage)::value;  // V_j in smem[S][1], K_{j+1} in smem[S^1][0]
    constexpr int NX = decltype(nxmode)::value;
    const bool more = NX == 1 || j + 1 < nt;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // K_{j+1}, V_j landed for every wave; step j-1's reads are done
    if (j + 2 < nt) issue1(Kb, j + 2, smem[S][0]);
    if (more) issue1(Vb, j + 1, smem[S ^ 1][1]);
    if constexpr (SCHED && NX == 1) {
      const float mt = fwd_step_fenced(smem[S ^ 1][0], smem[S][1], qf, cur, nxt, o0, o1, lacc, ones, m, c2, lane);
      const bool moved = mt > m + TAU;
      if (__any(moved)) {
        const float mn = moved ? mt : m;
        const float alpha = fast_exp2(m - mn);
#pragma unroll
        for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
        lacc[0] *= alpha;
        m = mn;
      }
      return;
    }
    if (more) qk_tile(smem[S ^ 1][0], qf, nxt, lane);
    bf16x8 p[4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)fast_exp2(fmaf(cur[t][8 * ss + e], c2, -m));
        p[2 * t + ss] = v;
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int rb = 32 * t + 16 * ss;
        const bf16x8 va0 = tr_acc_order(smem[S][1], rb, 0, lane);
        const bf16x8 va1 = tr_acc_order(smem[S][1], rb, 32, lane);
        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va0, p[2 * t + ss], o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va1, p[2 * t + ss], o1, 0, 0, 0);
        lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, p[2 * t + ss], lacc, 0, 0, 0);
      }
    if (more) {
      const float mt = (NX == 1 || j + 1 < nfull ? tile_rowmax<false>(nxt, (j + 1) * AK, N, lane)
                                                 : tile_rowmax<true>(nxt, (j + 1) * AK, N, lane)) * c2;
      const bool moved = mt > m + TAU;
      if (__any(moved)) {
        const float mn = moved ? mt : m;
        const float alpha = fast_exp2(m - mn);
#pragma unroll
        for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
        lacc[0] *= alpha;  // only element 0 is read back
        m = mn;
      }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I3 = std::integral_constant<int, 3>;
  int j = 0;
  for (; j + 2 < nfull; j += 2) {  // steps j, j+1: both next tiles (j+1, j+2) are full
    body(I0{}, I1{}, j, sc, sn);
    body(I1{}, I1{}, j + 1, sn, sc);
  }
  for (; j < nt; ++j) {  // at most three tail steps, generic body (NX = 3: decided at run time)
    if (j & 1) body(I1{}, I3{}, j, sn, sc);
    else body(I0{}, I3{}, j, sc, sn);
  }
  if (q < N) {
    const float l = lacc[0];
    const float inv = 1.f / l;
    bf16* orow = out + ((long)b * N + q) * D + h * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      Pack4 a, c;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a.h[e] = (bf16)(o0[4 * g + e] * inv);
        c.h[e] = (bf16)(o1[4 * g + e] * inv);
      }
      const int d = 8 * g + 4 * hl;
      *(uint2*)(orow + d) = a.u;
      *(uint2*)(orow + 32 + d) = c.u;
    }
    if (hl == 0) lse[(long)z * N + q] = (m + log2f(l)) * 0.69314718055994531f;
  }
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

IVIT_DEV float fwd_step_fenced6(const char* kimg, const char* vimg, const bf16x8 (&qf)[4], const f32x16 (&cur)[2],
                                f32x16 (&nxt)[2], f32x16& o0, f32x16& o1, f32x16& lacc, const bf16x8& ones,
                                const f32x16& negm, int lane) {
  const int hl = lane >> 5;
  auto kfrag = [&](int i) {
    return *(const bf16x8*)(kimg + t_off(32 * (i >> 2) + (lane & 31), 2 * (i & 3) + hl));
  };
  bf16x8 p[4];
  auto ex = [&](int i) { p[i >> 3][i & 7] = (bf16)fast_exp2(cur[i >> 4][i & 15]); };
  bf16x8 ka[8];
  ka[0] = kfrag(0);
  ka[1] = kfrag(1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i + 2 < 8) ka[i + 2] = kfrag(i + 2);
    const int t = i >> 2, ks = i & 3;
    nxt[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[i], qf[ks], ks == 0 ? negm : nxt[t], 0, 0, 0);
    ex(2 * i);
    ex(2 * i + 1);
    __builtin_amdgcn_sched_barrier(0);
  }
  bf16x8 vf[8];
  auto vread = [&](int f) { vf[f] = tr_acc_order(vimg, 16 * (f >> 1), 32 * (f & 1), lane); };
  vread(0);
  vread(1);
  __builtin_amdgcn_sched_barrier(0);
  constexpr int e0[7] = {16, 19, 22, 25, 28, 30, 32};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int g = k / 3, which = k % 3;
    if (k == 0) vread(2);
    if (k == 1) vread(3);
    if (k == 3) vread(4);
    if (k == 4) vread(5);
    if (which == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g], p[g], o0, 0, 0, 0);
    else if (which == 1) o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g + 1], p[g], o1, 0, 0, 0);
    else lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, p[g], lacc, 0, 0, 0);
#pragma unroll
    for (int i = e0[k]; i < e0[k + 1]; ++i) ex(i);
    __builtin_amdgcn_sched_barrier(0);
  }
  float a = NEG_BIG, bm = NEG_BIG;
#pragma unroll
  for (int k = 6; k < 12; ++k) {
    const int g = k / 3, which = k % 3;
    if (k == 6) vread(6);
    if (k == 7) vread(7);
    if (which == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g], p[g], o0, 0, 0, 0);
    else if (which == 1) o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[2 * g + 1], p[g], o1, 0, 0, 0);
    else lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, p[g], lacc, 0, 0, 0);
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

// PRE: prescale Q by c2 in the kernel (ivit_attn_fwd variant 11); otherwise the Q block of qkv
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
  int off[8 / W];
#pragma unroll
  for (int i = 0; i < 8 / W; ++i) off[i] = dma_off<W>(i, wv, lane, ld);
  auto issue1 = [&](const bf16* base, int kt, char* img) {
    if (kt < nfull) {
      const bf16* src = base + (long)kt * AK * ld;
#pragma unroll
      for (int i = 0; i < 8 / W; ++i) glds<16>((src + off[i]), img + (wv * (8 / W) + i) * 1024);
    } else {
      tile_glds_w<W>(base, ld, kt * AK, N, img, wv, lane);
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
#pragma unroll
      for (int r = 0; r < 16; ++r) negm[r] = -m;
    }
  };
  auto body = [&](auto stage, auto nxmode, int j, f32x16(&cur)[2], f32x16(&nxt)[2]) {
    constexpr int S = decltype(stage)::value;  // V_j in smem[S][1], K_{j+1} in smem[S^1][0]
    constexpr int NX = decltype(nxmode)::value;
    const bool more = NX == 1 || j + 1 < nt;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (j + 2 < nt) issue1(Kb, j + 2, smem[S][0]);
    if (more) issue1(Vb, j + 1, smem[S ^ 1][1]);
    if constexpr (NX == 1) {
      rescale(fwd_step_fenced6(smem[S ^ 1][0], smem[S][1], qf, cur, nxt, o0, o1, lacc, ones, negm, lane), nxt);
      return;
    }
    if (more) qk_tile_c(smem[S ^ 1][0], qf, negm, nxt, lane);
    bf16x8 p[4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)fast_exp2(cur[t][8 * ss + e]);
        p[2 * t + ss] = v;
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int rb = 32 * t + 16 * ss;
        const bf16x8 va0 = tr_acc_order(smem[S][1], rb, 0, lane);
        const bf16x8 va1 = tr_acc_order(smem[S][1], rb, 32, lane);
        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va0, p[2 * t + ss], o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va1, p[2 * t + ss], o1, 0, 0, 0);
        lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, p[2 * t + ss], lacc, 0, 0, 0);
      }
    if (more) {
      const float mt = NX == 1 || j + 1 < nfull ? tile_rowmax<false>(nxt, (j + 1) * AK, N, lane)
                                                : tile_rowmax<true>(nxt, (j + 1) * AK, N, lane);
      rescale(mt, nxt);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I3 = std::integral_constant<int, 3>;
  int j = 0;
  for (; j + 2 < nfull; j += 2) {
    body(I0{}, I1{}, j, sc, sn);
    body(I1{}, I1{}, j + 1, sn, sc);
  }
  for (; j < nt; ++j) {
    if (j & 1) body(I1{}, I3{}, j, sn, sc);
    else body(I0{}, I3{}, j, sc, sn);
  }
  if (q < N) {
    const float l = lacc[0];
    const float inv = 1.f / l;
    bf16* orow = out + ((long)b * N + q) * D + h * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      Pack4 a, c;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a.h[e] = (bf16)(o0[4 * g + e] * inv);
        c.h[e] = (bf16)(o1[4 * g + e] * inv);
      }
      const int d = 8 * g + 4 * hl;
      *(uint2*)(orow + d) = a.u;
      *(uint2*)(orow + 32 + d) = c.u;
    }
    if (hl == 0) lse[(long)z * N + q] = (m + log2f(l)) * 0.69314718055994531f;
  }
}

// ------------------------------------------------------------------------- dK, dV (bf16)
// (register-staged variant, IVIT_ATTN_DKV_VARIANT=1; rows from the padded lse2 / delta arrays)
__global__ __launch_bounds__(256, 2) void attn_bwd_dkv_bf16_kernel(const bf16* __restrict__ qkv,
                                                                   const bf16* __restrict__ dout,
                                                                   const float* __restrict__ lse2p,
                                                                   const float* __restrict__ deltap, int N, int Npad,
                                                                   int H, bf16* __restrict__ dqkv, float c2,
                                                                   float scale) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][8192];  // [stage][Q|dO]
  __shared__ float srow[2][2][AK];                                  // [stage][lse2|delta]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hl = lane >> 5;
  const int2 bid = attn_block_id();
  const int z = bid.y, b = z / H, h = z - b * H;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16* Qb = qkv + (long)b * N * ld + h * 64;
  const bf16* Kb = Qb + D;
  const bf16* Vb = Qb + 2 * D;
  const bf16* Gb = dout + (long)b * N * D + h * 64;
  const float* L = lse2p + (long)z * Npad;
  const float* Dl = deltap + (long)z * Npad;
  const int key = bid.x * AQ + wv * 32 + (lane & 31);
  bf16x8 kf[4], vf[4];
  load_row_frags(Kb + (long)key * ld, key < N, lane, kf);
  load_row_frags(Vb + (long)key * ld, key < N, lane, vf);

  f32x16 dk0 = zero16(), dk1 = zero16(), dv0 = zero16(), dv1 = zero16();  // [key][d]: col d, rows key
  const int nt = (N + AK - 1) / AK;
  uint4 rq[2], rg[2];
  float rl = 0.f, rd = 0.f;
  auto rows_load = [&](int q0) {
    if (tid < AK) {  // padded rows: lse2 = 1e30, delta = 0
      rl = L[q0 + tid];
      rd = Dl[q0 + tid];
    }
  };
  tile_gload(Qb, ld, 0, N, tid, rq);
  tile_gload(Gb, D, 0, N, tid, rg);
  rows_load(0);
  tile_sstore(smem[0][0], tid, rq);
  tile_sstore(smem[0][1], tid, rg);
  if (tid < AK) { srow[0][0][tid] = rl; srow[0][1][tid] = rd; }
  __syncthreads();
  for (int qt = 0; qt < nt; ++qt) {
    const int cur = qt & 1;
    if (qt + 1 < nt) {
      tile_gload(Qb, ld, (qt + 1) * AK, N, tid, rq);
      tile_gload(Gb, D, (qt + 1) * AK, N, tid, rg);
      rows_load((qt + 1) * AK);
    }
    const char* qimg = smem[cur][0];
    const char* gimg = smem[cur][1];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 s = zero16(), dp = zero16();  // [q][key]: col key (lane), rows q
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 qa = *(const bf16x8*)(qimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
        const bf16x8 ga = *(const bf16x8*)(gimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[ks], s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga, vf[ks], dp, 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int qi = 32 * t + 8 * g + 4 * hl;  // rows (r&3) + 8(r>>2) + 4h, r = 4g + j
        const float4 l4 = *(const float4*)&srow[cur][0][qi];
        const float4 d4 = *(const float4*)&srow[cur][1][qi];
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
        const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = fast_exp2(fmaf(s[4 * g + j], c2, -lv[j]));
          s[4 * g + j] = p;                               // P[q][key]
          dp[4 * g + j] = p * (dp[4 * g + j] - dv[j]);    // dS[q][key]
        }
      }
      // dV[key][d] += P^T dO ; dK[key][d] += dS^T Q   (X = P / dS as the A operand)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int rb = 32 * t + 16 * ss;
        const bf16x8 pa = pack_acc(s, ss);
        const bf16x8 g0 = tr_acc_order(gimg, rb, 0, lane);
        const bf16x8 g1 = tr_acc_order(gimg, rb, 32, lane);
        dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, g0, dv0, 0, 0, 0);
        dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, g1, dv1, 0, 0, 0);
        const bf16x8 da = pack_acc(dp, ss);
        const bf16x8 q0 = tr_acc_order(qimg, rb, 0, lane);
        const bf16x8 q1 = tr_acc_order(qimg, rb, 32, lane);
        dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, q0, dk0, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, q1, dk1, 0, 0, 0);
      }
    }
    if (qt + 1 < nt) {
      tile_sstore(smem[cur ^ 1][0], tid, rq);
      tile_sstore(smem[cur ^ 1][1], tid, rg);
      if (tid < AK) { srow[cur ^ 1][0][tid] = rl; srow[cur ^ 1][1][tid] = rd; }
    }
    __syncthreads();
  }
  const int kw = bid.x * AQ + wv * 32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int kk = kw + (r & 3) + 8 * (r >> 2) + 4 * hl;
    if (kk < N) {
      bf16* row = dqkv + ((long)b * N + kk) * ld + h * 64;
      row[D + (lane & 31)] = (bf16)(dk0[r] * scale);
      row[D + 32 + (lane & 31)] = (bf16)(dk1[r] * scale);
      row[2 * D + (lane & 31)] = (bf16)dv0[r];
      row[2 * D + 32 + (lane & 31)] = (bf16)dv1[r];
    }
  }
}

// ------------------------------------------------------------------------- backward v2 (bf16)
// Row constants for the backward in a padded layout [z][Npad] (Npad = N rounded up to 64):
// lse2 = lse * log2(e) (+1e30 on padding rows, so their probabilities are exactly 0) and
// delta = rowsum(dO * O) (0 on padding). 8 lanes per (z, padded row), one 16-B load of O
// and of dO each (a wave reads 8 whole 128-B row segments), reduced across the 8 lanes.
__global__ void attn_rows_v2_kernel(const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                    const float* __restrict__ lse, int B, int N, int Npad, int H,
                                    float* __restrict__ lse2p, float* __restrict__ deltap) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long i = t >> 3;  // (z, padded row)
  const int part = (int)(t & 7);
  if (i >= (long)B * H * Npad) return;
  // rows ordered n-major within (b, h): consecutive i share (b, h) -> contiguous stores
  const int z = (int)(i / Npad), n = (int)(i - (long)z * Npad);
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
    deltap[i] = s;
    lse2p[i] = n < N ? lse[(long)z * N + n] * LOG2E : 1e30f;
  }
}

// One dQ tile step: keys kbase.. of the K/V images against this wave's 32 queries.
// Q2: qf holds q * c2 and nl = -lse2 in every register: S' - lse2 comes straight out of the
// MFMA chain (nl as its initial accumulator) and p = exp2 of it, no per-score FMA.
template <bool MASK, bool Q2 = false>
IVIT_DEV void dq_tile(const char* kimg, const char* vimg, const bf16x8 (&qf)[4], const bf16x8 (&gf)[4], f32x16& a0,
                      f32x16& a1, float lse2, float dlt, int kbase, int N, float c2, int lane,
                      const f32x16& nl = f32x16{}) {
  const int hl = lane >> 5;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    f32x16 s = Q2 ? nl : zero16(), dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] = -dlt;  // row constant as the initial accumulator
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 ka = *(const bf16x8*)(kimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      const bf16x8 va = *(const bf16x8*)(vimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[ks], s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, gf[ks], dp, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float p = Q2 ? fast_exp2(s[r]) : fast_exp2(fmaf(s[r], c2, -lse2));
      if (MASK) {
        const int key = kbase + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (key >= N) p = 0.f;
      }
      s[r] = p * dp[r];  // dS^T[key][q]
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 xa = pack_acc(s, ss);
      const int rb = 32 * t + 16 * ss;
      const bf16x8 kb0 = tr_acc_order(kimg, rb, 0, lane);
      const bf16x8 kb1 = tr_acc_order(kimg, rb, 32, lane);
      a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa, kb0, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa, kb1, a1, 0, 0, 0);
    }
  }
}

// dQ: 4 waves x 32 queries; K/V tiles by LDS-DMA (k-invariant offsets, ragged tail guarded),
// tile loop unrolled by two so the LDS stage is a compile-time constant.
// V3ROWS: the row constants come from attn_rows_v3_kernel (lsn = -lse sqrt(Dh), dln = -delta).
// ROWS: this kernel also forms its queries' row constants (replacing attn_rows_v2_kernel):
// lse2 = lse * log2(e) and delta = rowsum(dO * O) from the dO fragments it already holds and
// the O rows, and writes both (padded rows: 1e30 / 0) for the dK/dV kernel that follows.
template <bool V3ROWS = false, bool Q2 = false, bool ROWS = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_v2_kernel(const bf16* __restrict__ qkv,
                                                                const bf16* __restrict__ dout,
                                                                float* __restrict__ lse2p,
                                                                float* __restrict__ deltap, int N, int Npad,
                                                                int H, bf16* __restrict__ dqkv, float c2,
                                                                float scale, const bf16* __restrict__ out = nullptr,
                                                                const float* __restrict__ lse = nullptr) {
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
  const int q = bid.x * AQ + wv * 32 + (lane & 31);
  const bool qv = q < N;
  bf16x8 qf[4], gf[4];
  load_row_frags(Qb + (long)q * ld, qv, lane, qf);
  load_row_frags(dout + ((long)b * N + q) * D + h * 64, qv, lane, gf);
  float lse2, dlt;
  if constexpr (ROWS) {
    bf16x8 of[4];
    load_row_frags(out + ((long)b * N + q) * D + h * 64, qv, lane, of);
    float d = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf((float)of[i][e], (float)gf[i][e], d);
    d = half_swap_sum(d);  // the other 32 of the 64 dims sit in lane ^ 32
    lse2 = qv ? lse[(long)z * N + q] * LOG2E : 1e30f;
    dlt = qv ? d : 0.f;
    if (hl == 0 && q < Npad) {
      lse2p[(long)z * Npad + q] = lse2;
      deltap[(long)z * Npad + q] = dlt;
    }
  } else {
    lse2 = qv ? lse2p[(long)z * Npad + q] : 1e30f;
    dlt = qv ? deltap[(long)z * Npad + q] : 0.f;
  }
  if (V3ROWS) {
    lse2 = qv ? -lse2 * c2 : 1e30f;  // -lsn * c2 = lse * log2(e)
    dlt = -dlt;
  }
  f32x16 a0 = zero16(), a1 = zero16();
  f32x16 nl;
#pragma unroll
  for (int r = 0; r < 16; ++r) nl[r] = -lse2;
  const int nt = (N + AK - 1) / AK, nfull = N / AK;
  int off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) off[i] = dma_off<4>(i, wv, lane, ld);
  auto issue = [&](int kt, char* kimg, char* vimg) {
    if (kt < nfull) {
      const bf16* kb = Kb + (long)kt * AK * ld;
      const bf16* vb = Vb + (long)kt * AK * ld;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int piece = wv * 2 + i;
        glds<16>((kb + off[i]), kimg + piece * 1024);
        glds<16>((vb + off[i]), vimg + piece * 1024);
      }
    } else {
      tile_glds_w<4>(Kb, ld, kt * AK, N, kimg, wv, lane);
      tile_glds_w<4>(Vb, ld, kt * AK, N, vimg, wv, lane);
    }
  };
  auto step = [&](auto stage, int kt) {
    constexpr int S = decltype(stage)::value;
    if (kt + 1 < nt) issue(kt + 1, smem[S ^ 1][0], smem[S ^ 1][1]);
    if (kt < nfull)
      dq_tile<false, Q2>(smem[S][0], smem[S][1], qf, gf, a0, a1, lse2, dlt, kt * AK, N, c2, lane, nl);
    else
      dq_tile<true, Q2>(smem[S][0], smem[S][1], qf, gf, a0, a1, lse2, dlt, kt * AK, N, c2, lane, nl);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  issue(0, smem[0][0], smem[0][1]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nt; kt += 2) {
    step(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < nt) step(std::integral_constant<int, 1>{}, kt + 1);
  }
  const int qw = bid.x * AQ + wv * 32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int qq = qw + (r & 3) + 8 * (r >> 2) + 4 * hl;
    if (qq < N) {
      bf16* row = dqkv + ((long)b * N + qq) * ld + h * 64;
      row[lane & 31] = (bf16)(a0[r] * scale);
      row[32 + (lane & 31)] = (bf16)(a1[r] * scale);
    }
  }
}

// One dK/dV tile step: queries of the Q/dO images (rows past N are zero with lse2 = 1e30,
// so P = 0 there and no mask is needed) against this wave's 32 keys.
IVIT_DEV void dkv_tile(const char* qimg, const char* gimg, const float* lrow, const float* drow,
                       const bf16x8 (&kf)[4], const bf16x8 (&vf)[4], f32x16& dk0, f32x16& dk1, f32x16& dv0,
                       f32x16& dv1, float c2, int lane) {
  const int hl = lane >> 5;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    f32x16 s = zero16(), dp = zero16();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 qa = *(const bf16x8*)(qimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      const bf16x8 ga = *(const bf16x8*)(gimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[ks], s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga, vf[ks], dp, 0, 0, 0);
    }
    // row constants read after the MFMA chains are issued (off the chains' critical path)
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // rows (r&3) + 8(r>>2) + 4h, r = 4g + j
      const float4 l4 = *(const float4*)(lrow + 32 * t + 8 * g + 4 * hl);
      const float4 d4 = *(const float4*)(drow + 32 * t + 8 * g + 4 * hl);
      const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
      const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = fast_exp2(fmaf(s[4 * g + j], c2, -lv[j]));
        s[4 * g + j] = p;                             // P[q][key]
        dp[4 * g + j] = p * (dp[4 * g + j] - dv[j]);  // dS[q][key]
      }
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const int rb = 32 * t + 16 * ss;
      const bf16x8 pa = pack_acc(s, ss);
      const bf16x8 g0 = tr_acc_order(gimg, rb, 0, lane);
      const bf16x8 g1 = tr_acc_order(gimg, rb, 32, lane);
      dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, g0, dv0, 0, 0, 0);
      dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, g1, dv1, 0, 0, 0);
      const bf16x8 da = pack_acc(dp, ss);
      const bf16x8 q0 = tr_acc_order(qimg, rb, 0, lane);
      const bf16x8 q1 = tr_acc_order(qimg, rb, 32, lane);
      dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, q0, dk0, 0, 0, 0);
      dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, q1, dk1, 0, 0, 0);
    }
  }
}

// dK/dV: 4 waves x 32 keys; Q, dO tiles and their lse2 / delta rows by LDS-DMA.
__global__ __launch_bounds__(256, 2) void attn_bwd_dkv_v2_kernel(const bf16* __restrict__ qkv,
                                                                 const bf16* __restrict__ dout,
                                                                 const float* __restrict__ lse2p,
                                                                 const float* __restrict__ deltap, int N, int Npad,
                                                                 int H, bf16* __restrict__ dqkv, float c2,
                                                                 float scale) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][8192];  // [stage][Q|dO]
  __shared__ __attribute__((aligned(16))) float srow[2][2][AK];    // [stage][lse2|delta]
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int2 bid = attn_block_id();
  const int z = bid.y, b = z / H, h = z - b * H;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16* Qb = qkv + (long)b * N * ld + h * 64;
  const bf16* Kb = Qb + D;
  const bf16* Vb = Qb + 2 * D;
  const bf16* Gb = dout + (long)b * N * D + h * 64;
  const float* L = lse2p + (long)z * Npad;
  const float* Dl = deltap + (long)z * Npad;
  const int key = bid.x * AQ + wv * 32 + (lane & 31);
  bf16x8 kf[4], vf[4];
  load_row_frags(Kb + (long)key * ld, key < N, lane, kf);
  load_row_frags(Vb + (long)key * ld, key < N, lane, vf);
  retire_loads(kf, vf);
  f32x16 dk0 = zero16(), dk1 = zero16(), dv0 = zero16(), dv1 = zero16();
  const int nt = (N + AK - 1) / AK, nfull = N / AK;
  int offq[2], offg[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    offq[i] = dma_off<4>(i, wv, lane, ld);
    offg[i] = dma_off<4>(i, wv, lane, D);
  }
  auto issue = [&](int qt, int S) {
    char* qimg = smem[S][0];
    char* gimg = smem[S][1];
    if (qt < nfull) {
      const bf16* qb = Qb + (long)qt * AK * ld;
      const bf16* gb = Gb + (long)qt * AK * D;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int piece = wv * 2 + i;
        glds<16>((qb + offq[i]), qimg + piece * 1024);
        glds<16>((gb + offg[i]), gimg + piece * 1024);
      }
    } else {
      tile_glds_w<4>(Qb, ld, qt * AK, N, qimg, wv, lane);
      tile_glds_w<4>(Gb, D, qt * AK, N, gimg, wv, lane);
    }
    if (wv == 0) {  // 64 lse2 + 64 delta floats (the padded arrays cover every tile row)
      glds<4>((L + qt * AK + lane), &srow[S][0][0]);
      glds<4>((Dl + qt * AK + lane), &srow[S][1][0]);
    }
  };
  auto step = [&](auto stage, int qt) {
    constexpr int S = decltype(stage)::value;
    if (qt + 1 < nt) issue(qt + 1, S ^ 1);
    dkv_tile(smem[S][0], smem[S][1], srow[S][0], srow[S][1], kf, vf, dk0, dk1, dv0, dv1, c2, lane);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int qt = 0; qt < nt; qt += 2) {
    step(std::integral_constant<int, 0>{}, qt);
    if (qt + 1 < nt) step(std::integral_constant<int, 1>{}, qt + 1);
  }
  const int kw = bid.x * AQ + wv * 32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int kk = kw + (r & 3) + 8 * (r >> 2) + 4 * hl;
    if (kk < N) {
      bf16* row = dqkv + ((long)b * N + kk) * ld + h * 64;
      row[D + (lane & 31)] = (bf16)(dk0[r] * scale);
      row[D + 32 + (lane & 31)] = (bf16)(dk1[r] * scale);
      row[2 * D + (lane & 31)] = (bf16)dv0[r];
      row[2 * D + 32 + (lane & 31)] = (bf16)dv1[r];
    }
  }
}

// ------------------------------------------------------------------------- backward v3 (bf16)
// Row constants as the initial accumulators (cdna_hip_programming.md, attention backward):
// lsn = -lse * sqrt(Dh), so S' = Q K^T + lsn and P = exp2(c2 S') with no subtraction, and
// dln = -delta, so dS = P * (dO V^T + dln) is one multiply. Padding rows (n >= N, up to Npad):
// lsn = -1e30 (P = 0 exactly), dln = 0.
__global__ void attn_rows_v3_kernel(const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                    const float* __restrict__ lse, int B, int N, int Npad, int H, float rs,
                                    float* __restrict__ lsn, float* __restrict__ dln) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long i = t >> 3;  // (z, padded row)
  const int part = (int)(t & 7);
  if (i >= (long)B * H * Npad) return;
  const int z = (int)(i / Npad), n = (int)(i - (long)z * Npad);
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
    dln[i] = -s;
    lsn[i] = n < N ? -lse[(long)z * N + n] * rs : -1e30f;
  }
}

// dK / dV v3: 4 waves x 32 keys; the query sweep is software-pipelined by 32-query halves —
// S', dP' of half u+1 (8 MFMA) are issued ahead of P, dS of half u (VALU) and its dV, dK
// products (8 MFMA), so one wave's matrix and vector pipes overlap. Q / dO tiles and their row
// constants arrive by LDS-DMA into a 3-stage ring: tile j+2 is issued at the top of step j
// and waited for one full step later; one barrier per 64-query tile.
__global__ __launch_bounds__(256, 2) void attn_bwd_dkv_v3_kernel(const bf16* __restrict__ qkv,
                                                                 const bf16* __restrict__ dout,
                                                                 const float* __restrict__ lsnp,
                                                                 const float* __restrict__ dlnp, int N, int Npad,
                                                                 int H, bf16* __restrict__ dqkv, float c2,
                                                                 float scale) {
  __shared__ __attribute__((aligned(16))) char smem[3][2][8192];  // [stage][Q|dO]
  __shared__ __attribute__((aligned(16))) float srow[3][2][AK];    // [stage][lsn|dln]
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int2 bid = attn_block_id();
  const int z = bid.y, b = z / H, h = z - b * H;
  const int D = H * 64;
  const long ld = 3L * D;
  const bf16* Qb = qkv + (long)b * N * ld + h * 64;
  const bf16* Kb = Qb + D;
  const bf16* Vb = Qb + 2 * D;
  const bf16* Gb = dout + (long)b * N * D + h * 64;
  const float* L = lsnp + (long)z * Npad;
  const float* Dl = dlnp + (long)z * Npad;
  const int key = bid.x * AQ + wv * 32 + (lane & 31);
  bf16x8 kf[4], vf[4];
  load_row_frags(Kb + (long)key * ld, key < N, lane, kf);
  load_row_frags(Vb + (long)key * ld, key < N, lane, vf);
  retire_loads(kf, vf);
  f32x16 dk0 = zero16(), dk1 = zero16(), dv0 = zero16(), dv1 = zero16();
  const int nt = (N + AK - 1) / AK, nfull = N / AK;
  int offq[2], offg[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    offq[i] = dma_off<4>(i, wv, lane, ld);
    offg[i] = dma_off<4>(i, wv, lane, D);
  }
  auto issue = [&](int qt, int S) {
    char* qimg = smem[S][0];
    char* gimg = smem[S][1];
    if (qt < nfull) {
      const bf16* qb = Qb + (long)qt * AK * ld;
      const bf16* gb = Gb + (long)qt * AK * D;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int piece = wv * 2 + i;
        glds<16>((qb + offq[i]), qimg + piece * 1024);
        glds<16>((gb + offg[i]), gimg + piece * 1024);
      }
    } else {
      tile_glds_w<4>(Qb, ld, qt * AK, N, qimg, wv, lane);
      tile_glds_w<4>(Gb, D, qt * AK, N, gimg, wv, lane);
    }
    if (wv == 0) {  // 64 lsn + 64 dln floats (the padded arrays cover every tile row)
      glds<4>((L + qt * AK + lane), &srow[S][0][0]);
      glds<4>((Dl + qt * AK + lane), &srow[S][1][0]);
    }
  };
  // S' and dP' of query half t of the tile in stage S (rows = queries, lane = key)
  auto sdp = [&](int S, int t, f32x16& s, f32x16& dp) {
    const char* qimg = smem[S][0];
    const char* gimg = smem[S][1];
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // rows 8g + 4h .. +3 = registers 4g .. 4g+3
      const float4 l4 = *(const float4*)(&srow[S][0][32 * t + 8 * g + 4 * hl]);
      const float4 d4 = *(const float4*)(&srow[S][1][32 * t + 8 * g + 4 * hl]);
      s[4 * g] = l4.x; s[4 * g + 1] = l4.y; s[4 * g + 2] = l4.z; s[4 * g + 3] = l4.w;
      dp[4 * g] = d4.x; dp[4 * g + 1] = d4.y; dp[4 * g + 2] = d4.z; dp[4 * g + 3] = d4.w;
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 qa = *(const bf16x8*)(qimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      const bf16x8 ga = *(const bf16x8*)(gimg + t_off(32 * t + (lane & 31), 2 * ks + hl));
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[ks], s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga, vf[ks], dp, 0, 0, 0);
    }
  };
  // P, dS of half t (from S', dP' in cs, cdp) and its dV^T += dO^T P, dK^T += Q^T dS products
  auto update = [&](int S, int t, const f32x16& cs, const f32x16& cdp) {
    const char* qimg = smem[S][0];
    const char* gimg = smem[S][1];
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      bf16x8 pa, da;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float p = fast_exp2(cs[8 * ss + e] * c2);
        pa[e] = (bf16)p;
        da[e] = (bf16)(p * cdp[8 * ss + e]);
      }
      const int rb = 32 * t + 16 * ss;
      const bf16x8 g0 = tr_acc_order(gimg, rb, 0, lane);
      const bf16x8 g1 = tr_acc_order(gimg, rb, 32, lane);
      dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, g0, dv0, 0, 0, 0);
      dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, g1, dv1, 0, 0, 0);
      const bf16x8 q0 = tr_acc_order(qimg, rb, 0, lane);
      const bf16x8 q1 = tr_acc_order(qimg, rb, 32, lane);
      dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, q0, dk0, 0, 0, 0);
      dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, q1, dk1, 0, 0, 0);
    }
  };
  f32x16 sA, dpA, sB, dpB;
  issue(0, 0);
  if (nt > 1) issue(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  sdp(0, 0, sA, dpA);
  auto step = [&](auto stage, int j) {
    constexpr int S = decltype(stage)::value;
    if (j > 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // tile j+1 landed for every wave; step j-1's reads are done
    }
    if (j + 2 < nt) issue(j + 2, (S + 2) % 3);
    sdp(S, 1, sB, dpB);   // half (j, 1) ahead of ...
    update(S, 0, sA, dpA);  // ... half (j, 0)
    if (j + 1 < nt) sdp((S + 1) % 3, 0, sA, dpA);  // half (j+1, 0) ahead of ...
    update(S, 1, sB, dpB);                           // ... half (j, 1)
  };
  for (int j = 0; j < nt; j += 3) {
    step(std::integral_constant<int, 0>{}, j);
    if (j + 1 < nt) step(std::integral_constant<int, 1>{}, j + 1);
    if (j + 2 < nt) step(std::integral_constant<int, 2>{}, j + 2);
  }
  const int kw = bid.x * AQ + wv * 32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int kk = kw + (r & 3) + 8 * (r >> 2) + 4 * hl;
    if (kk < N) {
      bf16* row = dqkv + ((long)b * N + kk) * ld + h * 64;
      row[D + (lane & 31)] = (bf16)(dk0[r] * scale);
      row[D + 32 + (lane & 31)] = (bf16)(dk1[r] * scale);
      row[2 * D + (lane & 31)] = (bf16)dv0[r];
      row[2 * D + 32 + (lane & 31)] = (bf16)dv1[r];
    }
  }
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

// Library-owned side streams for the dQ / dK-dV overlap: one per (device, caller stream),
// created lazily under a mutex, with a fork and a join event. Off by default
// (IVIT_ATTN_BWD_OVERLAP=1 enables): with the two ViT streams already concurrent, measured
// 6 % slower end to end (62.2 -> 66.4 ms/step, bench.py A/B in one call).
struct BwdSide {
  int device;
  hipStream_t caller, stream;
  hipEvent_t fork, join;
};
std::mutex g_side_mu;
BwdSide g_side[16];
int g_nside = 0;

bool bwd_overlap() {
  const char* v = getenv("IVIT_ATTN_BWD_OVERLAP");
  return v && v[0] == '1';
}

BwdSide* bwd_side_for(hipStream_t caller) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_side_mu);
  for (int i = 0; i < g_nside; ++i)
    if (g_side[i].device == dev && g_side[i].caller == caller) return &g_side[i];
  if (g_nside == 16) return nullptr;  // table full: run on the caller's stream
  BwdSide s{dev, caller, nullptr, nullptr, nullptr};
  if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
  if (hipEventCreateWithFlags(&s.fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s.join, hipEventDisableTiming) != hipSuccess)
    return nullptr;
  g_side[g_nside] = s;
  return &g_side[g_nside++];
}

}  // namespace

extern "C" long ivit_attn_workspace(int dtype, long B, long N, long H, long Dh, int backward) {
  if (dtype == IVIT_BF16) return backward ? 2 * B * H * ((N + AK - 1) / AK * AK) * 4 : 0;
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
    const char* ev = getenv("IVIT_ATTN_FWD_VARIANT");
    const int variant = ev ? atoi(ev) : 10;
    if (variant == 1) {
      dim3 g(ivit_cdiv(N, AQ), B * H);
      hipLaunchKernelGGL(attn_fwd_bf16_kernel, g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H, (bf16*)out,
                         lse, scale * LOG2E);
    } else if (variant == 2) {
      dim3 g(ivit_cdiv(N, AQ2), B * H);
      hipLaunchKernelGGL(attn_fwd_bf16_v2_kernel, g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H, (bf16*)out,
                         lse, scale * LOG2E);
    } else if (variant == 3) {
      dim3 g(ivit_cdiv(N, 128), B * H);
      hipLaunchKernelGGL(attn_fwd_bf16_v3_kernel<4>, g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H,
                         (bf16*)out, lse, scale * LOG2E);
    } else if (variant == 5) {
      dim3 g(ivit_cdiv(N, 128), B * H);
      hipLaunchKernelGGL(attn_fwd_bf16_v4_kernel<4>, g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H,
                         (bf16*)out, lse, scale * LOG2E);
    } else if (variant == 9) {  // software-pipelined (S_{j+1} || softmax_j), lazy rescale
      dim3 g(ivit_cdiv(N, 128), B * H);
      hipLaunchKernelGGL(attn_fwd_bf16_v5_kernel<4>, g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H,
                         (bf16*)out, lse, scale * LOG2E);
    } else if (variant == 10) {  // v5 with the interleave pinned by sched_group_barrier
      dim3 g(ivit_cdiv(N, 128), B * H);
      hipLaunchKernelGGL((attn_fwd_bf16_v5_kernel<4, true>), g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H,
                         (bf16*)out, lse, scale * LOG2E);
    } else if (variant == 11) {  // v6: prescaled Q, -m as the initial accumulator (no per-score FMA)
      dim3 g(ivit_cdiv(N, 128), B * H);
      hipLaunchKernelGGL((attn_fwd_bf16_v6_kernel<4, true>), g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H,
                         (bf16*)out, lse, scale * LOG2E);
    } else if (variant == 8) {  // v4 with the row sums on the MFMA pipe
      dim3 g(ivit_cdiv(N, 128), B * H);
      hipLaunchKernelGGL((attn_fwd_bf16_v4_kernel<4, 2, true>), g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H,
                         (bf16*)out, lse, scale * LOG2E);
    } else if (variant == 7) {  // v4 held to 3 workgroups (12 waves) per CU
      dim3 g(ivit_cdiv(N, 128), B * H);
      hipLaunchKernelGGL((attn_fwd_bf16_v4_kernel<4, 3>), g, dim3(256), 0, st, (const bf16*)qkv, (int)N, (int)H,
                         (bf16*)out, lse, scale * LOG2E);
    } else if (variant == 6) {
      dim3 g(ivit_cdiv(N, 256), B * H);
      hipLaunchKernelGGL(attn_fwd_bf16_v4_kernel<8>, g, dim3(512), 0, st, (const bf16*)qkv, (int)N, (int)H,
                         (bf16*)out, lse, scale * LOG2E);
    } else {
      dim3 g(ivit_cdiv(N, 256), B * H);
      hipLaunchKernelGGL(attn_fwd_bf16_v3_kernel<8>, g, dim3(512), 0, st, (const bf16*)qkv, (int)N, (int)H,
                         (bf16*)out, lse, scale * LOG2E);
    }
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
    const char* ev = getenv("IVIT_ATTN_DKV_VARIANT");
    const int dkv_variant = ev ? atoi(ev) : 2;
    dim3 g(ivit_cdiv(N, AQ), B * H);
    const long Npad = (N + AK - 1) / AK * AK;
    float* lse2p = (float*)work;
    float* deltap = lse2p + B * H * Npad;
    const bool v3 = dkv_variant == 3;  // v3: row constants as initial accumulators, pipelined dK/dV
    if (v3)
      hipLaunchKernelGGL(attn_rows_v3_kernel, dim3(ivit_cdiv(B * H * Npad * 8, 256)), dim3(256), 0, st,
                         (const bf16*)out, (const bf16*)dout, lse, (int)B, (int)N, (int)Npad, (int)H,
                         sqrtf((float)Dh), lse2p, deltap);
    else
      hipLaunchKernelGGL(attn_rows_v2_kernel, dim3(ivit_cdiv(B * H * Npad * 8, 256)), dim3(256), 0, st,
                         (const bf16*)out, (const bf16*)dout, lse, (int)B, (int)N, (int)Npad, (int)H, lse2p, deltap);
    // dQ and dK/dV are independent: optionally run dQ on a library-owned side stream so the two
    // latency-bound kernels overlap (the caller's stream waits for it before returning).
    hipStream_t sq = st;
    BwdSide* side = bwd_overlap() ? bwd_side_for(st) : nullptr;
    if (side) {
      if (hipEventRecord(side->fork, st) != hipSuccess || hipStreamWaitEvent(side->stream, side->fork, 0) != hipSuccess)
        IVIT_CHECK_ARG(false, "ivit_attn_bwd: side-stream fork failed");
      sq = side->stream;
    }
    if (v3)
      hipLaunchKernelGGL(attn_bwd_dq_v2_kernel<true>, g, dim3(256), 0, sq, (const bf16*)qkv, (const bf16*)dout, lse2p,
                         deltap, (int)N, (int)Npad, (int)H, (bf16*)dqkv, scale * LOG2E, scale);
    else
      hipLaunchKernelGGL(attn_bwd_dq_v2_kernel<false>, g, dim3(256), 0, sq, (const bf16*)qkv, (const bf16*)dout, lse2p,
                         deltap, (int)N, (int)Npad, (int)H, (bf16*)dqkv, scale * LOG2E, scale);
    if (side && hipEventRecord(side->join, sq) != hipSuccess) IVIT_CHECK_ARG(false, "ivit_attn_bwd: side-stream join failed");
    if (dkv_variant == 1)
      hipLaunchKernelGGL(attn_bwd_dkv_bf16_kernel, g, dim3(256), 0, st, (const bf16*)qkv, (const bf16*)dout, lse2p,
                         deltap, (int)N, (int)Npad, (int)H, (bf16*)dqkv, scale * LOG2E, scale);
    else if (v3)
      hipLaunchKernelGGL(attn_bwd_dkv_v3_kernel, g, dim3(256), 0, st, (const bf16*)qkv, (const bf16*)dout, lse2p,
                         deltap, (int)N, (int)Npad, (int)H, (bf16*)dqkv, scale * LOG2E, scale);
    else
      hipLaunchKernelGGL(attn_bwd_dkv_v2_kernel, g, dim3(256), 0, st, (const bf16*)qkv, (const bf16*)dout, lse2p,
                         deltap, (int)N, (int)Npad, (int)H, (bf16*)dqkv, scale * LOG2E, scale);
    if (side && hipStreamWaitEvent(st, side->join, 0) != hipSuccess)
      IVIT_CHECK_ARG(false, "ivit_attn_bwd: side-stream join failed");
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

// ------------------------------------------------------------------------- Q-prescaled bf16 path
extern "C" int ivit_attn_fwd_q2(const void* qkv, long B, long N, long H, long Dh, void* out, float* lse, void* work,
                                long work_bytes, void* stream) {
  IVIT_CHECK_ARG(Dh == 64, "ivit_attn_fwd_q2: head dim must be 64 (got %ld)", Dh);
  (void)work;
  (void)work_bytes;
  if (B * N * H == 0) return 0;
  dim3 g(ivit_cdiv(N, 128), B * H);
  hipLaunchKernelGGL((attn_fwd_bf16_v6_kernel<4, false>), g, dim3(256), 0, ivit_stream(stream), (const bf16*)qkv,
                     (int)N, (int)H, (bf16*)out, lse, 1.0f);
  IVIT_LAUNCH_CHECK();
  return 0;
}

// With q' = q c2 in qkv: P = exp2(q'k - lse2) (c2 = 1 in the kernels); dQ = scale dS K as before
// (the gradient w.r.t. the unscaled q); dK = ln2 dS^T q' = scale dS^T q.
extern "C" int ivit_attn_bwd_q2(const void* qkv, const void* out, const void* dout, const float* lse, long B, long N,
                                long H, long Dh, void* dqkv, void* work, long work_bytes, void* stream) {
  IVIT_CHECK_ARG(Dh == 64, "ivit_attn_bwd_q2: head dim must be 64 (got %ld)", Dh);
  IVIT_CHECK_ARG(work_bytes >= ivit_attn_workspace(IVIT_BF16, B, N, H, Dh, 1), "ivit_attn_bwd_q2: workspace too small");
  if (B * N * H == 0) return 0;
  hipStream_t st = ivit_stream(stream);
  const float scale = 1.0f / sqrtf((float)Dh);
  dim3 g(ivit_cdiv(N, AQ), B * H);
  const long Npad = (N + AK - 1) / AK * AK;
  float* lse2p = (float*)work;
  float* deltap = lse2p + B * H * Npad;
  // dQ also forms the row constants (lse2, delta) the dK/dV kernel reads: no rows kernel
  hipLaunchKernelGGL((attn_bwd_dq_v2_kernel<false, true, true>), g, dim3(256), 0, st, (const bf16*)qkv,
                     (const bf16*)dout, lse2p, deltap, (int)N, (int)Npad, (int)H, (bf16*)dqkv, 1.0f, scale,
                     (const bf16*)out, lse);
  hipLaunchKernelGGL(attn_bwd_dkv_v2_kernel, g, dim3(256), 0, st, (const bf16*)qkv, (const bf16*)dout, lse2p, deltap,
                     (int)N, (int)Npad, (int)H, (bf16*)dqkv, 1.0f, 0.69314718055994531f);
  IVIT_LAUNCH_CHECK();
  return 0;
}
