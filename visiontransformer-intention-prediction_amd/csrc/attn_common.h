// Helpers of the attention kernels (attention.hip: flash forward, the dQ and dK/dV backward
// kernels and the f32 parity path). gfx950 only.
#pragma once
#include "gemm_engine.h"
#include "panel_common.h"

using namespace ivit;

namespace {

constexpr int AQ = 128;  // queries per workgroup (4 waves x 32)
constexpr int AK = 64;   // keys per tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float NEG_BIG = -1.0e30f;

// LDS-DMA of 4 B per lane, saddr form: sbase + voff -> lds + 4 * lane.
IVIT_DEV void glds4_s(unsigned voff, const char* sbase, void* lds) {
  const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, %2" ::"v"(voff), "s"(a), "s"(sbase)
               : "memory");
}

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

// k-invariant per-lane DMA source offsets: a full tile is base + r0*ld + off (the row guard only
// on the ragged last tile), and tile loops unrolled by two so the LDS stage is a compile-time
// constant: every fragment read is a per-lane base plus an immediate offset.
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

// 16x16x32 forms (attention.hip v4 backward, v7 forward): 64-row x 128-B tile images with chunk c of
// row r at c ^ (r & 6) — conflict-free for the 16x16x32 row reads (16 rows x one chunk per 16-lane
// group) and the transposed reads of 8 rows x 2 chunks per half-wave.
IVIT_DEV int t16_off(int r, int c) { return r * 128 + ((c ^ (r & 6)) << 4); }

template <int W>
IVIT_DEV int dma_off16(int i, int wv, int lane, long ld) {
  const int piece = wv * (8 / W) + i;
  const int row = piece * 8 + (lane >> 3);
  const int c = (lane & 7) ^ (row & 6);
  return (int)(row * ld) + c * 8;
}

IVIT_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// max over the four lanes l, l ^ 16, l ^ 32, l ^ 48 (the 16x16 C layout's row groups)
IVIT_DEV float quad_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return half_swap_max(fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])));
}

}  // namespace
