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

// 16x16x32 forms (attention.hip v4 backward): 64-row x 128-B tile images with chunk c of
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

// Epilogue of the 16x16x32 backward kernels: one wave's [32 rows][64 columns] output tile, held in
// the C layout (lane (g, c16) holds rows 16i + 4g + r, column 16e + c16 of v[i][e][r]), goes through
// the wave's own 4.5-KiB LDS region (rows 144 B apart: the 2-byte writes of lane groups g and g + 1
// land 16 banks apart) and out as whole 128-B rows, 8 lanes per row, 16 B per lane: 4 stores per lane
// instead of 32 two-byte ones. The caller has passed a barrier after the last read of the region
// (it reuses the tile stages). Rows row0 + k < nrows are stored at dst + (row0 + k) * ld.
IVIT_DEV void wave_tile_store(char* lds, const f32x4 (&v)[2][4], float scale, bf16* dst, long ld, int row0, int nrows,
                              int lane) {
  const int g = lane >> 4, c16 = lane & 15;
  bf16* t = (bf16*)lds;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int r = 0; r < 4; ++r) t[(16 * i + 4 * g + r) * 72 + 16 * e + c16] = (bf16)(v[i][e][r] * scale);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int row = 8 * k + (lane >> 3), ch = lane & 7;
    const uint4 x = *(const uint4*)(lds + row * 144 + ch * 16);
    if (row0 + row < nrows) *(uint4*)(dst + (long)(row0 + row) * ld + ch * 8) = x;
  }
}

IVIT_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

}  // namespace
