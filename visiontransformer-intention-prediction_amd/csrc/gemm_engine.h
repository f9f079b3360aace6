// Generic tiled MFMA GEMM engine for gfx950 with gather loaders and fused epilogues.
//
//   C[m, n] = sum_k A[m, k] * B[k, n]      (per batch z; optional split-K)
//
// Operands are "loaders": functors returning 8 bf16 (load8) or 4 f32 (load4) that are
// contiguous along the loader's `c` argument. An operand is K-contiguous (LDS image
// [rows=M or N][K], read with ds_read_b128) or MN-contiguous (image [K][M or N], read
// with the CDNA4 transposing ds_read_b64_tr_b16). Gather loaders turn the patch
// embedding and 3x3 convolutions into implicit GEMMs without an im2col buffer.
//
// bf16 path: 128x128x64 tile, 4 waves (2x2) x 64x64, v_mfma_f32_32x32x16_bf16.
// f32  path: 128x128x16 tile, 4 waves (2x2) x 64x64, v_mfma_f32_32x32x2_f32 (exact f32).
#pragma once
#include <stdlib.h>

#include <type_traits>

#include "ivit_common.h"

namespace ivit {

constexpr int GBM = 128, GBN = 128;
constexpr int GBK16 = 64;  // bf16 K tile
constexpr int GBK32 = 16;  // f32 K tile

// z -> element offset: (z / zdiv) * s1 + (z % zdiv) * s2
// (32-bit index math only: a 64-bit division is a ~100-instruction software loop on CDNA.)
struct BatchOff {
  int zdiv;
  long s1, s2;
  __host__ __device__ BatchOff(long zd = 1, long a = 0, long b = 0) : zdiv((int)zd), s1(a), s2(b) {}
  IVIT_DEV long at(int z) const { return (long)(z / zdiv) * s1 + (long)(z % zdiv) * s2; }
};

// ----------------------------------------------------------------------------- loaders
// Dense matrix (optionally with a "row map" r -> (r / rpb) * rstride + roff + r % rpb,
// used to skip CLS token rows). Element (r, c) at p[rowaddr(r) * ld + c]; zero if r >= R
// or c >= C. C must be a multiple of 8 (bf16 chunks) / 4 (f32 chunks) — checked on host.
template <typename S>
struct LdDense {
  static constexpr bool kRowFast = false;
  static constexpr bool kGlds = sizeof(S) == 2;
  const S* p; long ld; int R, C; int rpb; long rstride; int roff; BatchOff bo;
  IVIT_DEV LdDense bind(int z) const {  // fold the batch offset into the base once per block
    LdDense t = *this;
    t.p = p + bo.at(z);
    return t;
  }
  IVIT_DEV long row_addr(int r) const { return rpb ? (long)(r / rpb) * rstride + roff + r % rpb : (long)r; }
  // LDS-DMA fast path (see gemm_bf16_glds_kernel): the per-lane source of an image piece is
  // a k-invariant 32-bit element offset plus a uniform per-K-tile advance. Rows / columns
  // past the matrix edge are clamped to the last valid one — they only feed output rows or
  // columns that the epilogue never stores; the K edge goes through the generic path.
  static constexpr bool kFast = true, kMayZero = false;
  using Pre = int;
  IVIT_DEV bool fast_ok(bool kc) const {
    return R > 0 && C >= 8 && (kc || rpb == 0) && (row_addr(R - 1) + 65) * ld + C < 0x7fffffffL;
  }
  IVIT_DEV Pre pre(bool kc, int piece, int lane, int o0) const {
    if (kc) {  // image rows = m/n (8 per piece), chunks along k
      const int row = piece * 8 + (lane >> 3), c = (lane & 7) ^ swz128_(row);
      return (int)(row_addr(min(o0 + row, R - 1)) * ld) + c * 8;
    }
    const int row = piece * 4 + (lane >> 4), c = (lane & 15) ^ ((row & 3) << 2);  // rows = k
    return (int)(row * ld) + min(o0 + c * 8, C - 8);
  }
  IVIT_DEV const void* fast_src(const Pre& o, bool kc, int k0) const {
    return p + (kc ? (long)k0 : (long)k0 * ld) + o;
  }
  IVIT_DEV static int swz128_(int r) { return (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 1) | ((r >> 2) & 1); }
  IVIT_DEV const void* src8(int, int r, int c) const {
    return (r >= R || c >= C) ? nullptr : (const void*)(p + row_addr(r) * ld + c);
  }
  IVIT_DEV uint4 load8(int, int r, int c) const {
    if (r >= R || c >= C) return make_uint4(0, 0, 0, 0);
    const S* q = p + row_addr(r) * ld + c;
    if constexpr (sizeof(S) == 2) {
      return *(const uint4*)q;
    } else {
      return f32x8_to_bf16x8(*(const float4*)q, *(const float4*)(q + 4));
    }
  }
  IVIT_DEV float4 load4(int, int r, int c) const {
    if (r >= R || c >= C) return make_float4(0.f, 0.f, 0.f, 0.f);
    const S* q = p + row_addr(r) * ld + c;
    if constexpr (sizeof(S) == 4) {
      return *(const float4*)q;
    } else {
      Pack4 t; t.u = *(const uint2*)q;
      return make_float4(bf2f(t.h[0]), bf2f(t.h[1]), bf2f(t.h[2]), bf2f(t.h[3]));
    }
  }
};

// Patch gather over an NCHW image (timm PatchEmbed conv k = s = P, P = 8):
// r = m = b*Np + gy*Wp + gx ; c = kk = (ch*P + ky)*P + kx  (chunk of 8 = one kx row).
template <typename S>
struct LdPatch {
  static constexpr bool kFast = false;
  static constexpr bool kRowFast = true;  // consecutive patches are consecutive 32-B runs
  static constexpr bool kGlds = false;    // f32 image converted to bf16 on the way: register staging
  IVIT_DEV LdPatch bind(int) const { return *this; }
  const S* img; int Bn, Cin, H, W, Wp, Np; int R, C;
  IVIT_DEV const S* addr(int r, int c) const {
    const int b = r / Np, pi = r - b * Np, gy = pi / Wp, gx = pi - gy * Wp;
    const int ch = c >> 6, ky = (c >> 3) & 7, kx = c & 7;
    return img + (((long)b * Cin + ch) * H + gy * 8 + ky) * (long)W + gx * 8 + kx;
  }
  IVIT_DEV uint4 load8(int, int r, int c) const {
    if (r >= R || c >= C) return make_uint4(0, 0, 0, 0);
    const S* q = addr(r, c);
    if constexpr (sizeof(S) == 2) return *(const uint4*)q;
    else return f32x8_to_bf16x8(*(const float4*)q, *(const float4*)(q + 4));
  }
  IVIT_DEV float4 load4(int, int r, int c) const {
    if (r >= R || c >= C) return make_float4(0.f, 0.f, 0.f, 0.f);
    const S* q = addr(r, c);
    if constexpr (sizeof(S) == 4) return *(const float4*)q;
    else {
      Pack4 t; t.u = *(const uint2*)q;
      return make_float4(bf2f(t.h[0]), bf2f(t.h[1]), bf2f(t.h[2]), bf2f(t.h[3]));
    }
  }
};

// k x k "same" convolution gather over an NHWC map (pad = k/2):
// r = m = (b*H + y)*W + x ; c = kk = (ky*k + kx)*Cin + ci   (Cin % 8 == 0).
// flip = true reads the spatially flipped tap (dgrad of the transposed conv).
template <typename S>
struct LdConv {
  static constexpr bool kRowFast = false;
  static constexpr bool kGlds = sizeof(S) == 2;
  const S* x; int H, W, Cin, ks; int R, C; long ldc;  // ldc = channel stride of a pixel
  IVIT_DEV LdConv bind(int) const { return *this; }
  // LDS-DMA fast path (K-contiguous image, Cin % 64 == 0, so a 64-wide K tile sits in one
  // tap): the pixel of each lane's row is decomposed once; per tile only the tap's (dy, dx)
  // bounds test and one add remain.
  static constexpr bool kFast = true, kMayZero = true;  // padding taps read the zero page
  struct Pre { int base; int yx; };
  IVIT_DEV bool fast_ok(bool kc) const {
    return kc && Cin % 64 == 0 && R > 0 && (long)R * ldc + C < 0x7fffffffL;
  }
  IVIT_DEV Pre pre(bool kc, int piece, int lane, int o0) const {
    const int row = piece * 8 + (lane >> 3), c = (lane & 7) ^ LdDense<S>::swz128_(row);
    const int r = min(o0 + row, R - 1);
    const int xw = r % W, y = (r / W) % H;
    return {(int)(r * ldc) + c * 8, (y << 16) | xw};
  }
  IVIT_DEV const void* fast_src(const Pre& o, bool, int k0) const {
    const int tap = k0 / Cin, ci0 = k0 - tap * Cin;
    const int ky = tap / ks, kx = tap - ky * ks, pad = ks >> 1;
    const int dy = ky - pad, dx = kx - pad;
    const int yy = (o.yx >> 16) + dy, xx = (o.yx & 0xffff) + dx;
    if (yy < 0 || yy >= H || xx < 0 || xx >= W) return nullptr;
    return x + o.base + (dy * W + dx) * ldc + ci0;
  }
  IVIT_DEV const void* src8(int, int r, int c) const {
    long off;
    return at(r, c, off) ? (const void*)(x + off) : nullptr;
  }
  IVIT_DEV bool at(int r, int c, long& off) const {
    if (r >= R || c >= C) return false;
    const int tap = c / Cin, ci = c - tap * Cin;
    const int ky = tap / ks, kx = tap - ky * ks, pad = ks >> 1;
    const int xw = r % W, t = r / W, y = t % H, b = t / H;
    const int yy = y + ky - pad, xx = xw + kx - pad;
    if (yy < 0 || yy >= H || xx < 0 || xx >= W) return false;
    off = (((long)b * H + yy) * W + xx) * ldc + ci;
    return true;
  }
  IVIT_DEV uint4 load8(int, int r, int c) const {
    long off;
    if (!at(r, c, off)) return make_uint4(0, 0, 0, 0);
    const S* q = x + off;
    if constexpr (sizeof(S) == 2) return *(const uint4*)q;
    else return f32x8_to_bf16x8(*(const float4*)q, *(const float4*)(q + 4));
  }
  IVIT_DEV float4 load4(int, int r, int c) const {
    long off;
    if (!at(r, c, off)) return make_float4(0.f, 0.f, 0.f, 0.f);
    const S* q = x + off;
    if constexpr (sizeof(S) == 4) return *(const float4*)q;
    else {
      Pack4 t; t.u = *(const uint2*)q;
      return make_float4(bf2f(t.h[0]), bf2f(t.h[1]), bf2f(t.h[2]), bf2f(t.h[3]));
    }
  }
};

// Weights [Cout][ks][ks][Cin] read as the dgrad B operand: row r = (ky'*ks + kx')*Cout + co
// (the flipped tap), col c = ci  ->  W[co][ks-1-ky'][ks-1-kx'][ci].
template <typename S>
struct LdConvWFlip {
  static constexpr bool kRowFast = false;
  static constexpr bool kGlds = sizeof(S) == 2;
  const S* w; int Cout, Cin, ks; int R, C;
  IVIT_DEV LdConvWFlip bind(int) const { return *this; }
  // LDS-DMA fast path (MN-contiguous image, Cout % 64 == 0: a 64-row K tile is one tap):
  // per lane a fixed (row, column) offset, per tile a uniform (co0, flipped tap) base.
  static constexpr bool kFast = true, kMayZero = false;
  using Pre = int;
  IVIT_DEV bool fast_ok(bool kc) const {
    return !kc && Cout % 64 == 0 && C >= 8 && (long)Cout * ks * ks * Cin < 0x7fffffffL;
  }
  IVIT_DEV Pre pre(bool, int piece, int lane, int o0) const {
    const int row = piece * 4 + (lane >> 4), c = (lane & 15) ^ ((row & 3) << 2);
    return row * ks * ks * Cin + min(o0 + c * 8, C - 8);
  }
  IVIT_DEV const void* fast_src(const Pre& o, bool, int k0) const {
    const int tap = k0 / Cout, co0 = k0 - tap * Cout;
    const int ky = tap / ks, kx = tap - ky * ks;
    return w + ((co0 * ks + (ks - 1 - ky)) * ks + (ks - 1 - kx)) * Cin + o;
  }
  IVIT_DEV const void* src8(int, int r, int c) const {
    return (r >= R || c >= C) ? nullptr : (const void*)addr(r, c);
  }
  IVIT_DEV const S* addr(int r, int c) const {
    const int tap = r / Cout, co = r - tap * Cout;
    const int ky = tap / ks, kx = tap - ky * ks;
    return w + (((long)co * ks + (ks - 1 - ky)) * ks + (ks - 1 - kx)) * Cin + c;
  }
  IVIT_DEV uint4 load8(int, int r, int c) const {
    if (r >= R || c >= C) return make_uint4(0, 0, 0, 0);
    const S* q = addr(r, c);
    if constexpr (sizeof(S) == 2) return *(const uint4*)q;
    else return f32x8_to_bf16x8(*(const float4*)q, *(const float4*)(q + 4));
  }
  IVIT_DEV float4 load4(int, int r, int c) const {
    if (r >= R || c >= C) return make_float4(0.f, 0.f, 0.f, 0.f);
    const S* q = addr(r, c);
    if constexpr (sizeof(S) == 4) return *(const float4*)q;
    else {
      Pack4 t; t.u = *(const uint2*)q;
      return make_float4(bf2f(t.h[0]), bf2f(t.h[1]), bf2f(t.h[2]), bf2f(t.h[3]));
    }
  }
};

// ----------------------------------------------------------------------------- epilogues
// apply8(z, split, m, n, v, nv): outputs (m, n .. n+nv-1), nv <= 8, m < M, n < N. The engine
// hands each lane 8 consecutive columns (accumulators transposed through LDS), so stores are
// 16-byte vectors whenever the destination is aligned.
//
// Two-phase form used by epilogue_tile: a lane's columns are the same for every row it
// stores, so col() loads the per-column operands (bias) ONCE per tile, and row() issues the
// per-row loads (residual, pre-activation, position rows) of all the lane's rows before any
// of them is consumed; out8() then only computes and stores. (Per-call loads behind a
// s_waitcnt made the epilogue a serial chain of ~8 exposed global-load latencies per wave.)
struct NoCol {};
struct NoRow {};
struct Bias8 { float b[8]; };
struct Row8 { float r[8]; };

// qcols > 0: columns n < qcols are additionally scaled by qscale (the attention's Q block of a
// fused qkv projection stored as q * log2(e)/sqrt(Dh); ivit_linear_fwd_qs). qcols % 8 == 0,
// so the factor is uniform over a lane's 8 columns.
struct BiasS { float b[8]; float s; };
template <typename O>
struct EpiStore {  // out = act(alpha*acc + bias[n]) [* qscale for n < qcols]; optional pre-activation copy
  O* out; long ldo; BatchOff bo; const float* bias; int act; O* pre; float alpha;
  int qcols = 0; float qscale = 1.f;
  using Col = BiasS;
  using Row = NoRow;
  IVIT_DEV EpiStore bind(int z) const {
    EpiStore t = *this;
    const long o = bo.at(z);
    t.out = out + o;
    t.pre = pre ? pre + o : nullptr;
    return t;
  }
  IVIT_DEV void col(int n, int nv, Col& c) const {
    if (bias) load8f(bias + n, c.b, nv);
    else {
#pragma unroll
      for (int k = 0; k < 8; ++k) c.b[k] = 0.f;
    }
    c.s = n < qcols ? qscale : 1.f;
  }
  IVIT_DEV void row(int, int, int, Row&) const {}
  IVIT_DEV void out8(int, int m, int n, const float (&v)[8], int nv, const Col& c, const Row&) const {
    float x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = (v[k] * alpha + c.b[k]) * c.s;
    const long o = (long)m * ldo + n;
    if (pre) store8(pre + o, x, nv);
    if (act == IVIT_ACT_GELU) {
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = gelu_t<O>(x[k]);
    } else if (act == IVIT_ACT_RELU) {
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = fmaxf(x[k], 0.f);
    }
    store8(out + o, x, nv);
  }
  IVIT_DEV void apply8(int, int, int m, int n, const float (&v)[8], int nv) const {
    Col c;
    col(n, nv, c);
    out8(0, m, n, v, nv, c, Row{});
  }
};

struct EpiResid {  // out(f32) = res + scale[m / rps] * (acc + bias[n])
  float* out; long ldo; const float* res; long ldr; const float* bias; const float* scale; int rps;
  using Col = Bias8;
  struct Row { float r[8]; float s; };
  IVIT_DEV EpiResid bind(int) const { return *this; }
  IVIT_DEV void col(int n, int nv, Col& c) const {
    if (bias) load8f(bias + n, c.b, nv);
    else {
#pragma unroll
      for (int k = 0; k < 8; ++k) c.b[k] = 0.f;
    }
  }
  IVIT_DEV void row(int m, int n, int nv, Row& r) const {
    load8f(res + (long)m * ldr + n, r.r, nv);
    r.s = scale ? scale[m / rps] : 1.f;
  }
  IVIT_DEV void out8(int, int m, int n, const float (&v)[8], int nv, const Col& c, const Row& r) const {
    float x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = r.r[k] + r.s * (v[k] + c.b[k]);
    store8(out + (long)m * ldo + n, x, nv);
  }
  IVIT_DEV void apply8(int, int, int m, int n, const float (&v)[8], int nv) const {
    Col c;
    Row r;
    col(n, nv, c);
    row(m, n, nv, r);
    out8(0, m, n, v, nv, c, r);
  }
};

template <typename O, typename P>
struct EpiGeluGrad {  // out = acc * gelu'(pre)
  O* out; long ldo; const P* pre; long ldp;
  using Col = NoCol;
  using Row = Row8;
  IVIT_DEV EpiGeluGrad bind(int) const { return *this; }
  IVIT_DEV void col(int, int, Col&) const {}
  IVIT_DEV void row(int m, int n, int nv, Row& r) const { load8f(pre + (long)m * ldp + n, r.r, nv); }
  IVIT_DEV void out8(int, int m, int n, const float (&v)[8], int nv, const Col&, const Row& r) const {
    float x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = v[k] * gelu_grad_t<O>(r.r[k]);
    store8(out + (long)m * ldo + n, x, nv);
  }
  IVIT_DEV void apply8(int, int, int m, int n, const float (&v)[8], int nv) const {
    Row r;
    row(m, n, nv, r);
    out8(0, m, n, v, nv, Col{}, r);
  }
};

struct EpiSlab {  // split-K partial slab [split][M][N] (f32)
  // bslab != null (bf16 LDS-DMA path, MN-contiguous A only): the blocks of the first column
  // tile also write per-split row sums of A, bslab[split][m] = sum_k A[m][k] — the bias
  // gradient of a wgrad (colsum of dY) — computed on the MFMA pipe against a ones operand.
  static constexpr bool kBiasOnes = true;
  float* slab; long M, N; float* bslab = nullptr;
  using Col = NoCol;
  using Row = NoRow;
  IVIT_DEV EpiSlab bind(int) const { return *this; }
  IVIT_DEV void col(int, int, Col&) const {}
  IVIT_DEV void row(int, int, int, Row&) const {}
  IVIT_DEV void out8(int split, int m, int n, const float (&v)[8], int nv, const Col&, const Row&) const {
    store8(slab + ((long)split * M + m) * N + n, v, nv);
  }
  IVIT_DEV void apply8(int, int split, int m, int n, const float (&v)[8], int nv) const {
    out8(split, m, n, v, nv, Col{}, Row{});
  }
};

struct EpiPatch {  // token (b, 1 + p) of x(f32) = acc + bias[n] + pos[1 + p][n]
  float* out; int Np, D; const float* bias; const float* pos;
  using Col = Bias8;
  using Row = Row8;
  IVIT_DEV EpiPatch bind(int) const { return *this; }
  IVIT_DEV void col(int n, int nv, Col& c) const { load8f(bias + n, c.b, nv); }
  IVIT_DEV void row(int m, int n, int nv, Row& r) const {
    const int p = m - (m / Np) * Np;
    load8f(pos + (long)(1 + p) * D + n, r.r, nv);
  }
  IVIT_DEV void out8(int, int m, int n, const float (&v)[8], int nv, const Col& c, const Row& r) const {
    const int b = m / Np, p = m - b * Np;
    const long row = (long)b * (Np + 1) + 1 + p;
    float x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = v[k] + c.b[k] + r.r[k];
    store8(out + row * D + n, x, nv);
  }
  IVIT_DEV void apply8(int, int, int m, int n, const float (&v)[8], int nv) const {
    Col c;
    Row r;
    col(n, nv, c);
    row(m, n, nv, r);
    out8(0, m, n, v, nv, c, r);
  }
};

// Wave-local accumulator transpose through LDS (the staging buffers are free after the
// main loop): 32-row halves of the wave's 64x64 tile, row stride 68 floats. Lane l stores
// columns nbase + 8(l & 7) .. +7 of rows (l >> 3) + 8t (t = 0..3) of each half: the column
// operands are loaded once, the 8 rows' operands all before the first LDS write.
constexpr int EP_LD = 68;
template <class EPI>
IVIT_DEV void epilogue_tile(float* ep, f32x16 (&acc)[2][2], const EPI& epi, int z, int split, int mbase, int nbase,
                            int M, int N, int lane) {
  const int h = lane >> 5;
  const int c0 = (lane & 7) * 8, n = nbase + c0, nv = min(8, N - n);
  const bool nok = n < N;
  typename EPI::Col col;
  if (nok) epi.col(n, nv, col);
  typename EPI::Row rows[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int m = mbase + 32 * i + (lane >> 3) + 8 * t;
      if (nok && m < M) epi.row(m, n, nv, rows[i][t]);
    }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ep[((r & 3) + 8 * (r >> 2) + 4 * h) * EP_LD + 32 * j + (lane & 31)] = acc[i][j][r];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes are complete
    float v[4][8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int row = (lane >> 3) + 8 * t;
      const float4 a = *(const float4*)(ep + row * EP_LD + c0);
      const float4 b = *(const float4*)(ep + row * EP_LD + c0 + 4);
      v[t][0] = a.x; v[t][1] = a.y; v[t][2] = a.z; v[t][3] = a.w;
      v[t][4] = b.x; v[t][5] = b.y; v[t][6] = b.z; v[t][7] = b.w;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int m = mbase + 32 * i + (lane >> 3) + 8 * t;
      if (nok && m < M) epi.out8(split, m, n, v[t], nv, col, rows[i][t]);
    }
  }
}

// ----------------------------------------------------------------------------- LDS images
// K-contiguous bf16 image: rows x 64 k (128-B rows); 16-B chunk c of row r stored at
// chunk c ^ f(r), f a bijection of (r>>1)&7 chosen so that both the 32x32x16 row reads
// (ds_read_b128 lane groups) and the transposed reads hit distinct bank slots.
IVIT_DEV int swz128(int r) { return (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 1) | ((r >> 2) & 1); }
IVIT_DEV int kc_off(int r, int c) { return r * 128 + ((c ^ swz128(r)) << 4); }
// MN-contiguous bf16 image: 64 k-rows x 128 columns (256-B rows); chunk c -> c ^ 4(r&3).
IVIT_DEV int mn_off(int r, int c) { return r * 256 + ((c ^ ((r & 3) << 2)) << 4); }

IVIT_DEV bf16x8 frag_kc(const char* img, int row, int chunk) {
  return *(const bf16x8*)(img + kc_off(row, chunk));
}

IVIT_DEV s16x4 ds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// 32x32x16 operand (lane l: row/col l&31, k = 8(l>>5) + j) from an MN-contiguous image:
// two transposing reads of 4 k-rows each.
IVIT_DEV bf16x8 frag_mn(const char* img, int kbase, int colbase, int lane) {
  const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = colbase + 16 * (G & 1) + 4 * p;
  const int r0 = kbase + 8 * (G >> 1) + q;
  const int c = col >> 3, e = (col & 7) * 2;
  s16x4 lo = ds_tr(img + mn_off(r0, c) + e);
  s16x4 hi = ds_tr(img + mn_off(r0 + 4, c) + e);
  union { s16x4 s[2]; bf16x8 v; } u;
  u.s[0] = lo; u.s[1] = hi;
  return u.v;
}

// ----------------------------------------------------------------------------- bf16 kernel
template <class LA, class LB, class EPI, bool A_KC, bool B_KC>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(LA la_, LB lb_, EPI epi_, int M, int N, int K,
                                                         int tilesM, int tilesN, int splits, int kchunk) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][16384];  // [stage][A|B][image]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin / tilesN, tn = lin - tm * tilesN;
  const int z = blockIdx.y / splits, split = blockIdx.y - z * splits;
  const LA la = la_.bind(z);
  const LB lb = lb_.bind(z);
  const EPI epi = epi_.bind(z);
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nk = (kend - kbeg + GBK16 - 1) / GBK16;

  uint4 ra[4], rb[4];
  auto gload = [&](const auto& ld, bool kc, int o0, int k0, uint4* r) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i;
      if (kc) {  // image rows = 128 (m/n), 8 chunks along k
        int row, ch;
        if (std::decay_t<decltype(ld)>::kRowFast) { row = idx & 127; ch = idx >> 7; }
        else { row = idx >> 3; ch = idx & 7; }
        const int kk = k0 + ch * 8;
        r[i] = kk < kend ? ld.load8(z, o0 + row, kk) : make_uint4(0, 0, 0, 0);
      } else {   // image rows = 64 (k), 16 chunks along m/n
        int row, ch;
        if (std::decay_t<decltype(ld)>::kRowFast) { row = idx & 63; ch = idx >> 6; }
        else { row = idx >> 4; ch = idx & 15; }
        const int kk = k0 + row;
        r[i] = kk < kend ? ld.load8(z, kk, o0 + ch * 8) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto sstore = [&](char* img, bool kc, bool rowfast, const uint4* r) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i;
      int off;
      if (kc) {
        int row, ch;
        if (rowfast) { row = idx & 127; ch = idx >> 7; } else { row = idx >> 3; ch = idx & 7; }
        off = kc_off(row, ch);
      } else {
        int row, ch;
        if (rowfast) { row = idx & 63; ch = idx >> 6; } else { row = idx >> 4; ch = idx & 15; }
        off = mn_off(row, ch);
      }
      *(uint4*)(img + off) = r[i];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    gload(la, A_KC, m0, kbeg, ra);
    gload(lb, B_KC, n0, kbeg, rb);
    sstore(smem[0][0], A_KC, LA::kRowFast, ra);
    sstore(smem[0][1], B_KC, LB::kRowFast, rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      gload(la, A_KC, m0, kbeg + (kt + 1) * GBK16, ra);
      gload(lb, B_KC, n0, kbeg + (kt + 1) * GBK16, rb);
    }
    const char* ia = smem[cur][0];
    const char* ib = smem[cur][1];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int rb0 = wm * 64 + 32 * i;
        fa[i] = A_KC ? frag_kc(ia, rb0 + (lane & 31), 2 * t + (lane >> 5)) : frag_mn(ia, 16 * t, rb0, lane);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cb0 = wn * 64 + 32 * j;
        fb[j] = B_KC ? frag_kc(ib, cb0 + (lane & 31), 2 * t + (lane >> 5)) : frag_mn(ib, 16 * t, cb0, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      sstore(smem[cur ^ 1][0], A_KC, LA::kRowFast, ra);
      sstore(smem[cur ^ 1][1], B_KC, LB::kRowFast, rb);
    }
    __syncthreads();
  }
  // C layout (32x32 f32): col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5); transposed via LDS
  epilogue_tile((float*)&smem[0][0][0] + wv * (32 * EP_LD), acc, epi, z, split, m0 + wm * 64, n0 + wn * 64, M, N,
                lane);
}

// ----------------------------------------------------------------------------- f32 kernel
// K-contiguous f32 image [128][17] (row pad -> conflict-free ds_read_b32 column reads);
// MN-contiguous f32 image [16][128].
template <class LA, class LB, class EPI, bool A_KC, bool B_KC>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(LA la_, LB lb_, EPI epi_, int M, int N, int K,
                                                        int tilesM, int tilesN, int splits, int kchunk) {
  constexpr int KCS = 17;                       // K-contig row stride (floats)
  constexpr int IMG = 128 * KCS > 16 * 128 ? 128 * KCS : 16 * 128;
  __shared__ __attribute__((aligned(16))) float smem[2][2][IMG];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin / tilesN, tn = lin - tm * tilesN;
  const int z = blockIdx.y / splits, split = blockIdx.y - z * splits;
  const LA la = la_.bind(z);
  const LB lb = lb_.bind(z);
  const EPI epi = epi_.bind(z);
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nk = (kend - kbeg + GBK32 - 1) / GBK32;

  float4 ra[2], rb[2];
  auto gload = [&](const auto& ld, bool kc, int o0, int k0, float4* r) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i;
      if (kc) {  // 128 rows x 4 chunks of 4 k
        int row, ch;
        if (std::decay_t<decltype(ld)>::kRowFast) { row = idx & 127; ch = idx >> 7; }
        else { row = idx >> 2; ch = idx & 3; }
        const int kk = k0 + ch * 4;
        r[i] = kk < kend ? ld.load4(z, o0 + row, kk) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {   // 16 k-rows x 32 chunks of 4
        int row, ch;
        if (std::decay_t<decltype(ld)>::kRowFast) { row = idx & 15; ch = idx >> 4; }
        else { row = idx >> 5; ch = idx & 31; }
        const int kk = k0 + row;
        r[i] = kk < kend ? ld.load4(z, kk, o0 + ch * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  auto sstore = [&](float* img, bool kc, bool rowfast, const float4* r) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i;
      if (kc) {
        int row, ch;
        if (rowfast) { row = idx & 127; ch = idx >> 7; } else { row = idx >> 2; ch = idx & 3; }
        float* d = img + row * KCS + ch * 4;
        d[0] = r[i].x; d[1] = r[i].y; d[2] = r[i].z; d[3] = r[i].w;
      } else {
        int row, ch;
        if (rowfast) { row = idx & 15; ch = idx >> 4; } else { row = idx >> 5; ch = idx & 31; }
        *(float4*)(img + row * 128 + ch * 4) = r[i];
      }
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    gload(la, A_KC, m0, kbeg, ra);
    gload(lb, B_KC, n0, kbeg, rb);
    sstore(smem[0][0], A_KC, LA::kRowFast, ra);
    sstore(smem[0][1], B_KC, LB::kRowFast, rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      gload(la, A_KC, m0, kbeg + (kt + 1) * GBK32, ra);
      gload(lb, B_KC, n0, kbeg + (kt + 1) * GBK32, rb);
    }
    const float* ia = smem[cur][0];
    const float* ib = smem[cur][1];
    const int kq = lane >> 5;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int k = 2 * s + kq;
      float fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 64 + 32 * i + (lane & 31);
        fa[i] = A_KC ? ia[row * KCS + k] : ia[k * 128 + row];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wn * 64 + 32 * j + (lane & 31);
        fb[j] = B_KC ? ib[col * KCS + k] : ib[k * 128 + col];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      sstore(smem[cur ^ 1][0], A_KC, LA::kRowFast, ra);
      sstore(smem[cur ^ 1][1], B_KC, LB::kRowFast, rb);
    }
    __syncthreads();
  }
  epilogue_tile(&smem[0][0][0] + wv * (32 * EP_LD), acc, epi, z, split, m0 + wm * 64, n0 + wn * 64, M, N, lane);
}

// ----------------------------------------------------------------------------- bf16 LDS-DMA kernel
// Same tiling/fragments/epilogue as gemm_bf16_kernel, but operands stream HBM -> LDS with
// global_load_lds_dwordx4 (no VGPR staging): the next K tile is in flight during the
// current tile's MFMAs, retired by a counted vmcnt and a raw s_barrier (no __syncthreads:
// its fence would drain the DMA). The swizzle moves to the per-lane SOURCE address: each
// 1-KiB wave piece is lane-linear in LDS (cdna_hip_programming.md §5 rule 21). Out-of-range
// rows/taps read a zero page.
static __device__ __attribute__((aligned(16))) uint4 g_zero16[4];

template <class L>
IVIT_DEV void glds_piece(const L& ld, int z, bool kc, char* img, int piece, int lane, int o0, int k0, int kend) {
  const void* src;
  if (kc) {  // image rows = m/n (128-B rows); a piece = 8 rows
    const int row = piece * 8 + (lane >> 3), c = (lane & 7) ^ swz128(row);
    const int kk = k0 + c * 8;
    src = kk < kend ? ld.src8(z, o0 + row, kk) : nullptr;
  } else {   // image rows = k (256-B rows); a piece = 4 rows
    const int row = piece * 4 + (lane >> 4), c = (lane & 15) ^ ((row & 3) << 2);
    const int kk = k0 + row;
    src = kk < kend ? ld.src8(z, kk, o0 + c * 8) : nullptr;
  }
  glds<16>(src ? src : (const void*)g_zero16, img + piece * 1024);
}

// One operand's P pieces of a K tile for this wave: fast (precomputed per-lane state) or the
// generic gather (bounds-checked per element chunk).
template <int P, class L>
IVIT_DEV void glds_operand(const L& ld, int z, bool kc, char* img, int wv, int lane, int o0, int k0, int kend,
                           bool fast, const typename L::Pre (&pre)[P]) {
  if (fast) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const void* src = ld.fast_src(pre[i], kc, k0);
      if constexpr (L::kMayZero) src = src ? src : (const void*)g_zero16;
      glds<16>(src, img + (wv * P + i) * 1024);
    }
  } else {
#pragma unroll
    for (int i = 0; i < P; ++i) glds_piece(ld, z, kc, img, wv * P + i, lane, o0, k0, kend);
  }
}

template <class E, class = void>
struct BiasOnes { static constexpr bool v = false; };
template <class E>
struct BiasOnes<E, std::void_t<decltype(E::kBiasOnes)>> { static constexpr bool v = E::kBiasOnes; };

// WM waves along M (tile BM = 64*WM rows) x 2 waves along N (BN = 128), each wave 64x64.
// WM = 2: 128x128 tile, 4 waves, two workgroups per CU. WM = 4: 256x128 tile, 8 waves, one
// workgroup per CU — half the B-tile traffic per flop and twice the work per K step for the
// skinny M = 36 008 token GEMMs (K-contiguous A only: the A image keeps 128-B rows).
template <class LA, class LB, class EPI, bool A_KC, bool B_KC, int WM>
__global__ __launch_bounds__(128 * WM, WM == 2 ? 2 : 1) void gemm_bf16_glds_kernel(LA la_, LB lb_, EPI epi_, int M,
                                                                                   int N, int K, int tilesM,
                                                                                   int tilesN, int splits,
                                                                                   int kchunk) {
  constexpr int BM = 64 * WM, NW = 2 * WM;
  constexpr int PA = BM / 8 / NW, PB = 16 / NW;  // 1-KiB pieces per wave per K tile
  constexpr int SA = BM * 128, STAGE = SA + 16384;
  constexpr int NS = WM == 2 ? 2 : 3;  // LDS stages: the 256-row tile keeps two K tiles in flight
  static_assert(WM == 2 || A_KC, "256-row tiles need a K-contiguous A image");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];  // [stage][A image | B image]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), wm = wv >> 1, wn = wv & 1;  // wave-uniform (SGPR)
  // Workgroups reach the XCDs round-robin in FLAT dispatch order (x fastest), so the remap runs
  // over the flattened (tile, batch*split) id: each XCD gets a contiguous run of work items,
  // tile-minor, i.e. whole splits — the K-chunk panels of one split are then fetched into one
  // L2 and shared by its tiles. (Remapping blockIdx.x alone scattered every split's tiles over
  // all 8 XCDs: split-K weight gradients read ~3x their operand bytes from HBM.)
  const int tiles = tilesM * tilesN;
  const int flat = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int zs = flat / tiles, lin = flat - zs * tiles;
  // Group the smaller tile dimension innermost: the workgroups an XCD runs together then share
  // the panel of the larger operand through its L2 (tm-major when tilesM >= tilesN). For the
  // LiDAR patch-embed weight gradient (3 x 145 tiles, B = 1.34 GB) tm-major re-read B 3 times.
  const bool tmin = tilesN > tilesM;
  const int tm = tmin ? lin % tilesM : lin / tilesN, tn = tmin ? lin / tilesM : lin - (lin / tilesN) * tilesN;
  const int z = zs / splits, split = zs - z * splits;
  const LA la = la_.bind(z);
  const LB lb = lb_.bind(z);
  const EPI epi = epi_.bind(z);
  const int m0 = tm * BM, n0 = tn * GBN;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nk = (kend - kbeg + GBK16 - 1) / GBK16;

  // Fast path: per-lane source state computed once (k-invariant), a uniform per-tile advance
  // (loader::fast_src). Generic gather when the loader declines and for a partial K tile.
  typename LA::Pre preA[PA];
  typename LB::Pre preB[PB];
  const bool fastA = la.fast_ok(A_KC), fastB = lb.fast_ok(B_KC);
#pragma unroll
  for (int i = 0; i < PA; ++i) preA[i] = la.pre(A_KC, wv * PA + i, lane, m0);
#pragma unroll
  for (int i = 0; i < PB; ++i) preB[i] = lb.pre(B_KC, wv * PB + i, lane, n0);
  auto issue = [&](int stage, int k0) {
    const bool full = k0 + GBK16 <= kend;
    glds_operand<PA>(la, z, A_KC, smem + stage * STAGE, wv, lane, m0, k0, kend, fastA && full, preA);
    glds_operand<PB>(lb, z, B_KC, smem + stage * STAGE + SA, wv, lane, n0, k0, kend, fastB && full, preB);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  f32x16 accb;
#pragma unroll
  for (int r = 0; r < 16; ++r) accb[r] = 0.f;
  bool dob = false;
  bf16x8 ones;
  if constexpr (BiasOnes<EPI>::v) {
    static_assert(!A_KC, "row sums of A need the MN-contiguous A image");
    dob = epi.bslab != nullptr && tn == 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
  }

  if (nk > 0) issue(0, kbeg);
  if constexpr (NS == 3) {
    if (nk > 1) issue(1, kbeg + GBK16);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = NS == 2 ? (kt & 1) : kt % 3;
    if constexpr (NS == 2) {
      if (kt + 1 < nk) {
        issue(cur ^ 1, kbeg + (kt + 1) * GBK16);
        // this tile's PA + PB pieces have landed (the next tile's stay in flight)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {  // 6 pieces per tile per wave; tiles kt+1 and kt+2 stay in flight
      if (kt + 2 < nk) {
        issue((kt + 2) % 3, kbeg + (kt + 2) * GBK16);
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      } else if (kt + 1 < nk) {
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __builtin_amdgcn_s_barrier();  // ... for every wave's pieces
    const char* ia = smem + cur * STAGE;
    const char* ib = ia + SA;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int rb0 = wm * 64 + 32 * i;
        fa[i] = A_KC ? frag_kc(ia, rb0 + (lane & 31), 2 * t + (lane >> 5)) : frag_mn(ia, 16 * t, rb0, lane);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cb0 = wn * 64 + 32 * j;
        fb[j] = B_KC ? frag_kc(ib, cb0 + (lane & 31), 2 * t + (lane >> 5)) : frag_mn(ib, 16 * t, cb0, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if constexpr (BiasOnes<EPI>::v) {
        if (dob) {  // wave (wm, wn) sums A rows wm*64 + 32*wn .. +31 (one extra MFMA per 4)
          if (wn == 0) accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], ones, accb, 0, 0, 0);
          else accb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], ones, accb, 0, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // my reads of this stage are done
    __builtin_amdgcn_s_barrier();                         // ... everyone's, before it is refilled
  }
  if constexpr (BiasOnes<EPI>::v) {
    if (dob && (lane & 31) == 0) {  // every column of accb holds the row sum; lanes 0 / 32 keep rows
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + 32 * wn + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < M) epi.bslab[(long)split * M + m] = accb[r];
      }
    }
  }
  epilogue_tile((float*)smem + wv * (32 * EP_LD), acc, epi, z, split, m0 + wm * 64, n0 + wn * 64, M, N, lane);
}

// ----------------------------------------------------------------------------- launcher
// dtype_bf16: which kernel. batch: number of z. splits: split-K factor (kchunk multiple
// of the K tile). Grid: x = tiles (XCD-remapped), y = batch * splits.
template <bool A_KC, bool B_KC, class LA, class LB, class EPI>
int launch_gemm(bool bf16_path, const LA& la, const LB& lb, const EPI& epi, int M, int N, int K, int batch,
                int splits, hipStream_t st) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  const int tilesM = ivit_cdiv(M, GBM), tilesN = ivit_cdiv(N, GBN);
  const int bk = bf16_path ? GBK16 : GBK32;
  if (splits < 1) splits = 1;
  int kchunk = ivit_cdiv(ivit_cdiv(K, splits), bk) * bk;
  if (kchunk <= 0) kchunk = bk;
  dim3 grid(tilesM * tilesN, batch * splits);
  if constexpr (BiasOnes<EPI>::v) {  // fused row sums exist only in the LDS-DMA kernel
    if (epi.bslab && !(bf16_path && LA::kGlds && LB::kGlds)) return IVIT_ERR_UNSUPPORTED;
  }
  if (bf16_path) {
    if constexpr (LA::kGlds && LB::kGlds) {
      // (a 256-row tile kernel, one workgroup per CU, was faster on 4096^3 only — 160 -> 140 us —
      // and slower or level on this model's shapes at one workgroup per CU; removed in round 6)
      hipLaunchKernelGGL((gemm_bf16_glds_kernel<LA, LB, EPI, A_KC, B_KC, 2>), grid, dim3(256), 0, st, la, lb, epi, M,
                         N, K, tilesM, tilesN, splits, kchunk);
    } else
      hipLaunchKernelGGL((gemm_bf16_kernel<LA, LB, EPI, A_KC, B_KC>), grid, dim3(256), 0, st, la, lb, epi, M, N, K,
                         tilesM, tilesN, splits, kchunk);
  } else
    hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, EPI, A_KC, B_KC>), grid, dim3(256), 0, st, la, lb, epi, M, N, K,
                       tilesM, tilesN, splits, kchunk);
  return 0;
}

}  // namespace ivit
