// Shared device/host helpers for libivit_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/ivit.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define IVIT_DEV __device__ __forceinline__

// ---------------------------------------------------------------- error plumbing
void ivit_set_error(const char* fmt, ...);
#define IVIT_CHECK_ARG(cond, ...)            \
  do {                                       \
    if (!(cond)) {                           \
      ivit_set_error(__VA_ARGS__);           \
      return IVIT_ERR_ARG;                   \
    }                                        \
  } while (0)
#define IVIT_LAUNCH_CHECK()                                                  \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess) {                                                  \
      ivit_set_error("%s: %s", __func__, hipGetErrorString(e_));             \
      return (int)e_;                                                        \
    }                                                                        \
  } while (0)

static inline hipStream_t ivit_stream(void* s) { return (hipStream_t)s; }

// Tuning knobs (ivit_set_knob / ivit_get_knob, ivit.h): process-wide ints read by the launchers.
int ivit_knob(int knob);
static inline int ivit_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------- LDS DMA
// global_load_lds_dword{,x4}: each lane's BYTES land at lds + lane * BYTES (lds wave-uniform,
// it goes to M0). Issued as inline asm, not __builtin_amdgcn_global_load_lds: with the builtin
// the compiler's waitcnt pass assumes every later ds_read_b64_tr_b16 may alias an outstanding
// DMA and puts s_waitcnt vmcnt(0) before it, which drains the NEXT tile's prefetch in every
// K step of the MN-contiguous GEMMs and of the attention kernels. Every kernel here retires its
// DMAs with explicit counted vmcnt waits + s_barrier, so the compiler needs no view of them.
// M0 is written only here (tools/check_m0.py verifies the emitted code); s_nop 0 covers the
// M0-write -> LDS-DMA hazard.
template <int BYTES>
IVIT_DEV void glds(const void* src, void* lds) {
  static_assert(BYTES == 16 || BYTES == 4, "global_load_lds: 4 or 16 bytes per lane");
  const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  if constexpr (BYTES == 16)
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(a) : "memory");
  else
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(a) : "memory");
}

// ---------------------------------------------------------------- numerics
IVIT_DEV float bf2f(bf16 x) { return (float)x; }
IVIT_DEV bf16 f2bf(float x) { return (bf16)x; }

template <typename T> IVIT_DEV T from_f32(float v);
template <> IVIT_DEV float from_f32<float>(float v) { return v; }
template <> IVIT_DEV bf16 from_f32<bf16>(float v) { return (bf16)v; }
template <typename T> IVIT_DEV float to_f32(T v) { return (float)v; }

IVIT_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
IVIT_DEV float gelu_erf_grad(float x) {
  // d/dx [0.5 x (1 + erf(x/sqrt2))] = 0.5(1+erf(x/sqrt2)) + x * exp(-x^2/2)/sqrt(2 pi)
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

// 8 bf16 <-> uint4 reinterpretation
union Pack8 {
  uint4 u;
  bf16x8 v;
  bf16 h[8];
};
union Pack4 {
  uint2 u;
  bf16x4 v;
  bf16 h[4];
};

// Fast GELU / GELU' for bf16 outputs: erf by Abramowitz-Stegun 7.1.26 (|err| <= 1.5e-7, far below
// bf16 resolution); erf(x/sqrt2) and the Gaussian density share one exp(-x^2/2).
IVIT_DEV float erf_as(float x, float e /* = exp(-x*x) */) {
  const float a = fabsf(x);
  // raw v_rcp_f32 (1 ulp): __frcp_rn compiles to the 8-instruction correctly-rounded division
  // sequence, the largest part of this epilogue function; the polynomial's own error is 1.5e-7
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * a);
  const float p = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float r = 1.0f - p * e;
  return x < 0.f ? -r : r;
}
IVIT_DEV float gelu_fast(float x) {
  const float e = __expf(-0.5f * x * x);
  return 0.5f * x * (1.0f + erf_as(x * 0.70710678118654752f, e));
}
IVIT_DEV float gelu_grad_fast(float x) {
  const float e = __expf(-0.5f * x * x);
  return 0.5f * (1.0f + erf_as(x * 0.70710678118654752f, e)) + x * 0.39894228040143268f * e;
}
// gelu(x) and gelu'(x) together (one exp, one erf): y = x c, dy = c + x phi(x), c = Phi(x)
IVIT_DEV void gelu_fast2(float x, float& y, float& dy) {
  const float e = __expf(-0.5f * x * x);
  const float c = 0.5f * (1.0f + erf_as(x * 0.70710678118654752f, e));
  y = x * c;
  dy = c + x * 0.39894228040143268f * e;
}
template <typename O> IVIT_DEV float gelu_t(float x) { return sizeof(O) == 2 ? gelu_fast(x) : gelu_erf(x); }
template <typename O> IVIT_DEV float gelu_grad_t(float x) {
  return sizeof(O) == 2 ? gelu_grad_fast(x) : gelu_erf_grad(x);
}

IVIT_DEV bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static inline bool hal16(const void* p) { return ((uintptr_t)p & 15) == 0; }  // host side

// ---------------------------------------------------------------- diagnostic stamps
// (ivit_debug_stamps) Kernels built with a stamping flag record clocks per workgroup; lane 0 of
// wave 0 writes them with an ordinary vector store into a buffer no other code reads.
typedef unsigned long long u64;
IVIT_DEV u64 clk_now() { return __builtin_amdgcn_s_memtime(); }
IVIT_DEV u64 rclk_now() { return __builtin_amdgcn_s_memrealtime(); }
IVIT_DEV u64 hw_ids() {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID, 32 bits
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
  return (u64)hw | ((u64)xcc << 32);
}
struct Stamps {
  u64 t0, t1, t2, r0;
  IVIT_DEV void begin() { t0 = clk_now(); r0 = rclk_now(); t1 = t2 = 0; }
  IVIT_DEV void end(u64* buf) {
    const u64 t3 = clk_now(), r3 = rclk_now();
    if (threadIdx.x == 0) {
      u64* o = buf + 8L * blockIdx.x;
      o[0] = t0; o[1] = t1; o[2] = t2; o[3] = t3; o[4] = r0; o[5] = r3; o[6] = hw_ids(); o[7] = 0;
    }
  }
};
u64* ivit_stamp_buffer(long blocks);  // host: the armed buffer if it holds `blocks` records, else null

// store 8 consecutive values (vectorised when aligned and complete)
template <typename O>
IVIT_DEV void store8(O* p, const float (&x)[8], int nv) {
  if (nv >= 8 && al16(p)) {
    if constexpr (sizeof(O) == 2) {
      Pack8 q;
#pragma unroll
      for (int k = 0; k < 8; ++k) q.h[k] = (bf16)x[k];
      *(uint4*)p = q.u;
    } else {
      *(float4*)p = make_float4(x[0], x[1], x[2], x[3]);
      *(float4*)(p + 4) = make_float4(x[4], x[5], x[6], x[7]);
    }
  } else {
    for (int k = 0; k < nv && k < 8; ++k) p[k] = from_f32<O>(x[k]);
  }
}
template <typename T>
IVIT_DEV void load8f(const T* p, float (&x)[8], int nv) {
  if (nv >= 8 && al16(p)) {
    if constexpr (sizeof(T) == 2) {
      Pack8 q;
      q.u = *(const uint4*)p;
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (float)q.h[k];
    } else {
      const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
      x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = k < nv ? to_f32(p[k]) : 0.f;
  }
}

// 8 consecutive elements of a bf16 / f32 buffer selected by a runtime dtype code (16-B aligned when
// the element offset is a multiple of 8 and the base is 16-B aligned)
IVIT_DEV void ld8dt(const void* p, int dt, long i, float (&x)[8]) {
  if (dt == IVIT_BF16) load8f((const bf16*)p + i, x, 8);
  else load8f((const float*)p + i, x, 8);
}
IVIT_DEV void st8dt(void* p, int dt, long i, const float (&x)[8]) {
  if (dt == IVIT_BF16) store8((bf16*)p + i, x, 8);
  else store8((float*)p + i, x, 8);
}

// Raw v_exp_f32 (2^x; results below 2^-126 flush to 0 — harmless for softmax weights).
// exp2f() adds a denormal range reduction: 4-5 VALU ops per call.
IVIT_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Combine a value with its lane^32 partner without LDS: v_permlane32_swap exchanges the
// wave halves, so max/sum of the pair is symmetric (cdna_hip_programming.md T12).
IVIT_DEV float half_swap_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
IVIT_DEV float half_swap_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

IVIT_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
IVIT_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}


// Two f32 -> packed bf16 pair (round to nearest even): one v_cvt_pk_bf16_f32. (Element-wise
// casts assembled into a vector compiled to the same conversions plus and/shift/or re-packing.)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
IVIT_DEV unsigned pk_bf16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}
IVIT_DEV uint4 f32x8_to_bf16x8(float4 a, float4 b) {
  return make_uint4(pk_bf16(a.x, a.y), pk_bf16(a.z, a.w), pk_bf16(b.x, b.y), pk_bf16(b.z, b.w));
}

// Column reduction of per-block partial sums: out[c] (+)= sum_b part[b * pstride + c].
// 256 threads = 16 columns x 16 partial phases (phase ph sums rows ph, ph + 16, ...; the phases are
// then added in order), so long partial lists reduce in parallel; narrow 4-wave workgroups, many of
// them (C / 16), find room on CUs that the other ViT stream's kernels hold. Columns >= C0 go to
// out1[c - C0] (two outputs packed in one partial row, e.g. dgamma|dbeta).
namespace {
constexpr int CR_COLS = 16;
__global__ __launch_bounds__(256) void colreduce_kernel(const float* __restrict__ part, int nb, long pstride, int C,
                                                        float* out0, int C0, float* out1, int acc) {
  const int cl = threadIdx.x & (CR_COLS - 1), ph = threadIdx.x / CR_COLS;
  const int c = blockIdx.x * CR_COLS + cl;
  float s = 0.f;
  if (c < C) {
    // this phase's rows in batches of 16 loads in flight per lane (the reduce is latency-bound: a
    // serial tail of one load per add took ~19 L2 round trips at nb = 563), each batch summed in
    // row order, so the result is the plain sequential sum over the phase's rows
    for (int b0 = ph; b0 < nb; b0 += 256) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int b = b0 + 16 * i;
        v[i] = b < nb ? part[(long)b * pstride + c] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (b0 + 16 * i < nb) s += v[i];
    }
  }
  __shared__ float red[16][CR_COLS];
  red[ph][cl] = s;
  __syncthreads();
  if (ph == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    float* o = c < C0 ? (out0 ? out0 + c : nullptr) : (out1 ? out1 + (c - C0) : nullptr);
    if (o) *o = acc ? *o + t : t;
  }
}
inline void launch_colreduce(hipStream_t st, const float* part, int nb, long pstride, int C, float* out0, int C0,
                             float* out1, int acc) {
  hipLaunchKernelGGL(colreduce_kernel, dim3((C + CR_COLS - 1) / CR_COLS), dim3(256), 0, st, part, nb, pstride, C,
                     out0, C0, out1, acc);
}
}  // namespace

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks b and b+8 share an XCD under round-robin dispatch, so give each
// XCD group a contiguous range of logical tile ids (shared A/B panels hit one L2).
IVIT_DEV int xcd_remap(int orig, int nwg) {
  if (nwg < 16) return orig;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}
