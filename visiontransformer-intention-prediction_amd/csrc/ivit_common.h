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
static inline int ivit_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

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

IVIT_DEV uint4 f32x8_to_bf16x8(float4 a, float4 b) {
  Pack8 p;
  p.h[0] = f2bf(a.x); p.h[1] = f2bf(a.y); p.h[2] = f2bf(a.z); p.h[3] = f2bf(a.w);
  p.h[4] = f2bf(b.x); p.h[5] = f2bf(b.y); p.h[6] = f2bf(b.z); p.h[7] = f2bf(b.w);
  return p.u;
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks b and b+8 share an XCD under round-robin dispatch, so give each
// XCD group a contiguous range of logical tile ids (shared A/B panels hit one L2).
IVIT_DEV int xcd_remap(int orig, int nwg) {
  if (nwg < 16) return orig;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}
