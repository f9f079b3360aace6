// Helpers of the row-panel MFMA kernels (patch_embed.hip, rowpanel.hip): a workgroup owns a panel
// of rows x ALL output columns; the shared operand (weights) is pre-packed in MFMA fragment order
// and loaded straight into VGPRs, the streamed operand goes to LDS by LDS-DMA. Every memory
// operation of the main loops is inline asm retired by counted vmcnt waits (the compiler's
// waitcnt pass cannot see the DMAs, and a compiler wait on a register load would drain the
// in-flight DMA: the counter retires in issue order). tools/asm_load_check.py verifies no
// instruction touches an asm-loaded register before its wait.
#pragma once
#include "ivit_common.h"

namespace ivit {
namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int NBW = 3;  // 16-column MFMA blocks per wave (48 columns)

// s_waitcnt vmcnt(n), n wave-uniform (the field is an immediate)
#define PANEL_VM(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
IVIT_DEV void wait_vm(int n) {
  switch (n) {
    PANEL_VM(1) PANEL_VM(2) PANEL_VM(3) PANEL_VM(4) PANEL_VM(5) PANEL_VM(6) PANEL_VM(7) PANEL_VM(8) PANEL_VM(9)
    PANEL_VM(10) PANEL_VM(11) PANEL_VM(12) PANEL_VM(13) PANEL_VM(14) PANEL_VM(15) PANEL_VM(16) PANEL_VM(17)
    PANEL_VM(18) PANEL_VM(19) PANEL_VM(20) PANEL_VM(21) PANEL_VM(22) PANEL_VM(23) PANEL_VM(24)
    PANEL_VM(25) PANEL_VM(26) PANEL_VM(27) PANEL_VM(28) PANEL_VM(29) PANEL_VM(30) PANEL_VM(31) PANEL_VM(32)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}
#undef PANEL_VM

// Workgroup barrier that also publishes this wave's LDS stores: a raw s_barrier does not wait for
// outstanding ds_write (the compiler inserts no lgkmcnt wait before it), so a partner wave could
// read the location before the store lands.
IVIT_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Wave-uniform 64-bit address -> SGPR pair (the saddr operand of the loads below).
IVIT_DEV const char* uniform_ptr(const void* p) {
  const unsigned long v = (unsigned long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (const char*)(((unsigned long)hi << 32) | lo);
}

// 16 B per lane from sbase + voff + OFF into VGPRs (saddr form: one VGPR of per-lane offset).
template <int OFF>
IVIT_DEV void gload_b128(u32x4& r, unsigned voff, const char* sbase) {
  static_assert(OFF >= 0 && OFF < 4096, "global offset field");
  asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3" : "=v"(r) : "v"(voff), "s"(sbase), "i"(OFF) : "memory");
}

// LDS-DMA, saddr form: lane's 16 B from sbase + voff land at lds + 16 * lane (lds wave-uniform
// -> M0). NT: non-temporal (a stream read once, e.g. the BEV raster).
template <bool NT = true>
IVIT_DEV void glds_s(unsigned voff, const char* sbase, void* lds) {
  const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  if constexpr (NT)
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2 nt" ::"v"(voff), "s"(a), "s"(sbase)
                 : "memory");
  else
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2" ::"v"(voff), "s"(a), "s"(sbase)
                 : "memory");
}

// LDS-DMA from a per-lane 64-bit address.
template <bool NT>
IVIT_DEV void glds_v(const void* src, void* lds) {
  const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  if constexpr (NT)
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(src), "s"(a) : "memory");
  else
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(a) : "memory");
}

// The 2*NBW weight-fragment registers of one K stage become visible to the compiler only here,
// after the counted wait that retired their loads.
IVIT_DEV void tie(u32x4 (&r)[2 * NBW]) {
  asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]));
}

// The wave's NBW 16-column fragments of 32-k step s of a packed weight (ivit_patch_weight_pack:
// wpack[s][nb][lane][8 bf16]): NBW contiguous KiB.
IVIT_DEV void load_wfrag(u32x4 (&r)[2 * NBW], int t, const char* sb, unsigned vb) {
  gload_b128<0>(r[t * NBW + 0], vb, sb);
  gload_b128<1024>(r[t * NBW + 1], vb, sb);
  gload_b128<2048>(r[t * NBW + 2], vb, sb);
}

}  // namespace
}  // namespace ivit
