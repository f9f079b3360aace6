// LDS-DMA ingest probe: how many bytes per clock can one CU take in by global_load_lds_dwordx4
// (1 KiB per wave-instruction), by waves per workgroup, pieces in flight per wave and source
// footprint (L2-resident vs streamed from HBM). One workgroup per CU (160 KiB LDS declared).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/dma_probe.hip -o tools/libdma_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int DEPTH>
__global__ __launch_bounds__(1024, 1) void dma_probe_kernel(const char* __restrict__ src, long span, int iters,
                                                           int* sink) {
  __shared__ __attribute__((aligned(16))) char smem[160 * 1024 - 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const unsigned ldsw = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)(smem + (wv % 16) * 8192);
  long off = ((long)blockIdx.x * nw + wv) * 65536;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const char* p = src + (off + (long)d * 1024) % span + lane * 16;
      const unsigned a = __builtin_amdgcn_readfirstlane(ldsw + (d & 7) * 1024);
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(p), "s"(a) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    off += (long)DEPTH * 1024 * 257;
  }
  if (threadIdx.x == 0 && iters < 0) sink[0] = smem[0];
}

// The same stream into VGPRs (global_load_dwordx4, 16 B per lane, DEPTH loads in flight per wave):
// the path the row-panel kernels' weight fragments take. The loaded words are folded into one
// value so the loads stay live.
template <int DEPTH>
__global__ __launch_bounds__(1024, 1) void vgpr_probe_kernel(const char* __restrict__ src, long span, int iters,
                                                            int* sink) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  long off = ((long)blockIdx.x * nw + wv) * 65536;
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint4 r[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) r[d] = *(const uint4*)(src + (off + (long)d * 1024) % span + lane * 16);
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) acc ^= r[d].x ^ r[d].w;
    off += (long)DEPTH * 1024 * 257;
  }
  if (acc == 0x12345678u && iters < 0) sink[0] = (int)acc;
}

extern "C" int vgpr_probe(const void* src, long span, int wgs, int waves, int depth, int iters, int* sink,
                          void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(wgs), b(64 * waves);
  switch (depth) {
    case 2: hipLaunchKernelGGL(vgpr_probe_kernel<2>, g, b, 0, st, (const char*)src, span, iters, sink); break;
    case 4: hipLaunchKernelGGL(vgpr_probe_kernel<4>, g, b, 0, st, (const char*)src, span, iters, sink); break;
    case 8: hipLaunchKernelGGL(vgpr_probe_kernel<8>, g, b, 0, st, (const char*)src, span, iters, sink); break;
    case 16: hipLaunchKernelGGL(vgpr_probe_kernel<16>, g, b, 0, st, (const char*)src, span, iters, sink); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int dma_probe(const void* src, long span, int wgs, int waves, int depth, int iters, int* sink, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(wgs), b(64 * waves);
  switch (depth) {
    case 1: hipLaunchKernelGGL(dma_probe_kernel<1>, g, b, 0, st, (const char*)src, span, iters, sink); break;
    case 2: hipLaunchKernelGGL(dma_probe_kernel<2>, g, b, 0, st, (const char*)src, span, iters, sink); break;
    case 4: hipLaunchKernelGGL(dma_probe_kernel<4>, g, b, 0, st, (const char*)src, span, iters, sink); break;
    case 8: hipLaunchKernelGGL(dma_probe_kernel<8>, g, b, 0, st, (const char*)src, span, iters, sink); break;
    case 16: hipLaunchKernelGGL(dma_probe_kernel<16>, g, b, 0, st, (const char*)src, span, iters, sink); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}
