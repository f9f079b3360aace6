"""LDS-DMA ingest rate per CU (tools/dma_probe.hip): GB/s per CU and B/clk at 2.4 GHz by waves per
workgroup, pieces in flight per wave and source footprint.

    python tools/dma_probe.py [dma|vgpr]   (vgpr: the same stream by global_load_dwordx4 into VGPRs)
"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libdma_probe.so"))
    lib.dma_probe.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_void_p]
    lib.vgpr_probe.argtypes = lib.dma_probe.argtypes
    big = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    mode = sys.argv[1] if len(sys.argv) > 1 else "dma"
    probe = lib.vgpr_probe if mode == "vgpr" else lib.dma_probe
    for span_name, span in (("L2 2MiB", 2 << 20), ("MALL 64MiB", 64 << 20), ("HBM 1GiB", 1 << 30)):
        for waves in (1, 2, 4, 8, 16):
            for depth in (2, 4, 8, 16):
                iters = max(4, 4096 // (waves * depth))
                fn = lambda: probe(big.data_ptr(), span, 256, waves, depth, iters, sink.data_ptr(), st)
                fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    fn()
                e.record()
                torch.cuda.synchronize()
                t = s.elapsed_time(e) / 5 * 1e-3
                by = 256.0 * waves * depth * iters * 1024
                per_cu = by / 256 / t / 1e9
                print(f"{span_name:11s} waves {waves:2d} depth {depth:2d}: chip {by / t / 1e12:6.2f} TB/s  per CU "
                      f"{per_cu:6.1f} GB/s = {per_cu / 2.4:5.1f} B/clk", flush=True)


if __name__ == "__main__":
    main()
