"""Isolated timing of one ViT block's four weight gradients (M = 36 008 tokens, bf16): the grouped
launch (ivit_vit_block_wgrad) vs the four split-K engine GEMMs (ivit_linear_wgrad), HIP events.

    python tools/wgrad_bench.py [--M 36008] [--iters 20]
"""
import argparse
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "visiontransformer-intention-prediction_amd"))


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    # anatomy: build libraries with -DIVIT_WB_ANATOMY=1 / 2 (tools/ab_build.sh) and run this under
    # tools/gpu_ab_libs.sh
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=36008)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import ops
    from _lib import BF16
    D, Hd, M = 384, 1536, a.M
    g = torch.Generator(device="cuda").manual_seed(0)
    mk = lambda c: torch.randn(M, c, device="cuda", generator=g).to(torch.bfloat16)
    t = [mk(D), mk(Hd), mk(Hd), mk(D), mk(D), mk(D), mk(3 * D), mk(D)]
    flops = 2.0 * M * (D * Hd * 2 + D * D + 3 * D * D)
    grouped = timeit(lambda: ops.vit_block_wgrad(*t), a.iters)
    sep = timeit(lambda: [ops.linear_wgrad(t[2 * q], t[2 * q + 1], BF16) for q in range(4)], a.iters)
    each = [timeit(lambda q=q: ops.linear_wgrad(t[2 * q], t[2 * q + 1], BF16), a.iters) for q in range(4)]
    print(f"M={M}: grouped {grouped:.1f} us ({flops / grouped / 1e6:.0f} TF/s), four engine GEMMs {sep:.1f} us "
          f"({flops / sep / 1e6:.0f} TF/s); each {[round(x, 1) for x in each]} us")


if __name__ == "__main__":
    main()
