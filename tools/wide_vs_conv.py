"""Token GEMMs of a ViT block (M = 36 008, bf16 in / bf16 out + bias) through the wide row-panel
kernel (ops.panel_fwd: 144-row x 192-column workgroups, two per CU) vs the 288 x 256 conv panel
kernel run as a 1 x 1 convolution (ops.conv_fwd with H = 1, W = M), HIP events, back to back.
Both epilogues here are the plain bias + bf16 store (act NONE).

    python tools/wide_vs_conv.py
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "visiontransformer-intention-prediction_amd"))


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    import ops
    from _lib import BF16
    dev = torch.device("cuda", 0)
    M = 36008
    for (K, N) in ((384, 1536), (384, 1152), (1536, 384), (384, 384)):
        x = (torch.randn(M, K, device=dev) * 0.5).bfloat16()
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev) * 0.1
        wc = ops.pack_conv(w.reshape(N, K, 1, 1), BF16)
        y1, _ = ops.panel_fwd(x, w, b)
        y2 = ops.conv_fwd(x, 1, 1, M, wc, b, BF16, torch.bfloat16)
        err = (y1.float() - y2.float()).abs().max().item()
        fl = 2.0 * M * N * K
        for rep in range(2):
            tw = timed(lambda: ops.panel_fwd(x, w, b))
            tc = timed(lambda: ops.conv_fwd(x, 1, 1, M, wc, b, BF16, torch.bfloat16))
            print(f"K={K:5d} N={N:5d}: wide {tw:7.1f} us ({fl / tw / 1e6:6.1f} TF/s)   conv 1x1 {tc:7.1f} us "
                  f"({fl / tc / 1e6:6.1f} TF/s)   max|diff| {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
