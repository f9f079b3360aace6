"""Fusion-block convolution timings (B = 8, 50 x 90 map): forward and data gradient through the
288 x 256 panel kernel (conv_panel.hip) and the 128 x 128 engine (ivit_set_knob(IVIT_KNOB_CONV_PANEL, 0)), alternating
in one process; HIP events around 20 back-to-back launches.

    python tools/conv_bench.py [--panel-only]   (--panel-only: the fusion shapes on the panel kernels)
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
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    panel_only = "--panel-only" in sys.argv
    import ops
    from _lib import BF16, KNOB_CONV_PANEL, lib
    dev = torch.device("cuda", 0)
    B, H, W = 8, 50, 90
    M = B * H * W
    for (cin, cout, k) in ((384, 512, 3), (512, 512, 3), (384, 512, 1)):
        x = (torch.randn(M, cin, device=dev) * 0.5).bfloat16()
        dy = (torch.randn(M, cout, device=dev) * 0.5).bfloat16()
        w = torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5
        wp = ops.pack_conv(w, BF16)
        fl = 2.0 * M * cout * cin * k * k
        for rep in range(2):
            for mode in (("1",) if panel_only else ("1", "0")):
                lib.ivit_set_knob(KNOB_CONV_PANEL, int(mode))
                tf = timed(lambda: ops.conv_fwd(x, B, H, W, wp, None, BF16, torch.float32))
                td = timed(lambda: ops.conv_dgrad(dy, B, H, W, wp, BF16, torch.float32, w=w))
                tw = timed(lambda: ops.conv_wgrad(dy, x, B, H, W, cin, cout, k, BF16))
                name = "panel " if mode == "1" else "engine"
                print(f"{cin}->{cout} k{k} {name}: fwd {tf:7.1f} us ({fl / tf / 1e6:6.1f} TF/s)  "
                      f"dgrad(+pack) {td:7.1f} us ({fl / td / 1e6:6.1f} TF/s)  "
                      f"wgrad(+reduce) {tw:7.1f} us ({fl / tw / 1e6:6.1f} TF/s)", flush=True)
    lib.ivit_set_knob(KNOB_CONV_PANEL, 1)
    if panel_only:
        return
    # head conv data gradient (75 channels packed to 80): engine vs the panel kernel on rows zero-padded to 128
    cin, cw, cp, cq = 512, 75, 80, 128
    w = torch.randn(cw, cin, 3, 3, device=dev) / (cin * 9) ** 0.5
    wp = ops.pack_conv(w, BF16, cout_pad=cp)
    dy = torch.zeros(M, cq, device=dev)
    dy[:, :cw] = torch.randn(M, cw, device=dev)
    dy = dy.bfloat16()
    fl = 2.0 * M * cw * cin * 9
    for rep in range(2):
        te = timed(lambda: ops.conv_dgrad(dy, B, H, W, wp, BF16, torch.float32))
        tp = timed(lambda: ops.conv_dgrad(dy, B, H, W, wp, BF16, torch.float32, w=w, dy_zero_pad=True))
        print(f"head {cin}->{cw} k3 dgrad: engine {te:7.1f} us ({fl / te / 1e6:6.1f} TF/s)  "
              f"panel(pad {cq}, +pack) {tp:7.1f} us ({fl / tp / 1e6:6.1f} TF/s)", flush=True)
    # head forward and weight gradient: engine on 80 channels vs panel on 128
    x = (torch.randn(M, cin, device=dev) * 0.5).bfloat16()
    wq = ops.pack_conv(w, BF16, cout_pad=cq)
    bp, bq = torch.zeros(cp, device=dev), torch.zeros(cq, device=dev)
    for rep in range(2):
        fe = timed(lambda: ops.conv_fwd(x, B, H, W, wp, bp, BF16, torch.float32))
        fp = timed(lambda: ops.conv_fwd(x, B, H, W, wq, bq, BF16, torch.float32))
        we = timed(lambda: ops.conv_wgrad(dy, x, B, H, W, cin, cp, 3, BF16, want_bias=True))
        wq_ = timed(lambda: ops.conv_wgrad(dy, x, B, H, W, cin, cq, 3, BF16, want_bias=True))
        print(f"head {cin}->{cw} k3 fwd: engine(80) {fe:7.1f} us  panel(128) {fp:7.1f} us   "
              f"wgrad: engine(80) {we:7.1f} us  panel(128) {wq_:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
