"""Micro-benchmark: attention kernels at the bench shape (B=8, N=4501, H=6), variants A/B in one process."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "visiontransformer-intention-prediction_amd"))
import torch
import ops
from _lib import BF16

B, N, H = 8, 4501, 6
torch.manual_seed(0)
qkv = torch.randn(B * N, 3 * H * 64, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * N, H * 64, device="cuda").to(torch.bfloat16)
fl = 4.0 * B * H * N * N * 64


def timeit(fn, it=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it


ref = None
for rnd in range(2):
    for v in sys.argv[1:] or ["1", "2"]:
        os.environ["IVIT_ATTN_FWD_VARIANT"] = v
        o, lse = ops.attn_fwd(qkv, B, N, H, BF16)
        if ref is None:
            ref = o.float()
        err = float((o.float() - ref).abs().max())
        ms = timeit(lambda: ops.attn_fwd(qkv, B, N, H, BF16))
        print(f"fwd variant {v}: {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s  max|diff vs v{sys.argv[1] if len(sys.argv) > 1 else 1}|={err:.3g}")
os.environ.pop("IVIT_ATTN_FWD_VARIANT")
o, lse = ops.attn_fwd(qkv, B, N, H, BF16)
dref = None
for rnd in range(2):
    for bv in os.environ.get("BWD_VARIANTS", "2,3").split(","):
        os.environ["IVIT_ATTN_DKV_VARIANT"] = bv
        d = ops.attn_bwd(qkv, o, dout, lse, B, N, H, BF16)
        if dref is None:
            dref = d.float()
        err = float((d.float() - dref).abs().max() / dref.abs().max())
        ms = timeit(lambda: ops.attn_bwd(qkv, o, dout, lse, B, N, H, BF16))
        print(f"bwd variant {bv} (rows+dq+dkv): {ms:.3f} ms  {2.5 * fl / ms / 1e9:.1f} TF/s algorithmic  rel diff vs first={err:.3g}")
