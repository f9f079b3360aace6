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
if os.environ.get("TORCH_SDPA", "1") == "1":  # vendor yardstick: torch SDPA (ROCm flash backend) on the same shape
    import torch.nn.functional as F
    q, k, v = (qkv.view(B, N, 3, H, 64)[:, :, i].transpose(1, 2).contiguous() for i in range(3))
    g = dout.view(B, N, H, 64).transpose(1, 2).contiguous()
    try:
        ms = timeit(lambda: F.scaled_dot_product_attention(q, k, v))
        print(f"torch sdpa fwd: {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s")
        qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
        out = F.scaled_dot_product_attention(qr, kr, vr)
        ms = timeit(lambda: torch.autograd.grad(out, (qr, kr, vr), g, retain_graph=True))
        print(f"torch sdpa bwd: {ms:.3f} ms  {2.5 * fl / ms / 1e9:.1f} TF/s algorithmic")
    except Exception as ex:  # noqa: BLE001
        print("torch sdpa unavailable:", type(ex).__name__, str(ex)[:200])
