"""Attention forward anatomy at the bench shape: product vs no-DMA (stale stages) vs DMA skeleton
(IVIT_ATTN_AN builds).   python tools/attn_anat.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "visiontransformer-intention-prediction_amd"))
import torch  # noqa: E402

import ops  # noqa: E402

B, H, N = 8, 6, 4501
torch.manual_seed(0)
qkv = torch.randn(B * N, 3 * H * 64, device="cuda").to(torch.bfloat16)
qkv[:, : H * 64] = (qkv[:, : H * 64].float() * ops.Q2_SCALE).to(torch.bfloat16)
fl = 4.0 * B * H * N * N * 64


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for an in ("0", "1", "2", "0"):
    os.environ["IVIT_ATTN_AN"] = an
    ms = timeit(lambda: ops.attn_fwd_q2(qkv, B, N, H))
    print(f"fwd IVIT_ATTN_AN={an}: {ms:.4f} ms  {fl / ms / 1e9:.1f} TF/s", flush=True)
