"""Wave-quantisation probe of the attention kernels: per-kernel execution time (ivit_ktime_*) at
B=8, H=6 for several N, with the workgroup rounds each launch needs (blocks of 128 rows,
two workgroups per CU). Time per N^2 flat across N => no tail loss; rising with the fractional
part of the rounds => the last partial round costs a full one.   python tools/attn_tail.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "visiontransformer-intention-prediction_amd"))
import torch  # noqa: E402

import ops  # noqa: E402

B, H = 8, 6
torch.manual_seed(0)
for N in [int(v) for v in (sys.argv[1:] or "4096 4097 4224 4352 4480 4501 4608".split())]:
    qkv = torch.randn(B * N, 3 * H * 64, device="cuda").to(torch.bfloat16)
    qkv[:, : H * 64] = (qkv[:, : H * 64].float() * ops.Q2_SCALE).to(torch.bfloat16)
    dout = torch.randn(B * N, H * 64, device="cuda").to(torch.bfloat16)
    o, lse = ops.attn_fwd_q2(qkv, B, N, H)
    ops.attn_bwd_q2(qkv, o, dout, lse, B, N, H)
    torch.cuda.synchronize()
    ops.ktime_arm(True)
    for _ in range(10):
        ops.attn_fwd_q2(qkv, B, N, H)
        ops.attn_bwd_q2(qkv, o, dout, lse, B, N, H)
    torch.cuda.synchronize()
    ops.ktime_arm(False)
    blocks = (N + 127) // 128
    rounds = B * H * blocks / 512
    res = []
    for tag, name in ((ops.KT_ATTN_FWD, "fwd"), (ops.KT_ATTN_BWD_DQ, "dq"), (ops.KT_ATTN_BWD_DKV, "dkv")):
        iv = ops.ktime_read(tag)
        ms = sum(b - a for a, b in iv) / len(iv)
        res.append(f"{name} {ms * 1e3:7.1f} us ({ms * 1e3 / (N / 4501) ** 2:7.1f} at N=4501 scale)")
    print(f"N={N:5d} blocks={blocks} rounds={rounds:.3f}  " + "  ".join(res), flush=True)
