"""Run the bench-shape q2 attention fwd (+ bwd unless FWD_ONLY=1) a few times (rocprofv3 passes)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "visiontransformer-intention-prediction_amd"))
import torch  # noqa: E402
import ops  # noqa: E402

B, N, H = 8, int(os.environ.get("ATTN_N", "4501")), 6
torch.manual_seed(0)
qkv = torch.randn(B * N, 3 * H * 64, device="cuda").to(torch.bfloat16)
qkv[:, : H * 64] = (qkv[:, : H * 64].float() * ops.Q2_SCALE).to(torch.bfloat16)
dout = torch.randn(B * N, H * 64, device="cuda").to(torch.bfloat16)
for _ in range(3):
    o, lse = ops.attn_fwd_q2(qkv, B, N, H)
    if os.environ.get("FWD_ONLY") != "1":
        ops.attn_bwd_q2(qkv, o, dout, lse, B, N, H)
torch.cuda.synchronize()
print("ok")
