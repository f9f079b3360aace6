"""Run the bench-shape attention fwd (+ bwd unless FWD_ONLY=1) a few times (rocprofv3 PMC passes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "visiontransformer-intention-prediction_amd"))
import torch
import ops
from _lib import BF16

B, N, H = 8, 4501, 6
torch.manual_seed(0)
qkv = torch.randn(B * N, 3 * H * 64, device="cuda").to(torch.bfloat16)
dout = torch.randn(B * N, H * 64, device="cuda").to(torch.bfloat16)
for _ in range(3):
    o, lse = ops.attn_fwd(qkv, B, N, H, BF16)
    if os.environ.get("FWD_ONLY") != "1":
        ops.attn_bwd(qkv, o, dout, lse, B, N, H, BF16)
torch.cuda.synchronize()
print("ok")
