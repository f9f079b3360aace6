"""qkv-shape forward GEMM a few times (for rocprofv3 PMC passes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "visiontransformer-intention-prediction_amd"))
import torch
import ops
from _lib import BF16
M = 8 * 4501
x = (torch.rand(M, 384, device="cuda") * 2 - 1).to(torch.bfloat16)
w = (torch.rand(1152, 384, device="cuda") * 2 - 1).to(torch.bfloat16)
b = torch.zeros(1152, device="cuda")
x4 = (torch.rand(4096, 4096, device="cuda") * 2 - 1).to(torch.bfloat16)
w4 = (torch.rand(4096, 4096, device="cuda") * 2 - 1).to(torch.bfloat16)
b4 = torch.zeros(4096, device="cuda")
for _ in range(5):
    ops.linear_fwd(x, w, b, BF16)
    ops.linear_fwd(x4, w4, b4, BF16)
torch.cuda.synchronize()
print("ok")
