"""One pass of each row-panel kernel of a bf16 ViT block at the bench shape (M = 8 x 4501, D = 384,
MLP 1536) for counter collection (tools/gpu_pmc_sq.sh TAG tools/wide_once.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "visiontransformer-intention-prediction_amd"))
import torch  # noqa: E402

import ops  # noqa: E402
from _lib import ACT_GELU  # noqa: E402

torch.manual_seed(0)
M, D, F = 8 * 4501, 384, 1536
dev = "cuda"
bf = lambda *s: torch.randn(*s, device=dev).to(torch.bfloat16)
ln, h, dy = bf(M, D), bf(M, F), bf(M, D)
wqkv, w1, w2 = torch.randn(3 * D, D, device=dev) / 20, torch.randn(F, D, device=dev) / 20, torch.randn(D, F, device=dev) / 40
b3, b1 = torch.zeros(3 * D, device=dev), torch.zeros(F, device=dev)
x32, scale = torch.randn(M, D, device=dev), torch.ones(8, device=dev)
g, beta = torch.ones(D, device=dev), torch.zeros(D, device=dev)
a = bf(M, F)
for _ in range(3):
    ops.panel_fwd(ln, wqkv, b3, qcols=D, qscale=ops.Q2_SCALE)
    ops.panel_fwd(ln, w1, b1, act=ACT_GELU, want_pre=True)
    ops.panel_dgrad_gelu(dy, w2, h)
    ops.linear_resid_ln_fwd(a, w2, torch.zeros(D, device=dev), x32, scale, 4501, g, beta, 1e-6)
torch.cuda.synchronize()
