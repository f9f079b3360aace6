import sys, math, torch
sys.path.insert(0, "visiontransformer-intention-prediction_amd")
import ops
from _lib import ACT_GELU, BF16
DEV="cuda"
for (M, N, K) in [(36008, 1152, 384), (300, 384, 128), (144*4, 384, 64), (144, 1152, 64)]:
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV)
    b = (0.1 * torch.randn(N, generator=g)).to(DEV)
    got, _ = ops.panel_fwd(x, w, b)
    ref = (x.float() @ w.to(torch.bfloat16).float().t() + b)
    err = (got.float() - ref).abs()
    print(M, N, K, "max", float(err.max()))
    for c in range(N // 192):
        e = err[:, c*192:(c+1)*192]
        rows = (e.max(1).values > 0.05).nonzero().flatten()
        print("  chunk", c, "max", round(float(e.max()), 4), "bad rows", rows.numel(), rows[:8].tolist(), "cols", (e.max(0).values > 0.05).nonzero().flatten()[:12].tolist())
