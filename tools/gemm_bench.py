"""Micro-benchmark: the ViT block GEMMs at the bench shape (M = 8 x 4501 tokens) through the
C-ABI (fwd / dgrad / wgrad), plus a square 4096^3 calibration shape. Prints TF/s per shape."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "visiontransformer-intention-prediction_amd"))
import torch

import ops
from _lib import ACT_GELU, ACT_NONE, BF16

torch.manual_seed(0)
M = 8 * 4501


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


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


rows = []
VARIANTS = os.environ.get("GEMM_VARIANTS", "").split(",") if os.environ.get("GEMM_VARIANTS") else [None]
for var in VARIANTS:
  if var is not None:
    os.environ["IVIT_GEMM_PERSIST"] = var
  for name, m, n, k, act in [("qkv", M, 1152, 384, ACT_NONE), ("fc1+gelu", M, 1536, 384, ACT_GELU),
                             ("proj", M, 384, 384, ACT_NONE), ("fc2", M, 384, 1536, ACT_NONE),
                             ("sq4096", 4096, 4096, 4096, ACT_NONE)]:
      x, w = rnd(m, k), rnd(n, k)
      b = torch.zeros(n, device="cuda")
      fl = 2.0 * m * n * k
      ms = timeit(lambda: ops.linear_fwd(x, w, b, BF16, act=act))
      rows.append((f"fwd   {name} p{var}", m, n, k, ms, fl))
      dy = rnd(m, n)
      ms = timeit(lambda: ops.linear_dgrad(dy, w, BF16, torch.bfloat16))
      rows.append((f"dgrad {name} p{var}", m, k, n, ms, fl))
      ms = timeit(lambda: ops.linear_wgrad(dy, x, BF16, want_bias=True))
      rows.append((f"wgrad {name} p{var}", n, k, m, ms, fl))
if "torch" in sys.argv[1:]:  # vendor-library yardstick (hipBLASLt via torch.mm), same shapes, no epilogue
    for name, m, n, k in [("qkv", M, 1152, 384), ("fc1", M, 1536, 384), ("proj", M, 384, 384), ("fc2", M, 384, 1536),
                          ("sq4096", 4096, 4096, 4096)]:
        x, w, dy = rnd(m, k), rnd(n, k), rnd(m, n)
        fl = 2.0 * m * n * k
        rows.append((f"torch fwd   {name}", m, n, k, timeit(lambda: torch.mm(x, w.t())), fl))
        rows.append((f"torch dgrad {name}", m, k, n, timeit(lambda: torch.mm(dy, w)), fl))
        rows.append((f"torch wgrad {name}", n, k, m, timeit(lambda: torch.mm(dy.t(), x)), fl))
if len(sys.argv) > 1 and sys.argv[1] == "resid":
    x, w = rnd(M, 1536), rnd(384, 1536)
    r = torch.randn(M, 384, device="cuda")
    ms = timeit(lambda: ops.linear_fwd(x, w, torch.zeros(384, device="cuda"), BF16, resid=r))
    rows.append(("fwd   fc2+resid", M, 384, 1536, ms, 2.0 * M * 384 * 1536))
for name, m, n, k, ms, fl in rows:
    print(f"{name:22s} M={m:6d} N={n:5d} K={k:6d}  {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s")
