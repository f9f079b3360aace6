"""Micro-benchmark: residual GEMM + LayerNorm as two kernels (EpiResid GEMM + ln_fwd_vec_kernel)
vs the fused row-panel kernel (ivit_linear_resid_ln_fwd), at the ViT token shape M = 8 x 4501,
N = 384, K = 384 (proj) and 1536 (fc2)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "visiontransformer-intention-prediction_amd"))
import torch

import ops
from _lib import BF16

M, N = 8 * 4501, 384


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for K in (384, 1536):
    a = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    wb = w.to(torch.bfloat16)
    b, g, bt = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")
    r = torch.randn(M, N, device="cuda")
    s = torch.ones(8, device="cuda")

    def two():
        x, _ = ops.linear_fwd(a, wb, b, BF16, resid=r, row_scale=s, rps=4501)
        return ops.layernorm_fwd(x, g, bt, 1e-6, torch.bfloat16)

    def fused():
        return ops.linear_resid_ln_fwd(a, w, b, r, s, 4501, g, bt, 1e-6)
    t_g = timeit(lambda: ops.linear_fwd(a, wb, b, BF16, resid=r, row_scale=s, rps=4501))
    t2 = timeit(two)
    t1 = timeit(fused)
    fl = 2.0 * M * N * K
    print(f"K={K:5d}  GEMM+resid {t_g:6.1f} us   + LayerNorm {t2:6.1f} us   fused {t1:6.1f} us "
          f"({fl / t1 / 1e6:.0f} TF/s)", flush=True)

# backward form: dgrad G = dY @ W (K = 1536: fc1's dgrad; 1152: qkv's) + LayerNorm backward, with
# the residual-stream gradient dres added and the bf16 copy written (the in-step call shapes)
for K in (1536, 1152):
    dy = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = torch.randn(K, N, device="cuda") / K ** 0.5
    x = torch.randn(M, N, device="cuda")
    g = torch.ones(N, device="cuda") + 0.1 * torch.randn(N, device="cuda")
    mean, rstd = x.mean(1), 1.0 / (x.var(1, unbiased=False) + 1e-6).sqrt()
    dres = torch.randn(M, N, device="cuda")
    dx = torch.empty_like(dres)
    s = torch.ones(8, device="cuda")
    t = timeit(lambda: ops.linear_dgrad_ln_bwd(dy, w, x, g, mean, rstd, dres=dres, dx=dx, xs_dtype=torch.bfloat16,
                                               row_scale=s, rps=4501))
    fl = 2.0 * M * N * K
    print(f"bwd K={K:5d}  dgrad + LN bwd (+ colreduce) {t:6.1f} us ({fl / t / 1e6:.0f} TF/s)", flush=True)
