"""Isolated timing of every token-GEMM kernel of one bf16 ViT block at the bench shape
(M = 8 x 4501 tokens, D = 384, MLP 1536) exactly as ops.ViTBlockFn launches them, with each
kernel's HBM floor (algorithmic bytes / 6.3 TB/s achievable) and MFMA floor (flops / 2516.6 TF/s).
python tools/block_bench.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "visiontransformer-intention-prediction_amd"))
import torch  # noqa: E402

import ops  # noqa: E402
from _lib import ACT_GELU, ACT_GELU_D, BF16  # noqa: E402

torch.manual_seed(0)
M, D, F = 8 * 4501, 384, 1536
dev = "cuda"


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


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


x32 = torch.randn(M, D, device=dev)
ln = bf(M, D)
wqkv, bqkv = torch.randn(3 * D, D, device=dev) / 20, torch.zeros(3 * D, device=dev)
wp, bp = torch.randn(D, D, device=dev) / 20, torch.zeros(D, device=dev)
w1, b1 = torch.randn(F, D, device=dev) / 20, torch.zeros(F, device=dev)
w2, b2 = torch.randn(D, F, device=dev) / 40, torch.zeros(D, device=dev)
g, beta = torch.ones(D, device=dev), torch.zeros(D, device=dev)
scale = torch.ones(8, device=dev)
mean, rstd = torch.zeros(M, device=dev), torch.ones(M, device=dev)
a_o = bf(M, D)
h, a = bf(M, F), bf(M, F)
dy = bf(M, D)
dh = bf(M, F)
dqkv = bf(M, 3 * D)
wb = {k: v.to(torch.bfloat16) for k, v in (("p", wp),)}

B2, F4 = 2, 4
rows = [
    # name, fn, bytes, flops
    ("fwd qkv (panel, Q prescaled)", lambda: ops.panel_fwd(ln, wqkv, bqkv, qcols=D, qscale=ops.Q2_SCALE),
     M * D * B2 + M * 3 * D * B2, 2.0 * M * 3 * D * D),
    ("fwd proj + resid + LN2", lambda: ops.linear_resid_ln_fwd(a_o, wp, bp, x32, scale, 4501, g, beta, 1e-6),
     M * D * (B2 + F4 + F4 + B2) + 8 * M, 2.0 * M * D * D),
    ("fwd fc1 + GELU (+pre)", lambda: ops.panel_fwd(ln, w1, b1, act=ACT_GELU, want_pre=True),
     M * D * B2 + 2 * M * F * B2, 2.0 * M * F * D),
    ("fwd fc2 + resid + LN1'", lambda: ops.linear_resid_ln_fwd(a, w2, b2, x32, scale, 4501, g, beta, 1e-6),
     M * F * B2 + M * D * (F4 + F4 + B2) + 8 * M, 2.0 * M * D * F),
    ("bwd fc2 dgrad x GELU'", lambda: ops.panel_dgrad_gelu(dy, w2, h), M * D * B2 + 2 * M * F * B2, 2.0 * M * D * F),
    ("fwd fc1 + GELU (+GELU') [train]", lambda: ops.panel_fwd(ln, w1, b1, act=ACT_GELU_D, want_pre=True),
     M * D * B2 + 2 * M * F * B2, 2.0 * M * F * D),
    ("bwd fc2 dgrad x G [train]", lambda: ops.panel_dgrad_mul(dy, w2, h), M * D * B2 + 2 * M * F * B2, 2.0 * M * D * F),
    ("bwd fc2 wgrad", lambda: ops.linear_wgrad(dy, a, BF16), M * (D + F) * B2, 2.0 * M * D * F),
    ("bwd fc1 dgrad + LN2 bwd", lambda: ops.linear_dgrad_ln_bwd(dh, w1, x32, g, mean, rstd, dres=x32.clone(),
                                                                xs_dtype=torch.bfloat16, row_scale=scale, rps=4501),
     M * F * B2 + M * D * (F4 + F4 + F4 + B2) + 8 * M, 2.0 * M * D * F),
    ("bwd fc1 wgrad", lambda: ops.linear_wgrad(dh, ln, BF16), M * (D + F) * B2, 2.0 * M * D * F),
    ("bwd proj dgrad", lambda: ops.linear_dgrad(dy, wb["p"], BF16, torch.bfloat16), 2 * M * D * B2, 2.0 * M * D * D),
    ("bwd proj wgrad", lambda: ops.linear_wgrad(dy, a_o, BF16), 2 * M * D * B2, 2.0 * M * D * D),
    ("bwd qkv dgrad + LN1 bwd", lambda: ops.linear_dgrad_ln_bwd(dqkv, wqkv, x32, g, mean, rstd, dres=x32.clone()),
     M * 3 * D * B2 + M * D * (F4 + F4 + F4) + 8 * M, 2.0 * M * D * 3 * D),
    ("bwd qkv wgrad", lambda: ops.linear_wgrad(dqkv, ln, BF16), M * 4 * D * B2, 2.0 * M * 3 * D * D),
]
# WIDE_AB="ENV=V;ENV=V;...": only the wide row-panel kernels, once per variant, twice over (same-call A/B)
if os.environ.get("WIDE_AB"):
    wide = [r for r in rows if r[0].startswith(("fwd qkv", "fwd fc1 + GELU (+GELU')", "bwd fc2 dgrad x G"))]
    for rep in range(2):
        for var in os.environ["WIDE_AB"].split(";"):
            for kv in var.split(","):
                k_, v_ = kv.split("=")
                os.environ[k_] = v_
            res = [(name, timeit(fn) * 1e3, max(by / 6.3e12, fl / 2516.6e12) * 1e6) for name, fn, by, fl in wide]
            print(f"[{var}] " + "; ".join(f"{n}: {t:.1f} us ({t / f:.2f}x floor)" for n, t, f in res))
    sys.exit(0)
tot = tot_floor = 0.0
print(f"{'kernel':32s} {'us':>8s} {'TF/s':>7s} {'GB/s':>7s} {'hbm-floor':>9s} {'mfma-floor':>10s}  ratio")
for name, fn, by, fl in rows:
    ms = timeit(fn)
    hb, mf = by / 6.3e12 * 1e6, fl / 2516.6e12 * 1e6
    floor = max(hb, mf)
    tot += ms * 1e3
    tot_floor += floor
    print(f"{name:32s} {ms * 1e3:8.1f} {fl / ms / 1e9:7.1f} {by / ms / 1e6:7.0f} {hb:9.1f} {mf:10.1f}  {ms * 1e3 / floor:5.2f}")
print(f"{'block total':32s} {tot:8.1f} us   floor {tot_floor:.1f} us  ({tot / tot_floor:.2f}x)")

# library reference points (torch.matmul -> hipBLASLt): the same GEMMs without the fused epilogues
if os.environ.get("BLAS_REF", "1") == "1":
    wq16, w116, w216 = wqkv.to(torch.bfloat16), w1.to(torch.bfloat16), w2.to(torch.bfloat16)
    refs = [("blas qkv  ln @ Wqkv^T", lambda: ln @ wq16.t(), M * D * B2 + M * 3 * D * B2, 2.0 * M * 3 * D * D),
            ("blas fc1  ln @ W1^T", lambda: ln @ w116.t(), M * D * B2 + M * F * B2, 2.0 * M * F * D),
            ("blas fc2  a @ W2^T", lambda: a @ w216.t(), M * F * B2 + M * D * B2, 2.0 * M * D * F),
            ("blas fc2 dgrad dy @ W2", lambda: dy @ w216, M * D * B2 + M * F * B2, 2.0 * M * D * F),
            ("blas qkv dgrad dqkv @ Wqkv", lambda: dqkv @ wq16, M * 3 * D * B2 + M * D * B2, 2.0 * M * 3 * D * D)]
    for name, fn, by, fl in refs:
        ms = timeit(fn)
        hb, mf = by / 6.3e12 * 1e6, fl / 2516.6e12 * 1e6
        print(f"{name:32s} {ms * 1e3:8.1f} {fl / ms / 1e9:7.1f} {by / ms / 1e6:7.0f} {hb:9.1f} {mf:10.1f}  "
              f"{ms * 1e3 / max(hb, mf):5.2f}")
