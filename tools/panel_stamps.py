"""Per-workgroup anatomy of the row-panel kernels from in-kernel clock stamps (ivit_debug_stamps;
stamping builds, diagnostic only): prologue (entry -> first K stage ready), main loop, epilogue,
per-CU occupancy and the idle time between a workgroup's exit and the next start on that CU.
    python tools/panel_stamps.py"""
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "visiontransformer-intention-prediction_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ops  # noqa: E402
from _lib import ACT_GELU, ACT_GELU_D, lib  # noqa: E402

torch.manual_seed(0)
M, D, F = 8 * 4501, 384, 1536
dev = "cuda"
bf = lambda *s: torch.randn(*s, device=dev).to(torch.bfloat16)
ln, h, dy, a, dh, dqkv = bf(M, D), bf(M, F), bf(M, D), bf(M, F), bf(M, F), bf(M, 3 * D)
wqkv, w1, w2 = torch.randn(3 * D, D, device=dev) / 20, torch.randn(F, D, device=dev) / 20, torch.randn(D, F, device=dev) / 40
b3, b1, bD = torch.zeros(3 * D, device=dev), torch.zeros(F, device=dev), torch.zeros(D, device=dev)
x32, scale = torch.randn(M, D, device=dev), torch.ones(8, device=dev)
g, beta = torch.ones(D, device=dev), torch.zeros(D, device=dev)
mean, rstd = torch.zeros(M, device=dev), torch.ones(M, device=dev)
cases = [("qkv fwd (wide QS)", lambda: ops.panel_fwd(ln, wqkv, b3, qcols=D, qscale=ops.Q2_SCALE)),
         ("fc1 fwd (wide GELU+pre)", lambda: ops.panel_fwd(ln, w1, b1, act=ACT_GELU, want_pre=True)),
         ("fc2 dgrad (wide DGELU)", lambda: ops.panel_dgrad_gelu(dy, w2, h)),
         ("fc1 fwd (wide GELU+GELU')", lambda: ops.panel_fwd(ln, w1, b1, act=ACT_GELU_D, want_pre=True)),
         ("fc2 dgrad (wide x GELU')", lambda: ops.panel_dgrad_mul(dy, w2, h)),
         ("fc2 fwd + LN (ln<false>)", lambda: ops.linear_resid_ln_fwd(a, w2, bD, x32, scale, 4501, g, beta, 1e-6)),
         ("fc1 dgrad + LN bwd (ln<true>)", lambda: ops.linear_dgrad_ln_bwd(dh, w1, x32, g, mean, rstd, dres=x32.clone(),
                                                                          xs_dtype=torch.bfloat16, row_scale=scale,
                                                                          rps=4501)),
         ("qkv dgrad + LN bwd (ln<true>)", lambda: ops.linear_dgrad_ln_bwd(dqkv, wqkv, x32, g, mean, rstd,
                                                                          dres=x32.clone()))]
buf = torch.zeros(8 * 4096, dtype=torch.int64, device=dev)
for name, fn in cases:
    fn()
    torch.cuda.synchronize()
    buf.zero_()
    lib.ivit_debug_stamps(buf.data_ptr(), buf.numel())
    fn()
    torch.cuda.synchronize()
    lib.ivit_debug_stamps(None, 0)
    r = buf.view(-1, 8).cpu().numpy().astype(np.uint64)
    r = r[r[:, 3] != 0].astype(np.int64)
    t0, t1, t2, t3, r0, r3, hw = (r[:, i] for i in range(7))
    ghz = np.median((t3 - t0) / np.maximum(r3 - r0, 1)) * 0.1  # shader clock ticks per 10 ns
    span_us = (r3.max() - r0.min()) / 100.0
    pro, main, epi = (t1 - t0) / ghz / 1e3, (t2 - t1) / ghz / 1e3, (t3 - t2) / ghz / 1e3
    cu = ((hw >> 32) << 16) | ((hw >> 13) & 7) << 8 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 15)
    per = defaultdict(list)
    for i in range(len(r)):
        per[cu[i]].append((r0[i], r3[i]))
    idle, conc = [], []
    for k, v in per.items():
        v.sort()
        ev = sorted([(s, 1) for s, e in v] + [(e, -1) for s, e in v])
        c, last, busy_hist = 0, ev[0][0], defaultdict(float)
        for tt, d in ev:
            busy_hist[c] += tt - last
            c += d
            last = tt
        tot = sum(busy_hist.values())
        conc.append(sum(kk * vv for kk, vv in busy_hist.items()) / max(tot, 1))
        idle.append(busy_hist[0] / 100.0)
    print(f"{name}: {len(r)} WGs on {len(per)} CUs, span {span_us:.1f} us at {ghz:.2f} GHz; per WG (us, median "
          f"[p10 p90]): prologue {np.median(pro):.2f} [{np.percentile(pro, 10):.2f} {np.percentile(pro, 90):.2f}]  "
          f"main {np.median(main):.2f} [{np.percentile(main, 10):.2f} {np.percentile(main, 90):.2f}]  "
          f"epilogue {np.median(epi):.2f} [{np.percentile(epi, 10):.2f} {np.percentile(epi, 90):.2f}]; "
          f"WGs per CU {len(r) / len(per):.2f}, mean concurrency {np.mean(conc):.2f}, CU idle inside span "
          f"{np.mean(idle):.2f} us; first start spread {(r0.max() - r0.min()) / 100.0 if len(per) >= len(r) else 0:.1f}",
          flush=True)
