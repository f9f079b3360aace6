"""Per-kernel parity on the MI355X: each HIP op (through the C ABI) against a CPU f64/f32
reference of the same op. f32 path: rel 1e-5-ish (exact-f32 MFMA); bf16 path: bf16 tolerance."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


def _lin_case(M, N, K, dtype):
    x = torch.randn(M, K)
    w = torch.randn(N, K) / math.sqrt(K)
    b = torch.randn(N) * 0.1
    return x, w, b


@pytest.mark.parametrize("M,N,K", [(300, 200, 136), (1000, 1152, 384), (77, 64, 1536), (9002, 384, 1152)])
@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
def test_linear_fwd_dgrad_wgrad(M, N, K, cd):
    import ops
    from _lib import ACT_GELU, BF16, F32
    cdt = BF16 if cd == torch.bfloat16 else F32
    x, w, b = _lin_case(M, N, K, cd)
    xd, wd, bd = ops.cast(x.to(DEV), cd), ops.cast(w.to(DEV), cd), b.to(DEV)
    ref = x.double() @ w.double().T + b.double()
    y, _ = ops.linear_fwd(xd, wd, bd, cdt, out_dtype=torch.float32)
    tol = 1e-5 if cdt == F32 else 2e-2
    assert _rel(y, ref) < tol
    a, pre = ops.linear_fwd(xd, wd, bd, cdt, act=ACT_GELU, want_pre=True)
    assert _rel(pre.float(), ref) < tol
    assert _rel(a.float(), F.gelu(ref)) < max(tol, 1e-5) * 2
    r = torch.randn(M, N).to(DEV)
    s = torch.tensor([0.5, 2.0]).to(DEV)
    yr, _ = ops.linear_fwd(xd, wd, bd, cdt, resid=r, row_scale=s, rps=(M + 1) // 2)
    sc = torch.where(torch.arange(M) < (M + 1) // 2, 0.5, 2.0).double()[:, None]
    assert _rel(yr, r.cpu().double() + sc * ref) < tol
    dy = torch.randn(M, N)
    dyd = ops.cast(dy.to(DEV), cd)
    dx = ops.linear_dgrad(dyd, wd, cdt, torch.float32)
    assert _rel(dx, dy.double() @ w.double()) < tol
    prek = ops.cast(torch.randn(M, K).to(DEV), cd)
    dxg = ops.linear_dgrad(dyd, wd, cdt, torch.float32, gelu_pre=prek)
    hp = prek.float().cpu().double().requires_grad_(True)
    F.gelu(hp).backward(dyd.float().cpu().double() @ wd.float().cpu().double())
    assert _rel(dxg, hp.grad) < tol * 2
    dw, db = ops.linear_wgrad(dyd, xd, cdt)
    assert _rel(dw, dy.double().T @ x.double()) < tol
    assert _rel(db, dy.double().sum(0)) < tol
    # the bias gradient is an f32 sum of the exact operand values (fused into the bf16 GEMM)
    assert _rel(db, dyd.float().cpu().double().sum(0)) < 1e-5
    assert _rel(dw, dyd.float().cpu().double().T @ xd.float().cpu().double()) < 1e-5


@pytest.mark.parametrize("M,N,K", [(4133, 512, 1024), (2100, 384, 520), (4096, 1152, 768)])
def test_linear_engine_ragged_shapes(M, N, K):
    """The LDS-DMA GEMM engine (KC and MN-contiguous B) through the linear fwd / GELU / residual /
    dgrad / GELU-grad entry points at ragged M, N and K edges and long K."""
    import ops
    from _lib import ACT_GELU, BF16
    x, w, b = _lin_case(M, N, K, torch.bfloat16)
    xd, wd, bd = ops.cast(x.to(DEV), torch.bfloat16), ops.cast(w.to(DEV), torch.bfloat16), b.to(DEV)
    xr, wr = xd.float().cpu().double(), wd.float().cpu().double()
    ref = xr @ wr.T + b.double()
    y, _ = ops.linear_fwd(xd, wd, bd, BF16, out_dtype=torch.float32)
    assert _rel(y, ref) < 1e-5
    a, pre = ops.linear_fwd(xd, wd, bd, BF16, act=ACT_GELU, want_pre=True)
    assert _rel(pre.float(), ref) < 1e-2 and _rel(a.float(), F.gelu(ref)) < 1e-2
    r = torch.randn(M, N).to(DEV)
    yr, _ = ops.linear_fwd(xd, wd, bd, BF16, resid=r)
    assert _rel(yr, r.cpu().double() + ref) < 1e-5
    dyd = ops.cast(torch.randn(M, K).to(DEV), torch.bfloat16)   # dX[M, N] = dY[M, K] W[K, N] (MN-contiguous W)
    w2 = ops.cast(torch.randn(K, N).to(DEV) / math.sqrt(K), torch.bfloat16)
    dx = ops.linear_dgrad(dyd, w2, BF16, torch.float32)
    assert _rel(dx, dyd.float().cpu().double() @ w2.float().cpu().double()) < 1e-5
    prek = ops.cast(torch.randn(M, N).to(DEV), torch.bfloat16)
    dxg = ops.linear_dgrad(dyd, w2, BF16, torch.float32, gelu_pre=prek)
    hp = prek.float().cpu().double().requires_grad_(True)
    F.gelu(hp).backward(dyd.float().cpu().double() @ w2.float().cpu().double())
    assert _rel(dxg, hp.grad) < 1e-3


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
def test_layernorm(cd):
    import ops
    M, D = 513, 384
    x = torch.randn(M, D) * 2 + 0.5
    g, b = 1 + 0.1 * torch.randn(D), 0.1 * torch.randn(D)
    y, m, r = ops.layernorm_fwd(x.to(DEV), g.to(DEV), b.to(DEV), 1e-6, cd)
    xr = x.double().requires_grad_(True)
    gr, br = g.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = F.layer_norm(xr, (D,), gr, br, 1e-6)
    assert _rel(y.float(), ref.detach()) < (2e-6 if cd == torch.float32 else 1e-2)
    dy = torch.randn(M, D)
    dres = torch.randn(M, D)
    ref.backward(dy.double())
    s = torch.tensor([0.5]).to(DEV)
    dx, dxs, dg, dbb = ops.layernorm_bwd(x.to(DEV), g.to(DEV), m, r, dy.to(DEV), dres=dres.to(DEV).clone(),
                                         xs_dtype=cd, row_scale=s, rps=M)
    assert _rel(dx, xr.grad + dres.double()) < 1e-5
    assert _rel(dxs.float(), 0.5 * (xr.grad + dres.double())) < (1e-5 if cd == torch.float32 else 1e-2)
    assert _rel(dg, gr.grad) < 1e-5 and _rel(dbb, br.grad) < 1e-5


def _attn_ref(qkv, B, N, H):
    q, k, v = qkv.double().reshape(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) / 8.0
    p = torch.softmax(s, -1)
    return (p @ v).transpose(1, 2).reshape(B * N, H * 64), torch.logsumexp(s, -1)


@pytest.mark.parametrize("B,N,H", [(2, 257, 2), (1, 4501, 6), (1, 64, 1)])
@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
def test_attention(B, N, H, cd):
    import ops
    from _lib import BF16, F32
    cdt = BF16 if cd == torch.bfloat16 else F32
    qkv = torch.randn(B * N, 3 * H * 64)
    q = ops.cast(qkv.to(DEV), cd)
    o, lse = ops.attn_fwd(q, B, N, H, cdt)
    qr = q.float().cpu().double().requires_grad_(True)
    oref, lref = _attn_ref(qr, B, N, H)
    tol = 1e-5 if cdt == F32 else 2e-2
    assert _rel(o.float(), oref.detach()) < tol
    # bf16 path: the row sums l are accumulated on the MFMA pipe over the bf16-rounded
    # probabilities (exactly the weights P.V uses), so lse = m + log l carries their rounding
    # (~1e-4 relative at N <= 4501), plus the in-kernel bf16 rounding of q * log2(e)/8 (the
    # prescaled-Q forward serves the plain entry point too, as in the q2 test below); the f32
    # path sums f32 probabilities.
    assert _rel(lse, lref.detach()) < (1e-5 if cdt == F32 else 6e-4)
    do = torch.randn(B * N, H * 64)
    dod = ops.cast(do.to(DEV), cd)
    oref.backward(dod.float().cpu().double())
    dq = ops.attn_bwd(q, o, dod, lse, B, N, H, cdt)
    g = qr.grad.reshape(B * N, 3, H * 64)
    d = dq.float().cpu().reshape(B * N, 3, H * 64)
    for i in range(3):
        assert _rel(d[:, i], g[:, i]) < (1e-4 if cdt == F32 else 3e-2), ("qkv"[i], _rel(d[:, i], g[:, i]))


@pytest.mark.parametrize("B,N,H", [(1, 64, 1), (2, 257, 3), (1, 4501, 2), (1, 1, 1), (1, 33, 1), (1, 128, 2),
                                   (1, 130, 1), (1, 200, 1), (1, 320, 2), (3, 449, 1)])
def test_attention_q2_prescaled_path(B, N, H):
    """bf16 ViT-block path: the qkv projection stores q * log2(e)/8 (ivit_linear_fwd_qs) and the
    attention kernels run on it (ivit_attn_fwd_q2 / _bwd_q2). Outputs, lse and the gradient w.r.t.
    the UNSCALED q, k, v against the f64 reference on the unscaled q (bf16 tolerances). The backward
    runs the v_mfma_f32_16x16x32_bf16 dQ and dK/dV kernels (incl. the masked ragged key tile)."""
    import ops
    from _lib import BF16
    D = H * 64
    M, K = B * N, 96
    x = torch.randn(M, K)
    w = torch.randn(3 * D, K) / math.sqrt(K)
    b = torch.randn(3 * D) * 0.1
    xd, wd = ops.cast(x.to(DEV), torch.bfloat16), ops.cast(w.to(DEV), torch.bfloat16)
    qkv_s = ops.qkv_fwd_q2(xd, wd, b.to(DEV), D)
    qkv, _ = ops.linear_fwd(xd, wd, b.to(DEV), BF16)
    ref_s = qkv.float().clone()
    ref_s[:, :D] *= ops.Q2_SCALE
    assert _rel(qkv_s.float(), ref_s) < 8e-3  # one bf16 rounding of (xW^T + b) * c on the Q block
    qs = qkv.clone()
    qs[:, :D] = (qkv[:, :D].float() * ops.Q2_SCALE).to(torch.bfloat16)
    o, lse = ops.attn_fwd_q2(qs, B, N, H)
    qr = qkv.float().cpu().double().requires_grad_(True)
    oref, lref = _attn_ref(qr, B, N, H)
    assert _rel(o.float(), oref.detach()) < 2e-2
    # the extra bf16 rounding of q * c (the f32 test rounds q once); few rows: a single score's rounding
    assert _rel(lse, lref.detach()) < (6e-4 if N >= 64 else 3e-3)
    dod = ops.cast(torch.randn(B * N, D).to(DEV), torch.bfloat16)
    oref.backward(dod.float().cpu().double())
    dq = ops.attn_bwd_q2(qs, o, dod, lse, B, N, H)
    g = qr.grad.reshape(B * N, 3, D)
    d = dq.float().cpu().reshape(B * N, 3, D)
    for i in range(3):
        assert _rel(d[:, i], g[:, i]) < 3e-2, ("qkv"[i], _rel(d[:, i], g[:, i]))


@pytest.mark.parametrize("B,N,H", [(1, 64, 1), (2, 257, 3), (1, 4501, 2), (1, 33, 1)])
def test_attention_plain_entry_is_the_v4_pair(B, N, H):
    """The reference-facing seam (ivit_attn_bwd, bf16; INTEGRATION.md binds timm Attention to it)
    runs the product's 16x16x32 v4 backward pair on a prescaled copy of Q: its dQ / dK / dV are
    bitwise those of ivit_attn_bwd_q2 on qkv with the Q block holding bf16(q * log2(e)/8), and the
    kernel-timing hook records exactly one dQ and one dK/dV v4 launch for it."""
    import ops
    from _lib import BF16
    D = H * 64
    qkv = torch.randn(B * N, 3 * D, device=DEV).to(torch.bfloat16)
    dod = torch.randn(B * N, D, device=DEV).to(torch.bfloat16)
    o, lse = ops.attn_fwd(qkv, B, N, H, BF16)
    qs = qkv.clone()
    qs[:, :D] = (qkv[:, :D].float() * ops.Q2_SCALE).to(torch.bfloat16)
    o2, l2 = ops.attn_fwd_q2(qs, B, N, H)
    assert torch.equal(o, o2) and torch.equal(lse, l2)  # the forward's in-kernel prescale rounds alike
    torch.cuda.synchronize()
    ops.ktime_arm(True)
    d_plain = ops.attn_bwd(qkv, o, dod, lse, B, N, H, BF16)
    ops.ktime_arm(False)
    torch.cuda.synchronize()
    assert len(ops.ktime_read(ops.KT_ATTN_BWD_DQ)) == 1 and len(ops.ktime_read(ops.KT_ATTN_BWD_DKV)) == 1
    d_q2 = ops.attn_bwd_q2(qs, o, dod, lse, B, N, H)
    assert torch.equal(d_plain, d_q2)


def test_kernel_exec_timing_hook():
    """ivit_ktime_*: armed launches go through hipExtLaunchKernel with kernel-bound events (one
    record per kernel, outputs unchanged); the kernel intervals lie inside the stream's own span
    and nothing is recorded once disarmed."""
    import ops
    B, N, H = 2, 1025, 2
    qkv = torch.randn(B * N, 3 * H * 64, device=DEV).to(torch.bfloat16)
    dod = torch.randn(B * N, H * 64, device=DEV).to(torch.bfloat16)
    o0, l0 = ops.attn_fwd_q2(qkv, B, N, H)
    d0 = ops.attn_bwd_q2(qkv, o0, dod, l0, B, N, H)
    torch.cuda.synchronize()
    ops.ktime_arm(True)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    o1, l1 = ops.attn_fwd_q2(qkv, B, N, H)
    d1 = ops.attn_bwd_q2(qkv, o1, dod, l1, B, N, H)
    e.record()
    ops.ktime_arm(False)
    ops.attn_fwd_q2(qkv, B, N, H)  # disarmed: not recorded
    torch.cuda.synchronize()
    assert torch.equal(o0, o1) and torch.equal(l0, l1) and torch.equal(d0, d1)
    span = s.elapsed_time(e)
    iv = []
    for tag in (ops.KT_ATTN_FWD, ops.KT_ATTN_BWD_DQ, ops.KT_ATTN_BWD_DKV):
        r = ops.ktime_read(tag)
        assert len(r) == 1 and 0.0 < r[0][1] - r[0][0] <= span, (tag, r, span)
        iv += r
    # one stream: the fwd, dQ and dK/dV kernels run in order, from the common origin
    assert iv[0][0] == 0.0 and all(a[1] <= b[0] + 1e-3 for a, b in zip(iv, iv[1:])), iv
    assert abs(ops.busy_ms(iv) - sum(b - a for a, b in iv)) < 1e-6
    assert iv[-1][1] <= span * 1.01, (iv, span)
    assert ops.busy_ms([(0.0, 2.0), (1.0, 3.0), (5.0, 6.0)]) == 4.0
    ops.ktime_arm(True)  # re-arming clears the records
    ops.ktime_arm(False)
    assert ops.ktime_read(ops.KT_ATTN_FWD) == []


@pytest.mark.parametrize("tag", ["up", "odd", "down"])
def test_bilinear_resize_vs_golden(tag):
    """ivit_bilinear_fwd / _bwd vs F.interpolate(bilinear, align_corners=False) and its autograd
    adjoint, run by the reference's torch (tests/golden/model_regrid.npz: the model's 2x
    upsampling, a ragged upsampling and a downsampling)."""
    import ops
    from conftest import golden
    z = golden("model_regrid.npz")
    x = torch.from_numpy(z[f"resize_{tag}_x"]).to(DEV)
    y = ops.bilinear_fwd(x, z[f"resize_{tag}_y"].shape[2:])
    np.testing.assert_allclose(y.cpu().numpy(), z[f"resize_{tag}_y"], rtol=1e-6, atol=1e-6)
    dx = ops.bilinear_bwd(torch.from_numpy(z[f"resize_{tag}_dy"]).to(DEV), x.shape[2:])
    np.testing.assert_allclose(dx.cpu().numpy(), z[f"resize_{tag}_dx"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,H,W,D", [(2, 9, 32, 48, 384), (1, 290, 64, 96, 384), (3, 5, 16, 80, 192)])
def test_patch_embed_patch16(cd, B, C, H, W, D):
    """PatchEmbed with patch 16 (ivit_patch_im2col_p + linear + ivit_patch_tokens, and the
    backward's ivit_patch_tokens_bwd + weight gradient) vs F.conv2d(k = s = 16) + CLS + pos_embed
    in f64 (f32 path: 1e-5; bf16: vs f64 of the same bf16-rounded operands)."""
    import ops
    from _lib import BF16, F32
    cdt = BF16 if cd == torch.bfloat16 else F32
    img = torch.rand(B, C, H, W)
    w = torch.randn(D, C, 16, 16) / math.sqrt(C * 256)
    b, pos, cls = torch.randn(D) * 0.1, torch.randn(1, (H // 16) * (W // 16) + 1, D) * 0.1, torch.randn(1, 1, D)
    wd = w.to(DEV).requires_grad_(True)
    out = ops.PatchEmbedFn.apply(img.to(DEV), wd, b.to(DEV), pos.to(DEV), cls.to(DEV), cdt)
    imr, wr = img.double(), w.double()
    if cd == torch.bfloat16:
        imr, wr = img.bfloat16().double(), w.bfloat16().double()
    imr.requires_grad_(False)
    wr.requires_grad_(True)
    br, pr, cr = b.double().requires_grad_(True), pos.double().requires_grad_(True), cls.double().requires_grad_(True)
    t = F.conv2d(imr, wr, br, stride=16).flatten(2).transpose(1, 2)
    ref = (torch.cat([cr.expand(B, -1, -1), t], 1) + pr).reshape(B * t.shape[1] + B, D)
    tol = 1e-5 if cd == torch.float32 else 2e-5
    assert _rel(out, ref.detach()) < tol
    g = torch.randn(out.shape)
    out.backward(g.to(DEV))
    gr = g.double() if cd == torch.float32 else g.bfloat16().double()
    ref.backward(gr)
    assert _rel(wd.grad, wr.grad) < (1e-5 if cd == torch.float32 else 1e-4)


def test_attention_large_grid_bf16():
    """BASELINE config 5 sequence length (800x1440 grid: N = 100*180 + 1 = 18001), bf16 flash
    kernels vs an f32 torch reference on the device (scores materialised per head)."""
    import ops
    from _lib import BF16
    B, N, H = 1, 18001, 2
    q = (torch.randn(B * N, 3 * H * 64, device=DEV)).to(torch.bfloat16)
    o, lse = ops.attn_fwd(q, B, N, H, BF16)
    dod = torch.randn(B * N, H * 64, device=DEV).to(torch.bfloat16)
    dq = ops.attn_bwd(q, o, dod, lse, B, N, H, BF16).float()
    qr = q.float().requires_grad_(True)
    qq, kk, vv = qr.reshape(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (qq @ kk.transpose(-1, -2)) / 8.0
    oref = (torch.softmax(s, -1) @ vv).transpose(1, 2).reshape(B * N, H * 64)
    lref = torch.logsumexp(s, -1)
    assert _rel(o.float(), oref.detach()) < 2e-2
    assert _rel(lse, lref.detach()) < 3e-4  # incl. the in-kernel bf16 rounding of q * log2(e)/8
    oref.backward(dod.float())
    g = qr.grad.reshape(B * N, 3, H * 64)
    d = dq.reshape(B * N, 3, H * 64)
    for i in range(3):
        assert _rel(d[:, i], g[:, i]) < 3e-2, ("qkv"[i], _rel(d[:, i], g[:, i]))


@pytest.mark.parametrize("k,Cin", [(1, 48), (3, 48), (5, 48), (5, 64)])  # 5: model_cnn.py stride-1 convs
@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
def test_conv_nhwc(k, Cin, cd):
    import ops
    from _lib import BF16, F32
    cdt = BF16 if cd == torch.bfloat16 else F32
    B, H, W, Cout = 2, 7, 9, 40
    x = torch.randn(B, Cin, H, W)
    w = torch.randn(Cout, Cin, k, k) / math.sqrt(Cin * k * k)
    bias = torch.randn(Cout) * 0.1
    xh = ops.cast(x.permute(0, 2, 3, 1).reshape(-1, Cin).contiguous().to(DEV), cd)
    wp = ops.pack_conv(w.to(DEV), cdt)
    y = ops.conv_fwd(xh, B, H, W, wp, bias.to(DEV), cdt, torch.float32)
    xr = xh.float().cpu().reshape(B, H, W, Cin).permute(0, 3, 1, 2).double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    ref = F.conv2d(xr, wr, bias.double(), padding=k // 2)
    tol = 1e-5 if cdt == F32 else 2e-2
    assert _rel(y.reshape(B, H, W, Cout).permute(0, 3, 1, 2), ref.detach()) < tol
    dy = torch.randn(B, Cout, H, W)
    dyh = ops.cast(dy.permute(0, 2, 3, 1).reshape(-1, Cout).contiguous().to(DEV), cd)
    ref.backward(dyh.float().cpu().reshape(B, H, W, Cout).permute(0, 3, 1, 2).double())
    dx = ops.conv_dgrad(dyh, B, H, W, wp, cdt, torch.float32)
    assert _rel(dx.reshape(B, H, W, Cin).permute(0, 3, 1, 2), xr.grad) < tol
    gp, db = ops.conv_wgrad(dyh, xh, B, H, W, Cin, Cout, k, cdt, want_bias=True)
    assert _rel(ops.unpack_conv_grad(gp, Cout, Cin, k), wr.grad) < tol
    assert _rel(db, dyh.float().cpu().double().sum(0)) < 1e-5


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,ybf", [(2, 13, 29, 128, 256, 3, False),   # ragged last pixel panel
                                                   (1, 17, 23, 64, 384, 1, True),     # ragged channel tile
                                                   (1, 19, 21, 64, 136, 5, False),    # partial 16-channel block
                                                   (1, 24, 12, 192, 512, 3, True)])
def test_conv_panel(B, H, W, Cin, Cout, k, ybf):
    """288 x 256 panel kernel (conv_panel.hip): forward through ivit_conv_fwd and the data gradient
    on the tap-flipped transposed pack (ivit_conv_dgrad_t) vs f64 of the same bf16 operands (the
    fusion block convs, model_vit.py:12-43)."""
    import ops
    from _lib import BF16
    torch.manual_seed(7)
    x = torch.randn(B, Cin, H, W)
    w = torch.randn(Cout, Cin, k, k) / math.sqrt(Cin * k * k)
    bias = torch.randn(Cout) * 0.1
    xh = ops.cast(x.permute(0, 2, 3, 1).reshape(-1, Cin).contiguous().to(DEV), torch.bfloat16)
    wd = w.to(DEV)
    wp = ops.pack_conv(wd, BF16)
    od = torch.bfloat16 if ybf else torch.float32
    y = ops.conv_fwd(xh, B, H, W, wp, bias.to(DEV), BF16, od)
    xr = xh.float().cpu().reshape(B, H, W, Cin).permute(0, 3, 1, 2).double().requires_grad_(True)
    wr = wp.float().cpu().reshape(Cout, k, k, Cin).permute(0, 3, 1, 2).double().requires_grad_(True)
    ref = F.conv2d(xr, wr, bias.double(), padding=k // 2)
    tol = 1e-2 if ybf else 1e-5
    assert _rel(y.float().reshape(B, H, W, Cout).permute(0, 3, 1, 2), ref.detach()) < tol
    dy = torch.randn(B, Cout, H, W)
    dyh = ops.cast(dy.permute(0, 2, 3, 1).reshape(-1, Cout).contiguous().to(DEV), torch.bfloat16)
    ref.backward(dyh.float().cpu().reshape(B, H, W, Cout).permute(0, 3, 1, 2).double())
    # reference gradient against the bf16-rounded weight the transposed pack holds
    wt = ops.pack_conv_t(wd, BF16)
    assert torch.equal(wt.float().cpu(), w.bfloat16().float().permute(1, 2, 3, 0).flip(1, 2))
    dx = ops.conv_dgrad(dyh, B, H, W, wp, BF16, torch.float32, w=wd)
    if Cout % 64 == 0:
        assert _rel(dx.reshape(B, H, W, Cin).permute(0, 3, 1, 2), xr.grad) < 1e-5
    dx0 = ops.conv_dgrad(dyh, B, H, W, wp, BF16, torch.float32)  # 128 x 128 engine
    assert _rel(dx, dx0) < 1e-5
    # weight gradient: 256 x 256 panel tiles with the pixel reduction split (ivit_conv_wgrad)
    gp, db = ops.conv_wgrad(dyh, xh, B, H, W, Cin, Cout, k, BF16, want_bias=True)
    assert _rel(ops.unpack_conv_grad(gp, Cout, Cin, k), wr.grad) < 1e-5
    assert _rel(db, dyh.float().cpu().double().sum(0)) < 1e-5


def test_conv_dgrad_zero_padded_head():
    """The head conv's data gradient (heads.py:16,37: 75 output channels, packed to 80) on the panel
    kernel: dy rows zero-padded to 128 channels and the transposed pack zero past channel 75
    (ivit_pack_conv_weight_t Cout_pad) vs the 128 x 128 engine on the forward pack and vs f64."""
    import ops
    from _lib import BF16
    torch.manual_seed(11)
    B, H, W, Cin, Cw, Cp, Cq = 2, 50, 90, 512, 75, 80, 128
    w = torch.randn(Cw, Cin, 3, 3) / math.sqrt(Cin * 9)
    wd = w.to(DEV)
    wp = ops.pack_conv(wd, BF16, cout_pad=Cp)
    dyq = torch.zeros(B * H * W, Cq)
    dyq[:, :Cw] = torch.randn(B * H * W, Cw)
    dyh = ops.cast(dyq.to(DEV), torch.bfloat16)
    wt = ops.pack_conv_t(wd, BF16, cout_pad=Cq)
    assert torch.equal(wt[..., Cw:].float().cpu(), torch.zeros(Cin, 3, 3, Cq - Cw))
    dx = ops.conv_dgrad(dyh, B, H, W, wp, BF16, torch.float32, w=wd, dy_zero_pad=True)
    dx0 = ops.conv_dgrad(dyh, B, H, W, wp, BF16, torch.float32)  # engine, reads the first 80 channels
    assert _rel(dx, dx0) < 1e-5
    wr = w.bfloat16().double()
    dyr = dyh.float().cpu().double()[:, :Cw].reshape(B, H, W, Cw).permute(0, 3, 1, 2)
    ref = F.conv_transpose2d(dyr, wr, padding=1)
    assert _rel(dx.reshape(B, H, W, Cin).permute(0, 3, 1, 2), ref) < 1e-5


@pytest.mark.parametrize("B,H,W,Cin,Cout,k", [(8, 50, 90, 384, 512, 3), (1, 19, 23, 64, 256, 1), (1, 7, 9, 48, 40, 3)])
def test_conv_bn_stats_fused(B, H, W, Cin, Cout, k):
    """ivit_conv_bn_fwd: the BatchNorm batch statistics out of the panel convolution's epilogue (per-
    tile sums and centred squares merged by Chan's update) vs the two-pass ivit_bn_stats on the same
    output, and the running-stat update; the last shape takes the fallback (engine + two passes)."""
    import ops
    from _lib import BF16
    torch.manual_seed(11)
    x = (torch.randn(B * H * W, Cin, device=DEV) + 0.5).bfloat16()
    w = torch.randn(Cout, Cin, k, k, device=DEV) / math.sqrt(Cin * k * k)
    wp = ops.pack_conv(w, BF16)
    rm1, rv1 = torch.randn(Cout, device=DEV), torch.rand(Cout, device=DEV) + 0.5
    rm0, rv0 = rm1.clone(), rv1.clone()
    y1, s1 = ops.conv_bn_fwd(x, B, H, W, wp, BF16, torch.float32, rm1, rv1, True)
    y0 = ops.conv_fwd(x, B, H, W, wp, None, BF16, torch.float32)
    s0 = ops.bn_forward(y0, None, None, rm0, rv0, True)
    assert torch.equal(y1, y0)
    assert _rel(s1.mean, s0.mean) < 1e-5 and _rel(s1.invstd, s0.invstd) < 1e-5
    assert _rel(rm1, rm0) < 1e-5 and _rel(rv1, rv0) < 1e-5
    ref = y0.double().cpu()
    assert _rel(s1.mean, ref.mean(0)) < 1e-5
    assert _rel(s1.invstd, 1.0 / torch.sqrt(ref.var(0, unbiased=False) + 1e-5)) < 1e-5


def test_conv_panel_fusion_shape_vs_engine(request):
    """Full fusion-block shape (B = 8, 50 x 90, 512 -> 512, k = 3): panel kernel vs the 128 x 128
    engine (ivit_set_knob(IVIT_KNOB_CONV_PANEL, 0)), forward and data gradient — same bf16 products,
    f32 sums."""
    import ops
    from _lib import BF16
    torch.manual_seed(3)
    B, H, W, C = 8, 50, 90, 512
    xh = (torch.randn(B * H * W, C, device=DEV) * 0.5).bfloat16()
    w = torch.randn(C, C, 3, 3, device=DEV) / math.sqrt(C * 9)
    wp = ops.pack_conv(w, BF16)
    y1 = ops.conv_fwd(xh, B, H, W, wp, None, BF16, torch.float32)
    d1 = ops.conv_dgrad(xh, B, H, W, wp, BF16, torch.float32, w=w)
    dy = (torch.randn(B * H * W, C, device=DEV) * 0.5).bfloat16()
    g1, _ = ops.conv_wgrad(dy, xh, B, H, W, C, C, 3, BF16)
    from _lib import KNOB_CONV_PANEL, lib
    lib.ivit_set_knob(KNOB_CONV_PANEL, 0)
    request.addfinalizer(lambda: lib.ivit_set_knob(KNOB_CONV_PANEL, 1))
    y0 = ops.conv_fwd(xh, B, H, W, wp, None, BF16, torch.float32)
    d0 = ops.conv_dgrad(xh, B, H, W, wp, BF16, torch.float32, w=w)
    g0, _ = ops.conv_wgrad(dy, xh, B, H, W, C, C, 3, BF16)
    assert _rel(y1, y0) < 1e-5 and _rel(d1, d0) < 1e-5 and _rel(g1, g0) < 1e-5


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [64, 384])
def test_patch_embed(cd, D):
    """D = 64: bf16 through the patch matrix (im2col + GEMM); D = 384: the fused forward
    (ivit_patch_embed_fwd_packed) and the raster-reading weight gradient."""
    import ops
    from _lib import BF16, F32
    cdt = BF16 if cd == torch.bfloat16 else F32
    B, C, H, W = 2, 20, 32, 48
    img = torch.rand(B, C, H, W)
    w = torch.randn(D, C, 8, 8) / math.sqrt(C * 64)
    b, pos, cls = 0.1 * torch.randn(D), 0.02 * torch.randn(1, 25, D), 0.02 * torch.randn(1, 1, D)
    params = [t.to(DEV).requires_grad_(True) for t in (w, b, pos, cls)]
    out = ops.PatchEmbedFn.apply(img.to(DEV), *params, cdt)
    wr, br, pr, cr = [t.double().requires_grad_(True) for t in (w, b, pos, cls)]
    t = F.conv2d(img.double(), wr, br, stride=8).flatten(2).transpose(1, 2)
    ref = torch.cat([cr.expand(B, -1, -1), t], 1) + pr
    tol = 1e-5 if cdt == F32 else 2e-2
    assert _rel(out.reshape(B, 25, D), ref.detach()) < tol
    g = torch.randn(B, 25, D)
    out.backward(g.reshape(B * 25, D).to(DEV))
    ref.backward(g.double())
    for p, r in zip(params, (wr, br, pr, cr)):
        assert _rel(p.grad, r.grad) < tol


@pytest.mark.parametrize("B,C,H,W,D", [(2, 9, 32, 48, 384), (3, 5, 64, 40, 192), (1, 1, 16, 16, 384),
                                       (2, 290, 96, 720, 384), (1, 7, 24, 1448, 192)])
def test_patch_embed_fused_exact(B, C, H, W, D):
    """Fused bf16 forward vs the same products in f64 (bf16-rounded raster and weight): only the
    f32 accumulation order differs. Tiles spanning several images (Np < 144), partial last
    tiles, a single channel, the LiDAR channel count and both widths."""
    from _lib import lib, ptr, stream
    g = torch.Generator().manual_seed(B * 1000 + C)
    img = torch.rand(B, C, H, W, generator=g)
    w = torch.randn(D, C, 8, 8, generator=g) / math.sqrt(C * 64)
    b, pos, cls = 0.1 * torch.randn(D, generator=g), torch.randn(1, (H // 8) * (W // 8) + 1, D, generator=g), \
        torch.randn(1, 1, D, generator=g)
    Np = (H // 8) * (W // 8)
    wd, imgd = w.to(DEV), img.to(DEV)
    wp = torch.empty(lib.ivit_patch_weight_pack_bytes(D, C) // 2, dtype=torch.bfloat16, device=DEV)
    assert lib.ivit_patch_weight_pack(ptr(wd), D, C, ptr(wp), stream()) == 0
    out = torch.full((B * (Np + 1), D), float("nan"), device=DEV)
    bd, pd, cd_ = b.to(DEV), pos.to(DEV), cls.to(DEV)
    assert lib.ivit_patch_embed_fwd_packed(ptr(imgd), B, C, H, W, ptr(wp), ptr(bd), ptr(pd), ptr(cd_), D, ptr(out),
                                           stream()) == 0
    t = F.conv2d(img.to(torch.bfloat16).double(), w.to(torch.bfloat16).double(), b.double(), stride=8)
    ref = torch.cat([cls.double().expand(B, -1, -1), t.flatten(2).transpose(1, 2)], 1) + pos.double()
    o = out.reshape(B, Np + 1, D).double().cpu()
    assert torch.isfinite(o).all()
    err = (o - ref).abs().max().item()
    assert err < 2e-5 * max(1.0, math.sqrt(C * 64) / 8), err
    # the patch-matrix path agrees to the same accuracy
    wc = w.to(torch.bfloat16).reshape(D, C * 64).to(DEV)
    cols = torch.empty((B * Np, C * 64), dtype=torch.bfloat16, device=DEV)
    out2 = torch.empty_like(out)
    assert lib.ivit_patch_im2col(ptr(imgd), B, C, H, W, ptr(cols), stream()) == 0
    assert lib.ivit_patch_embed_fwd_cols(ptr(cols), B, C, H, W, ptr(wc), ptr(bd), ptr(pd), ptr(cd_), D, ptr(out2),
                                         stream()) == 0
    assert (out2.double().cpu().reshape(B, Np + 1, D) - o).abs().max().item() < 2 * err + 1e-5


@pytest.mark.parametrize("B,C,H,W", [(2, 9, 32, 48), (3, 290, 24, 40), (2, 4, 400, 720), (1, 3, 16, 16),
                                     (2, 290, 64, 128), (1, 290, 160, 200), (2, 7, 264, 264), (1, 64, 256, 256),
                                     (3, 33, 200, 360), (2, 65, 256, 264), (1, 290, 400, 720)])
def test_patch_wgrad_raster_exact(B, C, H, W):
    """bf16 weight gradient straight from the raster (ivit_patch_embed_wgrad, D = 384: the
    persistent channel-pair kernels + slab reduction) vs the same products in f64: odd channel
    counts, 32-patch chunks crossing images and patch rows, workgroups spanning two / several
    channel pairs, tiny grids with idle workgroups; dbias / dpos / dcls as before. Patch grids at
    least 32 wide run the wave-specialised kernel — with >= 32 channel pairs and >= 64 chunks
    (the last two shapes: 33 pairs with an odd last channel, and one LiDAR frame) on the
    XCD-sharded schedule — narrower ones the all-waves form."""
    from _lib import BF16, lib, ptr, stream
    D = 384
    g = torch.Generator().manual_seed(7 * C + B)
    img = torch.rand(B, C, H, W, generator=g)
    Np = (H // 8) * (W // 8)
    dtok = torch.randn(B * (Np + 1), D, generator=g).to(torch.bfloat16)
    dw = torch.full((D, C, 8, 8), float("nan"), device=DEV)
    db, dpos, dcls = (torch.empty(D, device=DEV), torch.empty(Np + 1, D, device=DEV), torch.empty(D, device=DEV))
    nws = lib.ivit_patch_embed_wgrad_workspace(B, C, H, W, D)
    ws = torch.empty(nws, dtype=torch.uint8, device=DEV)
    imgd, dtd = img.to(DEV), dtok.to(DEV)
    assert lib.ivit_patch_embed_wgrad(BF16, ptr(dtd), ptr(imgd), B, C, H, W, D, ptr(dw), ptr(db), ptr(dpos),
                                      ptr(dcls), 0, ptr(ws), nws, stream()) == 0
    X = img.to(torch.bfloat16).double().reshape(B, C, H // 8, 8, W // 8, 8).permute(0, 2, 4, 1, 3, 5)
    X = X.reshape(B * Np, C * 64)
    dt = dtok.double().reshape(B, Np + 1, D)
    ref = dt[:, 1:].reshape(B * Np, D).t() @ X
    got = dw.double().cpu().reshape(D, C * 64)
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item()
    assert err < 1e-5 * max(1.0, (B * Np) ** 0.5), err
    assert _rel(db, dt[:, 1:].sum((0, 1))) < 1e-5 and _rel(dpos, dt.sum(0)) < 1e-5
    assert _rel(dcls, dt[:, 0].sum(0)) < 1e-5
    # accumulate = 1 adds onto the previous result
    assert lib.ivit_patch_embed_wgrad(BF16, ptr(dtd), ptr(imgd), B, C, H, W, D, ptr(dw), ptr(db), ptr(dpos),
                                      ptr(dcls), 1, ptr(ws), nws, stream()) == 0
    assert (dw.double().cpu().reshape(D, C * 64) - 2 * ref).abs().max().item() < 2 * err + 1e-5
    assert _rel(db, 2 * dt[:, 1:].sum((0, 1))) < 1e-5 and _rel(dpos, 2 * dt.sum(0)) < 1e-5
    assert _rel(dcls, 2 * dt[:, 0].sum(0)) < 1e-5


@pytest.mark.parametrize("M,K,scale", [(36008, 384, True), (300, 1536, False), (1, 64, True), (145, 128, True)])
def test_linear_resid_ln_fused(M, K, scale):
    """ivit_linear_resid_ln_fwd (proj + residual + DropPath scale + norm2 in one kernel) vs a
    torch f64 reference on the same bf16 operands: partial last row panel, one row, K = 64."""
    import ops
    g = torch.Generator().manual_seed(M + K)
    N = 384
    a = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = 0.1 * torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g)
    s = (torch.rand(max(1, M // 7 + 1), generator=g) + 0.5) if scale else None
    gm, bt = 1 + 0.1 * torch.randn(N, generator=g), 0.1 * torch.randn(N, generator=g)
    x, y, mean, rstd = ops.linear_resid_ln_fwd(a.to(DEV), w.to(DEV), b.to(DEV), r.to(DEV),
                                               s.to(DEV) if scale else None, 7, gm.to(DEV), bt.to(DEV), 1e-6)
    z = a.double() @ w.to(torch.bfloat16).double().t() + b.double()
    if scale:
        z = z * s.double()[torch.arange(M) // 7][:, None]
    xr = r.double() + z
    mu = xr.mean(1)
    var = ((xr - mu[:, None]) ** 2).mean(1)
    rs = 1 / torch.sqrt(var + 1e-6)
    yr = (xr - mu[:, None]) * rs[:, None] * gm.double() + bt.double()
    assert (x.double().cpu() - xr).abs().max().item() < 2e-5 * math.sqrt(K)
    assert (mean.double().cpu() - mu).abs().max().item() < 1e-5
    assert ((rstd.double().cpu() - rs).abs() / rs).max().item() < 1e-4
    assert (y.double().cpu() - yr).abs().max().item() < 0.02 * yr.abs().max().item()
    assert _rel(y.float(), yr) < 4e-3


@pytest.mark.parametrize("M,K,xs", [(36008, 1536, True), (300, 1152, False), (1, 64, True), (145, 128, False)])
def test_linear_dgrad_ln_bwd_fused(M, K, xs):
    """ivit_linear_dgrad_ln_bwd (fc1 / qkv dgrad with the norm2 / norm1 backward in the epilogue)
    vs torch autograd in f64 of LayerNorm(x) fed by the same bf16 dgrad product."""
    import ops
    g = torch.Generator().manual_seed(3 * M + K)
    N = 384
    dy = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = torch.randn(K, N, generator=g) / math.sqrt(K)
    x = torch.randn(M, N, generator=g) * 2 + 0.5
    gm, bt = 1 + 0.1 * torch.randn(N, generator=g), 0.1 * torch.randn(N, generator=g)
    dres = torch.randn(M, N, generator=g)
    sc = torch.rand(M // 5 + 1, generator=g) + 0.5
    mu = x.double().mean(1)
    rs = 1 / torch.sqrt(((x.double() - mu[:, None]) ** 2).mean(1) + 1e-6)
    dx, dxs, dg, db = ops.linear_dgrad_ln_bwd(dy.to(DEV), w.to(DEV), x.to(DEV), gm.to(DEV), mu.float().to(DEV),
                                              rs.float().to(DEV), dres=dres.to(DEV).clone(),
                                              xs_dtype=torch.bfloat16 if xs else None,
                                              row_scale=sc.to(DEV) if xs else None, rps=5)
    G = dy.double() @ w.to(torch.bfloat16).double()
    xr = x.double().requires_grad_(True)
    gr, br = gm.double().requires_grad_(True), bt.double().requires_grad_(True)
    y = torch.nn.functional.layer_norm(xr, (N,), gr, br, 1e-6)
    y.backward(G)
    ref = xr.grad + dres.double()
    assert (dx.double().cpu() - ref).abs().max().item() < 1e-4 * ref.abs().max().item()
    assert _rel(dg, gr.grad) < 1e-4 and _rel(db, br.grad) < 1e-4
    if xs:
        r2 = ref * sc.double()[torch.arange(M) // 5][:, None]
        assert _rel(dxs.float(), r2) < 4e-3


def _set_wide_epi(epi, request):
    """The wide row-panel epilogue form for one test (ivit_set_knob), back to 0 after it."""
    from _lib import KNOB_WIDE_EPI, lib
    lib.ivit_set_knob(KNOB_WIDE_EPI, int(epi))
    request.addfinalizer(lambda: lib.ivit_set_knob(KNOB_WIDE_EPI, 0))


@pytest.mark.parametrize("M,N,K,mode", [(36008, 1152, 384, "qs"), (36008, 1536, 384, "gelu"), (300, 768, 128, "gelu"),
                                        (145, 1536, 384, "dgelu"), (36008, 1536, 384, "dgelu"), (1, 384, 64, "qs"),
                                        (36008, 384, 384, "dgrad"), (77, 384, 384, "dgrad")])
@pytest.mark.parametrize("epi", ["0", "2"])
def test_panel_wide(M, N, K, mode, epi, request):
    """Row-panel wide GEMMs (ivit_linear_fwd_panel / ivit_linear_dgrad_gelu_panel) vs the generic
    engine on the same bf16 operands (qkv with the prescaled Q block, fc1 + GELU + pre-activation,
    fc2 dgrad x GELU'): equal up to f32 summation order and the bf16 rounding of the output. Both
    epilogue forms: ivit_set_knob(IVIT_KNOB_WIDE_EPI) 0 (the default LDS-tile form), 2 (transposed accumulators)."""
    _set_wide_epi(epi, request)
    import ops
    from _lib import ACT_GELU, BF16
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    if mode == "dgrad":  # ops.panel_dgrad: the proj dgrad (ivit_linear_fwd_panel on the transposed pack)
        w = (torch.randn(K, N, generator=g) / math.sqrt(K)).to(DEV)
        ref = ops.linear_dgrad(x, w.to(torch.bfloat16), BF16, torch.bfloat16)
        assert _rel(ops.panel_dgrad(x, w).float(), ref.float()) < 8e-3
        return
    if mode == "dgelu":
        w = (torch.randn(K, N, generator=g) / math.sqrt(K)).to(DEV)
        pre = torch.randn(M, N, generator=g).to(torch.bfloat16).to(DEV)
        got = ops.panel_dgrad_gelu(x, w, pre)
        ref = ops.linear_dgrad(x, w.to(torch.bfloat16), BF16, torch.bfloat16, gelu_pre=pre)
        assert _rel(got.float(), ref.float()) < 8e-3
        return
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV)
    b = (0.1 * torch.randn(N, generator=g)).to(DEV)
    wb = w.to(torch.bfloat16)
    if mode == "qs":
        got, _ = ops.panel_fwd(x, w, b, qcols=384, qscale=ops.Q2_SCALE)
        ref = ops.qkv_fwd_q2(x, wb, b, 384)
        assert _rel(got.float(), ref.float()) < 8e-3
    else:
        got, pre = ops.panel_fwd(x, w, b, act=ACT_GELU, want_pre=True)
        ref, rpre = ops.linear_fwd(x, wb, b, BF16, act=ACT_GELU, want_pre=True)
        assert _rel(pre.float(), rpre.float()) < 8e-3 and _rel(got.float(), ref.float()) < 8e-3


@pytest.mark.parametrize("M,N,K", [(36008, 1536, 384), (300, 768, 128), (145, 1536, 384), (1, 384, 64)])
@pytest.mark.parametrize("epi", ["0", "1", "2"])
def test_panel_gelu_derivative_pair(M, N, K, epi, request):
    """fc1 with GELU' as its second output (act GELU_D: y = gelu(z), g = gelu'(z) from the f32 z =
    x W^T + b) and the fc2 dgrad that multiplies by it (ivit_linear_dgrad_mul_panel), vs torch on
    the same bf16 operands: z in f64, exact-erf GELU / GELU' (bf16-output tolerance); every
    epilogue form (IVIT_KNOB_WIDE_EPI 0: LDS tile, 1: transposed GELU_D, 2: transposed for both)."""
    _set_wide_epi(epi, request)
    import ops
    from _lib import ACT_GELU_D, BF16
    g = torch.Generator().manual_seed(7 * M + N + K)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV)
    b = (0.1 * torch.randn(N, generator=g)).to(DEV)
    y, gp = ops.panel_fwd(x, w, b, act=ACT_GELU_D, want_pre=True)
    z = x.double().cpu() @ w.to(torch.bfloat16).double().cpu().t() + b.double().cpu()
    phi = torch.exp(-0.5 * z * z) / math.sqrt(2 * math.pi)
    cdf = 0.5 * (1 + torch.erf(z / math.sqrt(2)))
    assert _rel(y.float().cpu(), z * cdf) < 8e-3
    assert _rel(gp.float().cpu(), cdf + z * phi) < 8e-3
    # the dgrad side: dx = (dy @ W2) * g
    dy = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    w2 = (torch.randn(K, N, generator=g) / math.sqrt(K)).to(DEV)
    dx = ops.panel_dgrad_mul(dy, w2, gp)
    ref = (dy.double().cpu() @ w2.to(torch.bfloat16).double().cpu()) * gp.double().cpu()
    assert _rel(dx.float().cpu(), ref) < 8e-3
    assert dx.shape == (M, N) and dx.dtype == torch.bfloat16


def test_patch_im2col_bitexact():
    """bf16 patch matrix (the throughput path's GEMM operand) is exactly the rearranged, rounded raster."""
    from _lib import lib, ptr, stream
    B, C, H, W = 2, 290, 16, 24
    img = torch.rand(B, C, H, W, device=DEV)
    Np = (H // 8) * (W // 8)
    cols = torch.empty((B * Np, C * 64), dtype=torch.bfloat16, device=DEV)
    assert lib.ivit_patch_im2col(ptr(img), B, C, H, W, ptr(cols), stream()) == 0
    ref = img.reshape(B, C, H // 8, 8, W // 8, 8).permute(0, 2, 4, 1, 3, 5).reshape(B * Np, C * 64)
    assert torch.equal(cols.cpu(), ref.to(torch.bfloat16).cpu())


@pytest.mark.parametrize("M,C", [(1000, 96), (2_200_007, 16)])
def test_batchnorm_train(M, C):
    """Training-mode BatchNorm forward / backward vs f64 torch; 2.2 M rows is past 32 x 65 535, where
    the partial-sum blocks grow to 64 rows (a full-grid B = 8 CNN map has 2.3 M)."""
    import ops
    x = torch.randn(M, C) * 3 + 1
    g, b = 1 + 0.1 * torch.randn(C), 0.1 * torch.randn(C)
    rm, rv = torch.zeros(C), torch.ones(C)
    rmd, rvd = rm.to(DEV).clone(), rv.to(DEV).clone()
    res = torch.randn(M, C)
    st = ops.bn_forward(x.to(DEV), g.to(DEV), b.to(DEV), rmd, rvd, True)
    y = ops.bn_apply(x.to(DEV), st, g.to(DEV), b.to(DEV), torch.float32, resid=res.to(DEV), relu=True)
    xr = x.double().requires_grad_(True)
    gr, br = g.double().requires_grad_(True), b.double().requires_grad_(True)
    rr = res.double().requires_grad_(True)
    rm2, rv2 = rm.double().clone(), rv.double().clone()
    ref = F.relu(F.batch_norm(xr, rm2, rv2, gr, br, training=True) + rr)
    assert _rel(y, ref.detach()) < 1e-5
    assert _rel(rmd, rm2) < 1e-5 and _rel(rvd, rv2) < 1e-5
    dy = torch.randn(M, C)
    ref.backward(dy.double())
    dx, dr, dg, db = ops.bn_backward(x.to(DEV), y, dy.to(DEV), st, g.to(DEV), True, torch.float32, want_dr=True)
    assert _rel(dx, xr.grad) < 1e-4 and _rel(dr, rr.grad) < 1e-5
    assert _rel(dg, gr.grad) < 1e-4 and _rel(db, br.grad) < 1e-5


def test_adamw_matches_torch():
    from optim import FusedAdamW
    ps = [torch.randn(1000), torch.randn(37, 5)]
    gs = [[torch.randn_like(p) for p in ps] for _ in range(3)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    dev = [p.clone().to(DEV).requires_grad_(True) for p in ps]
    o1 = torch.optim.AdamW(ref, lr=1e-3, weight_decay=1e-2)
    o2 = FusedAdamW(dev, lr=1e-3, weight_decay=1e-2)
    for step in gs:
        for p, q, g in zip(ref, dev, step):
            p.grad = g.clone()
            q.grad = g.clone().to(DEV)
        o1.step()
        o2.step()
    for p, q in zip(ref, dev):
        assert _rel(q.detach(), p.detach()) < 1e-6


@pytest.mark.parametrize("guard", ["host", "device"])
def test_adamw_chunked_bit_identical_to_guarded(guard):
    """ivit_adamw_chunked (FusedAdamW's launch: one workgroup per 4096-element chunk, 16-B
    accesses where allowed) against the 2D-grid ivit_adamw_guarded on the same state: bit-identical
    parameters, moments, bf16 shadows and step counts — tensors of several chunks with a ragged
    last one, ones smaller than a chunk, 4-B-offset (scalar-path) views, shadows present / absent,
    the host bias correction and the device step counts with finite = 1 and 0."""
    from _lib import lib, ptr, stream
    g0 = torch.Generator().manual_seed(3)
    flat = [torch.randn(4 * 20000 + 7, generator=g0) for _ in range(4)]  # p, g, m, v storage
    shapes = [(9000,), (4096,), (37, 5), (1,), (12289,), (384,)]
    offs = [0, 9004, 13100, 13287, 13289, 25580]  # 13289, 25580 % 4 == 1 / 0: scalar / vector
    sizes = [int(torch.tensor(sh).prod()) for sh in shapes]
    states = []
    for run in range(2):
        P, G, M, V = [f.clone().to(DEV) for f in flat]
        M.abs_().mul_(0.1)
        V.abs_().mul_(0.01)
        sh = [torch.zeros(n, dtype=torch.bfloat16, device=DEV) if i % 2 == 0 else None for i, n in enumerate(sizes)]
        views = [[T[o:o + n] for o, n in zip(offs, sizes)] for T in (P, G, M, V)]
        tab = [torch.tensor([v.data_ptr() for v in vs], dtype=torch.int64, device=DEV) for vs in views]
        tsh = torch.tensor([x.data_ptr() if x is not None else 0 for x in sh], dtype=torch.int64, device=DEV)
        tsz = torch.tensor(sizes, dtype=torch.int64, device=DEV)
        steps = [torch.tensor([3.0, 0.0, 7.0, 1.0, 2.0, 5.0], device=DEV), torch.empty(6, device=DEV)]
        for it, fin in enumerate((1.0, 0.0, 1.0)):
            finite = torch.tensor(fin, device=DEV)
            args_d = (ptr(finite), ptr(steps[it % 2]), ptr(steps[1 - it % 2])) if guard == "device" else \
                (ptr(finite), 0, 0)
            if run == 0:
                assert lib.ivit_adamw_guarded(6, *[ptr(t) for t in tab], ptr(tsh), ptr(tsz), max(sizes), 1e-2, 0.9,
                                              0.999, 1e-8, 1e-2, 0.271, 0.0447, *args_d, stream()) == 0
            else:
                ce = lib.ivit_adamw_chunk_elems()
                rec = [(t, c) for t, n in enumerate(sizes) for c in range(-(-n // ce))]
                ch = torch.tensor(rec, dtype=torch.int32, device=DEV)
                assert lib.ivit_adamw_chunked(6, *[ptr(t) for t in tab], ptr(tsh), ptr(tsz), ptr(ch), len(rec), 1e-2,
                                              0.9, 0.999, 1e-8, 1e-2, 0.271, 0.0447, *args_d, stream()) == 0
        torch.cuda.synchronize()
        states.append((P, M, V, [x for x in sh if x is not None], steps[1] if guard == "device" else None))
    (P0, M0, V0, S0, st0), (P1, M1, V1, S1, st1) = states
    assert torch.equal(P0, P1) and torch.equal(M0, M1) and torch.equal(V0, V1)
    assert all(torch.equal(a, b) for a, b in zip(S0, S1))
    assert not torch.equal(P0.cpu(), flat[0])  # the updates happened
    if st0 is not None:
        assert torch.equal(st0, st1)


def test_adamw_device_guard_skips_step_count():
    """The sync-free guard path (Trainer with check_nan=False: step(finite=flag)): a finite = 0
    update changes nothing — weights, moments AND step counts — so the following updates match
    torch.optim.AdamW with that step never taken (bias correction included)."""
    from optim import FusedAdamW
    ps = [torch.randn(1000), torch.randn(37, 5)]
    gs = [[torch.randn_like(p) for p in ps] for _ in range(4)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    dev = [p.clone().to(DEV).requires_grad_(True) for p in ps]
    o1 = torch.optim.AdamW(ref, lr=1e-3, weight_decay=1e-2)
    o2 = FusedAdamW(dev, lr=1e-3, weight_decay=1e-2)
    one, zero = torch.ones((), device=DEV), torch.zeros((), device=DEV)
    for k, step in enumerate(gs):
        skip = k == 1
        for p, q, g in zip(ref, dev, step):
            p.grad = None if skip else g.clone()
            q.grad = g.clone().to(DEV)
        if skip:
            before = [q.detach().clone() for q in dev]
            o2.step(finite=zero)
            assert all(torch.equal(q.detach(), b) for q, b in zip(dev, before))
        else:
            o1.step()
            o2.step(finite=one)
    for p, q in zip(ref, dev):
        assert float(o2.state[q]["step"]) == 3.0 and float(o1.state[p]["step"]) == 3.0
        assert _rel(q.detach(), p.detach()) < 1e-6
        assert _rel(o2.state[q]["exp_avg_sq"], o1.state[p]["exp_avg_sq"]) < 1e-6
    o2.step()  # the host path continues from the device counts
    assert all(o2.state[q]["step"] == 4 for q in dev)


def test_adamw_refreshes_bf16_weight_shadows():
    """ops.cast_weight's cached bf16 copy is rewritten by the AdamW launch (ivit_adamw_chunked),
    so after every step it equals bf16(p) exactly; a parameter without a shadow is unaffected."""
    import ops
    from optim import FusedAdamW
    ps = [torch.randn(1152, 384, device=DEV, requires_grad=True), torch.randn(300, device=DEV, requires_grad=True)]
    opt = FusedAdamW(ps, lr=1e-2, weight_decay=1e-2)
    sh = ops.cast_weight(ps[0], torch.bfloat16)
    assert ops.cast_weight(ps[0], torch.bfloat16) is sh
    for _ in range(3):
        for p in ps:
            p.grad = torch.randn_like(p)
        opt.step()
        assert ops.shadow_of(ps[0]) is sh
        assert torch.equal(sh, ps[0].detach().to(torch.bfloat16))
    assert ops.shadow_of(ps[1]) is None
    with torch.no_grad():
        ps[0].mul_(0.5)  # an in-place change outside the optimizer invalidates the shadow
    assert ops.shadow_of(ps[0]) is None
    assert torch.equal(ops.cast_weight(ps[0], torch.bfloat16), ps[0].detach().to(torch.bfloat16))


@pytest.mark.parametrize("M", [1, 33, 194, 4501, 36008])
def test_vit_block_wgrad_grouped(M):
    """ivit_vit_block_wgrad (the four weight + bias gradients of a bf16 timm Block in one grouped
    launch + reduce) vs f64 of the same bf16 operands: dW = dY^T X, db = colsum(dY), for
    M tokens incl. ragged last K steps and fewer tokens than splits; deterministic (two runs equal)."""
    import ops
    D, Hd = 384, 1536
    g = torch.Generator(device=DEV).manual_seed(M)
    mk = lambda c: torch.randn(M, c, device=DEV, generator=g).to(torch.bfloat16)
    ops_ = [mk(D), mk(Hd), mk(Hd), mk(D), mk(D), mk(D), mk(3 * D), mk(D)]
    got = ops.vit_block_wgrad(*ops_)
    again = ops.vit_block_wgrad(*ops_)
    for (dw, db), (dw2, db2) in zip(got, again):
        assert torch.equal(dw, dw2) and torch.equal(db, db2)
    for q, (dw, db) in enumerate(got):
        dy, x = ops_[2 * q].double(), ops_[2 * q + 1].double()
        rw, rb = dy.T @ x, dy.sum(0)
        assert dw.shape == rw.shape and db.shape == rb.shape
        ew = float((dw.double() - rw).norm() / rw.norm())
        eb = float((db.double() - rb).norm() / rb.norm())
        assert ew < 1e-5 and eb < 1e-5, (q, ew, eb)


def test_adamw_packs_unaligned_grads():
    """FusedAdamW (ivit_adamw_chunked + ivit_weight_pack_multi) on a packed weight whose gradient
    is a view at a 4-B (not 16-B) offset (a DDP bucket view): the same update as
    torch.optim.AdamW and packs equal to freshly built ones."""
    import ops
    from optim import FusedAdamW
    p = torch.randn(384, 1536, device=DEV, requires_grad=True)
    ref = p.detach().clone().requires_grad_(True)
    flat = torch.zeros(p.numel() + 1, device=DEV)
    p.grad = flat[1:].view_as(p)
    ops.packed_weight(p)
    ops.packed_weight_t(p)
    opt, topt = FusedAdamW([p], lr=1e-2, weight_decay=1e-2), torch.optim.AdamW([ref], lr=1e-2, weight_decay=1e-2)
    for _ in range(2):
        gr = torch.randn_like(p)
        p.grad.copy_(gr)
        ref.grad = gr.clone()
        opt.step()
        topt.step()
    assert (p.detach() - ref.detach()).abs().max().item() < 1e-5
    pk, pkt = ops.packs_of(p)
    fresh, fresh_t = torch.empty_like(pk), torch.empty_like(pkt)
    ops.lib.ivit_patch_weight_pack(ops.ptr(p.detach()), 384, 1536 // 64, ops.ptr(fresh), ops.stream())
    ops.lib.ivit_weight_pack_t(ops.ptr(p.detach()), 384, 1536, ops.ptr(fresh_t), ops.stream())
    assert torch.equal(pk, fresh) and torch.equal(pkt, fresh_t)


def test_geometry_golden():
    from conftest import golden
    import utils
    z = golden("geometry.npz")
    a = utils.generate_anchors(400, 720, 8)
    assert np.array_equal(a.cpu().numpy(), z["anchors"])
    out = utils.decode_box_predictions(torch.from_numpy(z["dec_rel"]).to(DEV),
                                       a[torch.from_numpy(z["dec_idx"]).to(DEV)])
    np.testing.assert_allclose(out.cpu().numpy(), z["dec_out"], rtol=1e-6, atol=1e-6)
    r = utils.compute_rotated_iou(torch.from_numpy(z["rot_b1"]).to(DEV), torch.from_numpy(z["rot_b2"]).to(DEV))
    np.testing.assert_allclose(r.cpu().numpy(), z["rot_iou"], atol=1e-6)
    gt0 = torch.from_numpy(z["gt0_boxes"]).to(DEV)
    iou = utils.compute_axis_aligned_iou(a, gt0)
    mx, arg = iou.max(dim=1)
    assert np.array_equal(mx.cpu().numpy(), z["iou_max"])


def test_nms_bitexact_golden():
    from conftest import golden
    import utils
    z = golden("geometry.npz")
    for i in range(int(z["nms_cases"][0])):
        keep = utils.apply_nms(torch.from_numpy(z[f"nms{i}_boxes"]).to(DEV), torch.from_numpy(z[f"nms{i}_scores"]).to(DEV),
                               0.2)
        assert np.array_equal(keep.cpu().numpy(), z[f"nms{i}_keep"]), i


def test_nms_batched_equals_per_sample_golden_and_oracle():
    """ivit_nms_batched: all golden NMS cases (full 22 500, heavy ties, all-equal scores,
    IoU == 0.2f, empty) plus random ragged sets in ONE batch, each bit-exact."""
    from conftest import golden
    from oracle import ivit_oracle as O
    import utils
    z = golden("geometry.npz")
    bl, sl, want = [], [], []
    for i in range(int(z["nms_cases"][0])):
        bl.append(torch.from_numpy(z[f"nms{i}_boxes"]).to(DEV))
        sl.append(torch.from_numpy(z[f"nms{i}_scores"]).to(DEV))
        want.append(z[f"nms{i}_keep"])
    g = torch.Generator().manual_seed(9)
    for n in (1, 65, 700, 4097):
        b = torch.stack([10 * torch.rand(n, generator=g), 10 * torch.rand(n, generator=g),
                         0.5 + 2 * torch.rand(n, generator=g), 0.5 + 2 * torch.rand(n, generator=g),
                         torch.zeros(n)], 1)
        s = torch.round(torch.rand(n, generator=g) * 8) / 8
        bl.append(b.to(DEV))
        sl.append(s.to(DEV))
        want.append(O.nms_numpy(b.numpy(), s.numpy(), 0.2))
    keeps = utils.nms_batched(bl, sl, 0.2)
    for i, (k, w) in enumerate(zip(keeps, want)):
        assert np.array_equal(k.cpu().numpy(), w), i


@pytest.mark.parametrize("thr", [0.2, 0.0, -0.5])
def test_nms_random_vs_oracle(thr):
    """Single-sample and batched NMS vs the oracle; thr <= 0 takes the exact IoU path for disjoint
    boxes too (the kernel skips the division only when it cannot change the decision)."""
    from oracle import ivit_oracle as O
    import utils
    g = torch.Generator().manual_seed(3)
    bl, sl, want = [], [], []
    for n in (1, 63, 64, 65, 500, 4097):
        b = torch.stack([10 * torch.rand(n, generator=g), 10 * torch.rand(n, generator=g),
                         0.5 + 2 * torch.rand(n, generator=g), 0.5 + 2 * torch.rand(n, generator=g),
                         torch.zeros(n)], 1)
        s = torch.round(torch.rand(n, generator=g) * 8) / 8
        keep = utils.apply_nms(b.to(DEV), s.to(DEV), thr).cpu().numpy()
        ref = O.nms_numpy(b.numpy(), s.numpy(), thr)
        assert np.array_equal(keep, ref), n
        bl.append(b.to(DEV))
        sl.append(s.to(DEV))
        want.append(ref)
    for i, (k, w) in enumerate(zip(utils.nms_batched(bl, sl, thr), want)):
        assert np.array_equal(k.cpu().numpy(), w), i


def test_nms_past_the_held_words_and_many_kept_per_column():
    """n = 26 000 (407 mask words: the scan's later-word update past its two held words per thread)
    with dense overlaps and scores in descending blocks, so columns keep more than 8 boxes (the
    update's synchronous path): keep indices bit-exact vs the oracle, single and batched."""
    from oracle import ivit_oracle as O
    import utils
    g = torch.Generator().manual_seed(17)
    n = 26000
    b = torch.stack([60 * torch.rand(n, generator=g), 60 * torch.rand(n, generator=g),
                     0.3 + 1.5 * torch.rand(n, generator=g), 0.3 + 1.5 * torch.rand(n, generator=g),
                     torch.zeros(n)], 1)
    s = torch.round(torch.rand(n, generator=g) * 64) / 64
    ref = O.nms_numpy(b.numpy(), s.numpy(), 0.2)
    assert len(ref) > 700  # many columns keep more than 8
    assert np.array_equal(utils.apply_nms(b.to(DEV), s.to(DEV), 0.2).cpu().numpy(), ref)
    k = utils.nms_batched([b.to(DEV), b[:5000].to(DEV)], [s.to(DEV), s[:5000].to(DEV)], 0.2)
    assert np.array_equal(k[0].cpu().numpy(), ref)
    assert np.array_equal(k[1].cpu().numpy(), O.nms_numpy(b[:5000].numpy(), s[:5000].numpy(), 0.2))


def test_nms_huge_areas_take_the_exact_division():
    """Boxes with areas near FLT_MAX / 4 (decoded boxes with a huge exp(dw)): the union is >= 2^126,
    where rcp(u) would be subnormal, so the fast IoU test must defer to the exact division — keep
    indices bit-exact vs the oracle, single and batched."""
    from oracle import ivit_oracle as O
    import utils
    g = torch.Generator().manual_seed(21)
    n = 300
    side = 1.0e19  # area 1e38 ~ FLT_MAX / 3.4: the union of two such boxes is past 2^126 (8.5e37)
    cx = torch.rand(n, generator=g) * side * 2
    cy = torch.rand(n, generator=g) * side * 2
    w = side * (0.5 + torch.rand(n, generator=g))
    h = side * (0.5 + torch.rand(n, generator=g)) * 0.7
    b = torch.stack([cx, cy, w, h, torch.zeros(n)], 1).float()
    s = torch.round(torch.rand(n, generator=g) * 16) / 16
    for thr in (0.2, 0.05, 0.5):
        ref = O.nms_numpy(b.numpy(), s.numpy(), thr)
        assert np.array_equal(utils.apply_nms(b.to(DEV), s.to(DEV), thr).cpu().numpy(), ref), thr
        k = utils.nms_batched([b.to(DEV), b[:100].to(DEV)], [s.to(DEV), s[:100].to(DEV)], thr)
        assert np.array_equal(k[0].cpu().numpy(), ref)
        assert np.array_equal(k[1].cpu().numpy(), O.nms_numpy(b[:100].numpy(), s[:100].numpy(), thr))


def test_standalone_activation_and_head_modules():
    """Module forwards outside the fused path run the device kernels too: nn.GELU / nn.ReLU
    (ivit_act_fwd / _bwd) and the det / intention heads' 35 / 40-channel 3x3 convs (im2col +
    GEMM; heads.py:18-25,39-43 view / permute) vs torch f32 references."""
    import heads
    import layers
    x = torch.randn(3, 5, 7, 11)
    for mod, ref in ((layers.GELU(), torch.nn.functional.gelu), (layers.ReLU(), torch.relu)):
        xd = x.to(DEV).requires_grad_(True)
        y = mod(xd)
        y.backward(torch.ones_like(y))
        xr = x.clone().requires_grad_(True)
        yr = ref(xr)
        yr.backward(torch.ones_like(yr))
        assert _rel(y.detach(), yr.detach()) < 1e-6 and _rel(xd.grad, xr.grad) < 1e-6
    f = torch.randn(2, 64, 6, 9)
    dh = heads.DetectionHead(64).to(DEV)
    ih = heads.IntentionHead(64).to(DEV)
    c, b = dh(f.to(DEV))
    it = ih(f.to(DEV))
    w = {k: v.detach().cpu() for k, v in dh.state_dict().items()}
    o = torch.nn.functional.conv2d(f, w["conv.weight"], w["conv.bias"], padding=1)
    o = o.view(2, 5, 7, 6, 9).permute(0, 3, 4, 1, 2)
    assert c.shape == (2, 6, 9, 5) and b.shape == (2, 6, 9, 5, 6)
    assert _rel(c, o[..., 0]) < 1e-5 and _rel(b, o[..., 1:]) < 1e-5
    wi = {k: v.detach().cpu() for k, v in ih.state_dict().items()}
    oi = torch.nn.functional.conv2d(f, wi["conv.weight"], wi["conv.bias"], padding=1).view(2, 5, 8, 6, 9)
    assert _rel(it, oi.permute(0, 3, 4, 1, 2)) < 1e-5
