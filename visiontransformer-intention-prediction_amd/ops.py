"""Autograd layer over libivit_hip: every differentiable op of the IntentNetViT hot path
as a ``torch.autograd.Function`` whose forward and backward launch only the hand-written
HIP kernels (through the C ABI in ``include/ivit.h``). PyTorch is used for device memory,
streams and autograd plumbing; there is no eager/ATen fallback for the compute.

Granularity (fused for HBM traffic and launch count, coarse enough for DDP overlap):
  * ``PatchEmbedFn``  timm PatchEmbed + CLS + pos_embed            (model_vit.py:64,71 → timm)
  * ``ViTBlockFn``    one pre-norm transformer block                (timm Block, ×12 per stream)
  * ``NeckFn``        final norms + adapters + fusion BasicBlocks + heads
                      (model_vit.py:116-142, 179-185; heads.py)
  * ``DetLossFn``     DetectionIntentionLoss                        (loss.py:58-206)
plus single-op Functions used by the standalone module forwards.
"""
from __future__ import annotations

import ctypes

import torch
from torch.utils.weak import WeakIdKeyDictionary

from _lib import ACT_GELU, ACT_GELU_D, ACT_NONE, BF16, F32, KNOB_CONV_PANEL, dt, lib, ptr, stream, tdtype, workspace


def _code(dtype):
    return BF16 if dtype == torch.bfloat16 else F32


def cast(x, dtype):
    if x.dtype == dtype:
        return x
    y = torch.empty(x.shape, dtype=dtype, device=x.device)
    lib.ivit_cast(ptr(x), dt(x), ptr(y), dt(y), x.numel(), stream())
    return y


# Compute-dtype (bf16) copies of f32 parameters, kept across steps: FusedAdamW refreshes them in
# its own launch (ivit_adamw_chunked) when it updates the parameter, so a training step casts no
# weights. Any other in-place change of a parameter bumps its version counter and re-casts.
_SHADOWS = WeakIdKeyDictionary()


def cast_weight(w, dtype):
    """cast(w, dtype) for a parameter, cached across steps (see _SHADOWS)."""
    if w.dtype == dtype or not w.is_cuda or not w.is_contiguous():
        return cast(w, dtype)
    e = _SHADOWS.get(w)
    if e is not None and e[0] == w._version and e[1].dtype == dtype and e[1].shape == w.shape:
        return e[1]
    y = cast(w, dtype)
    _SHADOWS[w] = (w._version, y)
    return y


_PACKED = WeakIdKeyDictionary()


def packed_weight(w):
    """A [D, K] weight (PatchEmbed [D, C, 8, 8]: K = 64 C) f32 in the row-panel kernels' MFMA
    fragment order (bf16), rebuilt when the parameter changes (keyed by its version counter,
    like cast_weight)."""
    e = _PACKED.get(w)
    if e is not None and e[0] == w._version:
        return e[1]
    D, C = w.shape[0], w[0].numel() // 64
    wp = torch.empty(lib.ivit_patch_weight_pack_bytes(D, C) // 2, dtype=torch.bfloat16, device=w.device)
    lib.ivit_patch_weight_pack(ptr(w.float().contiguous()), D, C, ptr(wp), stream())
    _PACKED[w] = (w._version, wp)
    return wp


_PACKED_T = WeakIdKeyDictionary()


def packed_weight_t(w):
    """A [K, N] weight used as a dgrad operand (fc1 / qkv weights [out, in] with in = N) packed as
    its transpose in the row-panel fragment order, cached per parameter version."""
    e = _PACKED_T.get(w)
    if e is not None and e[0] == w._version:
        return e[1]
    K, N = w.shape
    wp = torch.empty(lib.ivit_patch_weight_pack_bytes(N, K // 64) // 2, dtype=torch.bfloat16, device=w.device)
    lib.ivit_weight_pack_t(ptr(w.float().contiguous()), K, N, ptr(wp), stream())
    _PACKED_T[w] = (w._version, wp)
    return wp


def shadow_of(p):
    """The live bf16 shadow of parameter p (None if there is none or it is stale)."""
    e = _SHADOWS.get(p)
    if e is None or e[0] != p._version or e[1].dtype != torch.bfloat16 or e[1].shape != p.shape:
        return None
    return e[1]


def packs_of(p):
    """(pack, transposed pack) of parameter p that are live (built at its current version), or
    None each. FusedAdamW rewrites them in its update launch (ivit_adamw_chunked): its pointer-table
    update does not move the version counter, so without that the packs would stay at the
    weights they were built from."""
    e, et = _PACKED.get(p), _PACKED_T.get(p)
    return (e[1] if e is not None and e[0] == p._version else None,
            et[1] if et is not None and et[0] == p._version else None)


# ------------------------------------------------------------------------------ primitives
def linear_fwd(x, w, b, cdt, act=ACT_NONE, out_dtype=None, want_pre=False, resid=None, row_scale=None, rps=1,
               out=None, pre=None):
    """x [M, K] (cdt), w [N, K] (cdt) → act(x w^T + b); resid → f32 residual form."""
    M, K = x.shape[0], x.shape[-1]
    N = w.shape[0]
    if resid is not None:
        out = torch.empty((M, N), dtype=torch.float32, device=x.device) if out is None else out
        lib.ivit_linear_fwd(cdt, ptr(x), x.stride(0), ptr(w), ptr(b), M, N, K, ACT_NONE, ptr(out), out.stride(0), F32,
                            None, ptr(resid), resid.stride(0), ptr(row_scale), rps, stream())
        return out, None
    od = tdtype(cdt) if out_dtype is None else out_dtype
    out = torch.empty((M, N), dtype=od, device=x.device) if out is None else out
    if want_pre and pre is None:
        pre = torch.empty((M, N), dtype=od, device=x.device)
    assert pre is None or pre.stride(0) == out.stride(0)
    lib.ivit_linear_fwd(cdt, ptr(x), x.stride(0), ptr(w), ptr(b), M, N, K, act, ptr(out), out.stride(0), dt(out),
                        ptr(pre), None, 0, None, 0, stream())
    return out, pre


def linear_dgrad(dy, w, cdt, out_dtype, gelu_pre=None, out=None):
    M, N = dy.shape[0], dy.shape[-1]
    K = w.shape[1]
    out = torch.empty((M, K), dtype=out_dtype, device=dy.device) if out is None else out
    lib.ivit_linear_dgrad(cdt, ptr(dy), dy.stride(0), ptr(w), M, N, K, ptr(out), out.stride(0), dt(out),
                          ptr(gelu_pre), gelu_pre.stride(0) if gelu_pre is not None else 0, stream())
    return out


def linear_wgrad(dy, x, cdt, want_bias=True):
    M, N = dy.shape[0], dy.shape[-1]
    K = x.shape[-1]
    dw = torch.empty((N, K), dtype=torch.float32, device=dy.device)
    db = torch.empty((N,), dtype=torch.float32, device=dy.device) if want_bias else None
    ws = workspace(lib.ivit_linear_wgrad_workspace(M, N, K), dy.device)
    lib.ivit_linear_wgrad(cdt, ptr(dy), dy.stride(0), ptr(x), x.stride(0), M, N, K, ptr(dw), ptr(db), 0, ptr(ws),
                          ws.numel(), stream())
    return dw, db


def vit_block_wgrad(dy2, a, dh, x2, dyp, o, dyq, x1, outs=None):
    """The four weight + bias gradients of one bf16 timm Block (fc2, fc1, proj, qkv) in one grouped
    launch + one reduce (ivit_vit_block_wgrad): dW = dY^T X, db = colsum(dY) for
    (dY, X) = (dx2s, a), (dh, ln2), (dx1s, o), (dqkv, ln1). -> [(dW, db)] * 4. ``outs``: the eight
    contiguous f32 destinations (dW2, db2, dW1, db1, dWp, dbp, dWq, dbq), e.g. gradient-bucket views."""
    M, D = dy2.shape
    Hd = a.shape[1]
    dev = dy2.device
    shapes = ((D, Hd), (Hd, D), (D, D), (3 * D, D))
    if outs is not None:
        dws, dbs = list(outs[0::2]), list(outs[1::2])
        assert all(t.is_contiguous() and t.dtype == torch.float32 and tuple(t.shape) == sh
                   for t, sh in zip(dws, shapes))
    else:
        dws = [torch.empty(sh, dtype=torch.float32, device=dev) for sh in shapes]
        dbs = [torch.empty((sh[0],), dtype=torch.float32, device=dev) for sh in shapes]
    ws = workspace(lib.ivit_vit_block_wgrad_workspace(M, D, Hd), dev)
    lib.ivit_vit_block_wgrad(M, D, Hd, ptr(dy2), ptr(a), ptr(dh), ptr(x2), ptr(dyp), ptr(o), ptr(dyq), ptr(x1),
                             ptr(dws[0]), ptr(dbs[0]), ptr(dws[1]), ptr(dbs[1]), ptr(dws[2]), ptr(dbs[2]), ptr(dws[3]),
                             ptr(dbs[3]), ptr(ws), ws.numel(), stream())
    return list(zip(dws, dbs))


def layernorm_fwd(x, g, b, eps, out_dtype, rowmap=(0, 0, 0), M=None):
    D = x.shape[-1]
    M = x.shape[0] if M is None else M
    y = torch.empty((M, D), dtype=out_dtype, device=x.device)
    mean = torch.empty((M,), dtype=torch.float32, device=x.device)
    rstd = torch.empty((M,), dtype=torch.float32, device=x.device)
    lib.ivit_layernorm_fwd(ptr(x), x.stride(0), rowmap[0], rowmap[1], rowmap[2], M, D, ptr(g), ptr(b), eps, ptr(y),
                           D, dt(y), ptr(mean), ptr(rstd), stream())
    return y, mean, rstd


def linear_resid_ln_fwd(a, w, b, resid, row_scale, rps, g, beta, eps):
    """bf16 a [M, K] @ w[384, K]^T + b, times row_scale[m / rps], plus the f32 residual → x (f32),
    then LayerNorm(x) → y (bf16), mean, rstd: one kernel (ivit_linear_resid_ln_fwd)."""
    M, K = a.shape
    N = w.shape[0]
    x = torch.empty((M, N), dtype=torch.float32, device=a.device)
    y = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    mean = torch.empty((M,), dtype=torch.float32, device=a.device)
    rstd = torch.empty((M,), dtype=torch.float32, device=a.device)
    lib.ivit_linear_resid_ln_fwd(ptr(a), a.stride(0), M, N, K, ptr(packed_weight(w)), ptr(b), ptr(resid),
                                 resid.stride(0), ptr(row_scale), rps, ptr(g), ptr(beta), eps, ptr(x), N, ptr(y), N,
                                 ptr(mean), ptr(rstd), stream())
    return x, y, mean, rstd


def linear_dgrad_ln_bwd(dy, w, x, g, mean, rstd, dres=None, dx=None, xs_dtype=None, row_scale=None, rps=1,
                        dg=None, db=None):
    """dgrad G = dy [M, K] (bf16) @ w [K, 384] with the LayerNorm backward of (x, g, mean, rstd) in
    the epilogue: dx = dres + LN_bwd(G) (f32, may alias dres), optional bf16 dxs = dx * row_scale,
    dgamma, dbeta (into ``dg`` / ``db`` when given) — one kernel + the column reduction
    (ivit_linear_dgrad_ln_bwd)."""
    M, K = dy.shape
    N = w.shape[1]
    if dx is None:
        dx = torch.empty((M, N), dtype=torch.float32, device=dy.device) if dres is None else dres
    dxs = torch.empty((M, N), dtype=xs_dtype, device=dy.device) if xs_dtype is not None else None
    dg = torch.empty((N,), dtype=torch.float32, device=dy.device) if dg is None else dg
    db = torch.empty((N,), dtype=torch.float32, device=dy.device) if db is None else db
    ws = workspace(lib.ivit_linear_dgrad_ln_bwd_workspace(M, N), dy.device)
    lib.ivit_linear_dgrad_ln_bwd(ptr(dy), dy.stride(0), M, N, K, ptr(packed_weight_t(w)), ptr(x), x.stride(0), ptr(g),
                                 ptr(mean), ptr(rstd), ptr(dres), dres.stride(0) if dres is not None else N, ptr(dx),
                                 dx.stride(0), ptr(dxs), ptr(row_scale), rps, ptr(dg), ptr(db), 0, ptr(ws),
                                 ws.numel(), stream())
    return dx, dxs, dg, db


def layernorm_bwd(x, g, mean, rstd, dy, dres=None, dx=None, xs_dtype=None, row_scale=None, rps=1, rowmap=(0, 0, 0)):
    M, D = dy.shape[0], dy.shape[-1]
    if dx is None:
        dx = torch.empty_like(x, dtype=torch.float32) if dres is None else dres
    dxs = torch.empty((M, D), dtype=xs_dtype, device=dy.device) if xs_dtype is not None else None
    dg = torch.empty((D,), dtype=torch.float32, device=dy.device)
    db = torch.empty((D,), dtype=torch.float32, device=dy.device)
    ws = workspace(lib.ivit_layernorm_bwd_workspace(M, D), dy.device)
    lib.ivit_layernorm_bwd(ptr(x), x.stride(0), rowmap[0], rowmap[1], rowmap[2], M, D, ptr(g), ptr(mean), ptr(rstd),
                           ptr(dy), dy.stride(0), dt(dy), ptr(dres), ptr(dx), dx.stride(0), ptr(dxs),
                           dt(dxs) if dxs is not None else F32, ptr(row_scale), rps, ptr(dg), ptr(db), 0, ptr(ws),
                           ws.numel(), stream())
    return dx, dxs, dg, db


class KernelTimer:
    """Optional HIP-event bracketing of selected C-ABI launches on the current stream
    (bench.py uses it to measure the roofline kernel's average duration in the timed loop)."""
    enabled = set()
    records = {}

    @classmethod
    def span(cls, name):
        """Record a start event on the CURRENT stream (the one the launch goes to) and return
        the end event for the caller to record after the launch; None when not enabled."""
        if name not in cls.enabled:
            return None
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        cls.records.setdefault(name, []).append((s, e))
        return e

    @classmethod
    def mean_ms(cls, name):
        r = cls.records.get(name, [])
        return sum(s.elapsed_time(e) for s, e in r) / len(r) if r else float("nan")

    @classmethod
    def count(cls, name):
        return len(cls.records.get(name, []))


KT_ATTN_FWD, KT_ATTN_BWD_DQ, KT_ATTN_BWD_DKV = 0, 1, 2


def ktime_arm(on):
    """Start (clearing earlier records) / stop kernel-execution timing of the attention entry
    points (ivit_ktime_arm: event pairs bound to the kernel commands themselves)."""
    lib.ivit_ktime_arm(1 if on else 0)


def ktime_read(tag):
    """-> [(start_ms, stop_ms), ...] of every recorded kernel of one IVIT_KT_* tag since the
    last arm, relative to the first recorded launch's start (common to all tags)."""
    n = ctypes.c_long(0)
    lib.ivit_ktime_read(tag, None, None, 0, ctypes.addressof(n))
    if n.value == 0:
        return []
    t0, t1 = (ctypes.c_double * n.value)(), (ctypes.c_double * n.value)()
    lib.ivit_ktime_read(tag, ctypes.addressof(t0), ctypes.addressof(t1), n.value, ctypes.addressof(n))
    return list(zip(t0, t1))


def busy_ms(intervals):
    """Length of the union of [start, stop) intervals (time at least one of them was running)."""
    tot, end = 0.0, None
    for a, b in sorted(intervals):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def bilinear_fwd(x, size):
    """F.interpolate(x, size, mode='bilinear', align_corners=False) of an f32 (B, C, Hi, Wi) map
    (ivit_bilinear_fwd; model_vit.py:139)."""
    B, C, Hi, Wi = x.shape
    Ho, Wo = size
    x = x.contiguous()
    y = torch.empty((B, C, Ho, Wo), dtype=torch.float32, device=x.device)
    lib.ivit_bilinear_fwd(ptr(x), B * C, Hi, Wi, ptr(y), Ho, Wo, stream())
    return y


def bilinear_bwd(dy, in_size):
    """Adjoint of bilinear_fwd (ivit_bilinear_bwd): dX (B, C, Hi, Wi) from dY (B, C, Ho, Wo)."""
    B, C, Ho, Wo = dy.shape
    Hi, Wi = in_size
    dy = dy.contiguous()
    dx = torch.empty((B, C, Hi, Wi), dtype=torch.float32, device=dy.device)
    lib.ivit_bilinear_bwd(ptr(dy), B * C, Hi, Wi, Ho, Wo, ptr(dx), stream())
    return dx


class BilinearFn(torch.autograd.Function):
    """The map features re-gridded onto the LiDAR grid when the two patch grids differ
    (model_vit.py:139: F.interpolate(..., mode='bilinear', align_corners=False))."""

    @staticmethod
    def forward(ctx, x, size):
        ctx.in_size = tuple(x.shape[2:])
        return bilinear_fwd(x.float(), size)

    @staticmethod
    def backward(ctx, dy):
        return bilinear_bwd(dy.float(), ctx.in_size), None


def attn_fwd(qkv, B, N, H, cdt):
    D = H * 64
    out = torch.empty((B * N, D), dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty((B, H, N), dtype=torch.float32, device=qkv.device)
    ws = workspace(lib.ivit_attn_workspace(cdt, B, N, H, 64, 0), qkv.device)
    ev = KernelTimer.span("attn_fwd")
    lib.ivit_attn_fwd(cdt, ptr(qkv), B, N, H, 64, ptr(out), ptr(lse), ptr(ws), ws.numel(), stream())
    if ev is not None:
        ev.record()
    return out, lse


# bf16 ViT blocks: the qkv projection writes its Q block as q * log2(e)/sqrt(64)
# (ivit_linear_fwd_qs) and attention runs on the prescaled Q (ivit_attn_fwd_q2 / _bwd_q2):
# no per-score scaling FMA in the forward and dQ kernels. The f32 parity path keeps the plain
# layout (ivit_attn_fwd / _bwd).
Q2_SCALE = 1.4426950408889634 / 8.0  # log2(e) / sqrt(Dh), Dh = 64


def qkv_fwd_q2(x, w, b, D):
    """x w^T + b with columns < D (the Q block) multiplied by Q2_SCALE; bf16 out."""
    M, K = x.shape[0], x.shape[-1]
    N = w.shape[0]
    out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    lib.ivit_linear_fwd_qs(BF16, ptr(x), x.stride(0), ptr(w), ptr(b), M, N, K, ptr(out), out.stride(0), BF16, D,
                           Q2_SCALE, stream())
    return out


def panel_fwd(x, w, b, act=ACT_NONE, want_pre=False, qcols=0, qscale=1.0):
    """Row-panel form of a wide bf16 token GEMM (ivit_linear_fwd_panel): x [M, K] bf16 @ w [N, K]
    (f32 master, packed) + b; act GELU with the pre-activation copy (act GELU_D: with GELU' of the
    pre-activation instead, what the backward needs), or columns < qcols scaled."""
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    pre = torch.empty((M, N), dtype=torch.bfloat16, device=x.device) if want_pre else None
    lib.ivit_linear_fwd_panel(ptr(x), x.stride(0), M, N, K, ptr(packed_weight(w)), ptr(b), act, qcols, qscale,
                              ptr(y), N, ptr(pre), N, stream())
    return y, pre


def panel_dgrad(dy, w):
    """dy [M, K] bf16 @ w [K, N] (f32 master [out, in], packed transposed) → bf16 [M, N]: the plain
    dgrad through the row-panel kernel (ivit_linear_fwd_panel on the transposed pack)."""
    M, K = dy.shape
    N = w.shape[1]
    dx = torch.empty((M, N), dtype=torch.bfloat16, device=dy.device)
    lib.ivit_linear_fwd_panel(ptr(dy), dy.stride(0), M, N, K, ptr(packed_weight_t(w)), None, ACT_NONE, 0, 1.0,
                              ptr(dx), N, None, 0, stream())
    return dx


def panel_dgrad_mul(dy, w, g):
    """dy [M, K] bf16 @ w [K, N] (f32 master, packed transposed) * g → bf16 [M, N], g = the GELU'
    panel_fwd(act=ACT_GELU_D) wrote (ivit_linear_dgrad_mul_panel: fc2 dgrad into fc1's pre-activation
    with no GELU' evaluation)."""
    M, K = dy.shape
    N = w.shape[1]
    dx = torch.empty((M, N), dtype=torch.bfloat16, device=dy.device)
    lib.ivit_linear_dgrad_mul_panel(ptr(dy), dy.stride(0), M, N, K, ptr(packed_weight_t(w)), ptr(g), g.stride(0),
                                    ptr(dx), N, stream())
    return dx


def panel_dgrad_gelu(dy, w, pre):
    """dy [M, K] bf16 @ w [K, N] (f32 master, packed transposed) * gelu'(pre) → bf16 [M, N]
    (ivit_linear_dgrad_gelu_panel: fc2 dgrad into fc1's pre-activation)."""
    M, K = dy.shape
    N = w.shape[1]
    dx = torch.empty((M, N), dtype=torch.bfloat16, device=dy.device)
    lib.ivit_linear_dgrad_gelu_panel(ptr(dy), dy.stride(0), M, N, K, ptr(packed_weight_t(w)), ptr(pre),
                                     pre.stride(0), ptr(dx), N, stream())
    return dx


def attn_fwd_q2(qkv, B, N, H):
    D = H * 64
    out = torch.empty((B * N, D), dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty((B, H, N), dtype=torch.float32, device=qkv.device)
    ev = KernelTimer.span("attn_fwd")
    lib.ivit_attn_fwd_q2(ptr(qkv), B, N, H, 64, ptr(out), ptr(lse), None, 0, stream())
    if ev is not None:
        ev.record()
    return out, lse


def attn_bwd_q2(qkv, out, dout, lse, B, N, H):
    dqkv = torch.empty_like(qkv)
    ws = workspace(lib.ivit_attn_workspace(BF16, B, N, H, 64, 1), qkv.device)
    ev = KernelTimer.span("attn_bwd")
    lib.ivit_attn_bwd_q2(ptr(qkv), ptr(out), ptr(dout), ptr(lse), B, N, H, 64, ptr(dqkv), ptr(ws), ws.numel(),
                         stream())
    if ev is not None:
        ev.record()
    return dqkv


def attn_bwd(qkv, out, dout, lse, B, N, H, cdt):
    dqkv = torch.empty_like(qkv)
    ws = workspace(lib.ivit_attn_workspace(cdt, B, N, H, 64, 1), qkv.device)
    lib.ivit_attn_bwd(cdt, ptr(qkv), ptr(out), ptr(dout), ptr(lse), B, N, H, 64, ptr(dqkv), ptr(ws), ws.numel(),
                      stream())
    return dqkv


def add_act_grad(a, b=None, pre=None, row_scale=None, row_elems=1, out_dtype=None):
    out = torch.empty(a.shape, dtype=out_dtype or a.dtype, device=a.device)
    lib.ivit_add_act_grad(ptr(a), dt(a), ptr(b), dt(b) if b is not None else F32, ptr(pre),
                          dt(pre) if pre is not None else F32, ptr(row_scale), row_elems, ptr(out), dt(out),
                          a.numel(), stream())
    return out


def pack_conv(w, cdt, cout_pad=None):
    Cout, Cin, k, _ = w.shape
    cp = Cout if cout_pad is None else cout_pad
    out = torch.empty((cp, k, k, Cin), dtype=tdtype(cdt), device=w.device)
    lib.ivit_pack_conv_weight(cdt, ptr(w), Cout, Cin, k, cp, ptr(out), stream())
    return out


def pack_conv_pair(w0, w1, cdt, cout_pad):
    """pack_conv of torch.cat([w0, w1], 0) without the concatenation: w0's rows, then w1's rows
    zero-padded to cout_pad (two ivit_pack_conv_weight launches into one buffer)."""
    C0, Cin, k, _ = w0.shape
    C1 = w1.shape[0]
    out = torch.empty((cout_pad, k, k, Cin), dtype=tdtype(cdt), device=w0.device)
    lib.ivit_pack_conv_weight(cdt, ptr(w0), C0, Cin, k, C0, ptr(out), stream())
    lib.ivit_pack_conv_weight(cdt, ptr(w1), C1, Cin, k, cout_pad - C0, ptr(out[C0:]), stream())
    return out


def unpack_conv_grad(gp, Cout, Cin, k):
    out = torch.empty((Cout, Cin, k, k), dtype=torch.float32, device=gp.device)
    lib.ivit_unpack_conv_grad(ptr(gp), Cout, Cin, k, ptr(out), 0, stream())
    return out


def conv_fwd(x, B, H, W, wp, bias, cdt, out_dtype):
    Cout, k, _, Cin = wp.shape
    y = torch.empty((B * H * W, Cout), dtype=out_dtype, device=x.device)
    lib.ivit_conv_fwd(cdt, ptr(x), B, H, W, Cin, ptr(wp), ptr(bias), Cout, k, ptr(y), Cout, dt(y), stream())
    return y


def conv_panel_enabled():
    """The stride-1 bf16 convolutions on the panel kernels (ivit_get_knob(IVIT_KNOB_CONV_PANEL))."""
    return lib.ivit_get_knob(KNOB_CONV_PANEL) != 0


def pack_conv_t(w, cdt, cout_pad=None):
    """torch [Cout][Cin][k][k] -> the data gradient's K-contiguous weight [Cin][k][k][Cout_pad], taps
    flipped, zero for channels >= Cout."""
    Cout, Cin, k, _ = w.shape
    cp = Cout if cout_pad is None else cout_pad
    out = torch.empty((Cin, k, k, cp), dtype=tdtype(cdt), device=w.device)
    lib.ivit_pack_conv_weight_t(cdt, ptr(w), Cout, Cin, k, cp, ptr(out), stream())
    return out


def conv_bn_fwd(x, B, H, W, wp, cdt, out_dtype, rmean, rvar, training, momentum=0.1, eps=1e-5, nbt=None):
    """conv (no bias) and the following BatchNorm2d's statistics: in training the batch statistics
    come out of the convolution's epilogue (ivit_conv_bn_fwd; BasicBlock conv -> bn,
    model_vit.py:24-27,35-43), in eval the running ones. -> (y, _BNState)."""
    if not training:
        y = conv_fwd(x, B, H, W, wp, None, cdt, out_dtype)
        return y, bn_forward(y, None, None, rmean, rvar, False, momentum, eps)
    Cout, k, _, Cin = wp.shape
    y = torch.empty((B * H * W, Cout), dtype=out_dtype, device=x.device)
    mean = torch.empty((Cout,), dtype=torch.float32, device=x.device)
    invstd = torch.empty_like(mean)
    ws = workspace(lib.ivit_conv_bn_fwd_workspace(B, H, W, Cout), x.device)
    lib.ivit_conv_bn_fwd(cdt, ptr(x), B, H, W, Cin, ptr(wp), Cout, k, ptr(y), Cout, dt(y), ptr(mean), ptr(invstd),
                         ptr(rmean), ptr(rvar), momentum, eps, ptr(ws), ws.numel(), stream())
    if nbt is not None:
        nbt.add_(1)
    return y, _BNState(mean, invstd)


def conv_dgrad(dy, B, H, W, wp, cdt, out_dtype, w=None, dy_zero_pad=False):
    """dX of a stride-1 'same' conv. With the f32 weight `w` (torch layout) and a bf16 shape the
    288 x 256 panel kernel takes (ivit_conv_dgrad_t: Cout % 64, Cin >= 128, >= 288 pixels), the
    tap-flipped transposed pack is built and the panel kernel runs; otherwise the 128 x 128 engine
    on the forward pack `wp`. dy_zero_pad: dy's rows hold zeros from channel w.shape[0] up to its
    row stride, so the panel kernel may run on the channel count rounded up to 64 (the pack's extra
    channels are zero too)."""
    Cout, k, _, Cin = wp.shape
    dx = torch.empty((B * H * W, Cin), dtype=out_dtype, device=dy.device)
    if w is not None and cdt == BF16 and conv_panel_enabled():
        Cw = w.shape[0]
        cpad = (Cw + 63) // 64 * 64 if dy_zero_pad else Cw
        if (cpad % 64 == 0 and cpad <= dy.stride(0) and Cw <= Cout and Cin >= 128 and Cin % 8 == 0
                and B * H * W >= 288 and dy.stride(0) % 8 == 0):
            wt = pack_conv_t(w, cdt, cout_pad=cpad)
            lib.ivit_conv_dgrad_t(cdt, ptr(dy), dy.stride(0), B, H, W, cpad, ptr(wt), Cin, k, ptr(dx), dt(dx),
                                  stream())
            return dx
    lib.ivit_conv_dgrad(cdt, ptr(dy), dy.stride(0), B, H, W, Cout, ptr(wp), Cin, k, ptr(dx), dt(dx), stream())
    return dx


def conv_wgrad(dy, x, B, H, W, Cin, Cout, k, cdt, want_bias=False):
    gp = torch.empty((Cout, k, k, Cin), dtype=torch.float32, device=dy.device)
    db = torch.empty((Cout,), dtype=torch.float32, device=dy.device) if want_bias else None
    ws = workspace(lib.ivit_conv_wgrad_workspace(B, H, W, Cin, Cout, k), dy.device)
    lib.ivit_conv_wgrad(cdt, ptr(dy), dy.stride(0), ptr(x), B, H, W, Cin, Cout, k, ptr(gp), ptr(db), 0, ptr(ws),
                        ws.numel(), stream())
    return gp, db


class _BNState:
    """Per-forward BatchNorm statistics (batch stats in train, running stats in eval)."""

    def __init__(self, mean, invstd):
        self.mean, self.invstd = mean, invstd


def bn_forward(x, g, b, rmean, rvar, training, momentum=0.1, eps=1e-5, nbt=None):
    M, C = x.shape
    if training:
        mean = torch.empty((C,), dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        ws = workspace(lib.ivit_bn_workspace(M, C), x.device)
        lib.ivit_bn_stats(ptr(x), dt(x), M, C, ptr(mean), ptr(invstd), ptr(rmean), ptr(rvar), momentum, eps, ptr(ws),
                          ws.numel(), stream())
        if nbt is not None:
            nbt.add_(1)
    else:
        mean = torch.empty((C,), dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        lib.ivit_bn_eval_stats(ptr(rmean), ptr(rvar), C, eps, ptr(mean), ptr(invstd), stream())
    return _BNState(mean, invstd)


def bn_apply(x, st, g, b, out_dtype, resid=None, relu=False):
    M, C = x.shape
    y = torch.empty((M, C), dtype=out_dtype, device=x.device)
    if resid is not None:
        assert resid.dtype == out_dtype
    lib.ivit_bn_apply(ptr(x), dt(x), M, C, ptr(st.mean), ptr(st.invstd), ptr(g), ptr(b), ptr(resid), int(relu), ptr(y),
                      dt(y), stream())
    return y


def bn_backward(x, y, dy, st, g, relu, out_dtype, want_dr=False):
    M, C = x.shape
    dx = torch.empty((M, C), dtype=out_dtype, device=x.device)
    dr = torch.empty((M, C), dtype=out_dtype, device=x.device) if want_dr else None
    dg = torch.empty((C,), dtype=torch.float32, device=x.device)
    db = torch.empty_like(dg)
    ws = workspace(lib.ivit_bn_workspace(M, C), x.device)
    lib.ivit_bn_bwd(ptr(x), dt(x), ptr(y), dt(y), ptr(dy), dt(dy), M, C, ptr(st.mean), ptr(st.invstd), ptr(g),
                    int(relu), ptr(dx), dt(dx), ptr(dr), ptr(dg), ptr(db), 0, ptr(ws), ws.numel(), stream())
    return dx, dr, dg, db


# ------------------------------------------------------------------------------ fused Functions
class PatchEmbedFn(torch.autograd.Function):
    """timm PatchEmbed(Conv2d k=s=8, bias) → flatten/transpose → cat(CLS) → +pos_embed.
    img (B, C, H, W) f32 → tokens (B*(Np+1), D) f32. No input gradient (the BEV raster)."""

    @staticmethod
    def forward(ctx, img, w, b, pos, cls, cdt, hand=None):
        B, C, H, W = img.shape
        D = w.shape[0]
        P = w.shape[-1]
        # hand (GradHandoff): block 0's qkv-dgrad + norm1-backward epilogue also writes bf16(dtok),
        # the weight gradient's operand, so the backward skips its own cast pass over dtok
        ctx.hand = hand
        if hand is not None:
            hand.scale, hand.g, hand.key = None, None, None
        if P != 8:
            # other patch sizes (timm vit_*_patch16_224 at model_vit.py:64,71): patch matrix in the
            # compute dtype, the linear GEMM, then the CLS / pos_embed assembly (ivit_patch_*)
            Np = (H // P) * (W // P)
            cols = torch.empty((B * Np, C * P * P), dtype=tdtype(cdt), device=img.device)
            lib.ivit_patch_im2col_p(ptr(img), B, C, H, W, P, ptr(cols), cdt, stream())
            y, _ = linear_fwd(cols, cast_weight(w, tdtype(cdt)).reshape(D, C * P * P), b, cdt,
                              out_dtype=torch.float32)
            out = torch.empty((B * (Np + 1), D), dtype=torch.float32, device=img.device)
            lib.ivit_patch_tokens(ptr(y), B, Np, D, ptr(pos), ptr(cls), ptr(out), stream())
            ctx.save_for_backward(cols)
            ctx.meta = (B, C, H, W, D, cdt, w.shape)
            ctx.generic = True
            return out
        ctx.generic = False
        Ntok = (H // 8) * (W // 8) + 1
        wc = cast_weight(w, tdtype(cdt)).reshape(D, C * 64)
        out = torch.empty((B * Ntok, D), dtype=torch.float32, device=img.device)
        if cdt == BF16 and (D == 384 or (D == 192 and not ctx.needs_input_grad[1])) and img.data_ptr() % 16 == 0:
            # bf16: fused forward, the raster streamed through LDS once (no patch matrix); the
            # weight gradient re-reads the raster (ivit_patch_embed_wgrad: D = 384 kernel)
            wp = packed_weight(w)
            lib.ivit_patch_embed_fwd_packed(ptr(img), B, C, H, W, ptr(wp), ptr(b), ptr(pos), ptr(cls), D, ptr(out),
                                            stream())
            ctx.save_for_backward(img)
            ctx.cols = False
        elif cdt == BF16:
            # bf16, other widths: one coalesced pass writes the bf16 patch matrix; forward and
            # weight gradient stream it by LDS-DMA (saved for backward instead of the f32 raster)
            cols = torch.empty((B * (Ntok - 1), C * 64), dtype=torch.bfloat16, device=img.device)
            lib.ivit_patch_im2col(ptr(img), B, C, H, W, ptr(cols), stream())
            lib.ivit_patch_embed_fwd_cols(ptr(cols), B, C, H, W, ptr(wc), ptr(b), ptr(pos), ptr(cls), D, ptr(out),
                                          stream())
            ctx.save_for_backward(cols)
            ctx.cols = True
        else:
            lib.ivit_patch_embed_fwd(cdt, ptr(img), B, C, H, W, ptr(wc), ptr(b), ptr(pos), ptr(cls), D, ptr(out),
                                     stream())
            ctx.save_for_backward(img)
            ctx.cols = False
        ctx.meta = (B, C, H, W, D, cdt, w.shape)
        return out

    @staticmethod
    def backward(ctx, dtok):
        (src,) = ctx.saved_tensors
        B, C, H, W, D, cdt, wshape = ctx.meta
        if ctx.generic:
            P = wshape[-1]
            Np = (H // P) * (W // P)
            dtok = dtok.contiguous()
            dy = torch.empty((B * Np, D), dtype=tdtype(cdt), device=src.device)
            dpos = torch.empty((1, Np + 1, D), dtype=torch.float32, device=src.device)
            dcls = torch.empty((1, 1, D), dtype=torch.float32, device=src.device)
            lib.ivit_patch_tokens_bwd(ptr(dtok), dt(dtok), B, Np, D, ptr(dy), cdt, ptr(dpos), ptr(dcls), 0, stream())
            dw, db = linear_wgrad(dy, src, cdt)
            return None, dw.reshape(wshape), db, dpos, dcls, None, None
        hd = ctx.hand
        if hd is not None and hd.g is not None and hd.g.dtype == tdtype(cdt) and hd.key == GradHandoff.ident(dtok):
            dtok = hd.g  # written by block 0's backward (unmodified dtok: same tensor and version)
            GradHandoff.used += 1
        else:
            dtok = cast(dtok.contiguous(), tdtype(cdt))
        if hd is not None:
            hd.g = hd.key = None
        Ntok = (H // 8) * (W // 8) + 1
        dw = torch.empty(wshape, dtype=torch.float32, device=src.device)
        db = torch.empty((D,), dtype=torch.float32, device=src.device)
        dpos = torch.empty((1, Ntok, D), dtype=torch.float32, device=src.device)
        dcls = torch.empty((1, 1, D), dtype=torch.float32, device=src.device)
        ws = workspace(lib.ivit_patch_embed_wgrad_workspace(B, C, H, W, D), src.device)
        if ctx.cols:
            lib.ivit_patch_embed_wgrad_cols(ptr(dtok), ptr(src), B, C, H, W, D, ptr(dw), ptr(db), ptr(dpos),
                                            ptr(dcls), 0, ptr(ws), ws.numel(), stream())
        else:
            lib.ivit_patch_embed_wgrad(cdt, ptr(dtok), ptr(src), B, C, H, W, D, ptr(dw), ptr(db), ptr(dpos),
                                       ptr(dcls), 0, ptr(ws), ws.numel(), stream())
        return None, dw, db, dpos, dcls, None, None


class GradHandoff:
    """Backward hand-off between consecutive fused ViT blocks: block i+1's qkv-dgrad + norm1-backward
    kernel also writes bf16(dx * s2_i) — block i's DropPath-scaled MLP-branch gradient, the fc2
    dgrad's operand — so block i skips that separate scale-and-cast pass over dx. `scale` is set
    by block i's forward; `g` / `key` by block i+1's backward; block i uses `g` only if the
    gradient it receives is that very tensor, unmodified — same TensorImpl, data pointer and
    version counter (a hook that edits it in place bumps the version; a different tensor at a
    reused address has another TensorImpl) — else it recomputes it."""
    __slots__ = ("scale", "g", "key")
    used = 0  # hand-offs taken (tests)

    def __init__(self):
        self.scale, self.g, self.key = None, None, None

    @staticmethod
    def ident(t):
        return (t._cdata, t.data_ptr(), t._version)


def grad_sinks(params):
    """Destinations for writing these parameters' gradients directly (ddp.GradSink: gradient-bucket
    views, freshly zeroed this step), or None when any parameter has none — the op then returns its
    gradients to autograd as usual."""
    sinks = [getattr(p, "_ivit_sink", None) for p in params]
    if any(sk is None for sk in sinks):
        return None
    views = [sk.claim() for sk in sinks]
    if any(v is None for v in views):
        return None
    return sinks, views


class ViTBlockFn(torch.autograd.Function):
    """timm Block: x + dp1(proj(attn(norm1 x))); x + dp2(fc2(gelu(fc1(norm2 x)))).
    x: (B*N, D) f32 residual stream; GEMM operands in the compute dtype (f32 or bf16).

    bf16 row-panel fusion (D = 384): the proj GEMM's epilogue also applies norm2, and — when
    the NEXT block's norm1 parameters are passed (nxw, nxb) — the fc2 GEMM's epilogue applies
    that norm1 too and returns (y, mean, rstd) as extra, non-differentiable outputs. The next
    block takes them as (ln_in, m_in, r_in) instead of running its norm1 and still does that
    LayerNorm's backward itself (from its input x and the handed-over statistics), exactly as
    in the unfused block. Without fusion the extra outputs are empty tensors."""

    @staticmethod
    def forward(ctx, x, ln_in, m_in, r_in, n1w, n1b, qkvw, qkvb, pw, pb, n2w, n2b, f1w, f1b, f2w, f2b, nxw, nxb,
                s1, s2, meta, hand_mine=None, hand_prev=None):
        B, N, H, cdt, eps = meta
        cd = tdtype(cdt)
        q2 = cdt == BF16
        panel = q2 and x.shape[1] == 384
        if panel:  # row-panel kernels read the packed weights
            wq = wp = w1 = w2 = None
        else:
            wq, wp, w1, w2 = cast_weight(qkvw, cd), cast_weight(pw, cd), cast_weight(f1w, cd), cast_weight(f2w, cd)
        if ln_in is None:
            ln1, m1, r1 = layernorm_fwd(x, n1w, n1b, eps, cd)
        else:
            ln1, m1, r1 = ln_in, m_in, r_in
        if panel:
            qkv, _ = panel_fwd(ln1, qkvw, qkvb, qcols=H * 64, qscale=Q2_SCALE)
            o, lse = attn_fwd_q2(qkv, B, N, H)
        elif q2:
            qkv = qkv_fwd_q2(ln1, wq, qkvb, H * 64)
            o, lse = attn_fwd_q2(qkv, B, N, H)
        else:
            qkv, _ = linear_fwd(ln1, wq, qkvb, cdt)
            o, lse = attn_fwd(qkv, B, N, H, cdt)
        if panel:
            x1, ln2, m2, r2 = linear_resid_ln_fwd(o, pw, pb, x, s1, N, n2w, n2b, eps)
        else:
            x1, _ = linear_fwd(o, wp, pb, cdt, resid=x, row_scale=s1, rps=N)
            ln2, m2, r2 = layernorm_fwd(x1, n2w, n2b, eps, cd)
        # inference (torch.inference_mode): nothing is saved, and fc1 skips its pre-activation copy
        infer = torch.is_inference_mode_enabled()
        if panel:
            # training: h = GELU'(fc1 pre-activation) for the fc2 dgrad (panel_dgrad_mul), computed
            # beside GELU from the f32 pre-activation instead of re-evaluated in the backward
            a, h = panel_fwd(ln2, f1w, f1b, act=ACT_GELU if infer else ACT_GELU_D, want_pre=not infer)
        else:
            a, h = linear_fwd(ln2, w1, f1b, cdt, act=ACT_GELU, want_pre=not infer)
        if nxw is not None and panel:
            x2, lnx, mx, rx = linear_resid_ln_fwd(a, f2w, f2b, x1, s2, N, nxw, nxb, eps)
        elif panel:
            # the last block: the same row-panel residual GEMM (its LayerNorm epilogue on unit
            # parameters, outputs discarded) instead of the 128 x 128 engine's EpiResid GEMM
            g1, b0 = _unit_ln_params(x.shape[1], x.device)
            x2 = linear_resid_ln_fwd(a, f2w, f2b, x1, s2, N, g1, b0, eps)[0]
            lnx = mx = rx = x2.new_empty(0)
        else:
            x2, _ = linear_fwd(a, w2, f2b, cdt, resid=x1, row_scale=s2, rps=N)
            lnx = mx = rx = x2.new_empty(0)
        ctx.mark_non_differentiable(lnx, mx, rx)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the three extra outputs
        if infer:
            ctx.meta, ctx.q2 = meta, q2
            return x2, lnx, mx, rx
        ctx.save_for_backward(x, ln1, qkv, o, lse, x1, ln2, h, a, m1, r1, m2, r2, n1w, n2w, wq, wp, w1, w2, s1, s2,
                              qkvw, f1w, f2w, pw)
        ctx.meta = meta
        ctx.q2 = q2
        ctx.panel = panel
        # the parameters themselves (not saved tensors): their gradient-bucket sinks, if any
        ctx.params = (n1w, n1b, qkvw, qkvb, pw, pb, n2w, n2b, f1w, f1b, f2w, f2b)
        ctx.hand_mine, ctx.hand_prev = (hand_mine, hand_prev) if panel else (None, None)
        if ctx.hand_mine is not None:
            ctx.hand_mine.scale, ctx.hand_mine.g, ctx.hand_mine.key = s2, None, None
        return x2, lnx, mx, rx

    @staticmethod
    def backward(ctx, dx2, *_unused):
        (x, ln1, qkv, o, lse, x1, ln2, h, a, m1, r1, m2, r2, n1w, n2w, wq, wp, w1, w2, s1, s2, qkvw,
         f1w, f2w, pw) = ctx.saved_tensors
        B, N, H, cdt, eps = ctx.meta
        cd = tdtype(cdt)
        dx2 = torch.zeros_like(x) if dx2 is None else dx2.contiguous()
        D = x.shape[1]
        hm, hp = ctx.hand_mine, ctx.hand_prev
        dx2s = None
        if hm is not None:
            if hm.g is not None and dx2 is not None and hm.key == GradHandoff.ident(dx2):
                dx2s = hm.g  # written by the next block's qkv-dgrad epilogue
                GradHandoff.used += 1
            hm.g = hm.key = None
        if dx2s is None:
            dx2s = add_act_grad(dx2, row_scale=s2, row_elems=N * D, out_dtype=cd)
        dh = panel_dgrad_mul(dx2s, f2w, h) if ctx.panel else linear_dgrad(dx2s, w2, cdt, cd, gelu_pre=h)
        # bf16 row-panel blocks: the four weight gradients in one grouped launch after the dgrads
        # (ivit_vit_block_wgrad) instead of four split-K engine GEMMs (-1.5 ms per step, round 3)
        group = ctx.panel
        # DDP: the twelve parameter gradients straight into their bucket views (no autograd add)
        direct = grad_sinks(ctx.params) if group else None
        dv = direct[1] if direct is not None else [None] * 12
        g2 = None if group else linear_wgrad(dx2s, a, cdt)
        if ctx.panel:  # fc1 dgrad with norm2's backward in the epilogue
            dx1, dx1s, dg2, dbe2 = linear_dgrad_ln_bwd(dh, f1w, x1, n2w, m2, r2, dres=dx2, dx=torch.empty_like(dx2),
                                                       xs_dtype=cd, row_scale=s1, rps=N, dg=dv[6], db=dv[7])
        else:
            dln2 = linear_dgrad(dh, w1, cdt, torch.float32)
            dx1, dx1s, dg2, dbe2 = layernorm_bwd(x1, n2w, m2, r2, dln2, dres=dx2, dx=torch.empty_like(dx2),
                                                 xs_dtype=cd, row_scale=s1, rps=N)
        g1 = None if group else linear_wgrad(dh, ln2, cdt)
        do = panel_dgrad(dx1s, pw) if ctx.panel else linear_dgrad(dx1s, wp, cdt, cd)
        gp = None if group else linear_wgrad(dx1s, o, cdt)
        dqkv = attn_bwd_q2(qkv, o, do, lse, B, N, H) if ctx.q2 else attn_bwd(qkv, o, do, lse, B, N, H, cdt)
        if ctx.panel:  # qkv dgrad with norm1's backward in the epilogue
            if hp is not None:  # also the previous block's bf16(dx0 * s2) (GradHandoff)
                dx0, dx0s, dg1, dbe1 = linear_dgrad_ln_bwd(dqkv, qkvw, x, n1w, m1, r1, dres=dx1, dx=dx1, xs_dtype=cd,
                                                           row_scale=hp.scale, rps=N, dg=dv[0], db=dv[1])
                hp.g, hp.key = dx0s, GradHandoff.ident(dx0)
            else:
                dx0, _, dg1, dbe1 = linear_dgrad_ln_bwd(dqkv, qkvw, x, n1w, m1, r1, dres=dx1, dx=dx1, dg=dv[0],
                                                        db=dv[1])
        else:
            dln1 = linear_dgrad(dqkv, wq, cdt, torch.float32)
            dx0, _, dg1, dbe1 = layernorm_bwd(x, n1w, m1, r1, dln1, dres=dx1, dx=dx1)
        if group:
            outs = None if direct is None else (dv[10], dv[11], dv[8], dv[9], dv[4], dv[5], dv[2], dv[3])
            g2, g1, gp, gq = vit_block_wgrad(dx2s, a, dh, ln2, dx1s, o, dqkv, ln1, outs=outs)
        else:
            gq = linear_wgrad(dqkv, ln1, cdt)
        if direct is not None:  # written into the buckets: nothing for autograd to accumulate
            for sk in direct[0]:
                sk.done()
            return (dx0,) + (None,) * 22
        (dW2, db2), (dW1, db1), (dWp, dbp), (dWq, dbq) = g2, g1, gp, gq
        return (dx0, None, None, None, dg1, dbe1, dWq, dbq, dWp, dbp, dg2, dbe2, dW1, db1, dW2, db2, None, None,
                None, None, None, None, None)


_UNIT_LN = {}


def _unit_ln_params(n, dev):
    """(ones, zeros) LayerNorm parameters of width n on dev, cached."""
    key = (n, str(dev))
    if key not in _UNIT_LN:
        _UNIT_LN[key] = (torch.ones(n, device=dev), torch.zeros(n, device=dev))
    return _UNIT_LN[key]


_ZEROS = {}


def _zeros(n, dev):
    """A cached all-zero f32 vector (never written)."""
    key = (n, str(dev))
    z = _ZEROS.get(key)
    if z is None:
        z = _ZEROS[key] = torch.zeros((n,), dtype=torch.float32, device=dev)
    return z


class NeckFn(torch.autograd.Function):
    """Everything after the ViT blocks (model_vit.py:116-142,179-185; heads.py):
    final ViT norm (eps 1e-6) → drop CLS → adapter LN(eps 1e-5) → Linear → GELU for each
    stream, concat to an NHWC (B, Hf, Wf, Cl+Cm) map, fusion BasicBlocks (conv3x3-BN-ReLU-
    conv3x3-BN + identity/1x1-BN, ReLU), then the det (A*7) + intention (A*K) 3x3 heads as
    one GEMM, split into (cls, box, intent)."""

    @staticmethod
    def forward(ctx, tl, tm, meta, *params):
        (B, Hf, Wf, cdt, training, A, K, layers, names) = meta
        P = dict(zip(names, params))
        cd = tdtype(cdt)
        Np = Hf * Wf
        Ntok = Np + 1
        M = B * Np
        dev = tl.device
        rm = (Np, Ntok, 1)
        saved = {}
        Cl = P["adapter_lidar.1.weight"].shape[0]
        Cm = P["adapter_map.1.weight"].shape[0]
        cat = torch.empty((M, Cl + Cm), dtype=cd, device=dev)
        pre = torch.empty((M, Cl + Cm), dtype=cd, device=dev)
        for s, t, c0, C in (("lidar", tl, 0, Cl), ("map", tm, Cl, Cm)):
            y, mf, rf = layernorm_fwd(t, P[f"vit_{s}.norm.weight"], P[f"vit_{s}.norm.bias"], 1e-6, torch.float32,
                                      rowmap=rm, M=M)
            z, ma, ra = layernorm_fwd(y, P[f"adapter_{s}.0.weight"], P[f"adapter_{s}.0.bias"], 1e-5, cd)
            wa = cast_weight(P[f"adapter_{s}.1.weight"], cd)
            linear_fwd(z, wa, P[f"adapter_{s}.1.bias"], cdt, act=ACT_GELU, out=cat[:, c0:c0 + C],
                       pre=pre[:, c0:c0 + C])
            saved[s] = (t, y, mf, rf, z, ma, ra, wa)
        x = cat
        bns = {}
        packs = {}
        acts = []
        nbts = []  # the BatchNorms' num_batches_tracked, advanced in one launch below
        for li in range(layers):
            p = f"fusion_block.{li}."
            w1 = pack_conv(P[p + "conv1.weight"], cdt)
            w2 = pack_conv(P[p + "conv2.weight"], cdt)
            c1, s1 = conv_bn_fwd(x, B, Hf, Wf, w1, cdt, torch.float32, P[p + "bn1.running_mean"],
                                 P[p + "bn1.running_var"], training)
            r1 = bn_apply(c1, s1, P[p + "bn1.weight"], P[p + "bn1.bias"], cd, relu=True)
            c2, s2 = conv_bn_fwd(r1, B, Hf, Wf, w2, cdt, torch.float32, P[p + "bn2.running_mean"],
                                 P[p + "bn2.running_var"], training)
            nbts += [P.get(p + "bn1.num_batches_tracked"), P.get(p + "bn2.num_batches_tracked")]
            if (p + "downsample.0.weight") in P:
                wd = pack_conv(P[p + "downsample.0.weight"], cdt)
                dd, sd = conv_bn_fwd(x, B, Hf, Wf, wd, cdt, torch.float32, P[p + "downsample.1.running_mean"],
                                     P[p + "downsample.1.running_var"], training)
                nbts.append(P.get(p + "downsample.1.num_batches_tracked"))
                idn = bn_apply(dd, sd, P[p + "downsample.1.weight"], P[p + "downsample.1.bias"], cd)
                bns[p + "ds"] = (dd, sd, idn)
                packs[p + "ds"] = wd
            else:
                idn = x
            out = bn_apply(c2, s2, P[p + "bn2.weight"], P[p + "bn2.bias"], cd, resid=idn, relu=True)
            acts.append((x, c1, s1, r1, c2, s2, out))
            packs[p + "1"], packs[p + "2"] = w1, w2
            x = out
        nbts = [t for t in nbts if t is not None]
        if training and nbts:  # BatchNorm2d's num_batches_tracked += 1 (model_vit.py:24-27 via torch)
            torch._foreach_add_(nbts, 1)
        if A == 0:  # backbone-only call (TwoStreamViTBackbone.forward): fused feature map
            ctx.st = (saved, cat, pre, acts, bns, packs, None, x, 0)
            ctx.meta, ctx.P = meta, P
            return (cast(x, torch.float32) if x.dtype != torch.float32 else x.clone(),)
        Cd, Ci = A * 7, A * K
        Cp = (Cd + Ci + 7) // 8 * 8
        wd_, wi_ = P["det_head.conv.weight"], P["intention_head.conv.weight"]
        wh = (wd_, wi_)  # both heads as one conv: packed into one [Cp][3][3][Cin] weight, rows Cd.. the intention head
        whp = pack_conv_pair(wd_, wi_, cdt, Cp)
        bh = torch.empty((Cp,), dtype=torch.float32, device=dev)
        bh[:Cd].copy_(P["det_head.conv.bias"])
        bh[Cd:Cd + Ci].copy_(P["intention_head.conv.bias"])
        bh[Cd + Ci:].copy_(_zeros(Cp - Cd - Ci, dev))
        hout = conv_fwd(x, B, Hf, Wf, whp, bh, cdt, torch.float32)
        cls = torch.empty((B, M // B * A, 1), dtype=torch.float32, device=dev)
        box = torch.empty((B, M // B * A, 6), dtype=torch.float32, device=dev)
        intent = torch.empty((B, M // B * A, K), dtype=torch.float32, device=dev)
        lib.ivit_split_heads(ptr(hout), Cp, M, A, K, ptr(cls), ptr(box), ptr(intent), stream())
        ctx.st = (saved, cat, pre, acts, bns, packs, (whp, wh), x, Cp)
        ctx.meta = meta
        ctx.P = P
        return cls, box, intent

    @staticmethod
    def backward(ctx, *gouts):
        (B, Hf, Wf, cdt, training, A, K, layers, names) = ctx.meta
        saved, cat, pre, acts, bns, packs, (whp, wh), x_last, Cp = ctx.st
        P = ctx.P
        cd = tdtype(cdt)
        Np = Hf * Wf
        M = B * Np
        dev = cat.device
        G = {}

        def cw(n_, dy_, x_, Cin_, Cout_, k_):
            # a fusion conv's weight gradient (+ unpack)
            gp_, _ = conv_wgrad(dy_, x_, B, Hf, Wf, Cin_, Cout_, k_, cdt)
            G[n_] = unpack_conv_grad(gp_, Cout_, Cin_, k_)

        if A == 0:
            dx = gouts[0].contiguous().float()
        else:
            dcls, dbox, dint = gouts
            # rows zero-padded to a multiple of 64 channels: the head conv's data gradient then runs
            # on the panel kernel; the weight gradient reads the first Cp
            Cq = (Cp + 63) // 64 * 64
            dh = torch.empty((M, Cq), dtype=cd, device=dev)
            lib.ivit_merge_heads_grad(ptr(dcls.contiguous()), ptr(dbox.contiguous()), ptr(dint.contiguous()), M, A,
                                      K, ptr(dh), Cq, dt(dh), stream())
            Cin = x_last.shape[1]
            Cd, Ci = A * 7, A * K

            def head_wgrad(dh, x_last):
                gp, dbh = conv_wgrad(dh, x_last, B, Hf, Wf, Cin, Cp, 3, cdt, want_bias=True)
                gw = unpack_conv_grad(gp, Cd + Ci, Cin, 3)
                return gw[:Cd], gw[Cd:], dbh[:Cd], dbh[Cd:Cd + Ci]  # views: no copy launches

            for n_, g_ in zip(("det_head.conv.weight", "intention_head.conv.weight", "det_head.conv.bias",
                               "intention_head.conv.bias"), head_wgrad(dh, x_last)):
                G[n_] = g_
            # the transposed pack of both heads' weights (the forward packs them without a concatenation)
            dx = conv_dgrad(dh, B, Hf, Wf, whp, cdt, torch.float32, w=torch.cat(wh, 0), dy_zero_pad=True)
        for li in reversed(range(layers)):
            p = f"fusion_block.{li}."
            x, c1, s1, r1, c2, s2, out = acts[li]
            has_ds = (p + "ds") in bns
            dc2, dres, G[p + "bn2.weight"], G[p + "bn2.bias"] = bn_backward(c2, out, dx, s2, P[p + "bn2.weight"], True,
                                                                            cd, want_dr=True)
            Cm_ = c2.shape[1]
            cw(p + "conv2.weight", dc2, r1, r1.shape[1], Cm_, 3)
            dr1 = conv_dgrad(dc2, B, Hf, Wf, packs[p + "2"], cdt, torch.float32, w=P[p + "conv2.weight"])
            dc1, _, G[p + "bn1.weight"], G[p + "bn1.bias"] = bn_backward(c1, r1, dr1, s1, P[p + "bn1.weight"], True, cd)
            cw(p + "conv1.weight", dc1, x, x.shape[1], Cm_, 3)
            dxa = conv_dgrad(dc1, B, Hf, Wf, packs[p + "1"], cdt, torch.float32, w=P[p + "conv1.weight"])
            if has_ds:
                dd, sd, idn = bns[p + "ds"]
                ddd, _, G[p + "downsample.1.weight"], G[p + "downsample.1.bias"] = bn_backward(
                    dd, idn, dres, sd, P[p + "downsample.1.weight"], False, cd)
                cw(p + "downsample.0.weight", ddd, x, x.shape[1], Cm_, 1)
                dxb = conv_dgrad(ddd, B, Hf, Wf, packs[p + "ds"], cdt, torch.float32,
                                 w=P[p + "downsample.0.weight"])
            else:
                dxb = dres
            if li == 0:
                # d(adapter pre-activation) = (dxa + dxb) * gelu'(pre)
                dx = add_act_grad(dxa, dxb, pre=pre, out_dtype=cd)
            else:
                dx = add_act_grad(dxa, dxb, out_dtype=torch.float32)
        dpre = dx
        Cl = P["adapter_lidar.1.weight"].shape[0]
        outs = {}
        for s, c0 in (("lidar", 0), ("map", Cl)):
            t, y, mf, rf, z, ma, ra, wa = saved[s]
            C = wa.shape[0]
            dp = dpre[:, c0:c0 + C]
            dz = linear_dgrad(dp, wa, cdt, torch.float32)
            G[f"adapter_{s}.1.weight"], G[f"adapter_{s}.1.bias"] = linear_wgrad(dp, z, cdt)
            dy, _, G[f"adapter_{s}.0.weight"], G[f"adapter_{s}.0.bias"] = layernorm_bwd(
                y, P[f"adapter_{s}.0.weight"], ma, ra, dz)
            dt_ = torch.empty_like(t)
            dt_.view(B, Np + 1, -1)[:, 0].zero_()  # CLS rows: the neck drops them (no gradient)
            _, _, G[f"vit_{s}.norm.weight"], G[f"vit_{s}.norm.bias"] = layernorm_bwd(
                t, P[f"vit_{s}.norm.weight"], mf, rf, dy, dx=dt_, rowmap=(Np, Np + 1, 1))
            outs[s] = dt_
        grads = [G.get(n) for n in names]
        del ctx.st, ctx.P
        return (outs["lidar"], outs["map"], None) + tuple(grads)


class DetLossFn(torch.autograd.Function):
    """DetectionIntentionLoss on device (loss.py:58-206). Returns the 16-float stats vector;
    element 5 is the loss (0 with no gradient when non-finite, loss.py:190-198); element 9 is
    the finite flag (1.0 / 0.0) the Trainer reads to skip backward + optimizer step."""

    @staticmethod
    def forward(ctx, cls, box, intent, anchors, gt, ngt, gint, keep, cfg):
        B, NA = cls.shape[0], cls.shape[1]
        K = intent.shape[-1]
        G = gt.shape[1]
        dev = cls.device
        stats = torch.zeros((16,), dtype=torch.float32, device=dev)
        ws = workspace(lib.ivit_det_loss_workspace(B, NA, G), dev)
        cls, box, intent = cls.contiguous(), box.contiguous(), intent.contiguous()
        lib.ivit_det_loss_fwd(ptr(cls), ptr(box), ptr(intent), ptr(anchors), B, NA, K, ptr(gt), ptr(ngt), ptr(gint), G,
                              ptr(keep), cfg["dominant_mask"], int(cfg["downsampling"]), ptr(cfg.get("class_w")),
                              cfg["pos_thr"], cfg["neg_thr"], cfg["alpha"], cfg["gamma"], cfg["beta"], cfg["w_cls"],
                              cfg["w_box"], cfg["w_int"], int(cfg["rotated"]), ptr(stats), ptr(ws), ws.numel(),
                              stream())
        ctx.save_for_backward(cls, box, intent, keep, stats, ws)
        ctx.cfg = cfg
        ctx.shape = (B, NA, K)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        loss = stats[5:6].clone().reshape(())
        return loss, stats

    @staticmethod
    def backward(ctx, gloss, _gstats):
        cls, box, intent, keep, stats, ws = ctx.saved_tensors
        B, NA, K = ctx.shape
        cfg = ctx.cfg
        if gloss is None:
            return None, None, None, None, None, None, None, None, None
        g = gloss.reshape(1).float().contiguous()
        dcls, dbox, dint = torch.empty_like(cls), torch.empty_like(box), torch.empty_like(intent)
        lib.ivit_det_loss_bwd(ptr(cls), ptr(box), ptr(intent), B, NA, K, ptr(keep), cfg["dominant_mask"],
                              int(cfg["downsampling"]), ptr(cfg.get("class_w")), cfg["alpha"], cfg["gamma"],
                              cfg["beta"], cfg["w_cls"], cfg["w_box"], cfg["w_int"], ptr(stats), ptr(g), ptr(dcls),
                              ptr(dbox), ptr(dint), ptr(ws), ws.numel(), stream())
        return dcls, dbox, dint, None, None, None, None, None, None
