"""Parameter-container modules with torch.nn-compatible names/shapes (so reference
checkpoints load) whose forwards run the ivit HIP kernels. The fused model path
(``model_vit.IntentNetViT.forward``) bypasses these per-module forwards and calls the fused
Functions in ``ops.py`` directly; these forwards serve standalone sub-module calls."""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

import ops
from _lib import ACT_GELU, ACT_NONE, ACT_RELU, BF16, F32, dt, lib, ptr, stream, tdtype


def _cdt(dtype):
    return BF16 if dtype == torch.bfloat16 else F32


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, cdt):
        shp = x.shape
        cd = torch.bfloat16 if cdt == BF16 else torch.float32
        x2 = ops.cast(x.reshape(-1, shp[-1]).contiguous(), cd)
        wc = ops.cast_weight(w, cd)
        y, _ = ops.linear_fwd(x2, wc, b, cdt, out_dtype=torch.float32)
        ctx.save_for_backward(x2, wc)
        ctx.cdt, ctx.shp = cdt, shp
        return y.reshape(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, wc = ctx.saved_tensors
        cd = torch.bfloat16 if ctx.cdt == BF16 else torch.float32
        d2 = ops.cast(dy.reshape(-1, dy.shape[-1]).contiguous(), cd)
        dx = ops.linear_dgrad(d2, wc, ctx.cdt, torch.float32)
        dw, db = ops.linear_wgrad(d2, x2, ctx.cdt)
        return dx.reshape(ctx.shp), dw, db, None


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, eps):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).float().contiguous()
        y, m, r = ops.layernorm_fwd(x2, g, b, eps, torch.float32)
        ctx.save_for_backward(x2, g, m, r)
        ctx.shp = shp
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, g, m, r = ctx.saved_tensors
        dx, _, dg, db = ops.layernorm_bwd(x2, g, m, r, dy.reshape(x2.shape).float().contiguous())
        return dx.reshape(ctx.shp), dg, db, None


class _Conv2dFn(torch.autograd.Function):
    """NCHW stride-1 same-padding conv through the NHWC implicit-GEMM kernels."""

    @staticmethod
    def forward(ctx, x, w, b, cdt):
        B, C, H, W = x.shape
        cd = torch.bfloat16 if cdt == BF16 else torch.float32
        xh = ops.cast(x.permute(0, 2, 3, 1).contiguous(), cd).reshape(B * H * W, C)
        wp = ops.pack_conv(w, cdt)
        y = ops.conv_fwd(xh, B, H, W, wp, b, cdt, torch.float32)
        ctx.save_for_backward(xh, wp)
        ctx.meta = (B, C, H, W, w.shape, cdt, b is not None)
        return y.reshape(B, H, W, -1).permute(0, 3, 1, 2).contiguous()

    @staticmethod
    def backward(ctx, dy):
        xh, wp = ctx.saved_tensors
        B, C, H, W, wshape, cdt, has_b = ctx.meta
        cd = torch.bfloat16 if cdt == BF16 else torch.float32
        Cout, k = wshape[0], wshape[2]
        dyh = ops.cast(dy.permute(0, 2, 3, 1).contiguous(), cd).reshape(B * H * W, Cout)
        dx = ops.conv_dgrad(dyh, B, H, W, wp, cdt, torch.float32)
        gp, db = ops.conv_wgrad(dyh, xh, B, H, W, C, Cout, k, cdt, want_bias=has_b)
        dw = ops.unpack_conv_grad(gp, Cout, C, k)
        return dx.reshape(B, H, W, C).permute(0, 3, 1, 2).contiguous(), dw, db, None


class _ConvColsFn(torch.autograd.Function):
    """NHWC conv, any k / stride / zero pad (nn.Conv2d geometry): im2col + GEMM. The GEMM's K
    (k*k*Cin) and N (Cout) are padded to multiples of 8 with zero columns / rows."""

    @staticmethod
    def forward(ctx, x, w, b, s, p, cdt):
        B, H, W, C = x.shape
        Cout, Cin, k, _ = w.shape
        if Cin != C:
            raise ValueError(f"conv expects {Cin} input channels, got {C}")
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        K = k * k * C
        Kp, Np = _r8(K), _r8(Cout)
        x = x.contiguous()
        cols = torch.empty((B * Ho * Wo, Kp), dtype=tdtype(cdt), device=x.device)
        lib.ivit_im2col(dt(x), ptr(x), B, H, W, C, k, s, p, Ho, Wo, ptr(cols), Kp, cdt, stream())
        wp = ops.pack_conv(w, cdt, cout_pad=Np).reshape(Np, K)
        if Kp != K:
            wp = F.pad(wp, (0, Kp - K))
        wp = wp.contiguous()
        bp = None if b is None else (b if Np == Cout else F.pad(b, (0, Np - Cout))).contiguous()
        y, _ = ops.linear_fwd(cols, wp, bp, cdt, out_dtype=torch.float32)
        ctx.save_for_backward(cols, wp)
        ctx.meta = (B, H, W, C, Cout, k, s, p, Ho, Wo, K, Kp, Np, cdt, b is not None)
        y = y.view(B, Ho, Wo, Np)
        return y if Np == Cout else y[..., :Cout].contiguous()

    @staticmethod
    def backward(ctx, dy):
        cols, wp = ctx.saved_tensors
        B, H, W, C, Cout, k, s, p, Ho, Wo, K, Kp, Np, cdt, has_b = ctx.meta
        dy = dy.contiguous()
        if Np != Cout:
            dy = F.pad(dy, (0, Np - Cout))
        d2 = ops.cast(dy.reshape(B * Ho * Wo, Np).contiguous(), tdtype(cdt))
        dx = None
        if ctx.needs_input_grad[0]:
            dcols = ops.linear_dgrad(d2, wp, cdt, torch.float32)
            dx = torch.empty((B, H, W, C), dtype=torch.float32, device=dy.device)
            lib.ivit_col2im(ptr(dcols), Kp, B, H, W, C, k, s, p, Ho, Wo, ptr(dx), stream())
        dw2, db = ops.linear_wgrad(d2, cols, cdt, want_bias=has_b)
        dw = ops.unpack_conv_grad(dw2[:Cout, :K].contiguous(), Cout, C, k)
        return dx, dw, (db[:Cout] if has_b else None), None, None, None


def _r8(n):
    return (n + 7) // 8 * 8


class _ActFn(torch.autograd.Function):
    """Standalone nn.GELU (exact erf) / nn.ReLU on the device (ivit_act_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, x, act):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        lib.ivit_act_fwd(act, ptr(xc), dt(xc), ptr(y), dt(y), xc.numel(), stream())
        ctx.save_for_backward(xc)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        lib.ivit_act_bwd(ctx.act, ptr(dy), dt(dy), ptr(x), dt(x), ptr(dx), dt(dx), x.numel(), stream())
        return dx, None


class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, rm, rv, nbt, training, momentum, eps, relu, resid):
        B, C, H, W = x.shape
        xh = x.permute(0, 2, 3, 1).contiguous().reshape(-1, C).float()
        st = ops.bn_forward(xh, g, b, rm, rv, training, momentum, eps, nbt=nbt if training else None)
        rh = None if resid is None else resid.permute(0, 2, 3, 1).contiguous().reshape(-1, C).float()
        y = ops.bn_apply(xh, st, g, b, torch.float32, resid=rh, relu=relu)
        ctx.save_for_backward(xh, y, g)
        ctx.st, ctx.meta = st, (B, C, H, W, relu, resid is not None)
        return y.reshape(B, H, W, C).permute(0, 3, 1, 2).contiguous()

    @staticmethod
    def backward(ctx, dy):
        xh, y, g = ctx.saved_tensors
        B, C, H, W, relu, has_r = ctx.meta
        dyh = dy.permute(0, 2, 3, 1).contiguous().reshape(-1, C).float()
        dx, dr, dg, db = ops.bn_backward(xh, y, dyh, ctx.st, g, relu, torch.float32, want_dr=has_r)

        def back(t):
            return None if t is None else t.reshape(B, H, W, C).permute(0, 3, 1, 2).contiguous()
        return back(dx), dg, db, None, None, None, None, None, None, None, back(dr)


class Linear(nn.Module):
    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None
        nn.init.trunc_normal_(self.weight, std=0.02)

    def forward(self, x):
        return _LinearFn.apply(x, self.weight, self.bias, _cdt(getattr(self, "compute_dtype", torch.float32)))


class LayerNorm(nn.Module):
    def __init__(self, dim, eps=1e-5):
        super().__init__()
        self.normalized_shape, self.eps = (dim,), eps
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))

    def forward(self, x):
        return _LayerNormFn.apply(x, self.weight, self.bias, self.eps)


class Conv2d(nn.Module):
    """Conv2d parameter container (k x k, stride s, padding p). Standalone forward (NCHW, as
    nn.Conv2d): stride-1 'same' convolutions with channel counts % 8 on the implicit-GEMM conv
    kernels, everything else (strided, odd channel counts, e.g. the 35 / 40-channel heads) as
    im2col + GEMM."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = (kernel_size, kernel_size), (stride, stride), (padding, padding)
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, kernel_size, kernel_size))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(in_channels * kernel_size * kernel_size)
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        k, s_, p = self.kernel_size[0], self.stride[0], self.padding[0]
        cdt = _cdt(getattr(self, "compute_dtype", torch.float32))
        if s_ == 1 and p == k // 2 and k in (1, 3, 5) and self.in_channels % 8 == 0 and self.out_channels % 8 == 0:
            return _Conv2dFn.apply(x, self.weight, self.bias, cdt)
        y = _ConvColsFn.apply(x.permute(0, 2, 3, 1).float().contiguous(), self.weight, self.bias, s_, p, cdt)
        return y.permute(0, 3, 1, 2).contiguous()


class BatchNorm2d(nn.Module):
    def __init__(self, num_features, eps=1e-5, momentum=0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def forward(self, x, relu=False, resid=None):
        return _BatchNormFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                                  self.num_batches_tracked, self.training, self.momentum, self.eps, relu, resid)


class GELU(nn.Module):
    """nn.GELU (exact erf). In the fused path it is the adapter GEMM epilogue; standalone it runs
    ivit_act_fwd."""

    def forward(self, x):
        return _ActFn.apply(x, ACT_GELU)


class ReLU(nn.Module):
    def __init__(self, inplace=False):
        super().__init__()

    def forward(self, x):
        return _ActFn.apply(x, ACT_RELU)
