"""IntentNetCNN — the reference's CNN variant (model_cnn.py) on the ivit
kernels. Same classes, constructor kwargs, attribute and state-dict names as the reference
(model_cnn.py:7-150), so its checkpoints load and train_cnn.py / eval_cnn.py-style callers work.

Stride-1 'same' convolutions (the 5x5 convs of every block after the first, the fusion 3x3s)
run on the implicit-GEMM conv kernels (``ivit_conv_fwd`` / ``_dgrad`` / ``_wgrad``); the strided
ones (stride-2 5x5 / 3x3 / 1x1, and any channel count not % 8, e.g. the 290-plane input) as
``ivit_im2col`` + the dense MFMA GEMMs (``ivit_linear_*``), backward through ``ivit_col2im``; BatchNorm (+ ReLU, + residual) through the ``ivit_bn_*`` kernels; both heads as
one GEMM over the fused feature map. Activations stay NHWC from the input permute to the heads.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import ops
from _lib import BF16, F32, dt, lib, ptr, stream, tdtype
from constants import LIDAR_TOTAL_CHANNELS, MAP_CHANNELS, NUM_INTENTION_CLASSES
from heads import DetectionHead, IntentionHead
from layers import BatchNorm2d, Conv2d, ReLU, _ConvColsFn, _r8


class _BNFn(torch.autograd.Function):
    """BatchNorm2d on an NHWC map [.., C] (batch stats in train), optional + resid, ReLU."""

    @staticmethod
    def forward(ctx, x, g, b, rm, rv, nbt, training, momentum, eps, relu, resid):
        shp = x.shape
        C = shp[-1]
        x2 = x.reshape(-1, C).float().contiguous()
        st = ops.bn_forward(x2, g, b, rm, rv, training, momentum, eps, nbt=nbt if training else None)
        r2 = None if resid is None else resid.reshape(-1, C).float().contiguous()
        y = ops.bn_apply(x2, st, g, b, torch.float32, resid=r2, relu=relu)
        ctx.save_for_backward(x2, y, g)
        ctx.st, ctx.meta = st, (shp, relu, resid is not None)
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, y, g = ctx.saved_tensors
        shp, relu, has_r = ctx.meta
        dx, dr, dg, db = ops.bn_backward(x2, y, dy.reshape(x2.shape).float().contiguous(), ctx.st, g, relu,
                                         torch.float32, want_dr=has_r)
        return (dx.view(shp), dg, db, None, None, None, None, None, None, None,
                None if dr is None else dr.view(shp))


class _ConvSameFn(torch.autograd.Function):
    """NHWC stride-1 'same' conv (k in {1, 3, 5}, Cin / Cout % 8): the implicit-GEMM kernels
    (ivit_conv_fwd / _dgrad / _wgrad) read the taps straight from the map, no im2col copy."""

    @staticmethod
    def forward(ctx, x, w, b, cdt):
        B, H, W, C = x.shape
        Cout, _, k, _ = w.shape
        xh = ops.cast(x.reshape(-1, C).contiguous(), tdtype(cdt))
        wp = ops.pack_conv(w, cdt)
        y = ops.conv_fwd(xh, B, H, W, wp, b, cdt, torch.float32)
        ctx.save_for_backward(xh, wp, w)
        ctx.meta = (B, H, W, C, Cout, k, cdt, b is not None)
        return y.view(B, H, W, Cout)

    @staticmethod
    def backward(ctx, dy):
        xh, wp, w = ctx.saved_tensors
        B, H, W, C, Cout, k, cdt, has_b = ctx.meta
        d2 = ops.cast(dy.reshape(-1, Cout).contiguous(), tdtype(cdt))
        dx = (ops.conv_dgrad(d2, B, H, W, wp, cdt, torch.float32, w=w).view(B, H, W, C)
              if ctx.needs_input_grad[0] else None)
        gp, db = ops.conv_wgrad(d2, xh, B, H, W, C, Cout, k, cdt, want_bias=has_b)
        return dx, ops.unpack_conv_grad(gp, Cout, C, k), db, None


def _conv(m: Conv2d, x, cdt):
    k, s, p = m.kernel_size[0], m.stride[0], m.padding[0]
    if s == 1 and p == k // 2 and k in (1, 3, 5) and x.shape[-1] % 8 == 0 and m.out_channels % 8 == 0:
        return _ConvSameFn.apply(x, m.weight, m.bias, cdt)
    return _ConvColsFn.apply(x, m.weight, m.bias, s, p, cdt)


def _bn(m: BatchNorm2d, x, relu=False, resid=None):
    return _BNFn.apply(x, m.weight, m.bias, m.running_mean, m.running_var, m.num_batches_tracked, m.training,
                       m.momentum, m.eps, relu, resid)


def _cdt(mod):
    return BF16 if getattr(mod, "compute_dtype", torch.float32) == torch.bfloat16 else F32


def conv3x3(in_planes: int, out_planes: int, stride: int = 1, kernel_size: int = 3) -> Conv2d:
    """model_cnn.py:7-9 (k x k, padding (k-1)//2, no bias)."""
    return Conv2d(in_planes, out_planes, kernel_size=kernel_size, stride=stride, padding=(kernel_size - 1) // 2,
                  bias=False)


def conv1x1(in_planes: int, out_planes: int, stride: int = 1) -> Conv2d:
    """model_cnn.py:11-12."""
    return Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, padding=0, bias=False)


class BasicBlock(nn.Module):
    """model_cnn.py:14-33: relu(bn2(conv2(relu(bn1(conv1 x)))) + identity), identity through
    the downsample (conv1x1 stride s + BN) when given."""
    expansion: int = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None,
                 kernel_size: int = 3):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride, kernel_size=kernel_size)
        self.bn1 = BatchNorm2d(planes)
        self.relu = ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes, kernel_size=kernel_size)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward_nhwc(self, x, cdt):
        out = _bn(self.bn1, _conv(self.conv1, x, cdt), relu=True)
        out = _conv(self.conv2, out, cdt)
        identity = x if self.downsample is None else _bn(self.downsample[1], _conv(self.downsample[0], x, cdt))
        return _bn(self.bn2, out, relu=True, resid=identity)

    def forward(self, x):
        y = self.forward_nhwc(x.permute(0, 2, 3, 1).contiguous(), _cdt(self))
        return y.permute(0, 3, 1, 2).contiguous()


def _run_stage(stage: nn.Sequential, x, cdt):
    for blk in stage:
        x = blk.forward_nhwc(x, cdt)
    return x


class CNNBackbone(nn.Module):
    """model_cnn.py:35-123: LiDAR and map streams of three BasicBlock stages (strides 2, 1, 2,
    k = res_block2_kernel_size), channel concat, fusion stage (stride 2) -> stride-8 features."""

    def __init__(self, block: type[BasicBlock] = BasicBlock, lidar_input_channels: int = LIDAR_TOTAL_CHANNELS,
                 map_input_channels: int = MAP_CHANNELS, lidar_s1_planes: int = 160, lidar_s2_planes: int = 192,
                 lidar_s3_planes: int = 224, map_s1_planes: int = 32, map_s2_planes: int = 64,
                 map_s3_planes: int = 96, fusion_block_planes: int = 512, fusion_block_layers: int = 2,
                 num_blocks_per_stage: int = 2, res_block2_kernel_size: int = 5, fusion_block_kernel_size: int = 3):
        super().__init__()
        self.block = block
        ks, nb = res_block2_kernel_size, num_blocks_per_stage
        self.lidar_stage1 = self._make_layer(block, lidar_s1_planes, nb, 2, lidar_input_channels, ks)
        self.lidar_stage2 = self._make_layer(block, lidar_s2_planes, nb, 1, lidar_s1_planes * block.expansion, ks)
        self.lidar_stage3 = self._make_layer(block, lidar_s3_planes, nb, 2, lidar_s2_planes * block.expansion, ks)
        self.lidar_output_channels = lidar_s3_planes * block.expansion
        self.map_stage1 = self._make_layer(block, map_s1_planes, nb, 2, map_input_channels, ks)
        self.map_stage2 = self._make_layer(block, map_s2_planes, nb, 1, map_s1_planes * block.expansion, ks)
        self.map_stage3 = self._make_layer(block, map_s3_planes, nb, 2, map_s2_planes * block.expansion, ks)
        self.map_output_channels = map_s3_planes * block.expansion
        self.fusion_inplanes = self.lidar_output_channels + self.map_output_channels
        self.fusion_block = self._make_layer(block, fusion_block_planes, fusion_block_layers, 2, self.fusion_inplanes,
                                             fusion_block_kernel_size)
        self.final_feature_channels = fusion_block_planes * block.expansion
        self._initialize_weights()

    def _make_layer(self, block, planes, num_blocks, stride=1, current_inplanes=0, kernel_size_for_block=3):
        """model_cnn.py:86-100."""
        out_ch = planes * block.expansion
        downsample = None
        if stride != 1 or current_inplanes != out_ch:
            downsample = nn.Sequential(conv1x1(current_inplanes, out_ch, stride), BatchNorm2d(out_ch))
        layers = [block(current_inplanes, planes, stride, downsample, kernel_size=kernel_size_for_block)]
        for _ in range(1, num_blocks):
            layers.append(block(out_ch, planes, kernel_size=kernel_size_for_block))
        return nn.Sequential(*layers)

    def _initialize_weights(self):
        """model_cnn.py:102-108: kaiming normal (fan_out, relu) convs; BN weight 1, bias 0."""
        for m in self.modules():
            if isinstance(m, Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def forward_nhwc(self, lidar_nhwc, map_nhwc, cdt):
        lf = _run_stage(self.lidar_stage3, _run_stage(self.lidar_stage2, _run_stage(self.lidar_stage1, lidar_nhwc,
                                                                                        cdt), cdt), cdt)
        mf = _run_stage(self.map_stage3, _run_stage(self.map_stage2, _run_stage(self.map_stage1, map_nhwc, cdt),
                                                    cdt), cdt)
        return _run_stage(self.fusion_block, torch.cat([lf, mf], dim=-1), cdt)

    def forward(self, lidar_bev: torch.Tensor, map_bev: torch.Tensor) -> torch.Tensor:
        """model_cnn.py:110-123 (NCHW in, NCHW out)."""
        f = self.forward_nhwc(lidar_bev.permute(0, 2, 3, 1).contiguous(), map_bev.permute(0, 2, 3, 1).contiguous(),
                              _cdt(self))
        return f.permute(0, 3, 1, 2).contiguous()


class IntentNetCNN(nn.Module):
    """model_cnn.py:125-150: CNNBackbone -> DetectionHead / IntentionHead (3x3 convs, one GEMM
    here) -> cls (B, Hf*Wf*A, 1), box (B, Hf*Wf*A, 6), intent (B, Hf*Wf*A, 8); flat index
    (y * Wf + x) * A + a."""

    def __init__(self, backbone_cfg: dict | None = None, head_cfg: dict | None = None):
        super().__init__()
        self.backbone = CNNBackbone(**(backbone_cfg or {}))
        fc = self.backbone.final_feature_channels
        head_cfg = head_cfg or {}
        self.det_head = DetectionHead(in_channels=fc, **head_cfg)
        self.intention_head = IntentionHead(in_channels=fc, num_classes=NUM_INTENTION_CLASSES, **head_cfg)
        self.compute_dtype = torch.float32

    def set_compute_dtype(self, dtype):
        """f32 (exact MFMA, the parity path) or bf16 (bf16 GEMM operands, f32 accumulation)."""
        for m in self.modules():
            m.compute_dtype = dtype
        return self

    def forward(self, lidar_bev: torch.Tensor, map_bev: torch.Tensor):
        cdt = _cdt(self)
        f = self.backbone.forward_nhwc(lidar_bev.permute(0, 2, 3, 1).contiguous(),
                                       map_bev.permute(0, 2, 3, 1).contiguous(), cdt)
        dh, ih = self.det_head, self.intention_head
        A, K = dh.num_anchors, ih.num_classes
        w = torch.cat([dh.conv.weight, ih.conv.weight], 0)
        b = torch.cat([dh.conv.bias, ih.conv.bias], 0)
        out = _ConvColsFn.apply(f, w, b, 1, 1, cdt)  # [B, Hf, Wf, A*7 + A*K]
        B = out.shape[0]
        det = out[..., : A * 7].reshape(B, -1, 7)
        return det[..., :1].contiguous(), det[..., 1:].contiguous(), out[..., A * 7:].reshape(B, -1, K).contiguous()


__all__ = ["conv3x3", "conv1x1", "BasicBlock", "CNNBackbone", "IntentNetCNN"]
