"""IntentNetViT / TwoStreamViTBackbone / BasicBlock with the reference's constructor
signatures, attributes and state_dict keys (model_vit.py:1-184), running on the MI355X
HIP kernels.

``IntentNetViT.forward`` = 2 x (PatchEmbedFn + 12 ViTBlockFn) + NeckFn (final norms,
adapters, fusion, both heads). ``set_compute_dtype(torch.bfloat16)`` selects the bf16 MFMA
path (f32 master weights, f32 residual stream / statistics / loss); the default f32 path is
the exact-f32 parity path.
"""
from __future__ import annotations

import os

import warnings

import torch
import torch.nn as nn

import ops
import vit as timm_like
from _lib import BF16, F32
from constants import GRID_HEIGHT_PX, GRID_WIDTH_PX, LIDAR_TOTAL_CHANNELS, MAP_CHANNELS, NUM_INTENTION_CLASSES
from heads import DetectionHead, IntentionHead
from layers import GELU, BatchNorm2d, Conv2d, LayerNorm, Linear, ReLU, _LayerNormFn


def conv3x3_for_basic(in_planes, out_planes, stride=1, kernel_size=3):
    return Conv2d(in_planes, out_planes, kernel_size=kernel_size, stride=stride, padding=(kernel_size - 1) // 2,
                  bias=False)


def conv1x1_for_basic(in_planes, out_planes, stride=1):
    return Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    """model_vit.py:19-34: relu(bn2(conv2(relu(bn1(conv1 x)))) + identity)."""
    expansion: int = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, kernel_size=3):
        super().__init__()
        self.conv1 = conv3x3_for_basic(inplanes, planes, stride, kernel_size=kernel_size)
        self.bn1 = BatchNorm2d(planes)
        self.relu = ReLU(inplace=True)
        self.conv2 = conv3x3_for_basic(planes, planes, kernel_size=kernel_size)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample[1](self.downsample[0](x))
        out = self.bn1(self.conv1(x), relu=True)
        return self.bn2(self.conv2(out), relu=True, resid=identity)


class TwoStreamViTBackbone(nn.Module):
    def __init__(self, lidar_input_channels=LIDAR_TOTAL_CHANNELS, map_input_channels=MAP_CHANNELS,
                 vit_model_name_lidar="vit_small_patch8_224", vit_model_name_map="vit_small_patch8_224",
                 pretrained_lidar=False, pretrained_map=False, img_size=(GRID_HEIGHT_PX, GRID_WIDTH_PX),
                 drop_path_rate_lidar=0.1, drop_path_rate_map=0.1, lidar_adapter_out_channels=192,
                 map_adapter_out_channels=192, fusion_block_planes=512, fusion_block_layers=2,
                 fusion_block_kernel_size=3, fusion_block_stride=1, res_block_type=BasicBlock):
        super().__init__()
        self.img_size = tuple(img_size)
        self.lidar_adapter_out_channels = lidar_adapter_out_channels
        self.map_adapter_out_channels = map_adapter_out_channels
        self.vit_lidar = timm_like.create_model(vit_model_name_lidar, pretrained=pretrained_lidar,
                                                in_chans=lidar_input_channels, img_size=self.img_size,
                                                drop_path_rate=drop_path_rate_lidar)
        self.vit_lidar.head = nn.Identity()
        self.lidar_embed_dim = self.vit_lidar.embed_dim
        self.lidar_num_prefix_tokens = self.vit_lidar.num_prefix_tokens
        self.lidar_grid_size = tuple(self.vit_lidar.patch_embed.grid_size)
        self.vit_map = timm_like.create_model(vit_model_name_map, pretrained=pretrained_map,
                                              in_chans=map_input_channels, img_size=self.img_size,
                                              drop_path_rate=drop_path_rate_map)
        self.vit_map.head = nn.Identity()
        self.map_embed_dim = self.vit_map.embed_dim
        self.map_num_prefix_tokens = self.vit_map.num_prefix_tokens
        self.map_grid_size = tuple(self.vit_map.patch_embed.grid_size)
        if self.lidar_grid_size != self.map_grid_size:
            # model_vit.py:76-77; forward re-grids the map features bilinearly (:139)
            warnings.warn(f"LiDAR patch grid {self.lidar_grid_size} and Map patch grid {self.map_grid_size} differ.")
        self.feature_map_grid_h, self.feature_map_grid_w = self.lidar_grid_size
        self.adapter_lidar = nn.Sequential(LayerNorm(self.lidar_embed_dim),
                                           Linear(self.lidar_embed_dim, lidar_adapter_out_channels), GELU())
        self.adapter_map = nn.Sequential(LayerNorm(self.map_embed_dim),
                                         Linear(self.map_embed_dim, map_adapter_out_channels), GELU())
        self.fusion_input_channels = lidar_adapter_out_channels + map_adapter_out_channels
        self.fusion_block_stride = fusion_block_stride
        self.fusion_block = self._make_fusion_layer(res_block_type, fusion_block_planes, fusion_block_layers,
                                                    stride=fusion_block_stride,
                                                    current_inplanes=self.fusion_input_channels,
                                                    kernel_size_for_block=fusion_block_kernel_size)
        self.final_feature_channels = fusion_block_planes * res_block_type.expansion
        self.fusion_layers = fusion_block_layers

    def _get_patch_info(self, vit_model, stream_name=""):
        pe = vit_model.patch_embed
        return tuple(pe.grid_size), pe.num_patches

    def _make_fusion_layer(self, block, planes, num_blocks, stride=1, current_inplanes=0, kernel_size_for_block=3):
        downsample = None
        outc = planes * block.expansion
        if stride != 1 or current_inplanes != outc:
            downsample = nn.Sequential(conv1x1_for_basic(current_inplanes, outc, stride), BatchNorm2d(outc))
        layers = [block(current_inplanes, planes, stride, downsample, kernel_size=kernel_size_for_block)]
        for _ in range(1, num_blocks):
            layers.append(block(outc, planes, kernel_size=kernel_size_for_block))
        return nn.Sequential(*layers)

    # neck parameters in NeckFn order (names relative to the backbone / model)
    def neck_names(self):
        names = []
        for s in ("lidar", "map"):
            names += [f"vit_{s}.norm.weight", f"vit_{s}.norm.bias"]
        for s in ("lidar", "map"):
            names += [f"adapter_{s}.0.weight", f"adapter_{s}.0.bias", f"adapter_{s}.1.weight", f"adapter_{s}.1.bias"]
        for n, _ in self.fusion_block.named_parameters():
            names.append("fusion_block." + n)
        for n, _ in self.fusion_block.named_buffers():
            names.append("fusion_block." + n)
        return names

    def _cdt(self):
        return BF16 if getattr(self, "compute_dtype", torch.float32) == torch.bfloat16 else F32

    # Profiling mode (IVIT_CONCURRENT_STREAMS=0): both ViTs on the caller's stream, one after the
    # other — the one-stream step whose kernel trace attributes time per kernel without the other
    # stream sharing the CUs (the concurrency is worth 3.7 ms per step)
    concurrent_streams = os.environ.get("IVIT_CONCURRENT_STREAMS", "1") == "1"

    def stream_tokens(self, lidar_bev, map_bev):
        """The LiDAR and map ViTs are independent until the fusion block: run them on two HIP
        streams so their kernels fill each other's gaps (tile tails, barriers, prologues).
        Autograd replays each backward op on its forward op's stream, so the two backward
        passes overlap the same way; backward() syncs them back to the caller's stream."""
        if not (self.concurrent_streams and lidar_bev.is_cuda):
            return self.vit_lidar.forward_tokens(lidar_bev), self.vit_map.forward_tokens(map_bev)
        main = torch.cuda.current_stream(lidar_bev.device)
        s1, s2 = _side_streams(lidar_bev.device)
        s1.wait_stream(main)
        s2.wait_stream(main)
        # block by block, alternating (vit.VisionTransformer.forward_tokens_steps): with each ViT
        # launched whole (round 3), the backward engine enqueued the map stream's entire backward
        # before the LiDAR stream's first kernel, and the LiDAR stream ran its last blocks alone
        out = {}
        live = [(s1, "l", self.vit_lidar.forward_tokens_steps(lidar_bev)),
                (s2, "m", self.vit_map.forward_tokens_steps(map_bev))]
        # the map stream's first LEAD steps before the alternation, so the backward engine (newest
        # node first) runs the LiDAR stream LEAD blocks ahead and its long patch-embedding weight
        # gradient overlaps the map stream's last blocks
        with torch.cuda.stream(s2):
            for _ in range(LEAD):  # a lead past the map ViT's depth finishes it here
                try:
                    next(live[1][2])
                except StopIteration as stop:
                    out["m"] = stop.value
                    live.pop(1)
                    break
        while live:
            for item in list(live):
                st, key, gen = item
                with torch.cuda.stream(st):
                    try:
                        next(gen)
                    except StopIteration as stop:
                        out[key] = stop.value
                        live.remove(item)
        tl, tm = out["l"], out["m"]
        main.wait_stream(s1)
        main.wait_stream(s2)
        lidar_bev.record_stream(s1)
        map_bev.record_stream(s2)
        tl.record_stream(main)
        tm.record_stream(main)
        return tl, tm

    @property
    def generic_neck(self):
        """The module-by-module neck (features_generic) instead of the fused NeckFn: for
        fusion_block_stride != 1 and for differing LiDAR / map patch grids."""
        return self.fusion_block_stride != 1 or self.lidar_grid_size != self.map_grid_size

    def _process_stream(self, x, vit_stream, num_prefix_tokens, grid_size, adapter, stream_name):
        """model_vit.py:116-122: the stream ViT's features (final norm included), prefix tokens
        dropped, adapter (LayerNorm -> Linear -> GELU), tokens -> (B, C, Hf, Wf) feature map with
        token n at (n // Wf, n % Wf); None (after the reference's message) when the token count
        does not match the patch grid."""
        tokens_all = vit_stream.forward_features(x)
        adapted = adapter(tokens_all[:, num_prefix_tokens:])
        B, N, C = adapted.shape
        if grid_size and N == grid_size[0] * grid_size[1]:
            Hf, Wf = grid_size
            return adapted.permute(0, 2, 1).contiguous().view(B, C, Hf, Wf)
        print(f"ERROR ({stream_name}): Token count {N} or grid_size {grid_size} issue.")
        return None

    def _process_streams(self, lidar_bev, map_bev):
        """The two _process_stream calls (model_vit.py:135,137), on the two side streams when the
        inputs are on the GPU (as stream_tokens)."""
        args_l = (lidar_bev, self.vit_lidar, self.lidar_num_prefix_tokens, self.lidar_grid_size, self.adapter_lidar,
                  "LiDAR")
        args_m = (map_bev, self.vit_map, self.map_num_prefix_tokens, self.map_grid_size, self.adapter_map, "Map")
        if not (self.concurrent_streams and lidar_bev.is_cuda):
            return self._process_stream(*args_l), self._process_stream(*args_m)
        main = torch.cuda.current_stream(lidar_bev.device)
        s1, s2 = _side_streams(lidar_bev.device)
        s1.wait_stream(main)
        s2.wait_stream(main)
        with torch.cuda.stream(s1):
            fl = self._process_stream(*args_l)
        with torch.cuda.stream(s2):
            fm = self._process_stream(*args_m)
        main.wait_stream(s1)
        main.wait_stream(s2)
        lidar_bev.record_stream(s1)
        map_bev.record_stream(s2)
        for f in (fl, fm):
            if f is not None:
                f.record_stream(main)
        return fl, fm

    def features_generic(self, lidar_bev, map_bev):
        """model_vit.py:134-142 through the modules' own forwards: _process_stream per stream (a
        None there gives the reference's zero feature map), the map features re-gridded bilinearly
        onto the LiDAR grid when the grids differ (:139, ops.BilinearFn), fusion BasicBlocks with
        their strides — the path for fusion_block_stride != 1 (strided block-0 convs as im2col +
        GEMM) and for differing patch grids."""
        fl, fm = self._process_streams(lidar_bev, map_bev)
        for f, x in ((fl, lidar_bev), (fm, map_bev)):
            if f is None:
                return torch.zeros(x.shape[0], self.final_feature_channels, self.feature_map_grid_h or 1,
                                   self.feature_map_grid_w or 1, device=x.device)
        if fl.shape[2:] != fm.shape[2:]:
            fm = ops.BilinearFn.apply(fm, tuple(fl.shape[2:]))
        return self.fusion_block(torch.cat([fl, fm], 1))

    def forward(self, lidar_bev, map_bev):
        """model_vit.py:134-142 → fused feature map (B, C, Hf', Wf') f32."""
        if self.generic_neck:
            return self.features_generic(lidar_bev, map_bev)
        tl, tm = self.stream_tokens(lidar_bev, map_bev)
        names = self.neck_names()
        tens = _lookup(self, names)
        B = lidar_bev.shape[0]
        Hf, Wf = self.feature_map_grid_h, self.feature_map_grid_w
        meta = (B, Hf, Wf, self._cdt(), self.training, 0, 0, self.fusion_layers, tuple(names))
        feat = ops.NeckFn.apply(tl, tm, meta, *tens)[0]
        return feat.reshape(B, Hf, Wf, -1).permute(0, 3, 1, 2)


_SIDE_STREAMS = {}
LEAD = 1  # 44.53-44.64 vs 44.65-44.67 ms (lead 0), lead 3 44.56-44.63, same call (round 4)


def _side_streams(device):
    """Two persistent side streams per device for the LiDAR / map ViT streams."""
    key = torch.device(device).index
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = (torch.cuda.Stream(device), torch.cuda.Stream(device))
    return _SIDE_STREAMS[key]


def _lookup(root, names):
    sd = dict(root.named_parameters())
    sd.update(dict(root.named_buffers()))
    return [sd[n] for n in names]


class IntentNetViT(nn.Module):
    def __init__(self, backbone_cfg: dict | None = None, head_cfg: dict | None = None):
        super().__init__()
        if backbone_cfg is None:
            backbone_cfg = {}
        backbone_cfg.setdefault("vit_model_name_lidar", "vit_small_patch8_224")
        backbone_cfg.setdefault("vit_model_name_map", "vit_small_patch8_224")
        backbone_cfg.setdefault("pretrained_lidar", False)
        backbone_cfg.setdefault("pretrained_map", False)
        backbone_cfg.setdefault("img_size", (GRID_HEIGHT_PX, GRID_WIDTH_PX))
        backbone_cfg.setdefault("lidar_adapter_out_channels", 192)
        backbone_cfg.setdefault("map_adapter_out_channels", 192)
        backbone_cfg.setdefault("fusion_block_planes", 512)
        backbone_cfg.setdefault("fusion_block_layers", 2)
        backbone_cfg.setdefault("fusion_block_kernel_size", 3)
        backbone_cfg.setdefault("fusion_block_stride", 1)
        self.backbone = TwoStreamViTBackbone(**backbone_cfg)
        fc = self.backbone.final_feature_channels
        if head_cfg is None:
            head_cfg = {}
        self.det_head = DetectionHead(in_channels=fc, **head_cfg)
        self.intention_head = IntentionHead(in_channels=fc, num_classes=NUM_INTENTION_CLASSES, **head_cfg)
        try:
            stride = int(backbone_cfg.get("vit_model_name_lidar", "vit_small_patch8_224").split("_patch")[-1]
                         .split("_")[0])
        except ValueError:
            stride = 8
            warnings.warn("Could not parse patch stride from ViT name, defaulting to 8.")
        self.effective_head_stride = stride * backbone_cfg.get("fusion_block_stride", 1)
        self.compute_dtype = torch.float32

    def set_compute_dtype(self, dtype):
        """torch.float32 (exact-f32 parity path) or torch.bfloat16 (bf16 MFMA throughput path)."""
        assert dtype in (torch.float32, torch.bfloat16)
        for m in self.modules():
            m.compute_dtype = dtype
        return self

    def _neck_meta(self, B):
        bb = self.backbone
        names = bb.neck_names() + ["det_head.conv.weight", "det_head.conv.bias", "intention_head.conv.weight",
                                   "intention_head.conv.bias"]
        cdt = BF16 if self.compute_dtype == torch.bfloat16 else F32
        meta = (B, bb.feature_map_grid_h, bb.feature_map_grid_w, cdt, self.training, self.det_head.num_anchors,
                self.intention_head.num_classes, bb.fusion_layers, tuple(names))
        return meta, names

    def forward(self, lidar_bev, map_bev):
        """model_vit.py:179-185 → cls (B, A*Hf*Wf, 1), box (.., 6), intent (.., K), all f32."""
        B = lidar_bev.shape[0]
        if self.backbone.generic_neck:  # strided fusion / differing grids: module forwards, heads at H/s x W/s
            f = self.backbone(lidar_bev, map_bev)
            c, b = self.det_head(f)
            it = self.intention_head(f)
            return c.reshape(B, -1, 1), b.reshape(B, -1, 6), it.reshape(B, -1, NUM_INTENTION_CLASSES)
        tl, tm = self.backbone.stream_tokens(lidar_bev, map_bev)
        meta, names = self._neck_meta(B)
        bb = dict(self.backbone.named_parameters())
        bb.update(dict(self.backbone.named_buffers()))
        hd = dict(self.named_parameters())
        tens = [hd[n] if n.startswith(("det_head", "intention_head")) else bb[n] for n in names]
        return ops.NeckFn.apply(tl, tm, meta, *tens)
