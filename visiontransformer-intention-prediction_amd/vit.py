"""timm-compatible VisionTransformer stream (the object ``timm.create_model`` returns at
model_vit.py:64,71): same attribute surface (``patch_embed.grid_size``, ``num_prefix_tokens``,
``embed_dim``, ``cls_token``, assignable ``head``, ``forward_features``) and the same
``state_dict`` keys as timm's ``vit_{small,tiny}_patch{8,16}_224``, so reference checkpoints load.
Compute runs in ``ops.PatchEmbedFn`` + ``ops.ViTBlockFn`` (HIP)."""
from __future__ import annotations

import math

import torch
import torch.nn as nn

import ops
from _lib import BF16, F32
from layers import Conv2d, LayerNorm, Linear, _LayerNormFn

VIT_ARCH = {
    "vit_small_patch8_224": dict(embed_dim=384, depth=12, num_heads=6, patch=8, mlp_ratio=4),
    "vit_tiny_patch8_224": dict(embed_dim=192, depth=12, num_heads=3, patch=8, mlp_ratio=4),
    # patch-16 variants (timm registry): a stream built from one of these has a coarser grid, which
    # model_vit.py:139 re-grids bilinearly onto the LiDAR grid (ops.BilinearFn)
    "vit_small_patch16_224": dict(embed_dim=384, depth=12, num_heads=6, patch=16, mlp_ratio=4),
    "vit_tiny_patch16_224": dict(embed_dim=192, depth=12, num_heads=3, patch=16, mlp_ratio=4),
}


class PatchEmbed(nn.Module):
    def __init__(self, img_size, patch_size, in_chans, embed_dim):
        super().__init__()
        self.img_size = tuple(img_size)
        self.patch_size = (patch_size, patch_size)
        self.grid_size = (self.img_size[0] // patch_size, self.img_size[1] // patch_size)
        self.num_patches = self.grid_size[0] * self.grid_size[1]
        self.proj = Conv2d(in_chans, embed_dim, patch_size, stride=patch_size)


class Attention(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads, self.head_dim = num_heads, dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = Linear(dim, dim * 3)
        self.proj = Linear(dim, dim)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = Linear(dim, hidden)
        self.fc2 = Linear(hidden, dim)


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio, drop_path):
        super().__init__()
        self.norm1 = LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads)
        self.norm2 = LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))
        self.drop_path_rate = drop_path
        # injection hook (parity tests): (attn_scale[B], mlp_scale[B]) used instead of the drawn
        # masks while training; the same per-sample factors oracle.vit_forward_features takes
        self.drop_path_scales = None
        self.last_scales = (None, None)

    def _scales(self, B, device, drawn=None):
        """timm DropPath: per-sample Bernoulli(1-p) / (1-p), independent per branch (identity
        in eval mode or at p = 0). ``drawn``: this block's [2, B] factors from the stream's one
        draw for all blocks (VisionTransformer._draw_drop_path)."""
        p = self.drop_path_rate
        if not self.training or p <= 0.0:
            self.last_scales = (None, None)
            return None, None
        if drawn is not None and self.drop_path_scales is None:
            self.last_scales = (drawn[0], drawn[1])
            return self.last_scales
        if self.drop_path_scales is not None:
            s = torch.stack([torch.as_tensor(v, dtype=torch.float32).reshape(B) for v in self.drop_path_scales])
            s = s.to(device)
        else:
            keep = 1.0 - p
            s = torch.empty((2, B), device=device).bernoulli_(keep).div_(keep)
        self.last_scales = (s[0].contiguous(), s[1].contiguous())
        return self.last_scales

    def forward_flat(self, x, B, N, cdt, ln_in=None, next_norm=None, hand_mine=None, hand_prev=None, drawn=None):
        """-> (x_out, (y, mean, rstd) of the next block's norm1 or empty tensors): `ln_in` is
        this block's (y, mean, rstd) of norm1 computed by the previous block's fc2 epilogue;
        `next_norm` the next block's norm1, whose forward this block's fc2 epilogue runs
        (ops.ViTBlockFn, bf16 row-panel path)."""
        s1, s2 = self._scales(B, x.device, drawn)
        nxw = next_norm.weight if next_norm is not None else None
        nxb = next_norm.bias if next_norm is not None else None
        li, mi, ri = ln_in if ln_in is not None else (None, None, None)
        out = ops.ViTBlockFn.apply(x, li, mi, ri, self.norm1.weight, self.norm1.bias, self.attn.qkv.weight,
                                    self.attn.qkv.bias, self.attn.proj.weight, self.attn.proj.bias, self.norm2.weight,
                                    self.norm2.bias, self.mlp.fc1.weight, self.mlp.fc1.bias, self.mlp.fc2.weight,
                                    self.mlp.fc2.bias, nxw, nxb, s1, s2, (B, N, self.attn.num_heads, cdt, 1e-6),
                                    hand_mine, hand_prev)
        return out[0], tuple(out[1:])

    def forward(self, x):
        B, N, D = x.shape
        cdt = BF16 if getattr(self, "compute_dtype", torch.float32) == torch.bfloat16 else F32
        return self.forward_flat(x.reshape(B * N, D).contiguous().float(), B, N, cdt)[0].reshape(B, N, D)


class VisionTransformer(nn.Module):
    def __init__(self, img_size=(224, 224), patch_size=8, in_chans=3, embed_dim=384, depth=12, num_heads=6,
                 mlp_ratio=4.0, drop_path_rate=0.0):
        super().__init__()
        self.embed_dim = self.num_features = embed_dim
        self.num_prefix_tokens = 1
        self.patch_embed = PatchEmbed(img_size, patch_size, in_chans, embed_dim)
        n_tok = self.patch_embed.num_patches + 1
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.randn(1, n_tok, embed_dim) * 0.02)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, depth)]
        self.blocks = nn.ModuleList([Block(embed_dim, num_heads, mlp_ratio, dpr[i]) for i in range(depth)])
        self.norm = LayerNorm(embed_dim, eps=1e-6)
        self.head = nn.Identity()
        nn.init.normal_(self.cls_token, std=1e-6)
        self.compute_dtype = torch.float32

    def set_drop_path_scales(self, scales):
        """Inject per-block DropPath factors: a list (one per block) of (attn_scale[B],
        mlp_scale[B]), or None to draw them again (timm semantics)."""
        for i, blk in enumerate(self.blocks):
            blk.drop_path_scales = None if scales is None else scales[i]

    def _draw_drop_path(self, B, device):
        """Every block's DropPath factors of this forward in ONE draw: torch.bernoulli over a cached
        device tensor of the per-block keep probabilities ([depth, 2, B]: attention / MLP branch),
        then one divide — 2 launches per stream instead of 2 per block (timm draws per block and
        branch, the same Bernoulli(1-p)/(1-p) law, a different stream). None when no block drops."""
        if not self.training or all(b.drop_path_rate <= 0.0 for b in self.blocks):
            return None
        # the per-block rates are part of the key: a drop-path schedule that changes them rebuilds it
        key = (device, B, tuple(float(b.drop_path_rate) for b in self.blocks))
        cache = getattr(self, "_keep_cache", None)
        if cache is None or cache[0] != key:
            keep = torch.tensor([1.0 - b.drop_path_rate for b in self.blocks], dtype=torch.float32)
            keep = keep.view(-1, 1, 1).expand(len(self.blocks), 2, B).contiguous().to(device)
            self._keep_cache = cache = (key, keep)
        keep = cache[1]
        return torch.bernoulli(keep).div_(keep)

    def _cdt(self):
        return BF16 if self.compute_dtype == torch.bfloat16 else F32

    def forward_tokens(self, x):
        """Patch embed + all blocks, without the final norm: (B*(Np+1), D) f32 residual stream."""
        steps = self.forward_tokens_steps(x)
        while True:
            try:
                next(steps)
            except StopIteration as stop:
                return stop.value

    def forward_tokens_steps(self, x):
        """forward_tokens as a generator that yields after the patch embedding and after every
        block (the launches of one step are all enqueued on the current stream when it yields) and
        returns the token stream: model_vit.stream_tokens interleaves the LiDAR and map ViTs block
        by block, so their autograd nodes interleave in creation order and the backward engine
        (which runs the ready node created last first) feeds both HIP streams evenly instead of
        enqueueing one stream's whole backward before the other's."""
        B, C, H, W = x.shape
        if (H, W) != self.patch_embed.img_size:
            raise ValueError(f"Input size {(H, W)} != model img_size {self.patch_embed.img_size} (timm strict size)")
        cdt = self._cdt()
        # bf16 at D = 384: block i's fc2 epilogue also produces block i+1's norm1 (ops.ViTBlockFn)
        fuse = cdt == BF16 and self.embed_dim == 384
        # ... and in the backward, block i+1 hands block i its DropPath-scaled bf16 gradient, and
        # block 0 hands the patch embedding its bf16 token gradient
        hands = [ops.GradHandoff() for _ in self.blocks] if fuse and torch.is_grad_enabled() else None
        # (only the fused patch-8 embedding reads it; the generic patch path takes its f32 dtok)
        hand_pe = ops.GradHandoff() if hands and self.patch_embed.proj.weight.shape[-1] == 8 else None
        t = ops.PatchEmbedFn.apply(x.float().contiguous(), self.patch_embed.proj.weight, self.patch_embed.proj.bias,
                                   self.pos_embed, self.cls_token, cdt, hand_pe)
        N = self.patch_embed.num_patches + 1
        ln = None
        drawn = self._draw_drop_path(B, x.device)
        yield
        for i, blk in enumerate(self.blocks):
            nxt = self.blocks[i + 1].norm1 if fuse and i + 1 < len(self.blocks) else None
            t, nxt_ln = blk.forward_flat(t, B, N, cdt, ln_in=ln, next_norm=nxt,
                                         hand_mine=hands[i] if hands else None,
                                         hand_prev=(hands[i - 1] if i > 0 else hand_pe) if hands else None,
                                         drawn=drawn[i] if drawn is not None else None)
            ln = nxt_ln if nxt is not None else None
            yield
        return t

    def forward_features(self, x):
        B = x.shape[0]
        t = self.forward_tokens(x)
        return _LayerNormFn.apply(t, self.norm.weight, self.norm.bias, 1e-6).reshape(B, -1, self.embed_dim)

    def forward(self, x):
        return self.head(self.forward_features(x)[:, 0])


def create_model(model_name, pretrained=False, in_chans=3, img_size=(224, 224), drop_path_rate=0.0, **_):
    """timm.create_model surface used by the reference (model_vit.py:64,71)."""
    if pretrained:
        raise RuntimeError("pretrained weights are not available offline; pass pretrained=False")
    a = VIT_ARCH[model_name]
    return VisionTransformer(img_size=img_size, patch_size=a["patch"], in_chans=in_chans, embed_dim=a["embed_dim"],
                             depth=a["depth"], num_heads=a["num_heads"], mlp_ratio=a["mlp_ratio"],
                             drop_path_rate=drop_path_rate)
