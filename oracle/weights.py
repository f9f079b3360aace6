"""Deterministic, seeded parameter filler (TEST INFRASTRUCTURE — oracle side).

Produces a timm-key-named ``state_dict`` for IntentNetViT so that the golden
generator (which runs the reference's own ``model_vit.py``), the CPU oracle and
the HIP product can all be fed bit-identical weights without any weight files.

Key names follow the reference checkpoint layout (SURVEY.md §8(b) "State-dict
keys"): ``backbone.vit_{lidar,map}.<timm key>``, ``backbone.adapter_*``,
``backbone.fusion_block.*``, ``det_head.conv.*``, ``intention_head.conv.*``.
"""
from __future__ import annotations

from collections import OrderedDict

import torch

# timm vit_{small,tiny}_patch8_224 geometry (timm model registry; used at
# model_vit.py:64,71 via timm.create_model)
VIT_ARCH = {
    "vit_small_patch8_224": dict(embed_dim=384, depth=12, num_heads=6, patch=8, mlp_ratio=4),
    "vit_tiny_patch8_224": dict(embed_dim=192, depth=12, num_heads=3, patch=8, mlp_ratio=4),
    "vit_small_patch16_224": dict(embed_dim=384, depth=12, num_heads=6, patch=16, mlp_ratio=4),
    "vit_tiny_patch16_224": dict(embed_dim=192, depth=12, num_heads=3, patch=16, mlp_ratio=4),
}


def model_cfg(img_size=(400, 720), lidar_ch=290, map_ch=9, vit_lidar="vit_small_patch8_224",
              vit_map="vit_small_patch8_224", lidar_adapter=192, map_adapter=192, planes=512,
              layers=2, num_anchors=5, num_classes=8, depth=None, fusion_stride=1):
    """Flat description of the IntentNetViT shapes (model_vit.py:145-177 defaults)."""
    return dict(img_size=tuple(img_size), lidar_ch=lidar_ch, map_ch=map_ch, vit_lidar=vit_lidar,
                vit_map=vit_map, lidar_adapter=lidar_adapter, map_adapter=map_adapter,
                planes=planes, layers=layers, num_anchors=num_anchors, num_classes=num_classes,
                depth=depth, fusion_stride=fusion_stride)


def _vit_shapes(prefix, arch, in_ch, img_size, depth_override=None):
    a = VIT_ARCH[arch]
    D, p = a["embed_dim"], a["patch"]
    depth = a["depth"] if depth_override is None else depth_override
    n_tok = (img_size[0] // p) * (img_size[1] // p) + 1
    hid = D * a["mlp_ratio"]
    out = [(prefix + "cls_token", (1, 1, D)), (prefix + "pos_embed", (1, n_tok, D)),
           (prefix + "patch_embed.proj.weight", (D, in_ch, p, p)), (prefix + "patch_embed.proj.bias", (D,))]
    for i in range(depth):
        b = f"{prefix}blocks.{i}."
        out += [(b + "norm1.weight", (D,)), (b + "norm1.bias", (D,)),
                (b + "attn.qkv.weight", (3 * D, D)), (b + "attn.qkv.bias", (3 * D,)),
                (b + "attn.proj.weight", (D, D)), (b + "attn.proj.bias", (D,)),
                (b + "norm2.weight", (D,)), (b + "norm2.bias", (D,)),
                (b + "mlp.fc1.weight", (hid, D)), (b + "mlp.fc1.bias", (hid,)),
                (b + "mlp.fc2.weight", (D, hid)), (b + "mlp.fc2.bias", (D,))]
    out += [(prefix + "norm.weight", (D,)), (prefix + "norm.bias", (D,))]
    return out


def _bn(prefix, c):
    return [(prefix + "weight", (c,)), (prefix + "bias", (c,)), (prefix + "running_mean", (c,)),
            (prefix + "running_var", (c,)), (prefix + "num_batches_tracked", ())]


def param_shapes(cfg):
    """Ordered (key, shape) list matching the reference module registration order."""
    shapes = []
    shapes += _vit_shapes("backbone.vit_lidar.", cfg["vit_lidar"], cfg["lidar_ch"], cfg["img_size"], cfg.get("depth"))
    shapes += _vit_shapes("backbone.vit_map.", cfg["vit_map"], cfg["map_ch"], cfg["img_size"], cfg.get("depth"))
    Dl = VIT_ARCH[cfg["vit_lidar"]]["embed_dim"]
    Dm = VIT_ARCH[cfg["vit_map"]]["embed_dim"]
    for name, D, C in (("lidar", Dl, cfg["lidar_adapter"]), ("map", Dm, cfg["map_adapter"])):
        p = f"backbone.adapter_{name}."
        shapes += [(p + "0.weight", (D,)), (p + "0.bias", (D,)), (p + "1.weight", (C, D)), (p + "1.bias", (C,))]
    cin = cfg["lidar_adapter"] + cfg["map_adapter"]
    P = cfg["planes"]
    for li in range(cfg["layers"]):
        p = f"backbone.fusion_block.{li}."
        ci = cin if li == 0 else P
        shapes += [(p + "conv1.weight", (P, ci, 3, 3))] + _bn(p + "bn1.", P)
        shapes += [(p + "conv2.weight", (P, P, 3, 3))] + _bn(p + "bn2.", P)
        if li == 0 and ci != P:
            shapes += [(p + "downsample.0.weight", (P, ci, 1, 1))] + _bn(p + "downsample.1.", P)
    A, K = cfg["num_anchors"], cfg["num_classes"]
    shapes += [("det_head.conv.weight", (A * 7, P, 3, 3)), ("det_head.conv.bias", (A * 7,)),
               ("intention_head.conv.weight", (A * K, P, 3, 3)), ("intention_head.conv.bias", (A * K,))]
    return shapes


def make_state_dict(cfg, seed=0):
    """Seeded filler. One torch CPU generator, consumed in ``param_shapes`` order.

    Scales keep activations O(1) through 12 pre-norm blocks so fp32 parity is
    meaningful (no saturation, no vanishing signal).
    """
    return fill_state_dict(param_shapes(cfg), seed)


def fill_state_dict(shapes, seed=0):
    """The filler over any ordered (key, shape) list (also the CNN variant's state dict)."""
    g = torch.Generator().manual_seed(seed)
    sd = OrderedDict()
    for key, shape in shapes:
        if key.endswith("num_batches_tracked"):
            sd[key] = torch.zeros((), dtype=torch.long)
            continue
        if key.endswith("running_mean"):
            sd[key] = 0.1 * torch.randn(shape, generator=g)
            continue
        if key.endswith("running_var"):
            sd[key] = 0.5 + torch.rand(shape, generator=g)
            continue
        leaf = key.rsplit(".", 1)[-1]
        if key.endswith("cls_token") or key.endswith("pos_embed"):
            t = 0.02 * torch.randn(shape, generator=g)
        elif leaf == "weight" and len(shape) == 1:      # LayerNorm / BatchNorm gamma
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif leaf == "bias":
            t = 0.02 * torch.randn(shape, generator=g)
        else:                                           # linear / conv weights: fan-in scaled
            fan_in = 1
            for s in shape[1:]:
                fan_in *= s
            t = torch.randn(shape, generator=g) / (fan_in ** 0.5)
        sd[key] = t.float().contiguous()
    return sd


def state_checksum(sd):
    """Order-sensitive float64 checksum over all float tensors (fixture sanity)."""
    acc = 0.0
    for i, (k, v) in enumerate(sd.items()):
        if v.is_floating_point():
            acc += (i + 1) * float(v.double().sum()) + float(v.double().abs().sum()) * 1e-3
    return acc
