"""``sys.modules`` stand-ins that let the reference's OWN modules import in this
container (TEST INFRASTRUCTURE; used only by ``oracle/make_golden.py``).

The reference needs timm, torchvision, cv2 and shapely, none of which are
installed. These stand-ins restate only what the hot path
calls:

* ``timm.create_model``: backed by ``transformers.ViTModel`` — an independent
  ViT implementation with timm ``forward_features`` semantics (pre-norm, CLS
  first, pos added after the concat, final LN, exact GELU, eps 1e-6). timm is
  unpinned in the reference (README.md:123).
* ``torchvision.ops.sigmoid_focal_loss`` / ``nms``: restated from torchvision's
  published source (unpinned, README.md:115); ``nms`` follows the CPU kernel.
* ``shapely.geometry.Polygon``: convex-polygon area/intersection in float64
  (GEOS restated for the convex rectangles ``utils.py:295-332`` builds).
* ``cv2``: ``getRotationMatrix2D`` / ``warpAffine`` / ``resize`` (INTER_LINEAR, BORDER_CONSTANT) and
  ``fillPoly`` / ``polylines`` (LINE_8, 1 px) backed by ``ivit_oracle``'s restatement of OpenCV's
  generic paths, so the reference's BEV augmentation (utils.py:394-517) and map rasterisation
  (utils.py:108-182) flows run here; the resampling / scan-conversion arithmetic itself is parity
  unpinned.
"""
from __future__ import annotations

import sys
import types

import numpy as np
import torch
import torch.nn as nn

from oracle import ivit_oracle as O
from oracle.weights import VIT_ARCH


class _PatchInfo:
    def __init__(self, grid, patch):
        self.grid_size = grid
        self.num_patches = grid[0] * grid[1]
        self.patch_size = (patch, patch)


class HFTimmViT(nn.Module):
    """timm ``VisionTransformer`` surface used at model_vit.py:64-73,101-119."""

    def __init__(self, name, pretrained=False, in_chans=3, img_size=(224, 224), drop_path_rate=0.0, **_):
        super().__init__()
        from transformers import ViTConfig, ViTModel
        a = VIT_ARCH[name]
        D = a["embed_dim"]
        cfg = ViTConfig(hidden_size=D, num_hidden_layers=a["depth"], num_attention_heads=a["num_heads"],
                        intermediate_size=D * a["mlp_ratio"], hidden_act="gelu", layer_norm_eps=1e-6,
                        image_size=tuple(img_size), patch_size=a["patch"], num_channels=in_chans, qkv_bias=True,
                        hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        self.hf = ViTModel(cfg, add_pooling_layer=False)
        self.embed_dim = D
        self.num_prefix_tokens = 1
        self.patch_embed = _PatchInfo((img_size[0] // a["patch"], img_size[1] // a["patch"]), a["patch"])
        self.head = nn.Identity()
        self.drop_path_rate = drop_path_rate

    @property
    def cls_token(self):
        return self.hf.embeddings.cls_token

    def forward_features(self, x):
        return self.hf(pixel_values=x).last_hidden_state


def timm_to_hf_state(sd):
    """Map timm-named ViT keys (``backbone.vit_*.<timm>``) onto the stand-in's HF keys."""
    out = {}
    for k, v in sd.items():
        for stream in ("backbone.vit_lidar.", "backbone.vit_map."):
            if not k.startswith(stream):
                continue
            t = k[len(stream):]
            h = stream + "hf."
            if t == "cls_token":
                out[h + "embeddings.cls_token"] = v
            elif t == "pos_embed":
                out[h + "embeddings.position_embeddings"] = v
            elif t.startswith("patch_embed.proj."):
                out[h + "embeddings.patch_embeddings.projection." + t.split(".")[-1]] = v
            elif t.startswith("norm."):
                out[h + "layernorm." + t.split(".")[-1]] = v
            elif t.startswith("blocks."):
                _, i, rest = t.split(".", 2)
                L = f"{h}layers.{i}."
                if rest.startswith("norm1."):
                    out[L + "layernorm_before." + rest.split(".")[-1]] = v
                elif rest.startswith("norm2."):
                    out[L + "layernorm_after." + rest.split(".")[-1]] = v
                elif rest.startswith("attn.qkv."):
                    leaf = rest.split(".")[-1]
                    q, kk, vv = v.chunk(3, dim=0)
                    out[L + "attention.q_proj." + leaf] = q.clone()
                    out[L + "attention.k_proj." + leaf] = kk.clone()
                    out[L + "attention.v_proj." + leaf] = vv.clone()
                elif rest.startswith("attn.proj."):
                    out[L + "attention.o_proj." + rest.split(".")[-1]] = v
                elif rest.startswith("mlp."):
                    out[L + rest] = v
                else:
                    raise KeyError(k)
            break
        else:
            out[k] = v
    return out


def hf_grads_to_timm(named_grads):
    """Inverse of ``timm_to_hf_state`` for gradients (re-fuses q/k/v into qkv)."""
    out = {}
    pend = {}
    for k, g in named_grads.items():
        if ".hf." not in k:
            out[k] = g
            continue
        stream, t = k.split("hf.", 1)
        if t == "embeddings.cls_token":
            out[stream + "cls_token"] = g
        elif t == "embeddings.position_embeddings":
            out[stream + "pos_embed"] = g
        elif t.startswith("embeddings.patch_embeddings.projection."):
            out[stream + "patch_embed.proj." + t.split(".")[-1]] = g
        elif t.startswith("layernorm."):
            out[stream + "norm." + t.split(".")[-1]] = g
        else:
            _, i, rest = t.split(".", 2)
            b = f"{stream}blocks.{i}."
            leaf = rest.split(".")[-1]
            if rest.startswith("layernorm_before."):
                out[b + "norm1." + leaf] = g
            elif rest.startswith("layernorm_after."):
                out[b + "norm2." + leaf] = g
            elif rest.startswith("attention.o_proj."):
                out[b + "attn.proj." + leaf] = g
            elif rest.split(".")[1] in ("q_proj", "k_proj", "v_proj"):
                pend.setdefault(b + "attn.qkv." + leaf, {})[rest.split(".")[1]] = g
            elif rest.startswith("mlp."):
                out[b + rest] = g
    for k, parts in pend.items():
        out[k] = torch.cat([parts["q_proj"], parts["k_proj"], parts["v_proj"]], dim=0)
    return out


class _Polygon:
    """Convex polygon with GEOS-like ``area``/``is_valid``/``intersection``/``buffer``."""

    def __init__(self, coords=None):
        self.coords = np.zeros((0, 2)) if coords is None else np.asarray(coords, np.float64).reshape(-1, 2)

    @property
    def area(self):
        return O._poly_area(self.coords)

    @property
    def is_valid(self):
        return self.coords.shape[0] >= 3 and self.area > 0.0

    def buffer(self, _d):
        return _Polygon(self.coords if self.is_valid else None)

    def intersection(self, other):
        return _Polygon(O.convex_clip(self.coords, other.coords))


def _focal(inputs, targets, alpha=0.25, gamma=2.0, reduction="none"):
    loss = O.sigmoid_focal_loss(inputs, targets, alpha, gamma)
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss


def _nms(boxes, scores, iou_threshold):
    b = boxes.detach().cpu().numpy()
    keep = O.nms_corners_numpy(b[:, 0], b[:, 1], b[:, 2], b[:, 3], scores.detach().cpu().numpy(), iou_threshold)
    return torch.from_numpy(keep).to(boxes.device)


def install(reference_dir="/root/reference"):
    """Register the stand-ins and put the reference directory on ``sys.path``."""
    import importlib.machinery
    import transformers.models.vit.modeling_vit  # noqa: F401  (import before the stand-ins exist)
    timm = types.ModuleType("timm")
    timm.create_model = lambda name, **kw: HFTimmViT(name, **kw)
    timm.__version__ = "standin-hf"
    tv = types.ModuleType("torchvision")
    ops = types.ModuleType("torchvision.ops")
    ops.sigmoid_focal_loss = _focal
    ops.nms = _nms
    tv.ops = ops
    cv2 = types.ModuleType("cv2")
    from oracle import ivit_oracle as _O
    cv2.INTER_LINEAR, cv2.BORDER_CONSTANT = 1, 0
    cv2.getRotationMatrix2D = _O.cv2_get_rotation_matrix_2d

    def _warp(src, M, dsize, flags=1, borderMode=0, borderValue=0):
        assert flags == 1 and borderMode == 0 and borderValue == 0, "stand-in: INTER_LINEAR / BORDER_CONSTANT 0"
        return _O.cv2_warp_affine_linear(src, M, dsize)

    def _resize(src, dsize, interpolation=1):
        assert interpolation == 1, "stand-in: INTER_LINEAR only"
        return _O.cv2_resize_linear(src, dsize)
    cv2.warpAffine, cv2.resize = _warp, _resize

    def _fill_poly(img, pts_list, color=1, *a, **k):
        assert color == 1 and not a and not k, "stand-in: color 1, LINE_8, shift 0"
        for pts in pts_list:
            _O.cv_fill_poly(img, np.asarray(pts).reshape(-1, 2))
        return img

    def _polylines(img, pts_list, isClosed, color=1, thickness=1, *a, **k):
        assert not isClosed and color == 1 and thickness == 1 and not a and not k, "stand-in: open, color 1, 1 px"
        for pts in pts_list:
            _O.cv_polyline(img, np.asarray(pts).reshape(-1, 2))
        return img
    cv2.fillPoly, cv2.polylines = _fill_poly, _polylines
    shp = types.ModuleType("shapely")
    geom = types.ModuleType("shapely.geometry")
    geom.Polygon = _Polygon
    geom.Point = lambda *a, **k: None
    vec = types.ModuleType("shapely.vectorized")
    vec.contains = lambda *a, **k: None
    shp.geometry, shp.vectorized = geom, vec
    for mod in (timm, tv, ops, cv2, shp, geom, vec):
        mod.__spec__ = importlib.machinery.ModuleSpec(mod.__name__, None)
    sys.modules.update({"timm": timm, "torchvision": tv, "torchvision.ops": ops, "cv2": cv2, "shapely": shp,
                        "shapely.geometry": geom, "shapely.vectorized": vec})
    if reference_dir not in sys.path:
        sys.path.insert(0, reference_dir)
