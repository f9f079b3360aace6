"""CPU oracle for the IntentNetViT hot path — TEST INFRASTRUCTURE ONLY.

A plain PyTorch-fp32 / numpy restatement of the reference algorithm, used by
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg as the checker and CPU baseline. The product (the HIP path in
``visiontransformer-intention-prediction_amd/``) never imports this file.

Pinning: every function here is checked against golden vectors produced by
running the reference's OWN ``model_vit.py`` / ``heads.py`` / ``loss.py`` /
``utils.py`` (``oracle/make_golden.py``; fixtures in ``tests/golden/``).
Third-party pieces that are absent from this image (timm ViT, torchvision
``nms``/``sigmoid_focal_loss``, shapely/GEOS) are restated from their
published algorithms; the timm ViT restatement is additionally cross-checked
against ``transformers.ViTModel`` (an independent implementation) inside the
golden generator. See DESIGN.md §Oracle.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# constants.py:18-25 (ANCHOR_CONFIGS_PAPER), :28-39 (grid / offsets), :72-77
ANCHOR_CONFIGS = [(2.0, 4.5, 0.0), (2.0, 4.5, math.pi / 2), (2.5, 2.5, 0.0), (1.5, 9.0, 0.0), (4.0, 2.0, 0.0)]
VOXEL = 0.2
DOMINANT = (0, 6, 7)  # iteration order of the reference's set({0, 7, 6}) for small ints


# --------------------------------------------------------------------------------------
# ViT stream (timm VisionTransformer.forward_features semantics, model_vit.py:64,71,119)
# --------------------------------------------------------------------------------------
def vit_forward_features(sd, prefix, x, num_heads, depth, drop_path_scales=None, eps=1e-6, attn="explicit",
                         checkpoint=False):
    """timm ``forward_features``: PatchEmbed conv k=s=patch → cat CLS → +pos_embed →
    ``depth`` pre-norm blocks (LN eps 1e-6, MHSA, exact-erf GELU MLP) → final LN.

    ``drop_path_scales``: optional list (per block) of (attn_scale[B], mlp_scale[B])
    standing in for timm DropPath's per-sample Bernoulli/keep_prob factors.
    ``attn``: "explicit" materialises softmax(q kᵀ · d^-0.5) (the golden-pinned form);
    "sdpa" calls ``F.scaled_dot_product_attention`` as timm's fused path does (timm
    ``Attention.fused_attn``), used by the CPU baseline and by large-grid checks.
    ``checkpoint``: recompute each block in backward (memory only; same arithmetic).
    """
    w = sd[prefix + "patch_embed.proj.weight"]
    p = w.shape[-1]
    t = F.conv2d(x, w, sd[prefix + "patch_embed.proj.bias"], stride=p)
    B, D = t.shape[0], t.shape[1]
    t = t.flatten(2).transpose(1, 2)
    cls = sd[prefix + "cls_token"].expand(B, -1, -1)
    t = torch.cat([cls, t], dim=1) + sd[prefix + "pos_embed"]
    for i in range(depth):
        sc = None if drop_path_scales is None else drop_path_scales[i]
        if checkpoint and torch.is_grad_enabled():
            from torch.utils.checkpoint import checkpoint as _ckpt
            t = _ckpt(_vit_block, sd, f"{prefix}blocks.{i}.", t, num_heads, sc, eps, attn, use_reentrant=False)
        else:
            t = _vit_block(sd, f"{prefix}blocks.{i}.", t, num_heads, sc, eps, attn)
    return F.layer_norm(t, (D,), sd[prefix + "norm.weight"], sd[prefix + "norm.bias"], eps)


def _vit_block(sd, b, t, num_heads, scales, eps, attn):
    """timm Block: x + dp(attn(LN1 x)); x + dp(mlp(LN2 x)); qkv rows [q heads; k; v]."""
    B, N, D = t.shape
    hd = D // num_heads
    h = F.layer_norm(t, (D,), sd[b + "norm1.weight"], sd[b + "norm1.bias"], eps)
    qkv = F.linear(h, sd[b + "attn.qkv.weight"], sd[b + "attn.qkv.bias"])
    q, k, v = qkv.reshape(B, N, 3, num_heads, hd).permute(2, 0, 3, 1, 4).unbind(0)
    if attn == "sdpa":
        a = F.scaled_dot_product_attention(q, k, v)
    else:
        s = (q @ k.transpose(-2, -1)) * (hd ** -0.5)
        a = torch.softmax(s, dim=-1) @ v
    a = a.transpose(1, 2).reshape(B, N, D)
    a = F.linear(a, sd[b + "attn.proj.weight"], sd[b + "attn.proj.bias"])
    if scales is not None:
        a = a * scales[0].view(B, 1, 1).to(a)
    t = t + a
    h = F.layer_norm(t, (D,), sd[b + "norm2.weight"], sd[b + "norm2.bias"], eps)
    h = F.gelu(F.linear(h, sd[b + "mlp.fc1.weight"], sd[b + "mlp.fc1.bias"]))
    h = F.linear(h, sd[b + "mlp.fc2.weight"], sd[b + "mlp.fc2.bias"])
    if scales is not None:
        h = h * scales[1].view(B, 1, 1).to(h)
    return t + h


def _stream(sd, name, x, num_heads, depth, dps, attn="explicit", checkpoint=False):
    """model_vit.py:116-122 (_process_stream): drop CLS, adapter LN(eps 1e-5)→Linear→GELU,
    tokens → (B, C, Hf, Wf) with token n = gy*Wf + gx."""
    pre = f"backbone.vit_{name}."
    tok = vit_forward_features(sd, pre, x, num_heads, depth, dps, attn=attn, checkpoint=checkpoint)[:, 1:]
    a = f"backbone.adapter_{name}."
    D = tok.shape[-1]
    y = F.layer_norm(tok, (D,), sd[a + "0.weight"], sd[a + "0.bias"], 1e-5)
    y = F.gelu(F.linear(y, sd[a + "1.weight"], sd[a + "1.bias"]))
    p = sd[pre + "patch_embed.proj.weight"].shape[-1]
    Hf, Wf = x.shape[2] // p, x.shape[3] // p
    B, Nn, C = y.shape
    return y.permute(0, 2, 1).contiguous().view(B, C, Hf, Wf)


def _bn(x, sd, p, training, momentum=0.1):
    return F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"], sd[p + "weight"], sd[p + "bias"],
                        training=training, momentum=momentum, eps=1e-5)


def fusion_forward(sd, x, layers=2, training=True, stride=1):
    """model_vit.py:19-34 BasicBlock ×layers (+1×1 downsample on block 0; block 0 carries
    fusion_block_stride on conv1 and the downsample), :125-132."""
    for li in range(layers):
        p = f"backbone.fusion_block.{li}."
        s = stride if li == 0 else 1
        idn = x
        o = F.relu(_bn(F.conv2d(x, sd[p + "conv1.weight"], padding=1, stride=s), sd, p + "bn1.", training))
        o = _bn(F.conv2d(o, sd[p + "conv2.weight"], padding=1), sd, p + "bn2.", training)
        if (p + "downsample.0.weight") in sd:
            idn = _bn(F.conv2d(x, sd[p + "downsample.0.weight"], stride=s), sd, p + "downsample.1.", training)
        x = F.relu(o + idn)
    return x


def heads_forward(sd, feat, num_anchors=5, num_classes=8):
    """heads.py:18-25,39-43 + model_vit.py:181-184: conv3x3 + view/permute → flat anchors."""
    B = feat.shape[0]
    d = F.conv2d(feat, sd["det_head.conv.weight"], sd["det_head.conv.bias"], padding=1)
    Hf, Wf = d.shape[2:]
    d = d.view(B, num_anchors, 7, Hf, Wf).permute(0, 3, 4, 1, 2).contiguous()
    it = F.conv2d(feat, sd["intention_head.conv.weight"], sd["intention_head.conv.bias"], padding=1)
    it = it.view(B, num_anchors, num_classes, Hf, Wf).permute(0, 3, 4, 1, 2).contiguous()
    return d[..., 0].reshape(B, -1, 1), d[..., 1:].reshape(B, -1, 6), it.reshape(B, -1, num_classes)


def intentnet_forward(sd, lidar, map_bev, cfg, training=False, drop_path_scales=None, attn="explicit",
                      checkpoint=False):
    """IntentNetViT.forward (model_vit.py:179-185) → (cls (B,A·HW,1), box (B,A·HW,6), intent)."""
    from oracle.weights import VIT_ARCH
    al, am = VIT_ARCH[cfg["vit_lidar"]], VIT_ARCH[cfg["vit_map"]]
    depth_l = cfg.get("depth") or al["depth"]
    depth_m = cfg.get("depth") or am["depth"]
    dl = dm = None
    if drop_path_scales is not None:
        dl, dm = drop_path_scales
    fl = _stream(sd, "lidar", lidar, al["num_heads"], depth_l, dl, attn, checkpoint)
    fm = _stream(sd, "map", map_bev, am["num_heads"], depth_m, dm, attn, checkpoint)
    if fm.shape[2:] != fl.shape[2:]:  # model_vit.py:139: differing patch grids
        fm = F.interpolate(fm, size=fl.shape[2:], mode="bilinear", align_corners=False)
    feat = fusion_forward(sd, torch.cat([fl, fm], dim=1), cfg["layers"], training, cfg.get("fusion_stride", 1))
    return heads_forward(sd, feat, cfg["num_anchors"], cfg["num_classes"])


# --------------------------------------------------------------------------------------
# Geometry (utils.py)
# --------------------------------------------------------------------------------------
def generate_anchors(bev_h=400, bev_w=720, stride=8, configs=ANCHOR_CONFIGS, voxel=VOXEL, off_x=None, off_y=None):
    """utils.py:519-562 — (Hf·Wf·A, 5) [cx, cy, w, l, yaw], location-major / anchor-minor.
    Offsets default to the constants.py:38-39 values of the *base* grid (400×720)."""
    off_x = 720 / 2.0 if off_x is None else off_x
    off_y = 400 * 3.0 / 4.0 if off_y is None else off_y
    fh, fw = bev_h // stride, bev_w // stride
    gy, gx = torch.meshgrid(torch.arange(fh), torch.arange(fw), indexing="ij")
    px = gx * stride + stride / 2.0
    py = gy * stride + stride / 2.0
    ey = (px - off_x) * voxel
    ex = (off_y - py) * voxel
    centers = torch.stack([ex, ey], dim=-1).reshape(-1, 2)
    per = []
    for (w, l, r) in configs:
        dims = torch.tensor([w, l, r], dtype=torch.float32).unsqueeze(0).repeat(centers.shape[0], 1)
        per.append(torch.cat([centers, dims], dim=1))
    return torch.stack(per, dim=0).transpose(0, 1).reshape(-1, 5)


def axis_aligned_iou(b1, b2):
    """utils.py:276-292 (cols 0..3 only; eps 1e-7 on the union)."""
    def corners(b):
        return torch.stack([b[:, 0] - b[:, 2] / 2, b[:, 1] - b[:, 3] / 2,
                            b[:, 0] + b[:, 2] / 2, b[:, 1] + b[:, 3] / 2], dim=1)
    c1, c2 = corners(b1), corners(b2)
    ix1 = torch.maximum(c1[:, None, 0], c2[None, :, 0])
    iy1 = torch.maximum(c1[:, None, 1], c2[None, :, 1])
    ix2 = torch.minimum(c1[:, None, 2], c2[None, :, 2])
    iy2 = torch.minimum(c1[:, None, 3], c2[None, :, 3])
    inter = torch.clamp(ix2 - ix1, min=0) * torch.clamp(iy2 - iy1, min=0)
    a1 = b1[:, 2] * b1[:, 3]
    a2 = b2[:, 2] * b2[:, 3]
    return inter / ((a1[:, None] + a2[None, :] - inter) + 1e-7)


def decode_boxes(rel, anchors):
    """utils.py:227-257."""
    if rel.shape[0] == 0:
        return torch.empty((0, 5))
    ax, ay, aw, al, ah = anchors.unbind(1)
    dx, dy, dw, dl, ds, dc = rel.unbind(1)
    yaw = ah + torch.atan2(ds, dc)
    yaw = torch.atan2(torch.sin(yaw), torch.cos(yaw))
    return torch.stack([dx * aw + ax, dy * al + ay, torch.exp(dw) * aw, torch.exp(dl) * al, yaw], dim=-1)


def nms_corners_numpy(x1, y1, x2, y2, scores, thr=0.2):
    """torchvision CPU ``nms`` (published C++ kernel ``nms_kernel_impl``) on x1y1x2y2:
    stable descending sort; f32 areas/IoU; suppress j if IoU > thr with the f32 IoU
    promoted to double. Returns kept indices (int64) in score order."""
    x1, y1, x2, y2 = [np.asarray(v, np.float32) for v in (x1, y1, x2, y2)]
    s = np.asarray(scores, dtype=np.float32)
    n = s.shape[0]
    if n == 0:
        return np.zeros((0,), np.int64)
    areas = (x2 - x1) * (y2 - y1)
    order = np.argsort(-s, kind="stable")
    sup = np.zeros(n, bool)
    keep = []
    zero = np.float32(0)
    for pos in range(n):
        i = order[pos]
        if sup[i]:
            continue
        keep.append(i)
        rest = order[pos + 1:]
        rest = rest[~sup[rest]]
        if rest.size == 0:
            continue
        w = np.maximum(zero, np.minimum(x2[i], x2[rest]) - np.maximum(x1[i], x1[rest]))
        h = np.maximum(zero, np.minimum(y2[i], y2[rest]) - np.maximum(y1[i], y1[rest]))
        inter = w * h
        ovr = inter / ((areas[i] + areas[rest]) - inter)
        sup[rest[ovr.astype(np.float64) > float(thr)]] = True
    return np.asarray(keep, dtype=np.int64)


def nms_numpy(boxes_xywha, scores, thr=0.2):
    """utils.py:259-274 (apply_nms): axis-aligned corners cx∓w/2, cy∓l/2 (yaw ignored) →
    ``nms_corners_numpy``."""
    b = np.asarray(boxes_xywha, dtype=np.float32)
    if b.shape[0] == 0:
        return np.zeros((0,), np.int64)
    half = np.float32(2)
    return nms_corners_numpy(b[:, 0] - b[:, 2] / half, b[:, 1] - b[:, 3] / half,
                             b[:, 0] + b[:, 2] / half, b[:, 1] + b[:, 3] / half, scores, thr)


def _rect_corners(box):
    """utils.py:295-332 — local corners [-w/2,-l/2],[w/2,-l/2],[w/2,l/2],[-w/2,l/2] rotated by yaw."""
    cx, cy, w, l, a = [float(v) for v in box]
    hw, hl = w / 2.0, l / 2.0
    loc = np.array([[-hw, -hl], [hw, -hl], [hw, hl], [-hw, hl]], dtype=np.float64)
    c, s = np.cos(a), np.sin(a)
    R = np.array([[c, -s], [s, c]])
    return loc @ R.T + np.array([cx, cy])


def _poly_area(P):
    if len(P) < 3:
        return 0.0
    x, y = P[:, 0], P[:, 1]
    return 0.5 * abs(float(np.dot(x, np.roll(y, -1)) - np.dot(y, np.roll(x, -1))))


def _ccw(P):
    x, y = P[:, 0], P[:, 1]
    sgn = float(np.dot(x, np.roll(y, -1)) - np.dot(y, np.roll(x, -1)))
    return P if sgn >= 0 else P[::-1]


def convex_clip(P, Q):
    """Sutherland–Hodgman clip of convex polygon P by convex polygon Q (float64)."""
    P, Q = _ccw(P), _ccw(Q)
    out = [tuple(p) for p in P]
    for i in range(len(Q)):
        if not out:
            break
        a, b = Q[i], Q[(i + 1) % len(Q)]
        inp, out = out, []
        ex, ey = b[0] - a[0], b[1] - a[1]

        def side(p):
            return ex * (p[1] - a[1]) - ey * (p[0] - a[0])
        for j in range(len(inp)):
            cur, prv = inp[j], inp[j - 1]
            sc, sp = side(cur), side(prv)
            if sc >= 0:
                if sp < 0:
                    t = sp / (sp - sc)
                    out.append((prv[0] + t * (cur[0] - prv[0]), prv[1] + t * (cur[1] - prv[1])))
                out.append(cur)
            elif sp >= 0:
                t = sp / (sp - sc)
                out.append((prv[0] + t * (cur[0] - prv[0]), prv[1] + t * (cur[1] - prv[1])))
    return np.array(out, dtype=np.float64).reshape(-1, 2)


def rotated_iou_numpy(b1, b2):
    """utils.py:335-392: area<1e-6 → 0; inter ≤ 1e-7 → 0; union ≤ 1e-6 → 0; output f32.
    GEOS intersection restated as convex clipping in float64 (inputs are rectangles)."""
    b1 = np.asarray(b1, np.float32)
    b2 = np.asarray(b2, np.float32)
    out = np.zeros((b1.shape[0], b2.shape[0]), np.float32)
    P1 = [_rect_corners(b) for b in b1]
    P2 = [_rect_corners(b) for b in b2]
    A1 = [_poly_area(p) for p in P1]
    A2 = [_poly_area(p) for p in P2]
    for i in range(len(P1)):
        if A1[i] < 1e-6:
            continue
        for j in range(len(P2)):
            if A2[j] < 1e-6:
                continue
            inter = _poly_area(convex_clip(P1[i], P2[j]))
            if inter > 1e-7:
                u = A1[i] + A2[j] - inter
                if u > 1e-6:
                    out[i, j] = inter / u
    return out


# --------------------------------------------------------------------------------------
# Loss (loss.py)
# --------------------------------------------------------------------------------------
def sigmoid_focal_loss(x, t, alpha=0.25, gamma=2.0):
    """torchvision.ops.sigmoid_focal_loss (published Python source), reduction='none'."""
    p = torch.sigmoid(x)
    ce = F.binary_cross_entropy_with_logits(x, t, reduction="none")
    p_t = p * t + (1 - p) * (1 - t)
    loss = ce * ((1 - p_t) ** gamma)
    if alpha >= 0:
        loss = (alpha * t + (1 - alpha) * (1 - t)) * loss
    return loss


def assign_targets(anchors, gt_list, pos_thr=0.6, neg_thr=0.45, iou_fn=axis_aligned_iou):
    """loss.py:58-126 — per-sample IoU assignment, force-match and delta encoding."""
    B, NA = len(gt_list), anchors.shape[0]
    cls_t = torch.full((B, NA), -1, dtype=torch.long)
    box_t = torch.zeros((B, NA, 6), dtype=anchors.dtype)
    int_t = torch.full((B, NA), -1, dtype=torch.long)
    for b in range(B):
        g = gt_list[b]
        if not isinstance(g, dict) or "boxes_xywha" not in g or "intentions" not in g or g["boxes_xywha"].shape[0] == 0:
            cls_t[b, :] = 0
            continue
        boxes, ints = g["boxes_xywha"].float(), g["intentions"].long()
        iou = iou_fn(anchors, boxes)
        mx, arg = iou.max(dim=1)
        cls_t[b, mx < neg_thr] = 0
        pos = mx >= pos_thr
        cls_t[b, pos] = 1
        _, best_anchor = iou.max(dim=0)
        for gi in range(boxes.shape[0]):
            ai = best_anchor[gi]
            if not pos[ai] and iou[ai, gi] >= neg_thr:
                pos[ai] = True
                cls_t[b, ai] = 1
        fin = cls_t[b] == 1
        idx = torch.where(fin)[0]
        if idx.numel():
            a, gbx = anchors[idx], boxes[arg[fin]]
            eps = 1e-6
            box_t[b, idx] = torch.stack([
                (gbx[:, 0] - a[:, 0]) / (a[:, 2] + eps), (gbx[:, 1] - a[:, 1]) / (a[:, 3] + eps),
                torch.log(gbx[:, 2] / (a[:, 2] + eps) + eps), torch.log(gbx[:, 3] / (a[:, 3] + eps) + eps),
                torch.sin(gbx[:, 4] - a[:, 4]), torch.cos(gbx[:, 4] - a[:, 4])], dim=1)
            int_t[b, idx] = ints[arg[fin]]
    return cls_t, box_t, int_t


def detection_loss(cls_logits, box_preds, intent_logits, anchors, gt_list, *, downsampling=True,
                   keep=None, keep_prob=0.15, dominant=DOMINANT, class_weights=None, alpha=0.25, gamma=2.0,
                   beta=1.0 / 9.0, w_cls=1.0, w_box=1.0, w_int=0.5, iou_fn=axis_aligned_iou):
    """loss.py:58-206. ``keep``: optional (B, NA) float 0/1 per-anchor keep mask applied to
    dominant-class positives (the product's device-RNG formulation); ``None`` reproduces
    the reference's global-RNG ``torch.rand`` draws in dominant-class order."""
    cls_t, box_t, int_t = assign_targets(anchors, gt_list, iou_fn=iou_fn)
    ct, bt, it = cls_t.reshape(-1), box_t.reshape(-1, 6), int_t.reshape(-1)
    cl = cls_logits.reshape(-1, 1)
    valid, pos = ct >= 0, ct == 1
    num_pos = pos.sum()
    cls_loss = torch.tensor(0.0)
    if valid.any():
        cls_loss = sigmoid_focal_loss(cl[valid], ct[valid].float().unsqueeze(1), alpha, gamma).sum() / max(1, num_pos)
    box_loss = torch.tensor(0.0)
    int_loss = torch.tensor(0.0)
    if num_pos > 0:
        box_loss = F.smooth_l1_loss(box_preds.reshape(-1, 6)[pos], bt[pos], beta=beta, reduction="sum") / max(1, num_pos)
        il = intent_logits.reshape(-1, intent_logits.shape[-1])[pos]
        itp = it[pos]
        ce = F.cross_entropy(il, itp, weight=None if downsampling else class_weights, reduction="none")
        if downsampling:
            with torch.no_grad():
                m = torch.ones_like(itp, dtype=torch.float32)
                if keep is not None:
                    kf = keep.reshape(-1)[pos].float()
                    for d in dominant:
                        sel = itp == d
                        m[sel] = kf[sel]
                else:
                    for d in dominant:
                        sel = itp == d
                        if sel.any():
                            m[sel] = (torch.rand(int(sel.sum().item())) < keep_prob).float()
            int_loss = (ce * m).sum() / max(1, m.sum())
        else:
            int_loss = ce.sum() / max(1, itp.numel())
    total = w_cls * cls_loss + w_box * box_loss + w_int * int_loss
    if torch.isnan(total).any() or torch.isinf(total).any():
        z = torch.tensor(0.0)
        return {"loss": torch.tensor(0.0, requires_grad=True), "cls_loss": z, "box_loss": z,
                "intent_loss": z, "num_pos_anchors": int(num_pos)}
    return {"loss": total, "cls_loss": cls_loss.detach(), "box_loss": box_loss.detach(),
            "intent_loss": int_loss.detach(), "num_pos_anchors": int(num_pos)}


# --------------------------------------------------------------------------------------
# Synthetic inputs (BASELINE.md "CPU baseline plan"; SURVEY.md §8(d) synthetic inputs)
# --------------------------------------------------------------------------------------
def synthetic_batch(B, img_size=(400, 720), lidar_ch=290, map_ch=9, seed=1234, G=20, grid_scale=1.0,
                    box_region=None):
    """lidar ~ U[0,1), map ~ Bernoulli(0.1), G boxes per sample. ``box_region`` =
    (xmin, xmax, ymin, ymax) overrides the metric box-centre range."""
    g = torch.Generator().manual_seed(seed)
    H, W = img_size
    lidar = torch.rand((B, lidar_ch, H, W), generator=g)
    mp = (torch.rand((B, map_ch, H, W), generator=g) < 0.1).float()
    if box_region is None:
        box_region = (-20.0 * grid_scale, 60.0 * grid_scale, -72.0 * grid_scale, 72.0 * grid_scale)
    x0, x1, y0, y1 = box_region
    gts = []
    for _ in range(B):
        u = torch.rand((G, 5), generator=g)
        boxes = torch.stack([x0 + (x1 - x0) * u[:, 0], y0 + (y1 - y0) * u[:, 1], 1.5 + 1.5 * u[:, 2],
                             3.5 + 3.0 * u[:, 3], -math.pi + 2 * math.pi * u[:, 4]], dim=1)
        ints = torch.randint(0, 8, (G,), generator=g)
        gts.append({"boxes_xywha": boxes.float(), "intentions": ints.long()})
    return lidar, mp, gts


# --------------------------------------------------------------------------------------
# LiDAR BEV voxelisation + sweep ego transform
# --------------------------------------------------------------------------------------
BEV_H, BEV_W, Z_MIN, Z_MAX, HEIGHT_CH, SWEEPS = 400, 720, -2.0, 3.8, 29, 10  # constants.py:28,40-43


def sweep_rel_transform(ego_pose, sweep_pose):
    """dataset.py:290-300 + :327-339: rel_tf = inv(world_SE3_ego) @ world_SE3_sweep, each SE3 from
    (tx, ty, tz, qx, qy, qz, qw) (scipy Rotation.from_quat, scalar-last)."""
    from scipy.spatial.transform import Rotation
    def se3(p):
        m = np.eye(4)
        m[:3, :3] = Rotation.from_quat(list(p[3:7])).as_matrix()
        m[:3, 3] = list(p[:3])
        return m
    return np.linalg.inv(se3(ego_pose)) @ se3(sweep_pose)


def transform_points_np(points, tf):
    """utils.py:27-33: (T @ [x y z 1]^T)^T[:, :3] in f64 (numpy matmul, as the reference)."""
    if points.shape[0] == 0:
        return np.empty((0, 3), dtype=points.dtype)
    h = np.hstack((points[:, :3], np.ones((points.shape[0], 1))))
    return (tf @ h.T).T[:, :3]


def lidar_bev_np(points_list, intensity_list, num_sweeps=SWEEPS, H=BEV_H, W=BEV_W):
    """utils.py:62-106: per sweep i, cells (floor(W/2 + y/0.2), floor(3H/4 - x/0.2)) inside the grid with
    z in [Z_MIN, Z_MAX) take max(cell, intensity) in channel i*29 + clip(floor((z-Z_MIN)/(Z_MAX-Z_MIN)*29))."""
    bev = np.zeros((HEIGHT_CH * num_sweeps, H, W), dtype=np.float32)
    for i in range(min(len(points_list), len(intensity_list))):
        p, v = points_list[i], intensity_list[i]
        if p is None or v is None or p.shape[0] == 0:
            continue
        x, y, z = p[:, 0], p[:, 1], p[:, 2]
        px = np.floor(W / 2.0 + y / VOXEL).astype(np.int64)          # utils.py:80
        py = np.floor(H * 3.0 / 4.0 - x / VOXEL).astype(np.int64)    # utils.py:81
        ok = (px >= 0) & (px < W) & (py >= 0) & (py < H) & (z >= Z_MIN) & (z < Z_MAX)
        if not ok.any():
            continue
        hz = np.clip(np.floor((z[ok] - Z_MIN) / (Z_MAX - Z_MIN) * HEIGHT_CH).astype(np.int64), 0, HEIGHT_CH - 1)
        flat = ((i * HEIGHT_CH + hz) * H + py[ok]) * W + px[ok]
        np.maximum.at(bev.reshape(-1), flat, v[ok].astype(np.float32))  # utils.py:99-104 (order-free max)
    return bev


# --------------------------------------------------------------------------------------
# BEV augmentations (utils.py:394-517)
# --------------------------------------------------------------------------------------
# cv2 is absent from this image, so the two OpenCV resamplers the reference calls are restated
# from OpenCV's long-standing generic scalar paths (imgwarp.cpp getRotationMatrix2D /
# WarpAffineInvoker / remapBilinear, resize.cpp resizeGeneric HResizeLinear / VResizeLinear, as
# in 3.x-4.10) for single-channel f32 planes: every product / sum rounds to f32 on its own (no
# fused multiply-add; SIMD-dispatched OpenCV builds may fuse and differ by an ulp).
# PARITY UNPINNED for that resampling arithmetic. The flow around it (random draw order,
# crop / pad offsets, dropout rectangles, GT box and intention updates) is pinned: make_golden.py
# runs the reference's OWN random_* / augment_bev with these functions as its cv2 stand-in.
import random as _random  # noqa: E402

_INTER_BITS, _INTER_TAB, _AB_BITS = 5, 32, 10


def cv2_get_rotation_matrix_2d(center, angle_deg, scale):
    """getRotationMatrix2D (f64): [[a, b, (1-a)cx - b cy], [-b, a, b cx + (1-a)cy]]; the centre is a
    Point2f, so it is rounded to f32 first."""
    ang = angle_deg * (math.pi / 180)
    a, b = math.cos(ang) * scale, math.sin(ang) * scale
    cx, cy = float(np.float32(center[0])), float(np.float32(center[1]))
    return np.array([[a, b, (1 - a) * cx - b * cy], [-b, a, b * cx + (1 - a) * cy]], dtype=np.float64)


def cv2_invert_affine(M):
    """warpAffine without WARP_INVERSE_MAP inverts M in f64 (dst -> src map), in this order."""
    m = [float(v) for v in np.asarray(M, np.float64).reshape(6)]
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    a11, a22 = m[4] * D, m[0] * D
    m[0] = a11
    m[1] *= -D
    m[3] *= -D
    m[4] = a22
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    return m


def _sat_i16(v):
    return np.clip(v, -32768, 32767)


def cv2_warp_affine_linear(img, M, dsize, flip_src=False):
    """cv2.warpAffine(img, M, dsize, INTER_LINEAR, BORDER_CONSTANT, 0) for one f32 plane (or a
    [C, H, W] stack, same map per plane). Source coordinates in 1/32-pixel fixed point:
    X = (round((m1 y + m2) 1024) + 16 + round(m0 x 1024)) >> 5 (round = half-to-even), tap
    (X >> 5, Y >> 5), weights from the exact 32x32 bilinear table; taps outside the image read 0.
    flip_src mirrors the source columns first (np.flip(axis=-1), fused)."""
    src = np.asarray(img, np.float32)
    Hs, Ws = src.shape[-2:]
    Wd, Hd = int(dsize[0]), int(dsize[1])
    m = cv2_invert_affine(M)
    xs, ys = np.arange(Wd, dtype=np.float64), np.arange(Hd, dtype=np.float64)
    adelta = np.rint(m[0] * xs * 1024.0).astype(np.int64)
    bdelta = np.rint(m[3] * xs * 1024.0).astype(np.int64)
    rd = (1 << _AB_BITS) // _INTER_TAB // 2
    X0 = np.rint((m[1] * ys + m[2]) * 1024.0).astype(np.int64) + rd
    Y0 = np.rint((m[4] * ys + m[5]) * 1024.0).astype(np.int64) + rd
    X = (X0[:, None] + adelta[None, :]) >> (_AB_BITS - _INTER_BITS)
    Y = (Y0[:, None] + bdelta[None, :]) >> (_AB_BITS - _INTER_BITS)
    sx, sy = _sat_i16(X >> _INTER_BITS), _sat_i16(Y >> _INTER_BITS)
    tx = (X & (_INTER_TAB - 1)).astype(np.float32) * np.float32(1.0 / _INTER_TAB)
    ty = (Y & (_INTER_TAB - 1)).astype(np.float32) * np.float32(1.0 / _INTER_TAB)
    one = np.float32(1.0)
    w = [(one - ty) * (one - tx), (one - ty) * tx, ty * (one - tx), ty * tx]
    flat = src.reshape(-1, Hs * Ws)
    out = np.zeros((flat.shape[0], Hd, Wd), np.float32)
    acc = None
    for k, (dy, dx) in enumerate(((0, 0), (0, 1), (1, 0), (1, 1))):
        cx, cy = sx + dx, sy + dy
        ok = (cx >= 0) & (cx < Ws) & (cy >= 0) & (cy < Hs)
        col = (Ws - 1 - cx) if flip_src else cx
        idx = np.where(ok, cy * Ws + col, 0)
        v = np.where(ok[None], flat[:, idx], np.float32(0.0))
        term = v * w[k][None]
        acc = term if acc is None else acc + term
    out[:] = acc
    return out.reshape(src.shape[:-2] + (Hd, Wd))


def _resize_axis(n_dst, n_src, scale):
    """resizeGeneric's per-axis source index / weights (INTER_LINEAR, f32 data)."""
    f = ((np.arange(n_dst, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = f - s.astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0, 0
    hi = s >= n_src - 1  # also xmax: HResizeLinear copies S[sx] from here on
    f[hi], s[hi] = 0, n_src - 1
    return s, np.float32(1.0) - f, f, hi


def cv2_resize_linear(img, dsize, flip_src=False):
    """cv2.resize(img, dsize, interpolation=INTER_LINEAR) for f32 planes ([.., H, W]): horizontal
    pass h = S[sx] a0 + S[sx+1] a1 (S[sx] alone at the right clamp), then vertical
    h[r0] b0 + h[r1] b1 with clipped rows; scale = 1 / (dst / src) in f64; same size -> copy."""
    src = np.asarray(img, np.float32)
    if flip_src:
        src = src[..., ::-1]
    Hs, Ws = src.shape[-2:]
    Wd, Hd = int(dsize[0]), int(dsize[1])
    if (Wd, Hd) == (Ws, Hs):
        return src.copy()
    sx, a0, a1, copy = _resize_axis(Wd, Ws, 1.0 / (Wd / Ws))
    sy, b0, b1, _ = _resize_axis(Hd, Hs, 1.0 / (Hd / Hs))
    sx1 = np.minimum(sx + 1, Ws - 1)
    h = np.where(copy, src[..., sx], src[..., sx] * a0 + src[..., sx1] * a1)  # [.., Hs, Wd]
    r1 = np.minimum(sy + 1, Hs - 1)
    return (h[..., sy, :] * b0[:, None] + h[..., r1, :] * b1[:, None]).astype(np.float32)


def resize_crop_pad(img, scale_factor, H=BEV_H, W=BEV_W, flip_src=False):
    """random_scale_bev's per-channel body (utils.py:460-474): resize to int(H s) x int(W s), then
    centre-crop (s > 1) or centre-pad with zeros (s <= 1) back to H x W."""
    new_h, new_w = int(H * scale_factor), int(W * scale_factor)
    r = cv2_resize_linear(img, (new_w, new_h), flip_src=flip_src)
    out = np.zeros(np.asarray(img).shape[:-2] + (H, W), np.float32)
    if scale_factor > 1.0:
        h0, w0 = (new_h - H) // 2, (new_w - W) // 2
        out[...] = r[..., h0:h0 + H, w0:w0 + W]
    else:
        h0, w0 = (H - new_h) // 2, (W - new_w) // 2
        out[..., h0:h0 + new_h, w0:w0 + new_w] = r
    return out


FLIP_INTENTION = np.array([0, 2, 1, 4, 3, 5, 6, 7], np.int64)  # utils.py:406-411 (constants.py:64-67)


def draw_augment_params(rng=_random, H=BEV_H, W=BEV_W):
    """The random draws of augment_bev (utils.py:500-511) in the reference's order: flip (:399),
    rotate (:422-423), scale (:451-452), dropout (:484-490)."""
    p = {"flip": rng.random() < 0.5, "angle": None, "scale": None, "rects": []}
    if rng.random() < 0.5:
        p["angle"] = rng.uniform(-15.0, 15.0)
    if rng.random() < 0.5:
        p["scale"] = rng.uniform(0.95, 1.05)
    if rng.random() < 0.1:
        for _ in range(rng.randint(1, 5)):
            ph, pw = rng.randint(20, 50), rng.randint(20, 50)
            p["rects"].append((rng.randint(0, max(0, H - ph)), rng.randint(0, max(0, W - pw)), ph, pw))
    return p


def augment_gt_np(boxes, intents, p):
    """GT updates of random_flip / rotate / scale_bev (utils.py:402-411, 440-447, 476-477)."""
    boxes = np.array(boxes, dtype=np.float32, copy=True)
    intents = np.array(intents, dtype=np.int64, copy=True)
    if p["flip"]:
        if boxes.shape[0] > 0:
            boxes[:, 1] *= -1
            boxes[:, 4] *= -1
            boxes[:, 4] = np.arctan2(np.sin(boxes[:, 4]), np.cos(boxes[:, 4]))
        if intents.shape[0] > 0:
            intents = FLIP_INTENTION[intents]
    if p["angle"] is not None and boxes.shape[0] > 0:
        rad = np.radians(p["angle"])
        cx, cy = boxes[:, 0].copy(), boxes[:, 1].copy()
        c, s = np.cos(rad), np.sin(rad)
        boxes[:, 0], boxes[:, 1] = cx * c - cy * s, cx * s + cy * c
        boxes[:, 4] += rad
        boxes[:, 4] = np.arctan2(np.sin(boxes[:, 4]), np.cos(boxes[:, 4]))
    if p["scale"] is not None and boxes.shape[0] > 0:
        boxes[:, :4] *= p["scale"]
    return boxes, intents


def augment_planes_np(x, p, H=BEV_H, W=BEV_W):
    """The raster side of augment_bev on one [C, H, W] f32 stack with drawn params p."""
    y = np.array(x, np.float32, copy=True)
    if p["flip"]:
        y = np.ascontiguousarray(y[..., ::-1])
    if p["angle"] is not None:
        M = cv2_get_rotation_matrix_2d((W / 2.0, H / 2.0), p["angle"], 1.0)
        y = cv2_warp_affine_linear(y, M, (W, H))
    if p["scale"] is not None:
        y = resize_crop_pad(y, p["scale"], H, W)
    for y0, x0, ph, pw in p["rects"]:
        y[..., y0:y0 + ph, x0:x0 + pw] = 0.0
    return y


def augment_bev_np(lidar, map_bev, boxes, intents, rng=_random):
    """utils.augment_bev (utils.py:500-517) restated: -> (lidar, map, boxes, intents, params)."""
    p = draw_augment_params(rng, *np.asarray(lidar).shape[-2:])
    H, W = np.asarray(lidar).shape[-2:]
    b, i = augment_gt_np(boxes, intents, p)
    return augment_planes_np(lidar, p, H, W), augment_planes_np(map_bev, p, H, W), b, i, p


def bev_augment_inputs(seed, lidar_ch=3, map_ch=2, G=20, H=BEV_H, W=BEV_W):
    """Seeded BEV-like planes + GT for the augmentation fixtures (regenerated on the GPU box):
    sparse lidar intensities in [0, 255), Bernoulli(0.1) map, G boxes as in bench's synthetic GT."""
    rng = np.random.default_rng(seed)
    lidar = (rng.random((lidar_ch, H, W), dtype=np.float32) * np.float32(255.0))
    lidar *= (rng.random((lidar_ch, H, W)) < 0.3)
    mp = (rng.random((map_ch, H, W)) < 0.1).astype(np.float32)
    boxes = np.stack([rng.uniform(-20, 60, G), rng.uniform(-72, 72, G), rng.uniform(1.5, 3.0, G),
                      rng.uniform(3.5, 6.5, G), rng.uniform(-math.pi, math.pi, G)], 1).astype(np.float32)
    intents = rng.integers(0, 8, G).astype(np.int64)
    return lidar, mp, boxes, intents


# --------------------------------------------------------------------------------------
# IntentNetCNN (model_cnn.py) — torch fp32 restatement
# --------------------------------------------------------------------------------------
CNN_STAGES = (("lidar", ((160, 2), (192, 1), (224, 2))), ("map", ((32, 2), (64, 1), (96, 2))))  # model_cnn.py:39-73


def _cnn_bn(sd, p, x, training):
    rm, rv = sd[p + "running_mean"], sd[p + "running_var"]
    return F.batch_norm(x, rm, rv, sd[p + "weight"], sd[p + "bias"], training, 0.1, 1e-5)


def cnn_block(sd, p, x, stride, k, training):
    """model_cnn.py:14-33: conv k x k (pad (k-1)//2, stride) -> BN -> ReLU -> conv k x k -> BN,
    + identity (conv1x1 stride + BN when p + 'downsample.0.weight' exists) -> ReLU."""
    pad = (k - 1) // 2
    out = F.relu(_cnn_bn(sd, p + "bn1.", F.conv2d(x, sd[p + "conv1.weight"], None, stride, pad), training))
    out = _cnn_bn(sd, p + "bn2.", F.conv2d(out, sd[p + "conv2.weight"], None, 1, pad), training)
    if p + "downsample.0.weight" in sd:
        x = _cnn_bn(sd, p + "downsample.1.", F.conv2d(x, sd[p + "downsample.0.weight"], None, stride), training)
    return F.relu(out + x)


def cnn_forward(sd, lidar, map_bev, training=False, ks=5, fusion_ks=3, blocks=2, fusion_layers=2):
    """IntentNetCNN.forward (model_cnn.py:110-150). BN running stats in sd update in place in
    training mode, as nn.BatchNorm2d's do."""
    def stage(name, x, stride, k, n):
        for i in range(n):
            x = cnn_block(sd, f"backbone.{name}.{i}.", x, stride if i == 0 else 1, k, training)
        return x
    feats = []
    for stream_name, stages in CNN_STAGES:
        x = lidar if stream_name == "lidar" else map_bev
        for si, (_, stride) in enumerate(stages):
            x = stage(f"{stream_name}_stage{si + 1}", x, stride, ks, blocks)
        feats.append(x)
    f = stage("fusion_block", torch.cat(feats, 1), 2, fusion_ks, fusion_layers)
    return heads_forward(sd, f)


# --------------------------------------------------------------------------------------
# HD-map rasterisation: utils.py:35-60 (ego transform, world → pixel)
# and utils.py:108-182 (rasterize_map_ego_centric), with OpenCV's integer fillPoly / polylines
# (LINE_8, thickness 1, shift 0) restated from OpenCV 4.x imgproc/drawing.cpp. cv2 is absent
# here: PARITY UNPINNED at the OpenCV level (the flow is pinned by tests/golden/map_raster.npz).
# --------------------------------------------------------------------------------------
CV_XY_SHIFT = 16
MAP_CH = 9


def cv_line8_pixels(p0, p1):
    """cv::LineIterator(connectivity 8, leftToRight) pixels of the segment p0 → p1 (x, y ints);
    both endpoints inside the image (the callers pre-filter points)."""
    (x0, y0), (x1, y1) = p0, p1
    dx, dy = x1 - x0, y1 - y0
    if dx < 0:  # leftToRight: iterate from the left endpoint
        dx, dy = -dx, -dy
        x0, y0, x1, y1 = x1, y1, x0, y0
    sy = 1
    if dy < 0:
        dy, sy = -dy, -1
    vert = dy > dx
    major, minor = (dy, dx) if vert else (dx, dy)
    err = major - 2 * minor
    out = []
    x, y = x0, y0
    for _ in range(major + 1):
        out.append((x, y))
        step = err < 0
        err += -2 * minor + (2 * major if step else 0)
        if vert:
            y += sy
            x += 1 if step else 0
        else:
            x += 1
            y += sy if step else 0
    return out


def _trunc_div(a, b):
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def cv_fill_poly(img, pts):
    """cv2.fillPoly(img, [pts], 1) for one polygon of integer (x, y) vertices, LINE_8, shift 0:
    CollectPolyEdges (every edge also drawn by Line) + FillEdgeCollection scanlines (edge x in
    16.16 fixed point, x += dx per scanline, spans [x_l >> 16, x_r >> 16] between sorted pairs,
    an edge active on y0 <= y < y1, horizontal edges skipped, fewer than 2 edges: no fill)."""
    H, W = img.shape
    pts = [(int(x), int(y)) for x, y in pts]
    n = len(pts)
    edges = []
    for i in range(n):
        (xa, ya), (xb, yb) = pts[i - 1], pts[i]
        for x, y in cv_line8_pixels((xa, ya), (xb, yb)):
            if 0 <= x < W and 0 <= y < H:
                img[y, x] = 1
        if ya == yb:
            continue
        Xa, Xb = xa << CV_XY_SHIFT, xb << CV_XY_SHIFT
        if ya < yb:
            e = (ya, yb, Xa)
        else:
            e = (yb, ya, Xb)
        edges.append((e[0], e[1], e[2], _trunc_div(Xb - Xa, yb - ya)))
    if len(edges) < 2:
        return img
    y_min = min(e[0] for e in edges)
    y_max = min(max(e[1] for e in edges), H)
    for y in range(max(y_min, 0), y_max):
        xs = sorted(x0 + (y - ya) * dx for ya, yb, x0, dx in edges if ya <= y < yb)
        for k in range(0, len(xs) - 1, 2):
            x1, x2 = xs[k] >> CV_XY_SHIFT, xs[k + 1] >> CV_XY_SHIFT
            if x1 < W and x2 >= 0:
                img[y, max(x1, 0):min(x2, W - 1) + 1] = 1
    return img


def cv_polyline(img, pts):
    """cv2.polylines(img, [pts], isClosed=False, 1, thickness=1): Line per consecutive pair."""
    H, W = img.shape
    pts = [(int(x), int(y)) for x, y in pts]
    for i in range(1, len(pts)):
        for x, y in cv_line8_pixels(pts[i - 1], pts[i]):
            if 0 <= x < W and 0 <= y < H:
                img[y, x] = 1
    return img


def ego_yaw_from_quat(qx, qy, qz, qw):
    """scipy Rotation.from_quat([qx, qy, qz, qw]).as_euler('xyz')[2] (utils.py:123)."""
    from scipy.spatial.transform import Rotation
    return float(Rotation.from_quat([qx, qy, qz, qw]).as_euler('xyz')[2])


def world_to_pixel_np(world_xy, ego_xy, ego_yaw, H=BEV_H, W=BEV_W, voxel=0.2):
    """utils.py:35-60: T = [R(-yaw) | -R(-yaw) t] (f64), pixel = round(offset ± ego / voxel)."""
    c, s = np.cos(-ego_yaw), np.sin(-ego_yaw)
    Rm = np.array([[c, -s], [s, c]])
    T = np.eye(3)
    T[:2, :2] = Rm
    T[:2, 2] = -Rm @ np.asarray(ego_xy, np.float64)
    homo = np.hstack([world_xy, np.ones((world_xy.shape[0], 1))])
    ego = (T @ homo.T).T[:, :2]
    px = W / 2.0 + ego[:, 1] / voxel
    py = H * 3.0 / 4.0 - ego[:, 0] / voxel
    return np.round(np.vstack([px, py]).T).astype(int)


def map_pixels_np(points, ego_xy, ego_yaw, H=BEV_H, W=BEV_W):
    """to_bev_pixel_local (utils.py:131-145): drop malformed points, transform, keep in-bounds."""
    if not points:
        return np.empty((0, 2), dtype=int)
    valid = [p for p in points if isinstance(p, dict) and 'x' in p and 'y' in p]
    if not valid:
        return np.empty((0, 2), dtype=int)
    xy = np.array([[p['x'], p['y']] for p in valid])
    pix = world_to_pixel_np(xy, ego_xy, ego_yaw, H, W)
    m = (pix[:, 0] >= 0) & (pix[:, 0] < W) & (pix[:, 1] >= 0) & (pix[:, 1] < H)
    return pix[m]


MARK_CHANNELS = {"DASHED_WHITE": 6, "SOLID_WHITE": 7, "SOLID_YELLOW": 8}


def rasterize_map_np(map_data, ego_pose, H=BEV_H, W=BEV_W):
    """rasterize_map_ego_centric (utils.py:108-182) on a parsed map dict and an ego pose mapping
    with tx_m, ty_m, qx, qy, qz, qw → (9, H, W) float32 {0, 1}."""
    out = np.zeros((MAP_CH, H, W), np.uint8)
    yaw = ego_yaw_from_quat(ego_pose['qx'], ego_pose['qy'], ego_pose['qz'], ego_pose['qw'])
    exy = (ego_pose['tx_m'], ego_pose['ty_m'])
    for _, lane in map_data.get("lane_segments", {}).items():
        lpx = map_pixels_np(lane.get("left_lane_boundary", []), exy, yaw, H, W)
        rpx = map_pixels_np(lane.get("right_lane_boundary", []), exy, yaw, H, W)
        if len(lpx) > 1 and len(rpx) > 1:
            poly = np.vstack([lpx, np.flipud(rpx)])
            if poly.shape[0] >= 3:
                cv_fill_poly(out[0], poly)
                if lane.get("is_intersection", False):
                    cv_fill_poly(out[4], poly)
                if lane.get("lane_type") == "BUS":
                    cv_fill_poly(out[5], poly)
        if len(lpx) > 1:
            cv_polyline(out[1], lpx)
        if len(rpx) > 1:
            cv_polyline(out[2], rpx)
        lm, rm = lane.get("left_lane_mark_type", ""), lane.get("right_lane_mark_type", "")
        if lm in MARK_CHANNELS and len(lpx) > 1:
            cv_polyline(out[MARK_CHANNELS[lm]], lpx)
        if rm in MARK_CHANNELS and len(rpx) > 1:
            cv_polyline(out[MARK_CHANNELS[rm]], rpx)
    for _, cw in map_data.get("pedestrian_crossings", {}).items():
        poly = cw.get('polygon', [])
        if poly:
            px = map_pixels_np(poly, exy, yaw, H, W)
            if len(px) >= 3:
                cv_fill_poly(out[3], px)
    return out.astype(np.float32)


def synthetic_map(seed, n_lanes=40, n_cross=6, center=(100.0, -50.0), spread=70.0):
    """A seeded Argoverse-2-style map dict: lanes with left / right boundaries of 2-12 points
    (some leaving the grid, some malformed), intersections, bus lanes, the three mark types and
    others, crosswalk polygons; plus degenerate cases (1-point / empty boundaries, collinear and
    horizontal polygons)."""
    rng = np.random.default_rng(seed)
    cx, cy = center
    lanes = {}
    marks = ["DASHED_WHITE", "SOLID_WHITE", "SOLID_YELLOW", "DOUBLE_SOLID_YELLOW", "NONE", ""]
    for i in range(n_lanes):
        n = int(rng.integers(2, 13))
        x0, y0 = cx + rng.uniform(-spread, spread), cy + rng.uniform(-spread, spread)
        ang = rng.uniform(-np.pi, np.pi)
        L = rng.uniform(5, 60)
        t = np.linspace(0, L, n)
        bend = rng.normal(0, 0.02)
        xs = x0 + t * np.cos(ang + bend * t)
        ys = y0 + t * np.sin(ang + bend * t)
        w = rng.uniform(2.5, 4.5)
        nx, ny = -np.sin(ang), np.cos(ang)
        left = [{"x": float(a + nx * w / 2), "y": float(b + ny * w / 2), "z": 0.0} for a, b in zip(xs, ys)]
        right = [{"x": float(a - nx * w / 2), "y": float(b - ny * w / 2), "z": 0.0} for a, b in zip(xs, ys)]
        if i % 13 == 5:
            left = left[:1]  # a 1-point boundary: no polygon, no polyline
        if i % 17 == 3:
            right = [{"y": 1.0}] + right  # a malformed point is dropped
        lanes[str(1000 + i)] = {"left_lane_boundary": left, "right_lane_boundary": right,
                                "is_intersection": bool(rng.random() < 0.25),
                                "lane_type": "BUS" if rng.random() < 0.15 else "VEHICLE",
                                "left_lane_mark_type": marks[int(rng.integers(len(marks)))],
                                "right_lane_mark_type": marks[int(rng.integers(len(marks)))]}
    # a horizontal-edge polygon (axis-aligned in the ego frame is not guaranteed; a sliver) and an empty lane
    lanes["9001"] = {"left_lane_boundary": [], "right_lane_boundary": []}
    crosses = {}
    for i in range(n_cross):
        x0, y0 = cx + rng.uniform(-spread / 2, spread / 2), cy + rng.uniform(-spread / 2, spread / 2)
        a = rng.uniform(-np.pi, np.pi)
        Lw, Ww = rng.uniform(4, 15), rng.uniform(2, 5)
        pts = [(0, 0), (Lw, 0), (Lw, Ww), (0, Ww)]
        c, s = np.cos(a), np.sin(a)
        crosses[str(2000 + i)] = {"polygon": [{"x": float(x0 + c * u - s * v), "y": float(y0 + s * u + c * v), "z": 0.0}
                                              for u, v in pts]}
    crosses["2999"] = {"polygon": []}
    return {"lane_segments": lanes, "pedestrian_crossings": crosses}


def synthetic_pose(seed, center=(100.0, -50.0)):
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(seed)
    q = Rotation.from_euler("xyz", [rng.normal(0, 0.01), rng.normal(0, 0.01), rng.uniform(-np.pi, np.pi)]).as_quat()
    return {"tx_m": center[0] + rng.normal(0, 5), "ty_m": center[1] + rng.normal(0, 5), "tz_m": 0.0,
            "qx": q[0], "qy": q[1], "qz": q[2], "qw": q[3]}
