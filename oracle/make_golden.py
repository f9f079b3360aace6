"""Generate golden vectors from the reference's OWN code (run HERE only).

    cd /root/repo && python -m oracle.make_golden

Imports ``model_vit``, ``heads``, ``loss``, ``utils``, ``constants`` from
/root/reference through ``oracle/refshim.py`` stand-ins, feeds them seeded
inputs and the ``oracle/weights.py`` filler, and writes small ``.npz``
fixtures (inputs as seeds + checksums, outputs as arrays / strided samples)
into ``tests/golden/``. The reference never travels to the GPU box: only these
data files do.
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

from oracle import ivit_oracle as O  # noqa: E402
from oracle import refshim  # noqa: E402
from oracle.weights import make_state_dict, model_cfg, state_checksum  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
SMALL_IMG = (32, 48)
N_SAMPLE = 64


def _sample(t):
    f = t.detach().reshape(-1).double()
    stride = max(1, f.numel() // N_SAMPLE)
    s = f[::stride][:N_SAMPLE].numpy()
    out = np.full(N_SAMPLE, np.nan)
    out[: s.size] = s
    return out, stride


def small_gt(seed=4321):
    """GT boxes inside the 32×48 grid's anchor footprint (x∈[54,60], y∈[-72,-62])."""
    g = torch.Generator().manual_seed(seed)
    gts = []
    for G in (6, 4):
        u = torch.rand((G, 5), generator=g)
        boxes = torch.stack([54.0 + 6.0 * u[:, 0], -72.0 + 10.0 * u[:, 1], 1.5 + 1.5 * u[:, 2],
                             3.5 + 3.0 * u[:, 3], -math.pi + 2 * math.pi * u[:, 4]], 1).float()
        gts.append({"boxes_xywha": boxes, "intentions": torch.randint(0, 8, (G,), generator=g)})
    return gts


def gen_model_small():
    import loss as ref_loss
    import model_vit as ref_model
    import utils as ref_utils
    cfg = model_cfg(img_size=SMALL_IMG)
    sd = make_state_dict(cfg, seed=0)
    lidar, mp, _ = O.synthetic_batch(2, SMALL_IMG, seed=1234)
    gts = small_gt()
    anchors = ref_utils.generate_anchors(SMALL_IMG[0], SMALL_IMG[1], 8)
    bcfg = {"img_size": SMALL_IMG, "lidar_input_channels": 290, "map_input_channels": 9,
            "drop_path_rate_lidar": 0.0, "drop_path_rate_map": 0.0}
    m = ref_model.IntentNetViT(backbone_cfg=dict(bcfg))
    m.load_state_dict(refshim.timm_to_hf_state(sd), strict=True)
    rec = {"cfg": json.dumps(cfg), "w_checksum": state_checksum(sd),
           "lidar_sum": float(lidar.double().sum()), "map_sum": float(mp.double().sum()),
           "anchors": anchors.numpy()}
    for i, g in enumerate(gts):
        rec[f"gt{i}_boxes"] = g["boxes_xywha"].numpy()
        rec[f"gt{i}_ints"] = g["intentions"].numpy()
    m.eval()
    with torch.no_grad():
        c, b, it = m(lidar, mp)
    rec.update(eval_cls=c.numpy(), eval_box=b.numpy(), eval_int=it.numpy())
    # train mode, DropPath 0, BN batch statistics, downsampling off
    m.train()
    c, b, it = m(lidar, mp)
    lf = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=False)
    d = lf(c, b, it, anchors, gts)
    d["loss"].backward()
    rec.update(train_cls=c.detach().numpy(), train_box=b.detach().numpy(), train_int=it.detach().numpy(),
               train_loss=np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]),
                                    float(d["intent_loss"]), float(d["num_pos_anchors"])]))
    grads = refshim.hf_grads_to_timm({k: p.grad for k, p in m.named_parameters() if p.grad is not None})
    names = sorted(grads)
    samples, strides = zip(*[_sample(grads[k]) for k in names])
    rec.update(grad_names=np.array(names), grad_sum=np.array([float(grads[k].double().sum()) for k in names]),
               grad_abssum=np.array([float(grads[k].double().abs().sum()) for k in names]),
               grad_samples=np.stack(samples), grad_strides=np.array(strides))
    bn = {k: v for k, v in m.state_dict().items() if "running_" in k}
    rec.update(bn_names=np.array(sorted(bn)), bn_values=np.stack([bn[k].numpy() for k in sorted(bn)]))
    # downsampling on: the reference's own torch.rand draws under a fixed global seed
    with torch.no_grad():
        torch.manual_seed(77)
        d2 = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=True)(c, b, it, anchors, gts)
    rec["train_loss_ds"] = np.array([float(d2["loss"]), float(d2["cls_loss"]), float(d2["box_loss"]),
                                     float(d2["intent_loss"]), float(d2["num_pos_anchors"])])
    np.savez_compressed(os.path.join(OUT, "model_small.npz"), **rec)
    print("model_small: loss", rec["train_loss"], "ds", rec["train_loss_ds"])


def gen_model_stride2():
    """The reference's OWN IntentNetViT with fusion_block_stride=2 (model_vit.py:55,125-128: block
    0's conv1 and downsample strided, heads at H/16 x W/16, effective_head_stride 16) at the
    32x48 grid: eval + train outputs, loss (downsampling off), gradient samples, BN stats."""
    import loss as ref_loss
    import model_vit as ref_model
    import utils as ref_utils
    cfg = model_cfg(img_size=SMALL_IMG, fusion_stride=2)
    sd = make_state_dict(cfg, seed=0)
    lidar, mp, _ = O.synthetic_batch(2, SMALL_IMG, seed=1234)
    gts = small_gt()
    anchors = ref_utils.generate_anchors(SMALL_IMG[0], SMALL_IMG[1], 16)
    m = ref_model.IntentNetViT(backbone_cfg={"img_size": SMALL_IMG, "lidar_input_channels": 290,
                                             "map_input_channels": 9, "drop_path_rate_lidar": 0.0,
                                             "drop_path_rate_map": 0.0, "fusion_block_stride": 2})
    assert m.effective_head_stride == 16
    m.load_state_dict(refshim.timm_to_hf_state(sd), strict=True)
    rec = {"cfg": json.dumps(cfg), "anchors": anchors.numpy()}
    m.eval()
    with torch.no_grad():
        c, b, it = m(lidar, mp)
    rec.update(eval_cls=c.numpy(), eval_box=b.numpy(), eval_int=it.numpy())
    m.train()
    c, b, it = m(lidar, mp)
    d = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=False)(c, b, it, anchors, gts)
    d["loss"].backward()
    rec.update(train_cls=c.detach().numpy(), train_box=b.detach().numpy(), train_int=it.detach().numpy(),
               train_loss=np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]),
                                    float(d["intent_loss"]), float(d["num_pos_anchors"])]))
    grads = refshim.hf_grads_to_timm({k: p.grad for k, p in m.named_parameters() if p.grad is not None})
    names = sorted(grads)
    samples, strides = zip(*[_sample(grads[k]) for k in names])
    rec.update(grad_names=np.array(names), grad_abssum=np.array([float(grads[k].double().abs().sum()) for k in names]),
               grad_samples=np.stack(samples), grad_strides=np.array(strides))
    bn = {k: v for k, v in m.state_dict().items() if "running_" in k}
    rec.update(bn_names=np.array(sorted(bn)), bn_values=np.stack([bn[k].numpy() for k in sorted(bn)]))
    osd = {k: v.clone() for k, v in sd.items()}
    with torch.no_grad():
        oc, _, _ = O.intentnet_forward(osd, lidar, mp, cfg, training=False)
    assert float((oc - torch.from_numpy(rec["eval_cls"])).abs().max()) < 1e-4, "oracle != reference (stride 2)"
    np.savez_compressed(os.path.join(OUT, "model_stride2.npz"), **rec)
    print("model_stride2: cls", c.shape, "loss", rec["train_loss"])


def gen_model_regrid():
    """The reference's OWN IntentNetViT with a patch-16 map ViT (vit_small_patch16_224 at
    model_vit.py:71): the map grid (2 x 3 at 32x48) differs from the LiDAR grid (4 x 6), so the
    forward re-grids the map features bilinearly (:139). Eval + train outputs, loss, gradient
    samples; plus a standalone F.interpolate case (up and down) for the resize kernel."""
    import loss as ref_loss
    import model_vit as ref_model
    import utils as ref_utils
    cfg = model_cfg(img_size=SMALL_IMG, vit_map="vit_small_patch16_224")
    sd = make_state_dict(cfg, seed=0)
    lidar, mp, _ = O.synthetic_batch(2, SMALL_IMG, seed=1234)
    gts = small_gt()
    anchors = ref_utils.generate_anchors(SMALL_IMG[0], SMALL_IMG[1], 8)
    m = ref_model.IntentNetViT(backbone_cfg={"img_size": SMALL_IMG, "lidar_input_channels": 290,
                                             "map_input_channels": 9, "drop_path_rate_lidar": 0.0,
                                             "drop_path_rate_map": 0.0,
                                             "vit_model_name_map": "vit_small_patch16_224"})
    assert m.backbone.map_grid_size != m.backbone.lidar_grid_size
    m.load_state_dict(refshim.timm_to_hf_state(sd), strict=True)
    rec = {"cfg": json.dumps(cfg), "anchors": anchors.numpy()}
    m.eval()
    with torch.no_grad():
        c, b, it = m(lidar, mp)
    rec.update(eval_cls=c.numpy(), eval_box=b.numpy(), eval_int=it.numpy())
    m.train()
    c, b, it = m(lidar, mp)
    d = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=False)(c, b, it, anchors, gts)
    d["loss"].backward()
    rec.update(train_cls=c.detach().numpy(), train_box=b.detach().numpy(), train_int=it.detach().numpy(),
               train_loss=np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]),
                                    float(d["intent_loss"]), float(d["num_pos_anchors"])]))
    grads = refshim.hf_grads_to_timm({k: p.grad for k, p in m.named_parameters() if p.grad is not None})
    names = sorted(grads)
    samples, strides = zip(*[_sample(grads[k]) for k in names])
    rec.update(grad_names=np.array(names), grad_abssum=np.array([float(grads[k].double().abs().sum()) for k in names]),
               grad_samples=np.stack(samples), grad_strides=np.array(strides))
    bn = {k: v for k, v in m.state_dict().items() if "running_" in k}
    rec.update(bn_names=np.array(sorted(bn)), bn_values=np.stack([bn[k].numpy() for k in sorted(bn)]))
    osd = {k: v.clone() for k, v in sd.items()}
    with torch.no_grad():
        oc, _, _ = O.intentnet_forward(osd, lidar, mp, cfg, training=False)
    assert float((oc - torch.from_numpy(rec["eval_cls"])).abs().max()) < 1e-4, "oracle != reference (re-grid)"
    # standalone resize cases: (Hi, Wi) -> (Ho, Wo), upsampling (the model's 2x) and ragged / down
    g = torch.Generator().manual_seed(77)
    for tag, (hi, wi, ho, wo) in {"up": (25, 45, 50, 90), "odd": (7, 5, 12, 13), "down": (9, 11, 4, 6)}.items():
        x = torch.randn(2, 3, hi, wi, generator=g, requires_grad=True)
        y = torch.nn.functional.interpolate(x, size=(ho, wo), mode="bilinear", align_corners=False)
        dy = torch.randn(y.shape, generator=g)
        y.backward(dy)
        rec.update({f"resize_{tag}_x": x.detach().numpy(), f"resize_{tag}_y": y.detach().numpy(),
                    f"resize_{tag}_dy": dy.numpy(), f"resize_{tag}_dx": x.grad.numpy()})
    np.savez_compressed(os.path.join(OUT, "model_regrid.npz"), **rec)
    print("model_regrid: cls", c.shape, "loss", rec["train_loss"])


def gen_geometry():
    import loss as ref_loss
    import utils as ref_utils
    rec = {}
    anchors = ref_utils.generate_anchors(400, 720, 8)
    rec["anchors"] = anchors.numpy()
    # --- full-size loss on seeded random head outputs ---
    g = torch.Generator().manual_seed(99)
    B, NA = 2, anchors.shape[0]
    cls = torch.randn((B, NA, 1), generator=g)
    box = 0.5 * torch.randn((B, NA, 6), generator=g)
    it = torch.randn((B, NA, 8), generator=g)
    rec["logits_seed"] = np.array([99])
    rec["logits_sums"] = np.array([float(cls.double().sum()), float(box.double().sum()), float(it.double().sum())])
    _, _, gts = O.synthetic_batch(B, seed=2024, G=20)
    # sample 1: GT centred exactly on anchors (ties between yaw-0 / yaw-90 anchors, force-match)
    sel = torch.tensor([5, 4005, 11117, 20000, 22499]) // 5
    a0 = anchors[sel * 5]
    gts[1]["boxes_xywha"] = torch.cat([gts[1]["boxes_xywha"][:15],
                                       torch.stack([a0[:, 0], a0[:, 1], torch.full((5,), 2.0),
                                                    torch.full((5,), 4.5), torch.zeros(5)], 1)])
    for i, gg in enumerate(gts):
        rec[f"gt{i}_boxes"] = gg["boxes_xywha"].numpy()
        rec[f"gt{i}_ints"] = gg["intentions"].numpy()
    iou = ref_utils.compute_axis_aligned_iou(anchors, gts[0]["boxes_xywha"])
    mx, arg = iou.max(dim=1)
    _, arg0 = iou.max(dim=0)
    rec.update(iou_max=mx.numpy(), iou_arg=arg.numpy(), iou_arg0=arg0.numpy(), iou_sample=iou[::97].numpy())
    lf = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=False)
    d = lf(cls, box, it, anchors, gts)
    rec["loss_full"] = np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]),
                                 float(d["intent_loss"]), float(d["num_pos_anchors"])])
    torch.manual_seed(5)
    d = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=True)(cls, box, it, anchors, gts)
    rec["loss_full_ds"] = np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]),
                                    float(d["intent_loss"]), float(d["num_pos_anchors"])])
    # empty / malformed GT → all anchors negative
    d = lf(cls, box, it, anchors, [{"boxes_xywha": torch.zeros((0, 5)), "intentions": torch.zeros((0,), dtype=torch.long)}, {}])
    rec["loss_empty"] = np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]),
                                  float(d["intent_loss"]), float(d["num_pos_anchors"])])
    # --- decode ---
    g = torch.Generator().manual_seed(7)
    idx = torch.randperm(NA, generator=g)[:1000]
    rel = 0.5 * torch.randn((1000, 6), generator=g)
    rec.update(dec_idx=idx.numpy(), dec_rel=rel.numpy(),
               dec_out=ref_utils.decode_box_predictions(rel, anchors[idx]).numpy())
    # --- NMS (apply_nms) cases ---
    cases = []
    g = torch.Generator().manual_seed(11)
    rel = 0.1 * torch.randn((NA, 6), generator=g)
    rel[:, 4:] = torch.randn((NA, 2), generator=g)
    boxes = ref_utils.decode_box_predictions(rel, anchors)
    scores = torch.sigmoid(0.5 * torch.randn(NA, generator=g))
    cases.append((boxes, scores))                                      # full 22500, eval-like
    cases.append((boxes[:3000], torch.round(scores[:3000] * 16) / 16))  # heavy score ties
    s1 = torch.full((3000,), 0.5)
    cases.append((boxes[:3000], s1))                                   # all equal scores
    ex = torch.tensor([[0.5, 0.5, 1.0, 1.0, 0.0], [0.5, 0.1, 1.0, 0.2, 0.0], [0.5, 0.9, 1.0, 0.2, 0.3],
                       [0.1, 0.5, 0.2, 1.0, 0.0], [3.0, 3.0, 1.0, 1.0, 0.0], [3.0, 3.0, 1.0, 1.0, 0.0],
                       [0.5, 0.5, 0.0, 1.0, 0.0]], dtype=torch.float32)
    cases.append((ex, torch.tensor([0.9, 0.8, 0.7, 0.6, 0.5, 0.5, 0.95])))  # IoU == 0.2f, dup, zero-area
    cases.append((torch.zeros((0, 5)), torch.zeros(0)))                # empty
    off = [0]
    keeps = []
    for i, (bx, sc) in enumerate(cases):
        rec[f"nms{i}_boxes"] = bx.numpy()
        rec[f"nms{i}_scores"] = sc.numpy()
        k = ref_utils.apply_nms(bx, sc, 0.2).numpy()
        rec[f"nms{i}_keep"] = k
        keeps.append(k.size)
    rec["nms_cases"] = np.array([len(cases)])
    # --- rotated IoU ---
    g = torch.Generator().manual_seed(13)
    b1 = torch.stack([10 * torch.rand(48, generator=g), 10 * torch.rand(48, generator=g),
                      0.5 + 3 * torch.rand(48, generator=g), 0.5 + 6 * torch.rand(48, generator=g),
                      -math.pi + 2 * math.pi * torch.rand(48, generator=g)], 1)
    b2 = b1[torch.randperm(48, generator=g)[:24]].clone()
    b2[:, :2] += 0.7 * torch.randn((24, 2), generator=g)
    b2[:, 4] += 0.3 * torch.randn(24, generator=g)
    b1[3, 2] = 0.0                                                    # degenerate box → 0 row
    rec.update(rot_b1=b1.numpy(), rot_b2=b2.numpy(), rot_iou=ref_utils.compute_rotated_iou(b1, b2).numpy())
    np.savez_compressed(os.path.join(OUT, "geometry.npz"), **rec)
    print("geometry: loss", rec["loss_full"], "ds", rec["loss_full_ds"], "nms keeps", keeps)


def _loss_vec(d):
    return np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
                     float(d["num_pos_anchors"])])


def gen_loss_options():
    """The reference's OWN DetectionIntentionLoss (loss.py) on its non-default option paths:
    * ``intention_class_weights`` with downsampling off (loss.py:40-45), full 400x720 anchors;
    * ``use_rotated_iou=True`` (loss.py:81, utils.py:335-392 with the convex-clip Polygon
      stand-in: GEOS absent) on an 80x120 grid (750 anchors, boxes inside its footprint);
    * the NaN / Inf guard (loss.py:190-198): a NaN class logit, an +Inf class logit on a
      negative anchor, an Inf intention logit on a positive anchor.
    Records the loss dicts and, where a gradient flows, d loss / d logits (full arrays)."""
    import loss as ref_loss
    import utils as ref_utils
    rec = {}
    # --- class weights, full grid ---
    anchors = ref_utils.generate_anchors(400, 720, 8)
    NA = anchors.shape[0]
    g = torch.Generator().manual_seed(31)
    cls = torch.randn((2, NA, 1), generator=g)
    box = 0.5 * torch.randn((2, NA, 6), generator=g)
    it = torch.randn((2, NA, 8), generator=g)
    _, _, gts = O.synthetic_batch(2, seed=2025, G=20)
    cw = torch.tensor([0.3, 1.7, 2.5, 0.9, 1.2, 3.1, 0.5, 0.6], dtype=torch.float32)
    for i, gg in enumerate(gts):
        rec[f"cw_gt{i}_boxes"] = gg["boxes_xywha"].numpy()
        rec[f"cw_gt{i}_ints"] = gg["intentions"].numpy()
    ts = [t.clone().requires_grad_(True) for t in (cls, box, it)]
    d = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=False, intention_class_weights=cw)(
        *ts, anchors, gts)
    d["loss"].backward()
    rec.update(cw_seed=np.array([31]), cw_weights=cw.numpy(), cw_loss=_loss_vec(d),
               cw_gcls=ts[0].grad.numpy(), cw_gbox=ts[1].grad.numpy(), cw_gint=ts[2].grad.numpy())
    # weights given but downsampling on: the reference ignores the weights (loss.py:41-42)
    torch.manual_seed(3)
    d = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=True, intention_class_weights=cw)(
        cls, box, it, anchors, gts)
    rec["cw_ds_loss_nods_terms"] = _loss_vec(d)[:3]  # cls / box terms do not depend on the draws
    # --- rotated IoU, 80x120 grid ---
    H, W = 80, 120
    anchors = ref_utils.generate_anchors(H, W, 8)
    NA = anchors.shape[0]
    g = torch.Generator().manual_seed(41)
    cls = torch.randn((2, NA, 1), generator=g)
    box = 0.5 * torch.randn((2, NA, 6), generator=g)
    it = torch.randn((2, NA, 8), generator=g)
    ax, ay = anchors[:, 0], anchors[:, 1]
    lo_x, hi_x, lo_y, hi_y = float(ax.min()), float(ax.max()), float(ay.min()), float(ay.max())
    gts = []
    for b, G in enumerate((8, 5)):
        u = torch.rand((G, 5), generator=g)
        boxes = torch.stack([lo_x + (hi_x - lo_x) * u[:, 0], lo_y + (hi_y - lo_y) * u[:, 1], 1.5 + 1.5 * u[:, 2],
                             3.5 + 3.0 * u[:, 3], -math.pi + 2 * math.pi * u[:, 4]], 1).float()
        if b == 0:  # two GTs exactly on anchors at yaw 0 / pi/2 (rotated IoU 1.0 on the matching anchor)
            boxes[0] = anchors[37].clone()
            boxes[1] = anchors[301].clone()
        gts.append({"boxes_xywha": boxes, "intentions": torch.randint(0, 8, (G,), generator=g)})
        rec[f"rot_gt{b}_boxes"] = boxes.numpy()
        rec[f"rot_gt{b}_ints"] = gts[-1]["intentions"].numpy()
    ts = [t.clone().requires_grad_(True) for t in (cls, box, it)]
    d = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=False, use_rotated_iou=True)(
        *ts, anchors, gts)
    d["loss"].backward()
    rec.update(rot_grid=np.array([H, W]), rot_anchors=anchors.numpy(), rot_cls=cls.numpy(), rot_box=box.numpy(),
               rot_int=it.numpy(), rot_loss=_loss_vec(d), rot_gcls=ts[0].grad.numpy(),
               rot_gbox=ts[1].grad.numpy(), rot_gint=ts[2].grad.numpy())
    # axis-aligned on the same inputs, to show the option changes the result
    d = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=False)(cls, box, it, anchors, gts)
    rec["rot_axis_loss"] = _loss_vec(d)
    # --- NaN / Inf guard (same 80x120 inputs) ---
    iou = ref_utils.compute_axis_aligned_iou(anchors, gts[0]["boxes_xywha"])
    pos_a = int(iou.max(dim=0)[1][0])  # force-matched positive of sample 0
    neg_a = int(torch.nonzero(iou.max(dim=1)[0] < 0.45)[0])
    cases = {"nan_cls": ("cls", 0, pos_a, 0, float("nan")), "inf_cls_neg": ("cls", 0, neg_a, 0, float("inf")),
             "inf_int_pos": ("int", 0, pos_a, 3, float("inf"))}
    for name, (which, b, a, k, v) in cases.items():
        c2, b2, i2 = cls.clone(), box.clone(), it.clone()
        (c2 if which == "cls" else i2)[b, a, k] = v
        ts = [t.requires_grad_(True) for t in (c2, b2, i2)]
        d = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=False)(*ts, anchors, gts)
        leaf = d["loss"].grad_fn is None and d["loss"].requires_grad
        d["loss"].backward()
        rec[f"guard_{name}"] = np.array([b, a, k, v], np.float64)
        rec[f"guard_{name}_loss"] = _loss_vec(d)
        rec[f"guard_{name}_leaf"] = np.array([int(leaf), int(all(t.grad is None for t in ts))])
    np.savez_compressed(os.path.join(OUT, "loss_options.npz"), **rec)
    print("loss_options: cw", rec["cw_loss"], "rot", rec["rot_loss"], "axis", rec["rot_axis_loss"],
          "guard", {k: rec[f"guard_{k}_loss"].tolist() + rec[f"guard_{k}_leaf"].tolist() for k in cases})


def _sparse(bev):
    flat = bev.reshape(-1)
    nz = np.flatnonzero(flat != 0)  # NaN != 0: NaN cells are kept
    return nz.astype(np.int64), flat[nz]


def gen_lidar_bev():
    """utils.create_intentnet_lidar_bev / transform_points (utils.py:27-33, 62-106) on seeded sweeps.
    Case A: the dataset path (dataset.py:290-347) -- 10 sweeps of sweep-frame f32 points, rel_tf from
    poses (host restatement O.sweep_rel_transform), the reference's transform_points, then its
    voxeliser; sweep 3 missing, sweep 5 empty, duplicate cells, zero / negative intensities.
    Case B: f32 points handed in directly (f32 binning), 2 sweeps, exact grid / z boundaries, NaN."""
    import utils as ref_utils
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(21)
    rec = {}
    ego = np.array([100.0, -50.0, 1.2] + list(Rotation.from_euler("xyz", [0.01, -0.02, 0.3]).as_quat()))
    pts_all, ints_all, counts, tfs, pts_ego, ints = [], [], [], [], [], []
    for i in range(10):
        if i == 3:
            counts.append(-1)
            pts_ego.append(None)
            ints.append(None)
            tfs.append(np.eye(4))
            continue
        n = 0 if i == 5 else 4000
        p = np.stack([rng.uniform(-30, 90, n), rng.uniform(-80, 80, n), rng.uniform(-3.5, 5.5, n)], 1).astype(np.float32)
        v = rng.uniform(0, 255, n).astype(np.float32)
        if n:
            v[rng.random(n) < 0.02] = 0.0
            v[rng.random(n) < 0.01] *= -1.0
            p[50:100] = p[:50]  # the same cells hit twice with different intensities
        sw = ego.copy()
        sw[:3] += rng.normal(0, 2.0, 3)
        sw[3:] = Rotation.from_euler("xyz", [rng.normal(0, 0.01), rng.normal(0, 0.01),
                                             0.3 + rng.normal(0, 0.05)]).as_quat()
        tf = O.sweep_rel_transform(ego, sw)
        counts.append(n)
        pts_all.append(p)
        ints_all.append(v)
        tfs.append(tf)
        pts_ego.append(ref_utils.transform_points(p, tf))
        ints.append(v)
    bev = ref_utils.create_intentnet_lidar_bev(pts_ego, ints)
    mine = O.lidar_bev_np(pts_ego, ints)
    assert np.array_equal(mine, bev), "oracle restatement != reference voxeliser"
    rec.update(a_points=np.concatenate(pts_all), a_intensity=np.concatenate(ints_all), a_counts=np.array(counts),
               a_tf=np.stack(tfs), a_ego_points_sample=np.concatenate([q for q in pts_ego if q is not None])[::97])
    rec["a_idx"], rec["a_val"] = _sparse(bev)
    rec["a_shape"] = np.array(bev.shape)
    # case B: f32 points straight in, boundaries of the f32 binning
    edge = np.array([[60.0, 0.0, 0.0], [-20.0, 0.0, 0.0], [0.0, 72.0, 0.0], [0.0, -72.0, 0.0],
                     [0.0, 0.0, 3.8], [0.0, 0.0, -2.0], [0.0, 0.0, 3.7999], [10.0, 10.0, -1.0],
                     [59.9, 71.9, 1.0], [-19.9, -71.9, 2.0], [0.1, 0.1, 0.0], [np.nan, 0.0, 0.0]], np.float32)
    pb = [np.concatenate([edge, np.stack([rng.uniform(-25, 65, 3000), rng.uniform(-75, 75, 3000),
                                          rng.uniform(-2.5, 4.3, 3000)], 1).astype(np.float32)]),
          np.stack([rng.uniform(-25, 65, 2000), rng.uniform(-75, 75, 2000), rng.uniform(-2.5, 4.3, 2000)],
                   1).astype(np.float32)]
    vb = [rng.uniform(0, 100, pb[0].shape[0]).astype(np.float32), rng.uniform(0, 100, 2000).astype(np.float32)]
    vb[1][7] = np.nan
    pb[1][7] = pb[1][8]  # NaN shares its cell with a finite value
    bev_b = ref_utils.create_intentnet_lidar_bev(pb, vb, num_expected_sweeps=2)
    mine = O.lidar_bev_np(pb, vb, num_sweeps=2)
    assert np.array_equal(mine, bev_b, equal_nan=True), "oracle restatement != reference voxeliser (case B)"
    rec.update(b_points0=pb[0], b_points1=pb[1], b_int0=vb[0], b_int1=vb[1], b_shape=np.array(bev_b.shape))
    rec["b_idx"], rec["b_val"] = _sparse(bev_b)
    np.savez_compressed(os.path.join(OUT, "lidar_bev.npz"), **rec)
    print("lidar_bev: case A nonzero", rec["a_idx"].size, "case B nonzero", rec["b_idx"].size,
          "NaN cells", int(np.isnan(rec["b_val"]).sum()))


def gen_bev_augment():
    """utils.augment_bev (utils.py:394-517): the reference's OWN flow (random draws, flip, rotate /
    scale per channel through cv2, crop / pad, dropout, GT updates) with cv2 backed by the oracle's
    OpenCV restatement (refshim). Per case: the python `random` seed, the drawn params, sha256 of
    the output rasters (+ a strided sample) and the GT outputs. Cases are chosen to cover every
    branch: none, flip only, rotate, scale up (crop), scale down (pad), rotate + scale, dropout."""
    import hashlib
    import random
    import torch as _t
    import utils as ref_utils
    want = {"none": lambda p: not p["flip"] and p["angle"] is None and p["scale"] is None and not p["rects"],
            "flip": lambda p: p["flip"] and p["angle"] is None and p["scale"] is None and not p["rects"],
            "rotate": lambda p: p["angle"] is not None and p["scale"] is None,
            "scale_up": lambda p: p["angle"] is None and p["scale"] is not None and p["scale"] > 1.0,
            "scale_down": lambda p: p["angle"] is None and p["scale"] is not None and p["scale"] <= 1.0,
            "rotate_scale_flip": lambda p: p["flip"] and p["angle"] is not None and p["scale"] is not None,
            "dropout": lambda p: len(p["rects"]) >= 2,
            "all": lambda p: p["flip"] and p["angle"] is not None and p["scale"] is not None and p["rects"]}
    seeds = {}
    for s in range(5000):
        random.seed(s)
        p = O.draw_augment_params(random)
        for k, f in want.items():
            if k not in seeds and f(p):
                seeds[k] = s
        if len(seeds) == len(want):
            break
    assert len(seeds) == len(want), seeds
    rec = {"cases": np.array(list(want))}
    for ci, (k, s) in enumerate(seeds.items()):
        lidar, mp, boxes, intents = O.bev_augment_inputs(100 + ci)
        random.seed(s)
        rl, rm, rg = ref_utils.augment_bev(lidar, mp, {"boxes_xywha": _t.from_numpy(boxes.copy()),
                                                       "intentions": _t.from_numpy(intents.copy())})
        random.seed(s)
        ol, om, ob, oi, p = O.augment_bev_np(lidar, mp, boxes, intents, random)
        assert np.array_equal(rl, ol) and np.array_equal(rm, om), f"oracle != reference rasters ({k})"
        assert np.array_equal(rg["boxes_xywha"].numpy(), ob) and np.array_equal(rg["intentions"].numpy(), oi), k
        rects = np.zeros((5, 4), np.int64)
        if p["rects"]:
            rects[:len(p["rects"])] = p["rects"]
        rec.update({f"{k}_seed": np.int64(s), f"{k}_input_seed": np.int64(100 + ci), f"{k}_flip": np.int64(p["flip"]),
                    f"{k}_angle": np.float64(np.nan if p["angle"] is None else p["angle"]),
                    f"{k}_scale": np.float64(np.nan if p["scale"] is None else p["scale"]),
                    f"{k}_nrect": np.int64(len(p["rects"])), f"{k}_rects": rects,
                    f"{k}_lidar_sha": np.array(hashlib.sha256(np.ascontiguousarray(rl).tobytes()).hexdigest()),
                    f"{k}_map_sha": np.array(hashlib.sha256(np.ascontiguousarray(rm).tobytes()).hexdigest()),
                    f"{k}_lidar_sample": np.ascontiguousarray(rl).reshape(-1)[::997].copy(),
                    f"{k}_map_sample": np.ascontiguousarray(rm).reshape(-1)[::997].copy(),
                    f"{k}_boxes": rg["boxes_xywha"].numpy(), f"{k}_intents": rg["intentions"].numpy()})
        print("bev_augment", k, "seed", s, {kk: v for kk, v in p.items() if kk != "rects"}, "rects", len(p["rects"]))
    np.savez_compressed(os.path.join(OUT, "bev_augment.npz"), **rec)


def gen_map_raster():
    """utils.rasterize_map_ego_centric (utils.py:108-182): the reference's OWN flow (JSON load,
    ego yaw from the quaternion, world -> pixel, point filtering, lane polygons / boundaries /
    mark types / intersections / bus lanes / crosswalks into the 9 channels) with cv2.fillPoly /
    polylines backed by the oracle's OpenCV restatement (parity unpinned at the OpenCV level).
    Cases: 4 seeded maps + poses, an empty map, a missing file and an invalid quaternion."""
    import json as _json
    import tempfile
    import pandas as pd
    import utils as ref_utils
    rec = {}
    cases = []
    for sd in range(4):
        cases.append((f"seed{sd}", O.synthetic_map(10 + sd, n_lanes=30 + 10 * sd), O.synthetic_pose(20 + sd)))
    cases.append(("empty", {}, O.synthetic_pose(7)))
    cases.append(("badquat", O.synthetic_map(3), dict(O.synthetic_pose(3), qx=0.0, qy=0.0, qz=0.0, qw=0.0)))
    with tempfile.TemporaryDirectory() as td:
        for name, m, pose in cases + [("missing", None, O.synthetic_pose(5))]:
            path = os.path.join(td, f"{name}.json")
            if m is not None:
                with open(path, "w") as fh:
                    _json.dump(m, fh)
            ser = pd.Series(pose)
            ref = ref_utils.rasterize_map_ego_centric(path, ser)
            mine = (O.rasterize_map_np(m, pose) if m is not None and name != "badquat"
                    else np.zeros((9, 400, 720), np.float32))
            assert ref.dtype == np.float32 and np.array_equal(ref, mine), f"oracle != reference map raster ({name})"
            nz = np.flatnonzero(ref.reshape(-1))
            rec[f"{name}_json"] = np.array(_json.dumps(m) if m is not None else "")
            rec[f"{name}_pose"] = np.array([pose[k] for k in ("tx_m", "ty_m", "qx", "qy", "qz", "qw")])
            rec[f"{name}_idx"] = nz.astype(np.int64)
            rec[f"{name}_per_channel"] = ref.reshape(9, -1).sum(1)
    rec["cases"] = np.array([c[0] for c in cases] + ["missing"])
    np.savez_compressed(os.path.join(OUT, "map_raster.npz"), **rec)
    print("map_raster:", {c: rec[f"{c}_per_channel"].astype(int).tolist() for c in rec["cases"]})


def gen_cnn_small():
    """The reference's OWN IntentNetCNN (model_cnn.py) at a 32x48 grid with its default channels,
    filled by the seeded filler in its state_dict order: eval outputs, train outputs + loss
    (downsampling off) + gradient samples + BN running stats; the oracle restatement agrees."""
    import loss as ref_loss
    import model_cnn as ref_cnn
    import utils as ref_utils
    from oracle.weights import fill_state_dict
    img = SMALL_IMG
    m = ref_cnn.IntentNetCNN()
    keys = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    sd = fill_state_dict(keys, seed=0)
    m.load_state_dict(sd, strict=True)
    lidar, mp, _ = O.synthetic_batch(2, img, seed=1234)
    gts = small_gt()
    anchors = ref_utils.generate_anchors(img[0], img[1], 8)
    rec = {"keys": np.array([k for k, _ in keys]), "w_checksum": state_checksum(sd)}
    for i, g in enumerate(gts):
        rec[f"gt{i}_boxes"] = g["boxes_xywha"].numpy()
        rec[f"gt{i}_ints"] = g["intentions"].numpy()
    m.eval()
    with torch.no_grad():
        c, b, it = m(lidar, mp)
        oc, ob, oi = O.cnn_forward({k: v.clone() for k, v in sd.items()}, lidar, mp, training=False)
    assert max(float((x - y).abs().max()) for x, y in ((c, oc), (b, ob), (it, oi))) < 1e-4
    rec.update(eval_cls=c.numpy(), eval_box=b.numpy(), eval_int=it.numpy())
    m.train()
    c, b, it = m(lidar, mp)
    d = ref_loss.DetectionIntentionLoss(apply_intention_downsampling=False)(c, b, it, anchors, gts)
    d["loss"].backward()
    rec.update(train_cls=c.detach().numpy(), train_box=b.detach().numpy(), train_int=it.detach().numpy(),
               train_loss=np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]),
                                    float(d["intent_loss"]), float(d["num_pos_anchors"])]))
    grads = {k: p.grad for k, p in m.named_parameters() if p.grad is not None}
    names = sorted(grads)
    samples, strides = zip(*[_sample(grads[k]) for k in names])
    rec.update(grad_names=np.array(names), grad_abssum=np.array([float(grads[k].double().abs().sum()) for k in names]),
               grad_samples=np.stack(samples), grad_strides=np.array(strides))
    bn = {k: v for k, v in m.state_dict().items() if "running_" in k}
    rec.update(bn_names=np.array(sorted(bn)), bn_values=np.concatenate([bn[k].numpy() for k in sorted(bn)]),
               bn_sizes=np.array([bn[k].numel() for k in sorted(bn)]))
    osd = {k: v.clone() for k, v in sd.items()}
    c2, _, _ = O.cnn_forward(osd, lidar, mp, training=True)
    assert float((c2 - c.detach()).abs().max()) < 1e-4
    np.savez_compressed(os.path.join(OUT, "cnn_small.npz"), **rec)
    print("cnn_small: params", sum(int(np.prod(s)) for _, s in keys), "loss", rec["train_loss"])


def gen_ap():
    """The reference's OWN calculate_ap (utils.py:564-575) on the recall / precision steps that
    eval_vit.py:249-255 builds from a TP-flag sequence (torch f32 cumsum, / (num_gt + 1e-9),
    / (arange + 1e-9)): seeded random walks, all-TP, all-FP, a single TP / FP, long FP runs (recall
    plateaus: tied recall values), a late-TP tail and the empty array pair."""
    import utils as ref_utils
    rng = np.random.default_rng(2468)
    cases = [(np.zeros(0, bool), 5), (np.ones(5, bool), 5), (np.zeros(6, bool), 3), (np.ones(1, bool), 1),
             (np.zeros(1, bool), 1), (np.array([0, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0, 1], bool), 4),
             (np.array([1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1], bool), 7)]
    for P, G, p_tp in ((50, 10, 0.2), (300, 25, 0.05), (700, 40, 0.04), (2000, 60, 0.02), (64, 64, 0.9)):
        tp = rng.random(P) < p_tp
        while tp.sum() > G:  # a GT is matched at most once
            tp[np.nonzero(tp)[0][-1]] = False
        cases.append((tp, G))
    rec = {"n_cases": np.array([len(cases)])}
    for k, (tp, G) in enumerate(cases):
        t = torch.from_numpy(tp)
        cum = torch.cumsum(t.float(), dim=0)
        recall = cum / (G + 1e-9)
        precision = cum / (torch.arange(1, t.numel() + 1).float() + 1e-9)
        rec[f"c{k}_tp"] = tp
        rec[f"c{k}_ngt"] = np.array([G])
        rec[f"c{k}_recall"] = recall.numpy()
        rec[f"c{k}_precision"] = precision.numpy()
        rec[f"c{k}_ap"] = np.array([ref_utils.calculate_ap(recall.numpy(), precision.numpy())])
    np.savez_compressed(os.path.join(OUT, "ap_reference.npz"), **rec)
    print("ap_reference:", [float(rec[f"c{k}_ap"][0]) for k in range(len(cases))])


def cross_check_vit():
    """HF ViTModel (stand-in) vs the oracle's timm restatement, 12 blocks, real widths."""
    cfg = model_cfg(img_size=SMALL_IMG)
    sd = make_state_dict(cfg, seed=0)
    vit = refshim.HFTimmViT("vit_small_patch8_224", in_chans=9, img_size=SMALL_IMG)
    pre = "backbone.vit_map."
    vit.load_state_dict({k[len(pre + "hf."):]: v for k, v in refshim.timm_to_hf_state(sd).items()
                         if k.startswith(pre + "hf.")} | {}, strict=False)
    hf_sd = {("hf." + k[len(pre + "hf."):]): v for k, v in refshim.timm_to_hf_state(sd).items() if k.startswith(pre + "hf.")}
    vit.load_state_dict(hf_sd, strict=True)
    _, mp, _ = O.synthetic_batch(2, SMALL_IMG, seed=1234)
    with torch.no_grad():
        a = vit.forward_features(mp)
        b = O.vit_forward_features(sd, pre, mp, 6, 12)
    err = float((a - b).abs().max())
    print("HF vs oracle ViT max abs diff", err)
    assert err < 1e-4, err


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    refshim.install()
    torch.set_num_threads(8)
    if len(sys.argv) > 1:  # python -m oracle.make_golden lidar_bev ...: only the named fixtures
        for name in sys.argv[1:]:
            globals()["gen_" + name]()
        sys.exit(0)
    cross_check_vit()
    gen_model_small()
    gen_geometry()
    gen_lidar_bev()
    gen_bev_augment()
    gen_cnn_small()
    gen_loss_options()
    gen_map_raster()
    gen_model_stride2()
    gen_model_regrid()
    gen_ap()
