"""Box geometry of the reference's utils.py (anchors, axis/rotated IoU, decode, NMS, AP) and
the LiDAR BEV voxelisation with its sweep ego transform (utils.py:27-33, 62-106; SURVEY.md §8f
rank 1) and the BEV augmentations (utils.py:394-517; §8f rank 3) on the MI355X kernels. Map
rasterisation (utils.py:108-225) belongs to the Argoverse-2 data pipeline, outside this build."""
from __future__ import annotations

import math
import random

import numpy as np
import torch

from _lib import lib, ptr, stream, workspace
from constants import (ANCHOR_CONFIGS_PAPER, BEV_PIXEL_OFFSET_X, BEV_PIXEL_OFFSET_Y, GRID_HEIGHT_PX, GRID_WIDTH_PX,
                       INTENTIONS_MAP, LIDAR_HEIGHT_CHANNELS, LIDAR_SWEEPS, MAP_CHANNELS, VOXEL_SIZE_M, Z_MAX, Z_MIN)


def _dev(device):
    d = torch.device(device if device is not None else "cuda")
    if d.type != "cuda":
        raise RuntimeError("ivit geometry runs on the GPU (no CPU fallback)")
    return d


def generate_anchors(bev_height: int = GRID_HEIGHT_PX, bev_width: int = GRID_WIDTH_PX, feature_map_stride: int = 8,
                     anchor_configs=ANCHOR_CONFIGS_PAPER, voxel_size: float = VOXEL_SIZE_M,
                     offset_x_px: float = BEV_PIXEL_OFFSET_X, offset_y_px: float = BEV_PIXEL_OFFSET_Y,
                     device=None) -> torch.Tensor:
    """utils.py:519-562 → (Hf*Wf*A, 5) [cx, cy, w, l, yaw], location-major, anchor-minor (device tensor)."""
    d = _dev(device)
    cfg = torch.tensor([list(c) for c in anchor_configs], dtype=torch.float32).reshape(-1).to(d)
    A = len(anchor_configs)
    n = (bev_height // feature_map_stride) * (bev_width // feature_map_stride) * A
    out = torch.empty((n, 5), dtype=torch.float32, device=d)
    lib.ivit_generate_anchors(bev_height, bev_width, feature_map_stride, ptr(cfg), A, float(voxel_size),
                              float(offset_x_px), float(offset_y_px), ptr(out), stream())
    return out


def compute_axis_aligned_iou(boxes1_xywh: torch.Tensor, boxes2_xywh: torch.Tensor) -> torch.Tensor:
    """utils.py:276-292 (uses columns 0..3)."""
    b1, b2 = _as5(boxes1_xywh), _as5(boxes2_xywh)
    out = torch.empty((b1.shape[0], b2.shape[0]), dtype=torch.float32, device=b1.device)
    lib.ivit_axis_iou(ptr(b1), b1.shape[0], ptr(b2), b2.shape[0], ptr(out), stream())
    return out


def compute_rotated_iou(boxes1_xywha: torch.Tensor, boxes2_xywha: torch.Tensor) -> torch.Tensor:
    """utils.py:335-392 semantics (area/intersection/union guards), convex clipping in f64 on device."""
    b1, b2 = _as5(boxes1_xywha), _as5(boxes2_xywha)
    out = torch.empty((b1.shape[0], b2.shape[0]), dtype=torch.float32, device=b1.device)
    lib.ivit_rotated_iou(ptr(b1), b1.shape[0], ptr(b2), b2.shape[0], ptr(out), stream())
    return out


def _as5(b):
    b = b.float()
    if b.shape[1] < 5:
        b = torch.cat([b, torch.zeros((b.shape[0], 5 - b.shape[1]), device=b.device)], 1)
    return b[:, :5].contiguous()


def decode_box_predictions(box_preds_rel: torch.Tensor, anchors_xywha: torch.Tensor) -> torch.Tensor:
    """utils.py:227-257."""
    n = box_preds_rel.shape[0]
    if n == 0:
        return torch.empty((0, 5), device=box_preds_rel.device)
    rel = box_preds_rel.float().contiguous()
    anc = anchors_xywha.float().contiguous()
    out = torch.empty((n, 5), dtype=torch.float32, device=rel.device)
    lib.ivit_decode_boxes(ptr(rel), ptr(anc), None, n, ptr(out), stream())
    return out


def nms_device(boxes_xywha: torch.Tensor, scores: torch.Tensor, iou_threshold: float = 0.2):
    """Kept indices (int64, descending-score order) padded to n, plus a device count: no host sync."""
    n = boxes_xywha.shape[0]
    dev = boxes_xywha.device
    keep = torch.empty((max(n, 1),), dtype=torch.int64, device=dev)
    count = torch.zeros((1,), dtype=torch.int64, device=dev)
    b = boxes_xywha.float().contiguous()
    s = scores.float().contiguous()
    ws = workspace(lib.ivit_nms_workspace(n), dev)
    lib.ivit_nms(ptr(b), ptr(s), n, float(iou_threshold), ptr(keep), ptr(count), ptr(ws), ws.numel(), stream())
    return keep, count


def apply_nms(boxes_xywha: torch.Tensor, scores: torch.Tensor, iou_threshold: float = 0.2) -> torch.Tensor:
    """utils.py:259-274 → torchvision CPU nms semantics on axis-aligned corners (bit-exact keep set/order)."""
    if boxes_xywha.shape[0] == 0:
        return torch.empty((0,), dtype=torch.long, device=boxes_xywha.device)
    keep, count = nms_device(boxes_xywha, scores, iou_threshold)
    return keep[: int(count.item())]


def nms_batched(boxes_list, scores_list, iou_threshold: float = 0.2):
    """apply_nms for every sample of a batch: one launch per NMS stage for all samples
    (ivit_nms_batched) and one host read of the kept counts. Returns per-sample kept LOCAL
    indices (int64 device tensors, descending-score order, torchvision CPU semantics)."""
    ns = [int(b.shape[0]) for b in boxes_list]
    S, total = len(ns), sum(ns)
    dev = boxes_list[0].device if S else torch.device("cuda")
    if total == 0:
        return [torch.empty((0,), dtype=torch.long, device=dev) for _ in ns]
    seg = np.concatenate([[0], np.cumsum(ns)]).astype(np.int64)
    words = [n * ((n + 63) // 64) for n in ns]
    moff = np.concatenate([[0], np.cumsum(words)[:-1]]).astype(np.int64)
    b = torch.cat([x.float() for x in boxes_list]).contiguous()
    sc = torch.cat([x.float() for x in scores_list]).contiguous()
    d_seg = torch.from_numpy(seg).to(dev, non_blocking=True)
    d_moff = torch.from_numpy(moff).to(dev, non_blocking=True)
    keep = torch.empty((total,), dtype=torch.int64, device=dev)
    count = torch.empty((S,), dtype=torch.int64, device=dev)
    ws = workspace(lib.ivit_nms_batched_workspace(S, total, sum(words)), dev)
    lib.ivit_nms_batched(ptr(b), ptr(sc), ptr(d_seg), ptr(d_moff), S, total, max(ns), sum(words),
                         float(iou_threshold), ptr(keep), ptr(count), ptr(ws), ws.numel(), stream())
    cnt = count.cpu().tolist()
    return [keep[seg[i]: seg[i] + cnt[i]] for i in range(S)]


def _post_launch(cls_logits, box_preds_rel, intent_logits, anchors, conf_threshold, nms_threshold):
    """ivit_eval_post for a batch on the current stream; returns what _post_collect needs."""
    B, NA = cls_logits.shape[0], anchors.shape[0]
    dev = cls_logits.device
    cls = cls_logits.reshape(B, NA).float().contiguous()  # no copy for the model's f32 outputs
    box = box_preds_rel.reshape(B, NA, 6).float().contiguous()
    it = intent_logits.reshape(B, NA, -1).float().contiguous()
    anc = anchors.float().contiguous()
    K = it.shape[2]
    sc = torch.empty((B, NA), dtype=torch.float32, device=dev)
    bx = torch.empty((B, NA, 5), dtype=torch.float32, device=dev)
    ii = torch.empty((B, NA), dtype=torch.int64, device=dev)
    cnt = torch.empty((B,), dtype=torch.int64, device=dev)
    ws = workspace(lib.ivit_eval_post_workspace(B, NA), dev)
    lib.ivit_eval_post(ptr(cls), ptr(box), ptr(it), ptr(anc), B, NA, K, float(conf_threshold), float(nms_threshold),
                       ptr(sc), ptr(bx), ptr(ii), ptr(cnt), ptr(ws), ws.numel(), stream())
    return sc, bx, ii, cnt


def _post_collect(launched):
    sc, bx, ii, cnt = launched
    n = cnt.cpu().tolist()  # the one host synchronisation
    return [{"pred_scores": sc[b, : n[b]], "pred_boxes_xywha": bx[b, : n[b]], "pred_intentions": ii[b, : n[b]]}
            for b in range(len(n))]


def _post_empty(B, dev):
    return [{"pred_scores": torch.empty((0,), device=dev), "pred_boxes_xywha": torch.empty((0, 5), device=dev),
             "pred_intentions": torch.empty((0,), dtype=torch.long, device=dev)} for _ in range(B)]


def postprocess_batch(cls_logits: torch.Tensor, box_preds_rel: torch.Tensor, intent_logits: torch.Tensor,
                      anchors: torch.Tensor, conf_threshold: float = 0.1, nms_threshold: float = 0.2):
    """eval_vit.py:156-176 for a whole batch on hand-written kernels (ivit_eval_post): sigmoid →
    score >= conf in anchor order → decode → NMS → argmax intention, every sample at once, four
    launches and ONE host read (the kept counts). Returns [{'pred_scores', 'pred_boxes_xywha',
    'pred_intentions'}] per sample as device tensors (views of the packed outputs; the caller
    moves them to the host when it needs them)."""
    B, NA = cls_logits.shape[0], anchors.shape[0]
    if NA == 0 or B == 0:
        return _post_empty(B, cls_logits.device)
    return _post_collect(_post_launch(cls_logits, box_preds_rel, intent_logits, anchors, conf_threshold,
                                      nms_threshold))


class PostPipeline:
    """postprocess_batch over consecutive batches, one batch deep (the eval loop, config 4): batch
    k's post-processing runs on its own HIP stream beside batch k+1's forward, and its kept counts
    are read once batch k+1's forward is enqueued — so the post-processing (sort, NMS mask and walk,
    ~4 ms of mostly serial kernels per B = 32 batch) no longer idles the ViT streams.
    ``push(cls, box, intent)`` returns the previous batch's predictions (None for the first);
    ``flush()`` returns the last one's. Same kernels and results as postprocess_batch."""

    def __init__(self, anchors, conf_threshold=0.1, nms_threshold=0.2):
        self.anchors, self.conf, self.nms = anchors, conf_threshold, nms_threshold
        self.stream = torch.cuda.Stream(anchors.device) if anchors.is_cuda else None
        if self.stream is not None:
            anchors.record_stream(self.stream)
        self.pending = None

    def _collect(self):
        if self.pending is None:
            return None
        p, self.pending = self.pending, None
        if isinstance(p, list):  # empty batch
            return p
        if self.stream is None:
            return _post_collect(p)
        with torch.cuda.stream(self.stream):  # the count read waits for this batch's kernels only
            return _post_collect(p)

    def push(self, cls_logits, box_preds_rel, intent_logits):
        prev = self._collect()  # batch k-1: its post-processing ran beside this batch's forward
        B, NA = cls_logits.shape[0], self.anchors.shape[0]
        if NA == 0 or B == 0:
            self.pending = _post_empty(B, cls_logits.device)
            return prev
        if self.stream is None:
            self.pending = _post_launch(cls_logits, box_preds_rel, intent_logits, self.anchors, self.conf, self.nms)
            return prev
        self.stream.wait_stream(torch.cuda.current_stream(cls_logits.device))  # this batch's forward
        for t in (cls_logits, box_preds_rel, intent_logits):
            t.record_stream(self.stream)
        with torch.cuda.stream(self.stream):
            self.pending = _post_launch(cls_logits, box_preds_rel, intent_logits, self.anchors, self.conf, self.nms)
        return prev

    def flush(self):
        return self._collect()


def calculate_ap(recall: np.ndarray, precision: np.ndarray) -> float:
    """utils.py:564-575 (VOC-style AP; host-side metric)."""
    mrec = np.concatenate(([0.0], recall, [1.0]))
    mpre = np.concatenate(([0.0], precision, [0.0]))
    mpre = np.maximum.accumulate(mpre[::-1])[::-1]
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return float(np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1]))


# ------------------------------------------------------------------------ LiDAR BEV (§8f rank 1)
def transform_points(points: np.ndarray, transform_matrix: np.ndarray) -> np.ndarray:
    """utils.py:27-33 (host numpy, f64): (T @ [p, 1]^T)^T[:, :3]. The device path fuses the same
    transform into the voxelisation kernel (create_intentnet_lidar_bev(..., transforms=...))."""
    if points.shape[0] == 0:
        return np.empty((0, 3), dtype=points.dtype)
    homogeneous_points = np.hstack((points[:, :3], np.ones((points.shape[0], 1))))
    return (transform_matrix @ homogeneous_points.T).T[:, :3]


def _sweep_rows(points, intensity):
    """One sweep's (points [n, ld] f32/f64 contiguous, intensity [n] f32) as numpy, or None."""
    if points is None or intensity is None:
        return None
    p = points.detach().cpu().numpy() if isinstance(points, torch.Tensor) else np.asarray(points)
    v = intensity.detach().cpu().numpy() if isinstance(intensity, torch.Tensor) else np.asarray(intensity)
    if p.shape[0] == 0:
        return None
    if p.ndim != 2 or p.shape[1] < 3:
        raise ValueError(f"LiDAR points must be [n, >=3] (got {tuple(p.shape)})")
    if v.shape[0] < p.shape[0]:
        raise ValueError(f"intensity has {v.shape[0]} values for {p.shape[0]} points")
    return p, v[: p.shape[0]].astype(np.float32)


def lidar_bev_batch(samples, num_expected_sweeps: int = LIDAR_SWEEPS, out: torch.Tensor | None = None,
                    device=None) -> torch.Tensor:
    """Voxelise a batch of samples into [B, C * num_expected_sweeps, H, W] f32 on the GPU, one launch.

    samples[b] = (points_list, intensity_list) or (points_list, intensity_list, transforms) with
    the semantics of create_intentnet_lidar_bev (utils.py:62-106): sweep i fills channels
    i*29 .. i*29+28; sweeps that are None or empty leave their channels zero; the number of
    sweeps used is min(len(points_list), len(intensity_list)). transforms[i] (4x4, or None for
    the whole sample) is the sweep's rel_tf of dataset.py:336-340, applied in the kernel in f64
    exactly as transform_points does. `out` (zero-filled here) may be the batch's lidar_bev slot.
    """
    dev = _dev(device if out is None else out.device)
    B = len(samples)
    C = LIDAR_HEIGHT_CHANNELS * num_expected_sweeps
    if out is None:
        out = torch.zeros((B, C, GRID_HEIGHT_PX, GRID_WIDTH_PX), dtype=torch.float32, device=dev)
    else:
        if tuple(out.shape) != (B, C, GRID_HEIGHT_PX, GRID_WIDTH_PX) or out.dtype != torch.float32 \
                or not out.is_contiguous():
            raise ValueError(f"out must be contiguous f32 {(B, C, GRID_HEIGHT_PX, GRID_WIDTH_PX)}")
        out.zero_()
    groups = {}  # point dtype -> sweeps; f32 and f64 sweeps bin in their own precision (bev.hip)
    with_tf = any(len(s) > 2 and s[2] is not None for s in samples)
    for b, smp in enumerate(samples):
        points_list, intensity_list = smp[0], smp[1]
        transforms = smp[2] if len(smp) > 2 else None
        n_loaded = min(len(points_list), len(intensity_list))
        if n_loaded > num_expected_sweeps:
            # the reference indexes past its raster (IndexError); refuse instead of dropping sweeps
            raise ValueError(f"sample {b}: {n_loaded} sweeps > num_expected_sweeps={num_expected_sweeps}")
        for i in range(n_loaded):
            rows = _sweep_rows(points_list[i], intensity_list[i])
            if rows is None:
                continue
            p, v = rows
            if p.dtype not in (np.float32, np.float64):
                p = p.astype(np.float64)
            t = None
            if with_tf:
                t = np.eye(4) if transforms is None or transforms[i] is None else np.asarray(transforms[i], np.float64)
                if t.shape != (4, 4):
                    raise ValueError(f"sample {b} sweep {i}: transform must be 4x4")
            groups.setdefault(p.dtype == np.float64, []).append((p, v, t, b * C + i * LIDAR_HEIGHT_CHANNELS))
    h2d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(dev, non_blocking=True)  # noqa: E731
    for f64, sw in groups.items():
        starts = np.cumsum([0] + [p.shape[0] for p, _, _, _ in sw]).astype(np.int64)
        ld = max(p.shape[1] for p, _, _, _ in sw)
        allp = np.zeros((int(starts[-1]), ld), dtype=np.float64 if f64 else np.float32)
        for (p, _, _, _), a, e in zip(sw, starts[:-1], starts[1:]):
            allp[a:e, : p.shape[1]] = p
        dp, dv, dst = h2d(allp), h2d(np.concatenate([v for _, v, _, _ in sw])), h2d(starts)
        dpl = h2d(np.asarray([pl for _, _, _, pl in sw], np.int32))
        dtf = h2d(np.stack([t for _, _, t, _ in sw])) if with_tf else None
        lib.ivit_lidar_bev(ptr(dp), int(f64), ld, ptr(dv), ptr(dst), len(sw), int(np.diff(starts).max()), ptr(dtf),
                           ptr(dpl), ptr(out), GRID_HEIGHT_PX, GRID_WIDTH_PX, LIDAR_HEIGHT_CHANNELS, VOXEL_SIZE_M,
                           BEV_PIXEL_OFFSET_X, BEV_PIXEL_OFFSET_Y, Z_MIN, Z_MAX, Z_MAX - Z_MIN, stream())
    return out


def create_intentnet_lidar_bev(points_list, intensity_list, num_expected_sweeps: int = LIDAR_SWEEPS,
                               transforms=None, device=None) -> torch.Tensor:
    """utils.py:62-106 on the GPU: (29 * num_expected_sweeps, 400, 720) f32 device tensor (the
    reference returns the same raster as a numpy array). transforms (optional): per-sweep 4x4
    rel_tf, fusing dataset.py:340's transform_points into the same kernel."""
    return lidar_bev_batch([(points_list, intensity_list, transforms)], num_expected_sweeps, device=device)[0]


# ------------------------------------------------------------------ BEV augmentations (§8f rank 3)
# The raster work runs as ivit_bev_augment passes (csrc/bev.hip): every stack of a batch in one
# launch per pass, the flip fused into the first pass's reads and the dropout rectangles into the
# last pass's writes (rotate + scale = 2 passes, anything else = 1). The random draws stay on the
# host in python `random`, in the reference's order, so a seeded run makes the reference's
# decisions; the GT updates (<= a few dozen boxes) stay host numpy as in the reference.
_BEV_PASS = np.dtype([("src", "<u8"), ("dst", "<u8"), ("C", "<i4"), ("op", "<i4"), ("flip", "<i4"),
                      ("n_rect", "<i4"), ("m", "<f8", (6,)), ("scale_x", "<f8"), ("scale_y", "<f8"),
                      ("new_w", "<i4"), ("new_h", "<i4"), ("off_x", "<i4"), ("off_y", "<i4"),
                      ("rect", "<i4", (5, 4))])
assert _BEV_PASS.itemsize == 192  # ivit_bev_pass (include/ivit.h)
_FLIP_INTENTION = np.arange(8, dtype=np.int64)
for _a, _b in (("TURN_LEFT", "TURN_RIGHT"), ("LEFT_CHANGE_LANE", "RIGHT_CHANGE_LANE")):  # utils.py:406-411
    _FLIP_INTENTION[INTENTIONS_MAP[_a]], _FLIP_INTENTION[INTENTIONS_MAP[_b]] = INTENTIONS_MAP[_b], INTENTIONS_MAP[_a]


def _rotation_inverse(angle_deg, H, W):
    """cv2.getRotationMatrix2D((W/2, H/2), angle, 1) (utils.py:429), inverted in f64 the way
    warpAffine inverts a forward map (dst -> src), as the 6 doubles of ivit_bev_pass.m."""
    ang = angle_deg * (math.pi / 180)
    a, b = math.cos(ang), math.sin(ang)
    cx, cy = float(np.float32(W / 2.0)), float(np.float32(H / 2.0))
    m = [a, b, (1 - a) * cx - b * cy, -b, a, b * cx + (1 - a) * cy]
    d = m[0] * m[4] - m[1] * m[3]
    d = 1.0 / d if d != 0 else 0.0
    m[0], m[4] = m[4] * d, m[0] * d
    m[1] *= -d
    m[3] *= -d
    m[2], m[5] = -m[0] * m[2] - m[1] * m[5], -m[3] * m[2] - m[4] * m[5]
    return m


def _draw_params(flip=True, rotate=True, scale=True, dropout=True, angle_range_deg=(-15.0, 15.0),
                 scale_range=(0.95, 1.05), dropout_prob=0.1, patch_size_range=(20, 50), num_patches_range=(1, 5),
                 H=GRID_HEIGHT_PX, W=GRID_WIDTH_PX):
    """One sample's draws from python `random`, in the order of utils.py:399, 422-423, 451-452, 484-490."""
    p = {"flip": False, "angle": None, "scale": None, "rects": []}
    if flip:
        p["flip"] = random.random() < 0.5
    if rotate and random.random() < 0.5:
        p["angle"] = random.uniform(angle_range_deg[0], angle_range_deg[1])
    if scale and random.random() < 0.5:
        p["scale"] = random.uniform(scale_range[0], scale_range[1])
    if dropout and random.random() < dropout_prob:
        for _ in range(random.randint(num_patches_range[0], num_patches_range[1])):
            ph = random.randint(patch_size_range[0], patch_size_range[1])
            pw = random.randint(patch_size_range[0], patch_size_range[1])
            p["rects"].append((random.randint(0, max(0, H - ph)), random.randint(0, max(0, W - pw)), ph, pw))
    return p


def _stages(p, H, W):
    """The passes one stack needs for params p: [(op, fields)]; flip goes on the first, rects on the last."""
    st = []
    if p["angle"] is not None:
        st.append((1, {"m": _rotation_inverse(p["angle"], H, W)}))
    if p["scale"] is not None:
        s = p["scale"]
        nh, nw = int(H * s), int(W * s)  # utils.py:453
        if (nh, nw) != (H, W):  # cv2.resize to the same size is a copy
            if s > 1.0:  # centre crop (utils.py:465-468)
                oy, ox = (nh - H) // 2, (nw - W) // 2
            else:  # centre pad (utils.py:469-472)
                oy, ox = -((H - nh) // 2), -((W - nw) // 2)
            st.append((2, {"scale_x": 1.0 / (nw / W), "scale_y": 1.0 / (nh / H), "new_w": nw, "new_h": nh,
                           "off_x": ox, "off_y": oy}))
    if not st:
        st.append((0, {}))
    if len(p["rects"]) > 5:
        raise ValueError("at most 5 dropout rectangles per stack")
    return st


def _run_bev_passes(jobs):
    """jobs: [(src [C,H,W] cuda f32, dst like src, params)] -> ivit_bev_augment once per pass depth
    (1 or 2) over every job; two-pass jobs go through a scratch stack."""
    if not jobs:
        return
    H, W = jobs[0][0].shape[-2:]
    levels, keep = [[], []], []
    for src, dst, p in jobs:
        for t in (src, dst):
            if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous() or t.dim() != 3 \
                    or tuple(t.shape[-2:]) != (H, W):
                raise ValueError(f"BEV stacks must be contiguous cuda f32 [C, {H}, {W}] (got {tuple(t.shape)})")
        if src.shape != dst.shape:
            raise ValueError("augmentation output must match its input")
        if src.data_ptr() == dst.data_ptr():
            raise ValueError("augmentation passes are out of place (src and dst share storage)")
        st = _stages(p, H, W)
        bufs = [src] + [torch.empty_like(src) for _ in st[:-1]] + [dst]
        keep += bufs[1:-1]
        for i, (op, f) in enumerate(st):
            e = np.zeros((), _BEV_PASS)
            e["src"], e["dst"], e["C"], e["op"] = bufs[i].data_ptr(), bufs[i + 1].data_ptr(), src.shape[0], op
            e["flip"] = int(p["flip"] and i == 0)
            if i == len(st) - 1 and p["rects"]:
                e["n_rect"] = len(p["rects"])
                e["rect"][: len(p["rects"])] = p["rects"]
            for k, v in f.items():
                e[k] = v
            levels[i].append(e)
    cur = torch.cuda.current_stream()
    for lv in levels:
        if not lv:
            continue
        tab = torch.from_numpy(np.stack(lv).view(np.uint8).reshape(-1)).pin_memory().to(jobs[0][0].device,
                                                                                           non_blocking=True)
        keep.append(tab)
        lib.ivit_bev_augment(ptr(tab), len(lv), H, W, max(int(e["C"]) for e in lv), stream())
    for t in keep:  # scratch stacks and pass tables stay allocated until the launches have run
        t.record_stream(cur)


def _bev_in(x, device=None):
    if isinstance(x, torch.Tensor):
        t = x if x.is_cuda else x.to(_dev(device))
    else:
        t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(_dev(device))
    return t.float().contiguous()


def _gt_update(boxes, intents, p):
    """GT side of utils.py:402-411 (flip), 440-447 (rotate), 476-477 (scale), in place on numpy."""
    if p["flip"]:
        if boxes.shape[0] > 0:
            boxes[:, 1] *= -1
            boxes[:, 4] *= -1
            boxes[:, 4] = np.arctan2(np.sin(boxes[:, 4]), np.cos(boxes[:, 4]))
        if intents is not None and intents.shape[0] > 0:
            intents[:] = _FLIP_INTENTION[intents]
    if p["angle"] is not None and boxes.shape[0] > 0:
        rad = np.radians(p["angle"])
        cos_a, sin_a = np.cos(rad), np.sin(rad)
        cx, cy = boxes[:, 0].copy(), boxes[:, 1].copy()
        boxes[:, 0] = cx * cos_a - cy * sin_a
        boxes[:, 1] = cx * sin_a + cy * cos_a
        boxes[:, 4] += rad
        boxes[:, 4] = np.arctan2(np.sin(boxes[:, 4]), np.cos(boxes[:, 4]))
    if p["scale"] is not None and boxes.shape[0] > 0:
        boxes[:, :4] *= p["scale"]


def _augment_stacks(lidar_bev, map_bev, p, device=None):
    lb, mb = _bev_in(lidar_bev, device), _bev_in(map_bev, device)
    lo, mo = torch.empty_like(lb), torch.empty_like(mb)
    _run_bev_passes([(lb, lo, p), (mb, mo, p)])
    return lo, mo


def random_flip_bev(lidar_bev, map_bev, gt_boxes_xywha: np.ndarray, gt_intentions: np.ndarray):
    """utils.py:394-415 on the GPU: the rasters come back as device tensors (mirrored when the draw
    says so); the GT arrays are updated in place and returned, as in the reference."""
    p = _draw_params(rotate=False, scale=False, dropout=False)
    if p["flip"]:
        lidar_bev, map_bev = _augment_stacks(lidar_bev, map_bev, p)
        _gt_update(gt_boxes_xywha, gt_intentions, p)
    return lidar_bev, map_bev, gt_boxes_xywha, gt_intentions


def random_rotate_bev(lidar_bev, map_bev, gt_boxes_xywha: np.ndarray, angle_range_deg=(-15.0, 15.0)):
    """utils.py:417-448 on the GPU: one warpAffine pass over every channel of both stacks."""
    p = _draw_params(flip=False, scale=False, dropout=False, angle_range_deg=angle_range_deg)
    if p["angle"] is not None:
        lidar_bev, map_bev = _augment_stacks(lidar_bev, map_bev, p)
        _gt_update(gt_boxes_xywha, None, p)
    return lidar_bev, map_bev, gt_boxes_xywha


def random_scale_bev(lidar_bev, map_bev, gt_boxes_xywha: np.ndarray, scale_range=(0.95, 1.05)):
    """utils.py:450-478 on the GPU: one resize + centre crop / pad pass over both stacks."""
    p = _draw_params(flip=False, rotate=False, dropout=False, scale_range=scale_range)
    if p["scale"] is not None:
        lidar_bev, map_bev = _augment_stacks(lidar_bev, map_bev, p)
        _gt_update(gt_boxes_xywha, None, p)
    return lidar_bev, map_bev, gt_boxes_xywha


def random_bev_dropout(lidar_bev, map_bev, dropout_prob: float = 0.1, patch_size_range=(20, 50),
                       num_patches_range=(1, 5)):
    """utils.py:480-494 on the GPU: the drawn rectangles zeroed in a copy pass."""
    p = _draw_params(flip=False, rotate=False, scale=False, dropout_prob=dropout_prob,
                     patch_size_range=patch_size_range, num_patches_range=num_patches_range)
    if p["rects"]:
        lidar_bev, map_bev = _augment_stacks(lidar_bev, map_bev, p)
    return lidar_bev, map_bev


def _gt_arrays(gt_dict):
    b, i = gt_dict["boxes_xywha"], gt_dict["intentions"]
    b = b.detach().cpu().numpy().copy() if isinstance(b, torch.Tensor) else np.array(b, copy=True)
    i = i.detach().cpu().numpy().copy() if isinstance(i, torch.Tensor) else np.array(i, copy=True)
    return b, i


def augment_bev(lidar_bev, map_bev, gt_dict: dict, device=None):
    """utils.py:500-517 on the GPU: flip -> rotate -> scale -> dropout fused into one or two passes
    (two when rotate and scale are both drawn). -> (lidar, map device tensors, GT dict f32 / int64)."""
    p = _draw_params()
    lo, mo = _augment_stacks(lidar_bev, map_bev, p, device)
    b, i = _gt_arrays(gt_dict)
    _gt_update(b, i, p)
    return lo, mo, {"boxes_xywha": torch.from_numpy(b).float(), "intentions": torch.from_numpy(i).long()}


def augment_bev_batch(lidar_bev: torch.Tensor, map_bev: torch.Tensor, gt_list, out=None):
    """augment_bev for every sample of a device batch ([B, C, H, W] f32 each), sample 0's draws
    first (the dataset's __getitem__ order); one launch per pass depth for all 2B stacks.
    -> (lidar_out, map_out, gt_list_out, params)."""
    if lidar_bev.dim() != 4 or map_bev.dim() != 4 or lidar_bev.shape[0] != map_bev.shape[0]:
        raise ValueError("augment_bev_batch takes [B, C, H, W] lidar and map batches")
    lo, mo = out if out is not None else (torch.empty_like(lidar_bev), torch.empty_like(map_bev))
    jobs, gts, params = [], [], []
    for b in range(lidar_bev.shape[0]):
        p = _draw_params(H=lidar_bev.shape[-2], W=lidar_bev.shape[-1])
        jobs += [(lidar_bev[b], lo[b], p), (map_bev[b], mo[b], p)]
        bx, it = _gt_arrays(gt_list[b])
        _gt_update(bx, it, p)
        gts.append({"boxes_xywha": torch.from_numpy(bx).float(), "intentions": torch.from_numpy(it).long()})
        params.append(p)
    _run_bev_passes(jobs)
    return lo, mo, gts, params


# ---------------------------------------------------------------------------- HD-map raster
# rasterize_map_ego_centric (utils.py:108-182). The host part is the
# reference's own flow (JSON, ego yaw from the quaternion, world -> pixel with np.round, in-grid
# point filtering, which primitive goes to which channel); the scan conversion — cv2.polylines /
# cv2.fillPoly, the CPU-heavy part — runs on the GPU (ivit_map_raster): one launch draws every
# segment and polygon edge (cv::Line, 8-connected), one fills every polygon scanline.
MAP_MARK_CHANNELS = {"DASHED_WHITE": 6, "SOLID_WHITE": 7, "SOLID_YELLOW": 8}


def get_ego_centric_transform_matrix(ego_translation_xy: np.ndarray, ego_yaw: float) -> np.ndarray:
    """utils.py:35-45: world -> ego 2-D homogeneous transform (rotation by -yaw)."""
    c, s = np.cos(-ego_yaw), np.sin(-ego_yaw)
    rot = np.array([[c, -s], [s, c]])
    T = np.eye(3)
    T[:2, :2] = rot
    T[:2, 2] = -rot @ ego_translation_xy
    return T


def world_to_bev_pixel(points_world_xy: np.ndarray, ego_tf_matrix: np.ndarray, H: int = GRID_HEIGHT_PX,
                       W: int = GRID_WIDTH_PX) -> np.ndarray:
    """utils.py:47-60: (x, y) world -> (col, row) pixels, np.round (half to even) then int."""
    if points_world_xy.shape[0] == 0:
        return np.empty((0, 2), dtype=int)
    homo = np.hstack([points_world_xy, np.ones((points_world_xy.shape[0], 1))])
    ego = (ego_tf_matrix @ homo.T).T[:, :2]
    px = W / 2.0 + ego[:, 1] / VOXEL_SIZE_M
    py = H * 3.0 / 4.0 - ego[:, 0] / VOXEL_SIZE_M
    return np.round(np.vstack([px, py]).T).astype(int)


def _map_pixels(points, T, H, W):
    """to_bev_pixel_local (utils.py:131-145)."""
    if not points:
        return np.empty((0, 2), dtype=int)
    valid = [p for p in points if isinstance(p, dict) and 'x' in p and 'y' in p]
    if not valid:
        return np.empty((0, 2), dtype=int)
    pix = world_to_bev_pixel(np.array([[p['x'], p['y']] for p in valid]), T, H, W)
    keep = (pix[:, 0] >= 0) & (pix[:, 0] < W) & (pix[:, 1] >= 0) & (pix[:, 1] < H)
    return pix[keep]


def _map_primitives(map_data, ego_pose, H, W):
    """-> (polylines [(pts, plane mask)], polygons [(pts, plane mask)]) in the reference's order
    (utils.py:147-180); None when the ego quaternion is invalid (the reference's empty map)."""
    from scipy.spatial.transform import Rotation
    q = [ego_pose['qx'], ego_pose['qy'], ego_pose['qz'], ego_pose['qw']]
    try:
        yaw = Rotation.from_quat(q).as_euler('xyz')[2]
    except ValueError:
        return None
    T = get_ego_centric_transform_matrix(np.array([ego_pose['tx_m'], ego_pose['ty_m']]), yaw)
    lines, polys = [], []
    for _, lane in map_data.get("lane_segments", {}).items():
        lpx = _map_pixels(lane.get("left_lane_boundary", []), T, H, W)
        rpx = _map_pixels(lane.get("right_lane_boundary", []), T, H, W)
        if len(lpx) > 1 and len(rpx) > 1:
            poly = np.vstack([lpx, np.flipud(rpx)])
            if poly.shape[0] >= 3:
                mask = 1 | (16 if lane.get("is_intersection", False) else 0) | (32 if lane.get("lane_type") == "BUS" else 0)
                polys.append((poly, mask))
        lm, rm = lane.get("left_lane_mark_type", ""), lane.get("right_lane_mark_type", "")
        if len(lpx) > 1:
            lines.append((lpx, 2 | (1 << MAP_MARK_CHANNELS[lm] if lm in MAP_MARK_CHANNELS else 0)))
        if len(rpx) > 1:
            lines.append((rpx, 4 | (1 << MAP_MARK_CHANNELS[rm] if rm in MAP_MARK_CHANNELS else 0)))
    for _, cw in map_data.get("pedestrian_crossings", {}).items():
        poly = cw.get('polygon', [])
        if poly:
            px = _map_pixels(poly, T, H, W)
            if len(px) >= 3:
                polys.append((px, 8))
    return lines, polys


def _map_tables(prims_per_image, H, W, img_stride):
    """Host tables of ivit_map_raster for a batch (image b's planes start at b * img_stride)."""
    seg, seg_base, edges, polys, poly_base, rows = [], [], [], [], [], []
    max_edges = 0
    for b, prims in enumerate(prims_per_image):
        if prims is None:
            continue
        lines, pgs = prims
        base = b * img_stride
        for pts, mask in lines:
            p = np.asarray(pts, np.int64)
            s = np.concatenate([p[:-1], p[1:], np.full((len(p) - 1, 1), mask)], 1)
            seg.append(s)
            seg_base.append(np.full(len(s), base))
        for pts, mask in pgs:
            p = np.asarray(pts, np.int64)
            prev = np.roll(p, 1, axis=0)  # edge i: vertex i-1 -> vertex i (the closing edge first)
            s = np.concatenate([prev, p, np.full((len(p), 1), mask)], 1)
            seg.append(s)
            seg_base.append(np.full(len(s), base))
            xa, ya, xb, yb = prev[:, 0], prev[:, 1], p[:, 0], p[:, 1]
            nh = ya != yb
            if nh.sum() < 2:
                continue
            xa, ya, xb, yb = xa[nh], ya[nh], xb[nh], yb[nh]
            num, den = (xb - xa) << 16, yb - ya
            dx = np.abs(num) // np.abs(den) * np.where((num >= 0) == (den > 0), 1, -1)  # C truncation
            top_a = ya < yb
            e = np.stack([np.where(top_a, ya, yb), np.where(top_a, yb, ya),
                          np.where(top_a, xa, xb) << 16, dx], 1)
            first = sum(len(x) for x in edges)
            edges.append(e)
            max_edges = max(max_edges, len(e))
            pi = len(polys)
            polys.append((first, len(e), mask))
            poly_base.append(base)
            y0, y1 = max(int(e[:, 0].min()), 0), min(int(e[:, 1].max()), H)
            if y1 > y0:
                rows.append(np.stack([np.full(y1 - y0, pi), np.arange(y0, y1)], 1))
    cat = (lambda xs, shape, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(shape, dt))
    return (cat(seg, (0, 5), np.int32), cat(seg_base, (0,), np.int64), cat(edges, (0, 4), np.int64),
            np.array(polys, np.int32).reshape(-1, 3), np.array(poly_base, np.int64), cat(rows, (0, 2), np.int32),
            max_edges)


def _load_map(m):
    import json
    if m is None or isinstance(m, dict):
        return m
    try:
        with open(m, "r") as f:
            return json.load(f)
    except Exception as e:  # noqa: BLE001  (the reference's behaviour, utils.py:111-116)
        print(f"Error loading map JSON {m}: {e}. Returning empty map.")
        return None


def rasterize_map_batch(items, H: int = GRID_HEIGHT_PX, W: int = GRID_WIDTH_PX, out: torch.Tensor | None = None,
                        device=None) -> torch.Tensor:
    """rasterize_map_ego_centric for a batch: items = [(map JSON path or parsed dict, ego pose
    with tx_m, ty_m, qx, qy, qz, qw)] -> (B, 9, H, W) f32 on the GPU (``out`` may be a collated
    map_bev tensor: it is zero-filled and drawn in place), one launch per stage."""
    d = _dev(device if out is None else out.device)
    B = len(items)
    if out is None:
        out = torch.zeros((B, MAP_CHANNELS, H, W), dtype=torch.float32, device=d)
    else:
        if out.shape != (B, MAP_CHANNELS, H, W) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("rasterize_map_batch: out must be a contiguous (B, 9, H, W) float32 tensor")
        out.zero_()
    prims = []
    for m, pose in items:
        md = _load_map(m)
        pr = None if md is None else _map_primitives(md, pose, H, W)
        if md is not None and pr is None:
            print("Warning: Invalid ego quaternion. Returning empty map.")
        prims.append(pr)
    seg, seg_base, edges, polys, poly_base, rows, max_edges = _map_tables(prims, H, W, MAP_CHANNELS * H * W)
    if len(seg) == 0 and len(rows) == 0:
        return out
    t = [torch.from_numpy(a).pin_memory().to(d, non_blocking=True) if a.size else None
         for a in (seg, seg_base, edges, polys, poly_base, rows)]
    lib.ivit_map_raster(ptr(t[0]), len(seg), ptr(t[1]), ptr(t[2]), ptr(t[3]), len(polys), ptr(t[4]), ptr(t[5]),
                        len(rows), max_edges, H, W, ptr(out), stream())
    return out


def rasterize_map_ego_centric(map_json_path, current_ego_pose, device=None) -> torch.Tensor:
    """utils.py:108-182 -> (9, GRID_H, GRID_W) float32 {0, 1} on the GPU (the reference returns
    the same array on the host). Channels: 0 lane area, 1 / 2 left / right boundaries, 3
    crosswalks, 4 intersections, 5 bus lanes, 6-8 dashed-white / solid-white / solid-yellow marks."""
    return rasterize_map_batch([(map_json_path, current_ego_pose)], device=device)[0]
