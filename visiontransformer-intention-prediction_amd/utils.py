"""Box geometry of the reference's utils.py (anchors, axis/rotated IoU, decode, NMS, AP) and
the LiDAR BEV voxelisation with its sweep ego transform (utils.py:27-33, 62-106; SURVEY.md §8f
rank 1) on the MI355X kernels. Map rasterisation and augmentations (utils.py:108-225, 394-517)
belong to the Argoverse-2 data pipeline, which is outside this build's scope."""
from __future__ import annotations

import numpy as np
import torch

from _lib import lib, ptr, stream, workspace
from constants import (ANCHOR_CONFIGS_PAPER, BEV_PIXEL_OFFSET_X, BEV_PIXEL_OFFSET_Y, GRID_HEIGHT_PX, GRID_WIDTH_PX,
                       LIDAR_HEIGHT_CHANNELS, LIDAR_SWEEPS, VOXEL_SIZE_M, Z_MAX, Z_MIN)


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
    ws = workspace(24 * total + 8 * sum(words) + 64, dev)
    lib.ivit_nms_batched(ptr(b), ptr(sc), ptr(d_seg), ptr(d_moff), S, total, max(ns), sum(words),
                         float(iou_threshold), ptr(keep), ptr(count), ptr(ws), ws.numel(), stream())
    cnt = count.cpu().tolist()
    return [keep[seg[i]: seg[i] + cnt[i]] for i in range(S)]


def postprocess_batch(cls_logits: torch.Tensor, box_preds_rel: torch.Tensor, intent_logits: torch.Tensor,
                      anchors: torch.Tensor, conf_threshold: float = 0.1, nms_threshold: float = 0.2):
    """eval_vit.py:157-180 for a whole batch: sigmoid → score >= conf → decode → NMS → argmax
    intention, per sample; returns [{'pred_scores', 'pred_boxes_xywha', 'pred_intentions'}]
    as device tensors (the caller moves them to the host when it needs them)."""
    B = cls_logits.shape[0]
    scores = torch.sigmoid(cls_logits.reshape(B, -1).float())
    box = box_preds_rel.reshape(B, scores.shape[1], -1)
    it = intent_logits.reshape(B, scores.shape[1], -1)
    idxs, sfs, decs = [], [], []
    for b in range(B):
        idx = torch.nonzero(scores[b] >= conf_threshold).squeeze(1)
        idxs.append(idx)
        sfs.append(scores[b].index_select(0, idx))
        decs.append(decode_box_predictions(box[b].index_select(0, idx), anchors.index_select(0, idx))
                    if idx.numel() > 0 else scores.new_empty((0, 5)))
    keeps = nms_batched(decs, sfs, nms_threshold)  # all samples' NMS in one batched launch per stage
    out = []
    for b in range(B):
        keep = keeps[b]
        if keep.numel() > 0:
            res = {"pred_scores": sfs[b][keep], "pred_boxes_xywha": decs[b][keep],
                   "pred_intentions": torch.argmax(it[b].index_select(0, idxs[b])[keep], dim=-1)}
        else:
            res = {"pred_scores": scores.new_empty((0,)), "pred_boxes_xywha": scores.new_empty((0, 5)),
                   "pred_intentions": torch.empty((0,), dtype=torch.long, device=scores.device)}
        out.append(res)
    return out


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
