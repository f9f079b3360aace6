"""Box geometry of the reference's utils.py (anchors, axis/rotated IoU, decode, NMS, AP)
on the MI355X kernels. BEV rasterisation, ego transforms and augmentations (utils.py:22-225,
394-517) belong to the Argoverse-2 data pipeline, which is outside this build's scope."""
from __future__ import annotations

import numpy as np
import torch

from _lib import lib, ptr, stream, workspace
from constants import (ANCHOR_CONFIGS_PAPER, BEV_PIXEL_OFFSET_X, BEV_PIXEL_OFFSET_Y, GRID_HEIGHT_PX, GRID_WIDTH_PX,
                       VOXEL_SIZE_M)


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


def postprocess_batch(cls_logits: torch.Tensor, box_preds_rel: torch.Tensor, intent_logits: torch.Tensor,
                      anchors: torch.Tensor, conf_threshold: float = 0.1, nms_threshold: float = 0.2):
    """eval_vit.py:157-180 for a whole batch: sigmoid → score >= conf → decode → NMS → argmax
    intention, per sample; returns [{'pred_scores', 'pred_boxes_xywha', 'pred_intentions'}]
    as device tensors (the caller moves them to the host when it needs them)."""
    B = cls_logits.shape[0]
    scores = torch.sigmoid(cls_logits.reshape(B, -1).float())
    box = box_preds_rel.reshape(B, scores.shape[1], -1)
    it = intent_logits.reshape(B, scores.shape[1], -1)
    out = []
    for b in range(B):
        idx = torch.nonzero(scores[b] >= conf_threshold).squeeze(1)
        res = {"pred_scores": scores.new_empty((0,)), "pred_boxes_xywha": scores.new_empty((0, 5)),
               "pred_intentions": torch.empty((0,), dtype=torch.long, device=scores.device)}
        if idx.numel() > 0:
            sf = scores[b].index_select(0, idx)
            dec = decode_box_predictions(box[b].index_select(0, idx), anchors.index_select(0, idx))
            keep = apply_nms(dec, sf, nms_threshold)
            if keep.numel() > 0:
                res = {"pred_scores": sf[keep], "pred_boxes_xywha": dec[keep],
                       "pred_intentions": torch.argmax(it[b].index_select(0, idx)[keep], dim=-1)}
        out.append(res)
    return out


def calculate_ap(recall: np.ndarray, precision: np.ndarray) -> float:
    """utils.py:564-575 (VOC-style AP; host-side metric)."""
    mrec = np.concatenate(([0.0], recall, [1.0]))
    mpre = np.concatenate(([0.0], precision, [0.0]))
    mpre = np.maximum.accumulate(mpre[::-1])[::-1]
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return float(np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1]))
