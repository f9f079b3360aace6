"""Detection mAP and intention-matching metrics of eval_vit.py:191-311 (host side).

The reference walks the score-sorted predictions one by one: a prediction is a true positive
when the IoU with its best GT (``torch.max`` over the row, first index on ties) reaches the
threshold and that GT is not matched yet. The best GT of a prediction does not depend on the
matching state, so the walk is exactly "the first qualifying prediction of each GT, in sorted
order" — computed here with one ``np.unique(return_index=True)`` per threshold instead of a
Python loop over up to 22 500 predictions.
"""
from __future__ import annotations

import numpy as np
import torch

from constants import DETECTION_IOU_THRESHOLDS, IOU_THRESHOLD_FOR_INTENTION_MATCH
from utils import calculate_ap, compute_axis_aligned_iou, compute_rotated_iou


def _iou(pred, gt, rotated):
    """(P,5) x (G,5) → (P,G) numpy f32; device kernels (utils.py:276-392 semantics)."""
    dev = torch.device("cuda")
    p = pred.to(dev).float()
    g = gt.to(dev).float()
    if rotated:
        return compute_rotated_iou(p, g).cpu().numpy()
    return compute_axis_aligned_iou(p[:, :4], g[:, :4]).cpu().numpy()


def _first_match(iou_sorted: np.ndarray, thr: float) -> np.ndarray:
    """TP flags of the sequential greedy matching (eval_vit.py:236-247) in sorted order."""
    best = iou_sorted.max(axis=1)
    arg = iou_sorted.argmax(axis=1)
    q = np.nonzero(best >= thr)[0]
    tp = np.zeros(iou_sorted.shape[0], dtype=bool)
    if q.size:
        _, first = np.unique(arg[q], return_index=True)
        tp[q[first]] = True
    return tp


def _stable_desc(scores: np.ndarray) -> np.ndarray:
    # torch.argsort(descending=True) on CPU is not guaranteed stable; a stable order is used
    # here (ties are measure-zero for sigmoid scores of distinct anchors).
    return np.argsort(-scores, kind="stable")


def detection_map(results, thresholds=DETECTION_IOU_THRESHOLDS, rotated=False):
    """results: list of dicts with pred_scores, pred_boxes_xywha, gt_boxes_xywha → {thr: mAP}."""
    aps = {t: [] for t in thresholds}
    for r in results:
        ps = np.asarray(r["pred_scores"].cpu(), dtype=np.float32)
        npred, ngt = ps.shape[0], r["gt_boxes_xywha"].shape[0]
        iou = None
        for t in thresholds:
            if npred == 0:
                aps[t].append(1.0 if ngt == 0 else 0.0)
                continue
            if ngt == 0:
                aps[t].append(0.0)
                continue
            if iou is None:
                order = _stable_desc(ps)
                iou = _iou(r["pred_boxes_xywha"][torch.from_numpy(order)], r["gt_boxes_xywha"], rotated)
            tp = _first_match(iou, t)
            cum = np.cumsum(tp.astype(np.float32))
            recall = cum / (ngt + 1e-9)
            precision = cum / (np.arange(1, npred + 1, dtype=np.float32) + 1e-9)
            aps[t].append(calculate_ap(recall, precision))
    return {t: (float(np.mean(v)) if v else 0.0) for t, v in aps.items()}


def intention_matches(results, thr=IOU_THRESHOLD_FOR_INTENTION_MATCH, rotated=False):
    """Matched (pred_intent, gt_intent) pairs of eval_vit.py:268-292."""
    mp, mg = [], []
    for r in results:
        npred, ngt = r["pred_boxes_xywha"].shape[0], r["gt_boxes_xywha"].shape[0]
        if npred == 0 or ngt == 0:
            continue
        ps = np.asarray(r["pred_scores"].cpu(), dtype=np.float32)
        order = _stable_desc(ps)
        iou = _iou(r["pred_boxes_xywha"], r["gt_boxes_xywha"], rotated)[order]
        tp = _first_match(iou, thr)
        gt_idx = iou.argmax(axis=1)
        pi = np.asarray(r["pred_intentions"].cpu())[order]
        gi = np.asarray(r["gt_intentions"].cpu())
        for k in np.nonzero(tp)[0]:
            mp.append(int(pi[k]))
            mg.append(int(gi[gt_idx[k]]))
    return mp, mg
