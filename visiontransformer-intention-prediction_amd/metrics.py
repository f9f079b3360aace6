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


# ---------------------------------------------------------------------------- device path (§8f-2)
def match_device(results, thresholds, rotated=False):
    """All samples' greedy matching + VOC AP in one launch (ivit_det_match).

    results: dicts with pred_scores / pred_boxes_xywha / gt_boxes_xywha (device tensors; the
    predictions are re-ordered by a stable descending score sort — postprocess_batch already
    emits them in that order). Returns (ap [S, T] float64 numpy, per-sample (order, tp [T, P]
    bool, best_gt [P]) on the device)."""
    from _lib import lib, ptr, stream, workspace
    dev = torch.device("cuda")
    S, T = len(results), len(thresholds)
    ious, npred, ngt, orders = [], [], [], []
    for r in results:
        ps = r["pred_scores"].to(dev)
        P, G = int(ps.shape[0]), int(r["gt_boxes_xywha"].shape[0])
        order = torch.sort(ps, descending=True, stable=True).indices if P else torch.zeros(0, dtype=torch.long,
                                                                                           device=dev)
        if P and G:
            pb = r["pred_boxes_xywha"].to(dev).float()[order]
            gb = r["gt_boxes_xywha"].to(dev).float()
            m = compute_rotated_iou(pb, gb) if rotated else compute_axis_aligned_iou(pb[:, :4], gb[:, :4])
            ious.append(m.reshape(-1))
        npred.append(P)
        ngt.append(G)
        orders.append(order)
    if max(ngt, default=0) > 4096:
        raise ValueError("device matching supports at most 4096 GT boxes per sample")
    iou = torch.cat(ious) if ious else torch.zeros(1, device=dev)
    sizes = [p * g if p and g else 0 for p, g in zip(npred, ngt)]
    iou_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64) if S else np.zeros(0, np.int64)
    pred_off = np.concatenate([[0], np.cumsum(npred)[:-1]]).astype(np.int64) if S else np.zeros(0, np.int64)
    tot = int(sum(npred))
    h2d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_iou_off, d_pred_off = h2d(iou_off), h2d(pred_off)
    d_np, d_ng = h2d(np.asarray(npred, np.int32)), h2d(np.asarray(ngt, np.int32))
    d_thr = h2d(np.asarray(thresholds, np.float32))
    ap = torch.empty((S, T), dtype=torch.float64, device=dev)
    best = torch.empty(max(tot, 1), dtype=torch.int32, device=dev)
    tp = torch.empty((T, max(tot, 1)), dtype=torch.uint8, device=dev)
    ws = workspace(8 * T * max(tot, 1), dev)
    lib.ivit_det_match(ptr(iou), ptr(d_iou_off), ptr(d_np), ptr(d_ng), ptr(d_pred_off), S, tot, ptr(d_thr), T,
                       ptr(ap), ptr(best), ptr(tp), ptr(ws), ws.numel(), max(ngt, default=0), stream())
    per = [(orders[i], tp[:, pred_off[i]:pred_off[i] + npred[i]].bool(), best[pred_off[i]:pred_off[i] + npred[i]])
           for i in range(S)]
    return ap.cpu().numpy(), per


def detection_map_device(results, thresholds=DETECTION_IOU_THRESHOLDS, rotated=False):
    """detection_map (eval_vit.py:191-262) with the matching and AP on the device."""
    if not results:
        return {t: 0.0 for t in thresholds}
    ap, _ = match_device(results, thresholds, rotated)
    return {t: float(np.mean(ap[:, i])) for i, t in enumerate(thresholds)}


def intention_matches_device(results, thr=IOU_THRESHOLD_FOR_INTENTION_MATCH, rotated=False):
    """intention_matches (eval_vit.py:268-292): the TPs at `thr` with their best GT, on the device."""
    if not results:
        return [], []
    _, per = match_device(results, [thr], rotated)
    mp, mg = [], []
    for r, (order, tp, best) in zip(results, per):
        if order.numel() == 0 or r["gt_boxes_xywha"].shape[0] == 0:
            continue
        k = torch.nonzero(tp[0]).flatten()
        pi = r["pred_intentions"].to(order.device)[order][k]
        gi = r["gt_intentions"].to(order.device)[best[k].long()]
        mp.extend(pi.cpu().tolist())
        mg.extend(gi.cpu().tolist())
    return mp, mg
