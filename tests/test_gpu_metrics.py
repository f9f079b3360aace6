"""Device mAP / intention matching (ivit_det_match) against a literal
restatement of the reference's sequential walk (eval_vit.py:224-257, 268-292) and calculate_ap
(utils.py:564-575), on the same device IoU matrices (the IoU kernels are pinned separately by
tests/golden/geometry.npz)."""
import numpy as np
import pytest
import torch

from test_cpu_host import _case

pytestmark = pytest.mark.gpu
THR = [0.5, 0.6, 0.7, 0.8, 0.9]


def _walk(scores, iou_sorted, ngt, thr):
    """eval_vit.py:224-257 with explicit loops on a score-sorted IoU matrix (numpy f32)."""
    from utils import calculate_ap
    npred = len(scores)
    if npred == 0:
        return 1.0 if ngt == 0 else 0.0, []
    if ngt == 0:
        return 0.0, []
    matched = np.zeros(ngt, bool)
    tp = np.zeros(npred, bool)
    pairs = []
    for k in range(npred):
        j = int(np.argmax(iou_sorted[k]))
        if iou_sorted[k, j] >= np.float32(thr) and not matched[j]:
            tp[k] = True
            matched[j] = True
            pairs.append((k, j))
    cum = np.cumsum(tp.astype(np.float32))
    rec = cum / (ngt + 1e-9)
    prec = cum / (np.arange(1, npred + 1, dtype=np.float32) + 1e-9)
    return calculate_ap(rec, prec), pairs


def _results(specs):
    res = []
    for seed, npred, ngt in specs:
        s, p, g, pi, gi = _case(seed, npred, ngt)
        if seed % 2 and npred > 4:
            s[1::3] = s[0]  # score ties: the stable descending order decides
        if ngt > 3:
            g[2] = g[1]     # duplicate GT: IoU ties, the first index wins
        res.append({"pred_scores": s.cuda(), "pred_boxes_xywha": p.cuda(), "gt_boxes_xywha": g.cuda(),
                    "pred_intentions": pi.cuda(), "gt_intentions": gi.cuda()})
    return res


SPECS = [(0, 50, 10), (1, 300, 25), (2, 0, 5), (3, 7, 0), (4, 0, 0), (5, 1, 1), (6, 700, 40), (7, 2000, 60)]


def test_det_match_map_equals_sequential_walk():
    import metrics
    from utils import compute_axis_aligned_iou
    res = _results(SPECS)
    ap, per = metrics.match_device(res, THR)
    for i, r in enumerate(res):
        sc = r["pred_scores"].cpu().numpy()
        order = np.argsort(-sc, kind="stable")
        assert np.array_equal(per[i][0].cpu().numpy(), order)
        ngt = r["gt_boxes_xywha"].shape[0]
        iou = (compute_axis_aligned_iou(r["pred_boxes_xywha"][torch.from_numpy(order).cuda()][:, :4],
                                        r["gt_boxes_xywha"][:, :4]).cpu().numpy() if len(sc) and ngt else None)
        for t, thr in enumerate(THR):
            want, pairs = _walk(sc, iou, ngt, thr)
            assert ap[i, t] == pytest.approx(want, abs=1e-12), (i, thr)
            if len(sc) and ngt:
                got_tp = np.nonzero(per[i][1][t].cpu().numpy())[0]
                assert got_tp.tolist() == [k for k, _ in pairs]
    maps = metrics.detection_map_device(res, THR)
    for t, thr in enumerate(THR):
        assert maps[thr] == pytest.approx(float(np.mean(ap[:, t])), abs=1e-15)


def test_intention_matches_device_equals_sequential_walk():
    import metrics
    from utils import compute_axis_aligned_iou
    res = _results([(11, 400, 30), (12, 90, 12), (13, 0, 3)])
    mp, mg = metrics.intention_matches_device(res, 0.5)
    ep, eg = [], []
    for r in res:
        sc = r["pred_scores"].cpu().numpy()
        ngt = r["gt_boxes_xywha"].shape[0]
        if len(sc) == 0 or ngt == 0:
            continue
        order = np.argsort(-sc, kind="stable")
        iou = compute_axis_aligned_iou(r["pred_boxes_xywha"][:, :4], r["gt_boxes_xywha"][:, :4]).cpu().numpy()
        _, pairs = _walk(sc[order], iou[order], ngt, 0.5)
        pi, gi = r["pred_intentions"].cpu().numpy(), r["gt_intentions"].cpu().numpy()
        ep += [int(pi[order[k]]) for k, _ in pairs]
        eg += [int(gi[j]) for _, j in pairs]
    assert (mp, mg) == (ep, eg) and len(ep) > 5


def test_det_match_agrees_with_host_vectorised_path():
    import metrics
    res = _results(SPECS[:6])
    host = metrics.detection_map(res, THR)
    dev = metrics.detection_map_device(res, THR)
    for thr in THR:
        assert dev[thr] == pytest.approx(host[thr], abs=1e-12)
