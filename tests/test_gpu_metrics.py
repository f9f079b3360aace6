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


def test_det_match_ap_vs_reference_fixture():
    """ivit_det_match's AP vs the reference's OWN calculate_ap (tests/golden/ap_reference.npz): each
    case's TP sequence is laid out as a score-ordered IoU matrix (a TP row: 0.95 with the next
    unmatched GT, 0 elsewhere; an FP row: 0.1 everywhere), all cases in one launch."""
    from conftest import golden
    from _lib import lib, ptr, stream, workspace
    z = golden("ap_reference.npz")
    n = int(z["n_cases"][0])
    mats, npred, ngt = [], [], []
    for k in range(n):
        tp, G = z[f"c{k}_tp"], int(z[f"c{k}_ngt"][0])
        m = np.full((tp.size, G), 0.1, np.float32)
        j = 0
        for r in np.nonzero(tp)[0]:
            m[r] = 0.0
            m[r, j] = 0.95
            j += 1
        mats.append(m.reshape(-1))
        npred.append(tp.size)
        ngt.append(G)
    sizes = [p * g for p, g in zip(npred, ngt)]
    iou = torch.from_numpy(np.concatenate(mats)).cuda()
    iou_off = torch.from_numpy(np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)).cuda()
    pred_off_np = np.concatenate([[0], np.cumsum(npred)[:-1]]).astype(np.int64)
    pred_off = torch.from_numpy(pred_off_np).cuda()
    d_np = torch.tensor(npred, dtype=torch.int32).cuda()
    d_ng = torch.tensor(ngt, dtype=torch.int32).cuda()
    thr = torch.tensor([0.5], dtype=torch.float32).cuda()
    tot = int(sum(npred))
    ap = torch.empty((n, 1), dtype=torch.float64, device="cuda")
    best = torch.empty(tot, dtype=torch.int32, device="cuda")
    tpo = torch.empty((1, tot), dtype=torch.uint8, device="cuda")
    ws = workspace(8 * tot, torch.device("cuda"))
    lib.ivit_det_match(ptr(iou), ptr(iou_off), ptr(d_np), ptr(d_ng), ptr(pred_off), n, tot, ptr(thr), 1, ptr(ap),
                       ptr(best), ptr(tpo), ptr(ws), ws.numel(), max(ngt), stream())
    ap = ap.cpu().numpy()[:, 0]
    tpo = tpo.cpu().numpy()[0].astype(bool)
    for k in range(n):
        tp = z[f"c{k}_tp"]
        np.testing.assert_array_equal(tpo[pred_off_np[k]:pred_off_np[k] + tp.size], tp)
        # P == 0 is the eval flow's own case (eval_vit.py:210-212: 1.0 / 0.0, calculate_ap not called)
        want = (1.0 if ngt[k] == 0 else 0.0) if tp.size == 0 else float(z[f"c{k}_ap"][0])
        assert abs(ap[k] - want) < 1e-12, (k, ap[k], want)
