"""Host-side logic of the eval / train entry points (CPU only): the vectorised mAP and
intention matching of metrics.py against a literal restatement of the reference's sequential
walk (eval_vit.py:224-257, 268-292), calculate_ap (utils.py:564-575), and the synthetic batch
format / distribution (dataset.py:137-150)."""
import math

import numpy as np
import pytest
import torch

import metrics
import synthetic
from oracle import ivit_oracle as O
from utils import calculate_ap


def _np_iou(pred, gt, rotated):
    p, g = pred.float(), gt.float()
    r = O.rotated_iou_numpy(p, g) if rotated else O.axis_aligned_iou(p[:, :4], g[:, :4])
    return np.asarray(r)


@pytest.fixture(autouse=True)
def host_iou(monkeypatch):
    monkeypatch.setattr(metrics, "_iou", _np_iou)


def _loop_ap(scores, boxes, gts, thr):
    """eval_vit.py:224-257 restated with explicit loops."""
    npred, ngt = len(scores), len(gts)
    if npred == 0:
        return 1.0 if ngt == 0 else 0.0
    if ngt == 0:
        return 0.0
    order = np.argsort(-scores, kind="stable")
    iou = _np_iou(boxes[torch.from_numpy(order)], gts, False)
    matched = np.zeros(ngt, bool)
    tp = np.zeros(npred, bool)
    for k in range(npred):
        j = int(np.argmax(iou[k]))
        if iou[k, j] >= thr and not matched[j]:
            tp[k] = True
            matched[j] = True
    cum = np.cumsum(tp.astype(np.float32))
    rec = cum / (ngt + 1e-9)
    prec = cum / (np.arange(1, npred + 1, dtype=np.float32) + 1e-9)
    return calculate_ap(rec, prec)


def _case(seed, npred, ngt):
    g = torch.Generator().manual_seed(seed)
    gt = torch.stack([torch.rand(ngt, generator=g) * 40, torch.rand(ngt, generator=g) * 40,
                      1.5 + torch.rand(ngt, generator=g) * 2, 3 + torch.rand(ngt, generator=g) * 3,
                      torch.zeros(ngt)], 1)
    # predictions: jittered copies of GTs (duplicates → FP after the first) plus clutter
    src = torch.randint(0, max(ngt, 1), (npred,), generator=g)
    pred = gt[src].clone() if ngt else torch.zeros((npred, 5))
    pred[:, :2] += torch.randn(npred, 2, generator=g) * 0.6
    pred[npred // 2:, :2] = torch.rand(npred - npred // 2, 2, generator=g) * 40
    return torch.rand(npred, generator=g), pred, gt, torch.randint(0, 8, (npred,), generator=g), \
        torch.randint(0, 8, (ngt,), generator=g)


@pytest.mark.parametrize("seed,npred,ngt", [(0, 50, 10), (1, 300, 25), (2, 0, 5), (3, 7, 0), (4, 0, 0), (5, 1, 1)])
def test_detection_map_matches_sequential_walk(seed, npred, ngt):
    s, p, g, _, _ = _case(seed, npred, ngt)
    res = [{"pred_scores": s, "pred_boxes_xywha": p, "gt_boxes_xywha": g}]
    got = metrics.detection_map(res, [0.3, 0.5, 0.7])
    for t in (0.3, 0.5, 0.7):
        assert got[t] == pytest.approx(_loop_ap(s.numpy(), p, g, t), abs=1e-12)


def test_intention_matches_sequential_walk():
    s, p, g, pi, gi = _case(7, 120, 15)
    res = [{"pred_scores": s, "pred_boxes_xywha": p, "pred_intentions": pi, "gt_boxes_xywha": g,
            "gt_intentions": gi}]
    mp_, mg_ = metrics.intention_matches(res, 0.5)
    # eval_vit.py:277-292 restated
    iou = _np_iou(p, g, False)
    order = np.argsort(-s.numpy(), kind="stable")
    matched = np.zeros(len(g), bool)
    ep, eg = [], []
    for k in order:
        j = int(np.argmax(iou[k]))
        if iou[k, j] >= 0.5 and not matched[j]:
            matched[j] = True
            ep.append(int(pi[k]))
            eg.append(int(gi[j]))
    assert (mp_, mg_) == (ep, eg)
    assert len(ep) > 3


def test_calculate_ap_known_values():
    assert calculate_ap(np.array([0.5, 1.0]), np.array([1.0, 1.0])) == pytest.approx(1.0)
    assert calculate_ap(np.array([0.0, 0.5]), np.array([0.0, 0.5])) == pytest.approx(0.25)


def _ap_cases():
    from conftest import golden
    z = golden("ap_reference.npz")
    return z, int(z["n_cases"][0])


def test_calculate_ap_vs_reference_fixture():
    """The build's calculate_ap and metrics' recall / precision steps vs the reference's OWN
    utils.calculate_ap (utils.py:564-575) on eval_vit.py:249-255's steps (tests/golden/ap_reference.npz,
    oracle/make_golden.py gen_ap): empty, all-TP, all-FP, single TP / FP, tied recall plateaus,
    seeded walks up to 2000 predictions."""
    z, n = _ap_cases()
    for k in range(n):
        tp, G = z[f"c{k}_tp"], int(z[f"c{k}_ngt"][0])
        cum = np.cumsum(tp.astype(np.float32))  # metrics.detection_map's steps
        rec = cum / (G + 1e-9)
        prec = cum / (np.arange(1, tp.size + 1, dtype=np.float32) + 1e-9)
        np.testing.assert_array_equal(rec, z[f"c{k}_recall"])
        np.testing.assert_array_equal(prec, z[f"c{k}_precision"])
        assert calculate_ap(z[f"c{k}_recall"], z[f"c{k}_precision"]) == float(z[f"c{k}_ap"][0]), k


def test_synthetic_batch_format_and_ranges():
    b = synthetic.synthetic_batch(2, (32, 48), torch.Generator().manual_seed(1234))
    assert b["lidar_bev"].shape == (2, 290, 32, 48) and b["lidar_bev"].dtype == torch.float32
    assert b["map_bev"].shape == (2, 9, 32, 48)
    assert set(torch.unique(b["map_bev"]).tolist()) <= {0.0, 1.0}
    assert float(b["lidar_bev"].min()) >= 0.0 and float(b["lidar_bev"].max()) < 1.0
    assert len(b["gt_list"]) == 2
    gt = b["gt_list"][0]
    assert gt["boxes_xywha"].shape == (20, 5) and gt["intentions"].dtype == torch.int64
    s = 32 / 400.0
    bx = gt["boxes_xywha"]
    assert float(bx[:, 0].min()) >= -20 * s and float(bx[:, 0].max()) < 60 * s
    assert float(bx[:, 2].min()) >= 1.5 and float(bx[:, 3].max()) < 6.5
    assert float(bx[:, 4].abs().max()) <= math.pi


def test_synthetic_loader_rank_shards_and_residency():
    a = list(synthetic.SyntheticBEVLoader(1, 2, (16, 16), rank=0))
    b = list(synthetic.SyntheticBEVLoader(1, 2, (16, 16), rank=1))
    assert a[0] is a[1]  # resident: one batch reused
    assert not torch.equal(a[0]["lidar_bev"], b[0]["lidar_bev"])
    f = list(synthetic.SyntheticBEVLoader(1, 2, (16, 16), rank=0, resident=False))
    assert torch.equal(f[0]["lidar_bev"], a[0]["lidar_bev"]) and not torch.equal(f[0]["lidar_bev"], f[1]["lidar_bev"])


def test_train_eval_entry_points_parse():
    import eval_vit
    import train_vit
    a = train_vit.parse_args(["--synthetic", "--epochs", "1", "--grid", "32x48"])
    assert a.synthetic and a.epochs == 1
    cfg = train_vit.backbone_cfg((32, 48))
    assert cfg["img_size"] == (32, 48) and cfg["lidar_input_channels"] == 290
    e = eval_vit.parse_args(["--synthetic", "--batch", "32"])
    assert e.batch == 32
    full = eval_vit.default_cfg({}, (400, 720))
    assert full["vit_model_name_map"] == "vit_tiny_patch8_224"  # eval_vit.py:77 default


def test_post_pipeline_order_and_flush(monkeypatch):
    """utils.PostPipeline's host logic (no kernels: launch / collect stubbed): push k returns batch k-1's
    predictions in order, an empty batch passes through as an empty list, flush returns the last one
    and then None."""
    import utils
    launched = []

    def fake_launch(cls, box, it, anchors, conf, nms):
        launched.append(int(cls[0, 0]))
        return ("batch", int(cls[0, 0]))

    monkeypatch.setattr(utils, "_post_launch", fake_launch)
    monkeypatch.setattr(utils, "_post_collect", lambda p: [{"id": p[1]}])
    anchors = torch.zeros(4, 5)
    pipe = utils.PostPipeline(anchors)
    assert pipe.stream is None  # CPU anchors: no side stream
    out = []
    for k in range(3):
        out.append(pipe.push(torch.full((2, 4), float(k)), torch.zeros(2, 4, 6), torch.zeros(2, 4, 8)))
    out.append(pipe.push(torch.zeros(0, 4), torch.zeros(0, 4, 6), torch.zeros(0, 4, 8)))  # empty batch
    out.append(pipe.flush())
    assert out == [None, [{"id": 0}], [{"id": 1}], [{"id": 2}], []]
    assert pipe.flush() is None and launched == [0, 1, 2]
