"""Pin the CPU oracle against golden vectors produced by the reference's own code
(``oracle/make_golden.py``). CPU only."""
import json

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ivit_oracle as O
from oracle.weights import make_state_dict, state_checksum


def _gts(z, n):
    return [{"boxes_xywha": torch.from_numpy(z[f"gt{i}_boxes"]), "intentions": torch.from_numpy(z[f"gt{i}_ints"])}
            for i in range(n)]


@pytest.fixture(scope="module")
def small():
    z = golden("model_small.npz")
    cfg = json.loads(str(z["cfg"]))
    cfg["img_size"] = tuple(cfg["img_size"])
    sd = make_state_dict(cfg, seed=0)
    lidar, mp, _ = O.synthetic_batch(2, cfg["img_size"], seed=1234)
    return z, cfg, sd, lidar, mp


def test_inputs_regenerate(small):
    z, cfg, sd, lidar, mp = small
    assert abs(state_checksum(sd) - float(z["w_checksum"])) < 1e-6 * abs(float(z["w_checksum"]))
    assert float(lidar.double().sum()) == pytest.approx(float(z["lidar_sum"]), rel=1e-12)
    assert float(mp.double().sum()) == pytest.approx(float(z["map_sum"]), rel=1e-12)


def test_anchors_bitexact():
    z = golden("geometry.npz")
    assert np.array_equal(O.generate_anchors(400, 720, 8).numpy(), z["anchors"])
    zs = golden("model_small.npz")
    assert np.array_equal(O.generate_anchors(32, 48, 8).numpy(), zs["anchors"])


def test_forward_eval(small):
    z, cfg, sd, lidar, mp = small
    sd = {k: v.clone() for k, v in sd.items()}
    with torch.no_grad():
        c, b, i = O.intentnet_forward(sd, lidar, mp, cfg, training=False)
    for got, key in ((c, "eval_cls"), (b, "eval_box"), (i, "eval_int")):
        ref = z[key]
        assert got.shape == ref.shape
        np.testing.assert_allclose(got.numpy(), ref, rtol=1e-4, atol=1e-4)


def test_train_forward_loss_grads(small):
    z, cfg, sd, lidar, mp = small
    sd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v.clone())
          for k, v in sd.items()}
    c, b, i = O.intentnet_forward(sd, lidar, mp, cfg, training=True)
    np.testing.assert_allclose(c.detach().numpy(), z["train_cls"], rtol=1e-4, atol=1e-4)
    anchors = torch.from_numpy(z["anchors"])
    gts = _gts(z, 2)
    d = O.detection_loss(c, b, i, anchors, gts, downsampling=False)
    got = np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
                    d["num_pos_anchors"]])
    np.testing.assert_allclose(got, z["train_loss"], rtol=1e-5)
    d["loss"].backward()
    for name, gs, gas, smp, st in zip(z["grad_names"], z["grad_sum"], z["grad_abssum"], z["grad_samples"],
                                      z["grad_strides"]):
        g = sd[str(name)].grad
        assert g is not None, name
        assert float(g.double().abs().sum()) == pytest.approx(gas, rel=1e-3, abs=1e-6), name
        s = g.reshape(-1).double()[:: int(st)][:64].numpy()
        m = ~np.isnan(smp)
        np.testing.assert_allclose(s, smp[m][: s.size], rtol=2e-3, atol=2e-5 * max(1.0, np.abs(smp[m]).max()),
                                   err_msg=str(name))
    for name, val in zip(z["bn_names"], z["bn_values"]):
        np.testing.assert_allclose(sd[str(name)].numpy(), val, rtol=1e-4, atol=1e-5)
    with torch.no_grad():
        torch.manual_seed(77)
        d2 = O.detection_loss(c, b, i, anchors, gts, downsampling=True)
    got = np.array([float(d2["loss"]), float(d2["cls_loss"]), float(d2["box_loss"]), float(d2["intent_loss"]),
                    d2["num_pos_anchors"]])
    np.testing.assert_allclose(got, z["train_loss_ds"], rtol=1e-5)


def _logits(z, NA):
    g = torch.Generator().manual_seed(int(z["logits_seed"][0]))
    cls = torch.randn((2, NA, 1), generator=g)
    box = 0.5 * torch.randn((2, NA, 6), generator=g)
    it = torch.randn((2, NA, 8), generator=g)
    sums = [float(t.double().sum()) for t in (cls, box, it)]
    np.testing.assert_allclose(sums, z["logits_sums"], rtol=1e-12)
    return cls, box, it


def test_full_size_assignment_and_loss():
    z = golden("geometry.npz")
    anchors = torch.from_numpy(z["anchors"])
    gts = _gts(z, 2)
    iou = O.axis_aligned_iou(anchors, gts[0]["boxes_xywha"])
    mx, arg = iou.max(dim=1)
    assert np.array_equal(mx.numpy(), z["iou_max"]) and np.array_equal(arg.numpy(), z["iou_arg"])
    assert np.array_equal(iou.max(dim=0)[1].numpy(), z["iou_arg0"])
    cls, box, it = _logits(z, anchors.shape[0])
    d = O.detection_loss(cls, box, it, anchors, gts, downsampling=False)
    got = [float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]), d["num_pos_anchors"]]
    np.testing.assert_allclose(got, z["loss_full"], rtol=1e-5)
    torch.manual_seed(5)
    d = O.detection_loss(cls, box, it, anchors, gts, downsampling=True)
    got = [float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]), d["num_pos_anchors"]]
    np.testing.assert_allclose(got, z["loss_full_ds"], rtol=1e-5)
    empty = [{"boxes_xywha": torch.zeros((0, 5)), "intentions": torch.zeros((0,), dtype=torch.long)}, {}]
    d = O.detection_loss(cls, box, it, anchors, empty, downsampling=False)
    got = [float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]), d["num_pos_anchors"]]
    np.testing.assert_allclose(got, z["loss_empty"], rtol=1e-5)


def test_decode():
    z = golden("geometry.npz")
    anchors = torch.from_numpy(z["anchors"])
    out = O.decode_boxes(torch.from_numpy(z["dec_rel"]), anchors[torch.from_numpy(z["dec_idx"])])
    np.testing.assert_array_equal(out.numpy(), z["dec_out"])


def test_nms_keep_bitexact():
    z = golden("geometry.npz")
    for i in range(int(z["nms_cases"][0])):
        keep = O.nms_numpy(z[f"nms{i}_boxes"], z[f"nms{i}_scores"], 0.2)
        assert np.array_equal(keep, z[f"nms{i}_keep"]), i


def test_rotated_iou():
    z = golden("geometry.npz")
    got = O.rotated_iou_numpy(z["rot_b1"], z["rot_b2"])
    np.testing.assert_allclose(got, z["rot_iou"], atol=1e-6)
    assert np.all(got[3] == 0)


def _opt_logits(seed, NA):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn((2, NA, 1), generator=g), 0.5 * torch.randn((2, NA, 6), generator=g),
            torch.randn((2, NA, 8), generator=g))


def _opt_gts(z, pre, n=2):
    return [{"boxes_xywha": torch.from_numpy(z[f"{pre}_gt{i}_boxes"]),
             "intentions": torch.from_numpy(z[f"{pre}_gt{i}_ints"])} for i in range(n)]


def _rot_iou(a, b):
    return torch.from_numpy(O.rotated_iou_numpy(a.detach().float().numpy(), b.detach().float().numpy()))


def _vec(d):
    return np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
                     float(d["num_pos_anchors"])])


def test_loss_class_weights_vs_golden():
    """loss.py:40-45: intention_class_weights with downsampling off (full 400x720 anchors)."""
    z = golden("loss_options.npz")
    anchors = O.generate_anchors(400, 720, 8)
    ts = [t.requires_grad_(True) for t in _opt_logits(int(z["cw_seed"][0]), anchors.shape[0])]
    d = O.detection_loss(*ts, anchors, _opt_gts(z, "cw"), downsampling=False,
                         class_weights=torch.from_numpy(z["cw_weights"]))
    np.testing.assert_allclose(_vec(d), z["cw_loss"], rtol=1e-5)
    d["loss"].backward()
    for t, k in zip(ts, ("cw_gcls", "cw_gbox", "cw_gint")):
        np.testing.assert_allclose(t.grad.numpy(), z[k], rtol=1e-4, atol=1e-6 * np.abs(z[k]).max())


def test_loss_rotated_iou_vs_golden():
    """loss.py:81 use_rotated_iou=True (80x120 grid, GEOS restated as f64 convex clipping)."""
    z = golden("loss_options.npz")
    anchors = torch.from_numpy(z["rot_anchors"])
    assert np.array_equal(O.generate_anchors(80, 120, 8).numpy(), z["rot_anchors"])
    ts = [torch.from_numpy(z[k]).clone().requires_grad_(True) for k in ("rot_cls", "rot_box", "rot_int")]
    d = O.detection_loss(*ts, anchors, _opt_gts(z, "rot"), downsampling=False, iou_fn=_rot_iou)
    np.testing.assert_allclose(_vec(d), z["rot_loss"], rtol=1e-5)
    assert not np.allclose(z["rot_loss"], z["rot_axis_loss"])
    d["loss"].backward()
    for t, k in zip(ts, ("rot_gcls", "rot_gbox", "rot_gint")):
        np.testing.assert_allclose(t.grad.numpy(), z[k], rtol=1e-4, atol=1e-6 * np.abs(z[k]).max())


@pytest.mark.parametrize("case", ["nan_cls", "inf_cls_neg", "inf_int_pos"])
def test_loss_guard_vs_golden(case):
    """loss.py:190-198: a non-finite total returns zeros and a disconnected leaf (no gradient)."""
    z = golden("loss_options.npz")
    anchors = torch.from_numpy(z["rot_anchors"])
    b, a, k, v = z[f"guard_{case}"]
    ts = [torch.from_numpy(z[n]).clone() for n in ("rot_cls", "rot_box", "rot_int")]
    ts[0 if case.endswith(("cls", "cls_neg")) else 2][int(b), int(a), int(k)] = v
    ts = [t.requires_grad_(True) for t in ts]
    d = O.detection_loss(*ts, anchors, _opt_gts(z, "rot"), downsampling=False)
    np.testing.assert_array_equal(_vec(d), z[f"guard_{case}_loss"])
    d["loss"].backward()
    assert all(t.grad is None for t in ts) and bool(z[f"guard_{case}_leaf"][1])


def test_forward_sdpa_variant_matches_golden(small):
    """The oracle's timm-fused-path variant (F.scaled_dot_product_attention, used by the CPU
    baseline and the large-grid checks) against the same reference goldens."""
    z, cfg, sd, lidar, mp = small
    sd = {k: v.clone() for k, v in sd.items()}
    with torch.no_grad():
        c, b, i = O.intentnet_forward(sd, lidar, mp, cfg, training=False, attn="sdpa")
    for got, key in ((c, "eval_cls"), (b, "eval_box"), (i, "eval_int")):
        np.testing.assert_allclose(got.numpy(), z[key], rtol=1e-4, atol=1e-4)


def _map_case(z, name):
    import json as _json
    s = str(z[f"{name}_json"])
    pose = dict(zip(("tx_m", "ty_m", "qx", "qy", "qz", "qw"), z[f"{name}_pose"].tolist()))
    return (_json.loads(s) if s else None), pose


def test_map_raster_oracle_vs_golden():
    """rasterize_map_ego_centric (utils.py:108-182): the oracle reproduces the reference's own flow
    (golden from the reference with cv2 backed by the oracle's OpenCV restatement)."""
    z = golden("map_raster.npz")
    for name in z["cases"]:
        name = str(name)
        m, pose = _map_case(z, name)
        if m is None or name == "badquat":
            assert z[f"{name}_idx"].size == 0
            continue
        got = O.rasterize_map_np(m, pose)
        assert np.array_equal(np.flatnonzero(got.reshape(-1)), z[f"{name}_idx"]), name
        assert np.array_equal(got.reshape(9, -1).sum(1), z[f"{name}_per_channel"]), name


def test_cv_raster_primitives():
    """The OpenCV LINE_8 / fillPoly restatement on hand-checked cases (parity unpinned: cv2 absent)."""
    assert O.cv_line8_pixels((0, 0), (4, 2)) == [(0, 0), (1, 0), (2, 1), (3, 1), (4, 2)]
    assert O.cv_line8_pixels((4, 2), (0, 0)) == O.cv_line8_pixels((0, 0), (4, 2))  # leftToRight
    assert O.cv_line8_pixels((3, 0), (3, 3)) == [(3, 0), (3, 1), (3, 2), (3, 3)]
    img = np.zeros((6, 6), np.uint8)
    O.cv_fill_poly(img, [(1, 1), (4, 1), (4, 4), (1, 4)])  # axis-aligned square: rows 1..4, cols 1..4
    assert img[1:5, 1:5].all() and img.sum() == 16
    img = np.zeros((6, 6), np.uint8)
    O.cv_fill_poly(img, [(0, 2), (5, 2), (3, 2)])  # all on one row: only the edge lines
    assert img.sum() == 6 and img[2].all()


# Triangle A(0,0) B(7,3) C(2,5), edges C->A, A->B, B->C, derived by hand from OpenCV's
# drawing.cpp semantics (LINE_8, shift 0) — not from the restatement:
#  CollectPolyEdges: x = x_top << 16, dx = (X_b - X_a) / (y_b - y_a) in C integer division
#    (truncates toward 0): C->A dx = 131072 / 5 = 26214 (not 26214.4), A->B dx = 458752 / 3 =
#    152917, B->C dx = -327680 / 2 = -163840; an edge is active on y0 <= y < y1.
#  FillEdgeCollection (delta = 0 for LINE_8): span [x_l >> 16, x_r >> 16] (floor, no rounding):
#    y0: [0, 0]; y1: [0, 26214 >> 16 = 0 .. 152917 >> 16 = 2]; y2: [0, 305834 >> 16 = 4]
#    (4.67 -> 4); y3: A->B retired, [78642 >> 16 = 1, 458752 >> 16 = 7];
#    y4: [104856 >> 16 = 1, 294912 >> 16 = 4] (4.5 -> 4); y5 = y_max: no span.
#  Line (LineIterator, 8-connected, left to right, err = major - 2 minor) for each edge:
#    C->A (0,0)(0,1)(1,2)(1,3)(2,4)(2,5); A->B (0,0)(1,0)(2,1)(3,1)(4,2)(5,2)(6,3)(7,3);
#    B->C (2,5)(3,5)(4,4)(5,4)(6,3)(7,3).
ODD_SLOPE_TRIANGLE = [(0, 0), (7, 3), (2, 5)]
ODD_SLOPE_ROWS = {0: (0, 1), 1: (0, 3), 2: (0, 5), 3: (1, 7), 4: (1, 5), 5: (2, 3)}  # row: (x_first, x_last)


def odd_slope_expected(H=10, W=10, ox=0, oy=0):
    img = np.zeros((H, W), np.uint8)
    for y, (a, b) in ODD_SLOPE_ROWS.items():
        img[oy + y, ox + a:ox + b + 1] = 1
    return img


def test_cv_fill_poly_odd_slopes_hand_derived():
    """fillPoly's fixed-point conventions asserted explicitly on odd slopes (truncated dx, floor
    spans, half-open edge rows): the restatement reproduces the hand-derived pixel set. The map
    rasteriser's outputs remain parity unpinned at the OpenCV level (cv2 absent here); this pins
    the convention, tests/test_gpu_map.py checks the kernel on the same triangle."""
    img = np.zeros((10, 10), np.uint8)
    O.cv_fill_poly(img, ODD_SLOPE_TRIANGLE)
    assert np.array_equal(img, odd_slope_expected()), np.argwhere(img != odd_slope_expected())
    for rot in (1, 2):  # vertex order does not matter
        img = np.zeros((10, 10), np.uint8)
        O.cv_fill_poly(img, ODD_SLOPE_TRIANGLE[rot:] + ODD_SLOPE_TRIANGLE[:rot])
        assert np.array_equal(img, odd_slope_expected())


def test_fusion_stride2_oracle_vs_golden():
    """fusion_block_stride=2 (model_vit.py:55,125-128): the oracle's strided fusion block vs the
    reference's own model."""
    z = golden("model_stride2.npz")
    cfg = json.loads(str(z["cfg"]))
    cfg["img_size"] = tuple(cfg["img_size"])
    sd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v.clone())
          for k, v in make_state_dict(cfg, seed=0).items()}
    lidar, mp, _ = O.synthetic_batch(2, cfg["img_size"], seed=1234)
    c, b, i = O.intentnet_forward(sd, lidar, mp, cfg, training=True)
    np.testing.assert_allclose(c.detach().numpy(), z["train_cls"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(i.detach().numpy(), z["train_int"], rtol=1e-4, atol=1e-4)
    d = O.detection_loss(c, b, i, torch.from_numpy(z["anchors"]), _gts(golden("model_small.npz"), 2),
                         downsampling=False)
    np.testing.assert_allclose(_vec(d), z["train_loss"], rtol=1e-5)


def test_regrid_oracle_vs_golden():
    """Patch-16 map ViT (vit_small_patch16_224, model_vit.py:71): the map grid differs from the
    LiDAR grid and the oracle re-grids bilinearly (:139) — vs the reference's own model; and the
    standalone F.interpolate cases the resize kernel is tested against."""
    z = golden("model_regrid.npz")
    cfg = json.loads(str(z["cfg"]))
    cfg["img_size"] = tuple(cfg["img_size"])
    assert cfg["vit_map"] == "vit_small_patch16_224"
    sd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v.clone())
          for k, v in make_state_dict(cfg, seed=0).items()}
    lidar, mp, _ = O.synthetic_batch(2, cfg["img_size"], seed=1234)
    c, b, i = O.intentnet_forward(sd, lidar, mp, cfg, training=True)
    np.testing.assert_allclose(c.detach().numpy(), z["train_cls"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(i.detach().numpy(), z["train_int"], rtol=1e-4, atol=1e-4)
    d = O.detection_loss(c, b, i, torch.from_numpy(z["anchors"]), _gts(golden("model_small.npz"), 2),
                         downsampling=False)
    np.testing.assert_allclose(_vec(d), z["train_loss"], rtol=1e-5)
    for tag in ("up", "odd", "down"):
        x = torch.from_numpy(z[f"resize_{tag}_x"])
        y = torch.nn.functional.interpolate(x, size=z[f"resize_{tag}_y"].shape[2:], mode="bilinear",
                                            align_corners=False)
        np.testing.assert_array_equal(y.numpy(), z[f"resize_{tag}_y"])
