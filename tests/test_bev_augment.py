"""BEV augmentations (utils.py:394-517): np.flip, per-channel cv2.warpAffine /
cv2.resize + centre crop / pad, dropout rectangles, GT updates.

Golden vectors: tests/golden/bev_augment.npz, written by oracle/make_golden.py from the reference's
OWN random_* / augment_bev (seeded python `random`) with cv2 backed by the oracle's OpenCV
restatement (cv2 is absent here: the resampling arithmetic is PARITY UNPINNED; the draw order,
crop / pad offsets, dropout and GT updates are pinned). GPU bar: bit-exact against the oracle on
the same inputs (rasters, NaN / inf / -0 included); GT boxes within 1e-6 (host numpy f32 trig)."""
import hashlib
import random

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ivit_oracle as O


def _cases(z):
    for k in z["cases"]:
        k = str(k)
        angle, scale = float(z[k + "_angle"]), float(z[k + "_scale"])
        p = {"flip": bool(z[k + "_flip"]), "angle": None if np.isnan(angle) else angle,
             "scale": None if np.isnan(scale) else scale,
             "rects": [tuple(int(v) for v in r) for r in z[k + "_rects"][: int(z[k + "_nrect"])]]}
        yield k, int(z[k + "_seed"]), int(z[k + "_input_seed"]), p


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


# ------------------------------------------------------------------ CPU: the oracle is pinned
def test_oracle_augment_matches_reference_golden():
    z = golden("bev_augment.npz")
    for k, seed, iseed, p in _cases(z):
        lidar, mp, boxes, intents = O.bev_augment_inputs(iseed)
        random.seed(seed)
        ol, om, ob, oi, op = O.augment_bev_np(lidar, mp, boxes, intents, random)
        assert op == p, k
        assert _sha(ol) == str(z[k + "_lidar_sha"]) and _sha(om) == str(z[k + "_map_sha"]), k
        assert np.array_equal(ol.reshape(-1)[::997], z[k + "_lidar_sample"]), k
        np.testing.assert_allclose(ob, z[k + "_boxes"], rtol=0, atol=1e-6)
        assert np.array_equal(oi, z[k + "_intents"]), k


def test_host_draws_follow_reference_order():
    """The product's host draw sequence equals the oracle's (hence the reference's) for every seed."""
    import utils
    for s in range(300):
        random.seed(s)
        a = O.draw_augment_params(random)
        random.seed(s)
        b = utils._draw_params()
        assert a == b, s


def test_host_gt_update_and_pass_table():
    import utils
    z = golden("bev_augment.npz")
    for k, seed, iseed, p in _cases(z):
        _, _, boxes, intents = O.bev_augment_inputs(iseed)
        b, i = boxes.copy(), intents.copy()
        utils._gt_update(b, i, p)
        np.testing.assert_allclose(b, z[k + "_boxes"], rtol=0, atol=1e-6)
        assert np.array_equal(i, z[k + "_intents"])
    d = utils._BEV_PASS  # ivit_bev_pass layout (include/ivit.h)
    assert d.itemsize == 192 and d.fields["m"][1] == 32 and d.fields["scale_x"][1] == 80
    assert d.fields["new_w"][1] == 96 and d.fields["rect"][1] == 112
    m = utils._rotation_inverse(-12.5, 400, 720)
    assert m == O.cv2_invert_affine(O.cv2_get_rotation_matrix_2d((360.0, 200.0), -12.5, 1.0))
    assert [op for op, _ in utils._stages({"flip": True, "angle": 3.0, "scale": 0.97, "rects": []}, 400, 720)] == [1, 2]
    assert [op for op, _ in utils._stages({"flip": False, "angle": None, "scale": 1.001, "rects": []}, 400, 720)] == [0]


def test_oracle_resamplers_identities():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, 40, 72)).astype(np.float32)
    M = O.cv2_get_rotation_matrix_2d((36.0, 20.0), 0.0, 1.0)
    assert np.array_equal(O.cv2_warp_affine_linear(x, M, (72, 40)), x)
    assert np.array_equal(O.cv2_resize_linear(x, (72, 40)), x)
    assert np.array_equal(O.cv2_warp_affine_linear(x, M, (72, 40), flip_src=True), x[..., ::-1])
    up = O.cv2_resize_linear(x, (144, 80))  # 2x up: centres land on quarter pixels
    assert np.allclose(up[:, 1:-1:2, 1:-1:2], 0.75 * 0.75 * x[:, :-1, :-1] + 0.75 * 0.25 * x[:, :-1, 1:]
                       + 0.25 * 0.75 * x[:, 1:, :-1] + 0.0625 * x[:, 1:, 1:], atol=1e-5)


# ------------------------------------------------------------------ GPU: the HIP passes
@pytest.mark.gpu
def test_augment_bev_golden_cases_bit_exact():
    import utils
    z = golden("bev_augment.npz")
    for k, seed, iseed, p in _cases(z):
        lidar, mp, boxes, intents = O.bev_augment_inputs(iseed)
        random.seed(seed)
        gl, gm, gg = utils.augment_bev(lidar, mp, {"boxes_xywha": torch.from_numpy(boxes),
                                                   "intentions": torch.from_numpy(intents)})
        assert gl.is_cuda and gm.is_cuda
        gl, gm = gl.cpu().numpy(), gm.cpu().numpy()
        assert np.array_equal(gl.reshape(-1)[::997], z[k + "_lidar_sample"]), k
        assert _sha(gl) == str(z[k + "_lidar_sha"]) and _sha(gm) == str(z[k + "_map_sha"]), k
        np.testing.assert_allclose(gg["boxes_xywha"].numpy(), z[k + "_boxes"], rtol=0, atol=1e-6)
        assert np.array_equal(gg["intentions"].numpy(), z[k + "_intents"])


@pytest.mark.gpu
def test_augment_batch_full_channels_vs_oracle():
    """A full-size batch (290 LiDAR + 9 map planes; the 290 % 8 plane tail) of 3 samples in one
    launch per pass depth, seeded so the draws include a two-pass (rotate + scale) sample."""
    import utils
    lid, mps, gts, ins = [], [], [], []
    for b in range(3):
        l, m, bx, it = O.bev_augment_inputs(200 + b, lidar_ch=290, map_ch=9)
        lid.append(l), mps.append(m), gts.append({"boxes_xywha": bx, "intentions": it}), ins.append((bx, it))
    L, M = torch.from_numpy(np.stack(lid)).cuda(), torch.from_numpy(np.stack(mps)).cuda()
    random.seed(45)  # sample 0 draws flip + rotate + scale + dropout ("all" golden case)
    lo, mo, go, params = utils.augment_bev_batch(L, M, gts)
    assert params[0]["angle"] is not None and params[0]["scale"] is not None
    random.seed(45)
    for b in range(3):
        ol, om, ob, oi, p = O.augment_bev_np(lid[b], mps[b], *ins[b], rng=random)
        assert p == params[b]
        assert np.array_equal(lo[b].cpu().numpy(), ol), b
        assert np.array_equal(mo[b].cpu().numpy(), om), b
        np.testing.assert_allclose(go[b]["boxes_xywha"].numpy(), ob, rtol=0, atol=1e-6)
        assert np.array_equal(go[b]["intentions"].numpy(), oi)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [
    {"flip": True, "angle": 45.0, "scale": 1.05, "rects": [(0, 0, 50, 50), (350, 670, 50, 50)]},
    {"flip": False, "angle": -15.0, "scale": None, "rects": []},
    {"flip": True, "angle": None, "scale": 0.95, "rects": [(10, 700, 20, 20)]},
    {"flip": False, "angle": None, "scale": 1.0499, "rects": []},
    {"flip": True, "angle": None, "scale": None, "rects": [(380, 0, 20, 720)]},
])
def test_bev_passes_special_values_vs_oracle(p):
    """Hand-set params (beyond the drawn ranges too) on planes holding NaN, +-inf and -0."""
    import utils
    rng = np.random.default_rng(7)
    x = rng.standard_normal((11, 400, 720)).astype(np.float32)
    flat = x.reshape(-1)
    for v in (np.nan, np.inf, -np.inf, -0.0):
        flat[rng.integers(0, flat.size, 200)] = v
    ref = O.augment_planes_np(x, p)
    src = torch.from_numpy(x).cuda()
    dst = torch.empty_like(src)
    utils._run_bev_passes([(src, dst, p)])
    got = dst.cpu().numpy()
    assert np.array_equal(got, ref, equal_nan=True)
    assert np.array_equal(np.signbit(got[~np.isnan(got)]), np.signbit(ref[~np.isnan(ref)]))


@pytest.mark.gpu
def test_individual_random_functions_match_oracle():
    import utils
    lidar, mp, boxes, intents = O.bev_augment_inputs(300)
    for seed in range(6):
        random.seed(seed)
        gl, gm, gb, gi = utils.random_flip_bev(lidar, mp, boxes.copy(), intents.copy())
        random.seed(seed)
        flip = random.random() < 0.5
        p = {"flip": flip, "angle": None, "scale": None, "rects": []}
        assert np.array_equal(torch.as_tensor(gl).cpu().numpy(), O.augment_planes_np(lidar, p))
        rb, ri = O.augment_gt_np(boxes, intents, p)
        np.testing.assert_allclose(gb, rb, atol=1e-6, rtol=0)
        assert np.array_equal(gi, ri)
        random.seed(seed)
        rl, rm, rb2 = utils.random_rotate_bev(lidar, mp, boxes.copy())
        random.seed(seed)
        ang = random.uniform(-15.0, 15.0) if random.random() < 0.5 else None
        p = {"flip": False, "angle": ang, "scale": None, "rects": []}
        assert np.array_equal(torch.as_tensor(rm).cpu().numpy(), O.augment_planes_np(mp, p))
        random.seed(seed)
        sl, sm, sb = utils.random_scale_bev(lidar, mp, boxes.copy())
        random.seed(seed)
        sc = random.uniform(0.95, 1.05) if random.random() < 0.5 else None
        p = {"flip": False, "angle": None, "scale": sc, "rects": []}
        assert np.array_equal(torch.as_tensor(sl).cpu().numpy(), O.augment_planes_np(lidar, p))
    random.seed(6)  # 6: the dropout draw fires (golden "dropout" case's seed)
    dl, dm = utils.random_bev_dropout(lidar, mp, dropout_prob=1.0)
    random.seed(6)
    random.random()
    rects = []
    for _ in range(random.randint(1, 5)):
        ph, pw = random.randint(20, 50), random.randint(20, 50)
        rects.append((random.randint(0, 400 - ph), random.randint(0, 720 - pw), ph, pw))
    p = {"flip": False, "angle": None, "scale": None, "rects": rects}
    assert np.array_equal(dm.cpu().numpy(), O.augment_planes_np(mp, p))


@pytest.mark.gpu
def test_bev_passes_reject_in_place_and_bad_shapes():
    import utils
    x = torch.zeros(3, 400, 720, device="cuda")
    p = {"flip": True, "angle": None, "scale": None, "rects": []}
    with pytest.raises(ValueError):
        utils._run_bev_passes([(x, x, p)])
    with pytest.raises(ValueError):
        utils._run_bev_passes([(x, torch.zeros(3, 400, 721, device="cuda"), p)])
