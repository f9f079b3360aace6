"""LiDAR BEV voxelisation + sweep ego transform (utils.py:27-33, 62-106,
dataset.py:290-347). Golden vectors: tests/golden/lidar_bev.npz, written by
oracle/make_golden.py from the reference's own transform_points / create_intentnet_lidar_bev.
The bar is bit-exact (every cell, NaN included): the binning is integer index work."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ivit_oracle as O


def _case_a(z):
    """Per-sweep (points, intensity, tf) of case A; a count of -1 is a missing sweep (None)."""
    pts, ints, tfs, off = [], [], [], 0
    for n, tf in zip(z["a_counts"], z["a_tf"]):
        if n < 0:
            pts.append(None)
            ints.append(None)
        else:
            pts.append(z["a_points"][off:off + n])
            ints.append(z["a_intensity"][off:off + n])
            off += n
        tfs.append(tf)
    return pts, ints, tfs


def _dense(z, pre):
    out = np.zeros(int(np.prod(z[pre + "_shape"])), np.float32)
    out[z[pre + "_idx"]] = z[pre + "_val"]
    return out.reshape(tuple(z[pre + "_shape"]))


# ------------------------------------------------------------------ CPU: the oracle is pinned
def test_oracle_transform_and_voxelise_match_reference_golden():
    z = golden("lidar_bev.npz")
    pts, ints, tfs = _case_a(z)
    ego = [O.transform_points_np(p, t) if p is not None else None for p, t in zip(pts, tfs)]
    got = np.concatenate([q for q in ego if q is not None])[::97]
    assert np.array_equal(got, z["a_ego_points_sample"])
    assert np.array_equal(O.lidar_bev_np(ego, ints), _dense(z, "a"))
    bev_b = O.lidar_bev_np([z["b_points0"], z["b_points1"]], [z["b_int0"], z["b_int1"]], num_sweeps=2)
    assert np.array_equal(bev_b, _dense(z, "b"), equal_nan=True)


def test_sweep_rel_transform_is_rigid():
    from scipy.spatial.transform import Rotation
    a = [1.0, 2.0, 0.5] + list(Rotation.from_euler("z", 0.4).as_quat())
    b = [3.0, -1.0, 0.7] + list(Rotation.from_euler("xyz", [0.01, 0.02, 0.5]).as_quat())
    t = O.sweep_rel_transform(a, b)
    assert np.allclose(t[:3, :3] @ t[:3, :3].T, np.eye(3), atol=1e-12)
    assert np.allclose(O.sweep_rel_transform(a, a), np.eye(4), atol=1e-12)


# ------------------------------------------------------------------ GPU: the HIP kernel
@pytest.mark.gpu
def test_lidar_bev_fused_transform_matches_golden():
    import utils
    z = golden("lidar_bev.npz")
    pts, ints, tfs = _case_a(z)
    bev = utils.create_intentnet_lidar_bev(pts, ints, transforms=tfs)
    assert bev.shape == (290, 400, 720) and bev.is_cuda
    assert np.array_equal(bev.cpu().numpy(), _dense(z, "a"))


@pytest.mark.gpu
def test_lidar_bev_pretransformed_f64_and_f32_points_match_golden():
    import utils
    z = golden("lidar_bev.npz")
    pts, ints, tfs = _case_a(z)
    ego = [utils.transform_points(p, t) if p is not None else None for p, t in zip(pts, tfs)]  # f64 rows
    assert np.array_equal(utils.create_intentnet_lidar_bev(ego, ints).cpu().numpy(), _dense(z, "a"))
    bev_b = utils.create_intentnet_lidar_bev([z["b_points0"], z["b_points1"]], [z["b_int0"], z["b_int1"]],
                                             num_expected_sweeps=2)
    assert np.array_equal(bev_b.cpu().numpy(), _dense(z, "b"), equal_nan=True)


@pytest.mark.gpu
def test_lidar_bev_batch_one_launch_and_row_stride():
    """Two samples into one [B, 290, H, W] raster (planes b*290 + i*29); points with an extra
    intensity column (ld = 4) and torch inputs; an all-missing sample stays zero."""
    import utils
    z = golden("lidar_bev.npz")
    pts, ints, tfs = _case_a(z)
    pts4 = [np.hstack([p, v[:, None]]) if p is not None else None for p, v in zip(pts, ints)]
    ints_t = [torch.from_numpy(v) if v is not None else None for v in ints]
    out = torch.full((3, 290, 400, 720), 7.0, device="cuda")
    utils.lidar_bev_batch([([None] * 10, [None] * 10), (pts4, ints_t, tfs), (pts, ints, tfs)], out=out)
    a = _dense(z, "a")
    assert float(out[0].abs().max()) == 0.0
    assert np.array_equal(out[1].cpu().numpy(), a) and np.array_equal(out[2].cpu().numpy(), a)


@pytest.mark.gpu
def test_lidar_bev_full_size_random_vs_oracle():
    """10 sweeps x 120k points (an Argoverse-2-sized frame), fused transform, against the oracle."""
    import utils
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(5)
    ego = np.array([10.0, 20.0, 0.0] + list(Rotation.from_euler("z", 1.0).as_quat()))
    pts, ints, tfs = [], [], []
    for _ in range(10):
        n = 120_000
        pts.append(np.stack([rng.uniform(-40, 100, n), rng.uniform(-90, 90, n), rng.uniform(-3, 5, n)],
                            1).astype(np.float32))
        ints.append(rng.uniform(0, 255, n).astype(np.float32))
        sw = ego.copy()
        sw[:3] += rng.normal(0, 3.0, 3)
        tfs.append(O.sweep_rel_transform(ego, sw))
    ref = O.lidar_bev_np([O.transform_points_np(p, t) for p, t in zip(pts, tfs)], ints)
    got = utils.create_intentnet_lidar_bev(pts, ints, transforms=tfs).cpu().numpy()
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_lidar_bev_rejects_more_sweeps_than_channels():
    import utils
    p = np.zeros((4, 3), np.float32)
    v = np.ones(4, np.float32)
    with pytest.raises(ValueError):
        utils.create_intentnet_lidar_bev([p] * 3, [v] * 3, num_expected_sweeps=2)
