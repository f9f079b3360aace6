"""Synthetic BEV batches in the reference's collate_fn format (dataset.py:137-150):
``{"lidar_bev": (B,290,H,W) f32, "map_bev": (B,9,H,W) f32, "gt_list": [{"boxes_xywha": (G,5),
"intentions": (G,) int64}, ...]}``.

Distribution: LiDAR occupancy U[0,1), map rasters Bernoulli(0.1) in {0,1},
G=20 boxes per sample with cx~U[-20,60)·s, cy~U[-72,72)·s (s = H/400, so the 2x grid of
config 5 doubles the ranges), w~U[1.5,3.0), l~U[3.5,6.5), yaw~U[-pi,pi), intentions~U{0..7}.
Seeded by ``torch.Generator('cpu').manual_seed(1234 + rank)`` so every DDP rank draws its
own shard. The Argoverse-2 loader (dataset.py) is outside this build's scope.
"""
from __future__ import annotations

import math

import torch

from constants import GRID_HEIGHT_PX, GRID_WIDTH_PX, LIDAR_TOTAL_CHANNELS, MAP_CHANNELS, NUM_INTENTION_CLASSES


def synthetic_gt(gen: torch.Generator, n_boxes: int = 20, grid=(GRID_HEIGHT_PX, GRID_WIDTH_PX)) -> dict:
    s = grid[0] / float(GRID_HEIGHT_PX)
    u = torch.rand((n_boxes, 5), generator=gen)
    boxes = torch.stack([-20.0 * s + 80.0 * s * u[:, 0], -72.0 * s + 144.0 * s * u[:, 1], 1.5 + 1.5 * u[:, 2],
                         3.5 + 3.0 * u[:, 3], -math.pi + 2.0 * math.pi * u[:, 4]], 1)
    return {"boxes_xywha": boxes, "intentions": torch.randint(0, NUM_INTENTION_CLASSES, (n_boxes,), generator=gen)}


def synthetic_batch(batch: int, grid=(GRID_HEIGHT_PX, GRID_WIDTH_PX), gen: torch.Generator | None = None,
                    n_boxes: int = 20, device=None) -> dict:
    gen = gen if gen is not None else torch.Generator().manual_seed(1234)
    H, W = grid
    lidar = torch.rand((batch, LIDAR_TOTAL_CHANNELS, H, W), generator=gen)
    mp = (torch.rand((batch, MAP_CHANNELS, H, W), generator=gen) < 0.1).float()
    gts = [synthetic_gt(gen, n_boxes, grid) for _ in range(batch)]
    if device is not None:
        lidar = lidar.to(device, non_blocking=True)
        mp = mp.to(device, non_blocking=True)
    return {"lidar_bev": lidar, "map_bev": mp, "gt_list": gts}


class SyntheticBEVLoader:
    """Iterable of ``num_batches`` synthetic batches (a stand-in for the reference DataLoader).
    ``resident=True`` draws one batch and yields it every time (inputs stay in HBM: the
    benchmark's primary placement); otherwise each batch is drawn fresh on the host.
    ``augment=True`` applies the training-time augment_bev of dataset.py:352-353 to every
    yielded batch on the GPU (utils.augment_bev_batch; python `random` draws, reference order)."""

    def __init__(self, batch: int, num_batches: int, grid=(GRID_HEIGHT_PX, GRID_WIDTH_PX), rank: int = 0,
                 device=None, resident: bool = True, n_boxes: int = 20, augment: bool = False):
        self.batch, self.num_batches, self.grid = batch, num_batches, tuple(grid)
        self.device, self.resident, self.n_boxes = device, resident, n_boxes
        self.augment, self._aug_out = augment, None
        self.gen = torch.Generator().manual_seed(1234 + rank)
        self._fixed = None

    def __len__(self):
        return self.num_batches

    def _augmented(self, b):
        import utils
        if self._aug_out is None:
            self._aug_out = (torch.empty_like(b["lidar_bev"]), torch.empty_like(b["map_bev"]))
        lo, mo, gts, _ = utils.augment_bev_batch(b["lidar_bev"], b["map_bev"], b["gt_list"], out=self._aug_out)
        return {"lidar_bev": lo, "map_bev": mo, "gt_list": gts}

    def __iter__(self):
        for _ in range(self.num_batches):
            if self.resident:
                if self._fixed is None:
                    self._fixed = synthetic_batch(self.batch, self.grid, self.gen, self.n_boxes, self.device)
                b = self._fixed
            else:
                b = synthetic_batch(self.batch, self.grid, self.gen, self.n_boxes, self.device)
            yield self._augmented(b) if self.augment else b
