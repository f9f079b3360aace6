"""One IntentNetViT training step — the loop body of train_vit.py:151-187 — shared by
train_vit.py and bench.py.

zero_grad → forward → (NaN skip) → DetectionIntentionLoss → (NaN skip) → backward (gradient
buckets all-reduce while it runs when world > 1) → FusedAdamW. The NaN skips are taken
collectively across ranks (ddp.any_rank) so every rank stays on the same step; they cost one
host sync each, as the reference's ``torch.isnan(...)`` checks do, and the benchmark turns
them off (``check_nan=False``) — nothing else in the step is skipped.
"""
from __future__ import annotations

import torch

from ddp import GradBuckets, any_rank


class Trainer:
    def __init__(self, model, loss_fn, optimizer, anchors, world: int = 1, bucket_mb: float = 64.0,
                 check_nan: bool = True):
        self.model, self.loss_fn, self.optimizer, self.anchors = model, loss_fn, optimizer, anchors
        self.world = world
        self.check_nan = check_nan
        self.buckets = GradBuckets(model.parameters(), bucket_mb) if world > 1 else None
        self.skipped = 0

    def zero_grad(self):
        if self.buckets is not None:
            self.buckets.zero_grad()
        else:
            self.optimizer.zero_grad(set_to_none=True)

    def step(self, batch: dict):
        """Returns the loss dict, or None when the batch was skipped (NaN outputs or loss)."""
        lidar, mp, gts = batch["lidar_bev"], batch["map_bev"], batch["gt_list"]
        self.zero_grad()
        cls, box, intent = self.model(lidar, mp)
        dev = cls.device
        if self.check_nan:
            bad = torch.isnan(cls).any() | torch.isnan(box).any() | torch.isnan(intent).any()
            if any_rank(bool(bad), dev):
                self.skipped += 1
                return None
        d = self.loss_fn(cls, box, intent, self.anchors, gts)
        if self.check_nan and any_rank(bool(torch.isnan(d["loss"])), dev):
            self.skipped += 1
            return None
        d["loss"].backward()
        if self.buckets is not None:
            self.buckets.finish()
        self.optimizer.step()
        return d
