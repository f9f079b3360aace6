"""One IntentNetViT training step — the loop body of train_vit.py:151-187 — shared by
train_vit.py and bench.py.

zero_grad → forward → (NaN skip) → DetectionIntentionLoss → (non-finite-loss no-op) → backward
(gradient buckets all-reduce while it runs when world > 1) → FusedAdamW.

* NaN in the model outputs skips the batch (train_vit.py:160-162): ``step`` returns None.
* A non-finite total loss comes back from the loss as a zero (loss.py:190-198 returns a
  disconnected zero leaf): the reference's ``loss.backward()`` then produces no gradient and
  ``optimizer.step()`` updates nothing (AdamW skips parameters whose ``.grad`` is None, step
  counters included). Here backward and the optimizer step are skipped outright, so the
  weights, the Adam moments and the step counters stay bit-identical; the zero loss dict is
  returned, and the caller accumulates it as the reference's loop does.

Both checks are taken collectively across ranks (ddp.any_rank) so every rank stays on the same
step; under DDP one rank's non-finite loss therefore skips the update on every rank (the
replicas stay identical). They cost one host sync each, as the reference's ``torch.isnan``
checks do; the benchmark turns them off (``check_nan=False``) — nothing else is skipped. Without
the host checks a non-finite loss still zeroes the update: backward runs (exact-zero gradients
from the loss kernel) and FusedAdamW's launch reads the loss's device finite flag (min over ranks
under DDP) and leaves weights and moments untouched; only its host step counters advance.
"""
from __future__ import annotations

import torch

from ddp import GradBuckets, any_rank, broadcast_state, grad_order, min_on_device
from loss import device_guard
from optim import FusedAdamW


class Trainer:
    def __init__(self, model, loss_fn, optimizer, anchors, world: int = 1, bucket_mb: float = 64.0,
                 check_nan: bool = True, force_buckets: bool = False):
        self.model, self.loss_fn, self.optimizer, self.anchors = model, loss_fn, optimizer, anchors
        self.world = world
        self.check_nan = check_nan
        if world > 1:
            # identical replicas from the first step, whatever each rank's RNG did
            broadcast_state(model)
        # force_buckets: the bucketed all-reduce path even at world 1 (tests on one GPU over RCCL)
        # buckets in the order the interleaved backward produces gradients, the last ones in a
        # 32-MB bucket of their own (the collective left after the backward)
        self.buckets = GradBuckets(grad_order(model), bucket_mb, force_collectives=force_buckets,
                                   last_bucket_mb=min(32.0, bucket_mb)) if world > 1 or force_buckets else None
        self.skipped = 0
        self.nonfinite = 0

    def zero_grad(self):
        if self.buckets is not None:
            self.buckets.zero_grad()
        else:
            self.optimizer.zero_grad(set_to_none=True)

    def _loss_finite(self, d):
        fin = getattr(self.loss_fn, "last_finite", None)
        if fin is None:
            return bool(torch.isfinite(d["loss"]).all())
        return bool(fin) and not bool(torch.isnan(d["loss"]))

    def step(self, batch: dict):
        """Returns the loss dict, or None when the batch was skipped (NaN in the outputs)."""
        lidar, mp, gts = batch["lidar_bev"], batch["map_bev"], batch["gt_list"]
        self.zero_grad()
        cls, box, intent = self.model(lidar, mp)
        dev = cls.device
        if self.check_nan:
            bad = torch.isnan(cls).any() | torch.isnan(box).any() | torch.isnan(intent).any()
            if any_rank(bool(bad), dev):
                self.skipped += 1
                return None
        with device_guard():  # the sync-free guard: last_finite decides below (loss.py docstring)
            d = self.loss_fn(cls, box, intent, self.anchors, gts)
        if self.check_nan and any_rank(not self._loss_finite(d), dev):
            self.nonfinite += 1
            return d
        d["loss"].backward()
        if self.buckets is not None:
            self.buckets.finish()
        fin = getattr(self.loss_fn, "last_finite", None)
        if not self.check_nan and fin is not None and isinstance(self.optimizer, FusedAdamW):
            # no host sync: the update launch itself reads the loss's finite flag and does nothing
            # on 0 (weights and moments unchanged, as with the reference's disconnected zero loss)
            if self.buckets is not None and self.world > 1:
                fin = min_on_device(fin)  # every rank skips together (replicas stay identical)
            self.optimizer.step(finite=fin)
        else:
            self.optimizer.step()
        return d
