"""DetectionIntentionLoss (loss.py:10-206 of the reference) on device.

Same constructor arguments, same forward signature and the same returned dict keys. The
whole assignment + focal/Smooth-L1/CE computation is four HIP kernels with no host
synchronisation (the reference syncs per GT and per `.item()`).

The non-finite guard (loss.py:190-206), two forms:
  * ``sync_guard=True`` (the default outside ``trainer.Trainer``, and under ``run_with_ivit.py``):
    exactly the reference's contract. The device finite flag and the positive-anchor count are
    read once (one host sync, where the reference syncs too: ``torch.isnan(...).any()`` and
    ``num_pos_total_batch.item()``); ``num_pos_anchors`` is a Python int and a non-finite total
    returns a disconnected ``requires_grad`` zero leaf, so a reference-style
    ``loss.backward(); torch.optim.AdamW.step()`` leaves ``.grad`` None and updates nothing.
  * ``sync_guard=False`` (what ``Trainer.step`` selects through ``device_guard()``): no host
    sync. ``num_pos_anchors`` is a 0-d device tensor, a non-finite total returns a zero loss still
    connected to the logits with exact-zero gradients, and ``last_finite`` (device 1.0 / 0.0)
    tells the Trainer / FusedAdamW to skip the update.

Intention down-sampling (loss.py:169-182), two random streams:
  * ``downsample_rng="device"`` (default): one uniform per anchor on the device
    (``keep_generator``), no host sync — the same Bernoulli(keep) law as the reference, a
    different stream;
  * ``downsample_rng="reference"``: the reference's own draws — per dominant class in the set's
    iteration order, ``torch.rand(k, device=device)`` over that class's positive anchors in
    flattened (sample, anchor) order — so the same torch seed drops the same anchors. It costs an
    assignment pass and a host sync per class (the reference's ``.item()``).
``forward(..., intent_keep=mask)`` injects the mask for parity tests.
"""
from __future__ import annotations

import contextlib
import threading

import torch
import torch.nn as nn

import ops
from constants import DOMINANT_CLASSES_FOR_DOWNSAMPLING, INTENTION_DOWNSAMPLE_RATIO


_TLS = threading.local()


@contextlib.contextmanager
def device_guard():
    """Inside this block a loss built with ``sync_guard=None`` (the default) takes the sync-free
    device guard; ``trainer.Trainer.step`` wraps its loss call in it (wrappers around the loss
    included). An explicit ``sync_guard=True / False`` on the module always wins."""
    prev = getattr(_TLS, "device", False)
    _TLS.device = True
    try:
        yield
    finally:
        _TLS.device = prev


def pack_gt(gt_list, device):
    """gt_list[b] = {'boxes_xywha': (G,5), 'intentions': (G,)} → padded device tensors.
    A missing/malformed entry or G == 0 means "all anchors negative" (loss.py:69-79)."""
    B = len(gt_list)
    ok = [isinstance(g, dict) and "boxes_xywha" in g and "intentions" in g for g in gt_list]
    counts = [int(g["boxes_xywha"].shape[0]) if o else 0 for g, o in zip(gt_list, ok)]
    G = max(1, max(counts) if counts else 1)
    # pinned staging so the three copies are truly asynchronous (no host/GPU drain per step)
    pin = torch.device(device).type == "cuda"
    gt = torch.zeros((B, G, 5), dtype=torch.float32, pin_memory=pin)
    gi = torch.zeros((B, G), dtype=torch.int32, pin_memory=pin)
    for b, (g, o, n) in enumerate(zip(gt_list, ok, counts)):
        if o and n:
            gt[b, :n] = g["boxes_xywha"].detach().float().cpu()
            gi[b, :n] = g["intentions"].detach().cpu().to(torch.int32)
    ng = torch.tensor(counts, dtype=torch.int32)
    if pin:
        ng = ng.pin_memory()
    return (gt.to(device, non_blocking=True), ng.to(device, non_blocking=True), gi.to(device, non_blocking=True))


class DetectionIntentionLoss(nn.Module):
    def __init__(self, iou_threshold=0.6, neg_iou_threshold=0.45, box_weight=1.0, cls_weight=1.0, intent_weight=0.5,
                 intention_class_weights=None, use_rotated_iou=False, focal_loss_alpha=0.25, focal_loss_gamma=2.0,
                 smooth_l1_beta=1.0 / 9.0, apply_intention_downsampling=True,
                 dominant_intentions=DOMINANT_CLASSES_FOR_DOWNSAMPLING,
                 intention_downsample_ratio=INTENTION_DOWNSAMPLE_RATIO, downsample_rng="device",
                 sync_guard=None):
        super().__init__()
        if sync_guard not in (None, True, False):
            raise ValueError(f"sync_guard must be None, True or False, got {sync_guard!r}")
        self.sync_guard = sync_guard
        if downsample_rng not in ("device", "reference"):
            raise ValueError(f"downsample_rng must be 'device' or 'reference', got {downsample_rng!r}")
        self.downsample_rng = downsample_rng
        self.iou_threshold, self.neg_iou_threshold = iou_threshold, neg_iou_threshold
        self.box_weight, self.cls_weight, self.intent_weight = box_weight, cls_weight, intent_weight
        self.use_rotated_iou = use_rotated_iou
        self.focal_loss_alpha, self.focal_loss_gamma, self.smooth_l1_beta = focal_loss_alpha, focal_loss_gamma, smooth_l1_beta
        self.apply_intention_downsampling = apply_intention_downsampling
        self.dominant_intentions = set(dominant_intentions)
        self.intention_downsample_keep_prob = 1.0 - intention_downsample_ratio
        w = None
        if not apply_intention_downsampling and intention_class_weights is not None:
            w = torch.as_tensor(intention_class_weights, dtype=torch.float32)
        self.register_buffer("final_intention_class_weights", w)
        self.keep_generator = None
        self.last_finite = None
        self.last_keep = None

    def _cfg(self, device):
        dom = 0
        for d in self.dominant_intentions:
            dom |= 1 << int(d)
        cw = self.final_intention_class_weights
        return {"dominant_mask": dom, "downsampling": self.apply_intention_downsampling,
                "class_w": None if cw is None else cw.to(device).float().contiguous(),
                "pos_thr": self.iou_threshold, "neg_thr": self.neg_iou_threshold, "alpha": self.focal_loss_alpha,
                "gamma": self.focal_loss_gamma, "beta": self.smooth_l1_beta, "w_cls": self.cls_weight,
                "w_box": self.box_weight, "w_int": self.intent_weight, "rotated": self.use_rotated_iou}

    def forward(self, cls_logits, box_preds, intention_logits, anchors, gt_list, intent_keep=None):
        B = cls_logits.shape[0]
        NA = anchors.shape[0]
        dev = cls_logits.device
        anchors = anchors.to(dev).float().contiguous()
        gt, ng, gi = pack_gt(gt_list, dev)
        keep = None
        if self.apply_intention_downsampling:
            if intent_keep is not None:
                keep = intent_keep.to(dev).float().reshape(B, NA).contiguous()
            elif self.downsample_rng == "reference":
                keep = self._reference_keep(cls_logits, box_preds, intention_logits, anchors, gt, ng, gi)
            else:
                u = torch.rand((B, NA), device=dev, generator=self.keep_generator)
                keep = (u < self.intention_downsample_keep_prob).float()
        self.last_keep = keep
        cls = cls_logits.float().reshape(B, NA)
        box = box_preds.float().reshape(B, NA, 6)
        it = intention_logits.float().reshape(B, NA, -1)
        loss, stats = ops.DetLossFn.apply(cls, box, it, anchors, gt, ng, gi, keep, self._cfg(dev))
        # 1.0 / 0.0 on device: 0 means the guard of loss.py:190-198 fired (loss and terms are 0,
        # and the backward writes exact zero gradients); trainer.Trainer skips the update on it
        self.last_finite = stats[9].detach()
        sync = self.sync_guard if self.sync_guard is not None else not getattr(_TLS, "device", False)
        if sync:
            return self._reference_guard(loss, stats, dev)
        return {"loss": loss, "cls_loss": stats[6].detach(), "box_loss": stats[7].detach(),
                "intent_loss": stats[8].detach(), "num_pos_anchors": stats[3].detach().round().long()}

    def _reference_guard(self, loss, stats, dev):
        """loss.py:190-206 with one host read of (finite flag, positive count, raw terms)."""
        h = stats.detach()[:16].cpu()
        num_pos = int(round(float(h[3])))
        if float(h[9]) == 0.0:
            # the reference prints the raw (non-finite) terms before zeroing them: rebuilt from
            # the device's raw sums and denominators (loss_final_kernel: slots 0-4, 10, 11)
            cden, iden = float(h[10]), float(h[11])
            cl = float(h[0]) / cden
            bl = float(h[1]) / cden if num_pos > 0 else 0.0
            il = float(h[2]) / iden if num_pos > 0 else 0.0
            print(f"NaN or Inf DETECTED IN LOSS! Cls: {cl}, Box: {bl}, Intent: {il}")
            z = torch.tensor(0.0, device=dev)
            return {"loss": torch.tensor(0.0, device=dev, requires_grad=True), "cls_loss": z,
                    "box_loss": z.clone(), "intent_loss": z.clone(), "num_pos_anchors": num_pos}
        return {"loss": loss, "cls_loss": stats[6].detach(), "box_loss": stats[7].detach(),
                "intent_loss": stats[8].detach(), "num_pos_anchors": num_pos}

    def _reference_keep(self, cls_logits, box_preds, intention_logits, anchors, gt, ng, gi):
        """The keep mask of the reference's draws (loss.py:170-178): the per-anchor targets from one
        assignment pass (ivit_det_loss_fwd with no mask; its workspace starts with them), then per
        dominant class, in ``self.dominant_intentions``' iteration order, ``torch.rand(k)`` on the
        logits' device for its k positives in flattened order, kept where < keep probability."""
        from _lib import lib, ptr, stream, workspace
        B, NA = cls_logits.shape[0], anchors.shape[0]
        dev = cls_logits.device
        cls = cls_logits.detach().float().reshape(B, NA).contiguous()
        box = box_preds.detach().float().reshape(B, NA, 6).contiguous()
        it = intention_logits.detach().float().reshape(B, NA, -1).contiguous()
        cfg = self._cfg(dev)
        ws = workspace(lib.ivit_det_loss_workspace(B, NA, gt.shape[1]), dev)
        stats = torch.empty((16,), dtype=torch.float32, device=dev)
        lib.ivit_det_loss_fwd(ptr(cls), ptr(box), ptr(it), ptr(anchors), B, NA, it.shape[-1], ptr(gt), ptr(ng), ptr(gi),
                              gt.shape[1], None, cfg["dominant_mask"], 0, None, cfg["pos_thr"], cfg["neg_thr"],
                              cfg["alpha"], cfg["gamma"], cfg["beta"], cfg["w_cls"], cfg["w_box"], cfg["w_int"],
                              int(cfg["rotated"]), ptr(stats), ptr(ws), ws.numel(), stream())
        tgt = ws[:B * NA * 4].view(torch.int32)
        pos_idx = torch.nonzero((tgt & 3) == 2).squeeze(1)  # cls target 1, in flattened order
        it_pos = (tgt[pos_idx] >> 2) - 1
        keep = torch.ones((B * NA,), dtype=torch.float32, device=dev)
        for d in self.dominant_intentions:
            m = it_pos == d
            k = int(m.sum().item())
            if k:
                r = torch.rand(k, device=dev)
                keep[pos_idx[m]] = (r < self.intention_downsample_keep_prob).float()
        return keep.reshape(B, NA)
