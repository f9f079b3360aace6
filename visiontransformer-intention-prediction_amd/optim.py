"""Fused AdamW (torch.optim.AdamW semantics as used at train_vit.py:130: lr 1e-4, wd 1e-4,
betas (0.9, 0.999), eps 1e-8, decoupled weight decay) — one HIP launch per parameter group
over device pointer tables instead of torch's per-tensor foreach kernels."""
from __future__ import annotations

import math

import torch

import ops
from _lib import lib, ptr, stream


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._tables = {}

    def _table(self, tensors, device):
        key = tuple(t.data_ptr() for t in tensors)
        tab = self._tables.get(key)
        if tab is None:
            # pinned staging + non_blocking: a pageable H2D copy would stall the host until the
            # GPU drains (a bubble every step when gradient buffers move)
            tab = torch.tensor(key, dtype=torch.int64).pin_memory().to(device, non_blocking=True)
            if len(self._tables) > 64:
                self._tables.clear()
            self._tables[key] = tab
        return tab

    @torch.no_grad()
    def step(self, closure=None, finite=None):
        """One AdamW update. ``finite``: optional device scalar (f32); when it holds 0 the launch
        updates nothing — the guard of loss.py:190-198 without a host sync (trainer.Trainer passes
        the loss's flag when it does not sync). On that path the step counts live on the device
        (``state['step']`` is a 0-d f32 device tensor, as torch's capturable AdamW keeps it) and a
        skipped update does not advance them, so the bias correction of every later step is the one
        torch.optim.AdamW applies when the reference's disconnected zero loss left no gradient."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            live = [p for p in group["params"] if p.grad is not None]
            for p in live:
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32 or not p.is_contiguous() \
                        or not p.grad.is_contiguous():
                    raise TypeError("FusedAdamW: contiguous f32 params/grads required")
            self._init_state([p for p in live if not self.state[p]])
            if not live:
                continue
            if finite is None:
                by_step = {}
                for p in live:
                    st = self.state[p]
                    st["step"] = int(st["step"]) + 1  # a device count (sync-free path) is read once
                    by_step.setdefault(st["step"], []).append(p)
                for step, ps in by_step.items():
                    b1, b2 = group["betas"]
                    self._launch(group, ps, 1.0 - b1 ** step, math.sqrt(1.0 - b2 ** step), None, None, None)
            else:
                sin, sout = self._device_steps(live)
                self._launch(group, live, 1.0, 1.0, finite, sin, sout)
                for i, p in enumerate(live):
                    self.state[p]["step"] = sout[i]  # 0-d view; the other buffer is next step's output
        return loss

    def _device_steps(self, ps):
        """(steps_in, steps_out) device f32 buffers for this parameter list: steps_in holds every
        parameter's current count. Reused across steps (the two buffers alternate), rebuilt from the
        state (one host read) when the list changes or a count was set elsewhere."""
        key = ("steps",) + tuple(id(p) for p in ps)
        bufs = self._tables.get(key)
        cur = [self.state[p]["step"] for p in ps]
        if bufs is not None:
            for b in bufs:
                if all(torch.is_tensor(c) and c.data_ptr() == b[i].data_ptr() for i, c in enumerate(cur)):
                    other = bufs[1] if b is bufs[0] else bufs[0]
                    return b, other
        dev = ps[0].device
        sin = torch.tensor([float(c) for c in cur], dtype=torch.float32, device=dev)
        bufs = (sin, torch.empty_like(sin))
        if len(self._tables) > 64:
            self._tables.clear()
        self._tables[key] = bufs
        return bufs

    def _launch(self, group, ps, bc1, bc2s, finite, sin, sout):
        """The update of ``ps`` through the chunked streaming kernel (live bf16 compute copies,
        ops.cast_weight, rewritten in it), then every live row-panel weight pack (ops.packed_weight /
        packed_weight_t) rebuilt from the updated f32 weights in ONE launch: the pointer-table update
        moves no version counter, so without it the packs would stay at the old weights."""
        b1, b2 = group["betas"]
        dev = ps[0].device
        st = [self.state[p] for p in ps]
        tp = self._table(ps, dev)
        tg = self._table([p.grad for p in ps], dev)
        tm = self._table([s["exp_avg"] for s in st], dev)
        tv = self._table([s["exp_avg_sq"] for s in st], dev)
        sizes = self._table_sizes(ps, dev)
        shadows, jobs, big = [], [], 0
        for p in ps:
            sh = ops.shadow_of(p)
            shadows.append(sh.data_ptr() if sh is not None else 0)
            pk, pkt = ops.packs_of(p)
            rows, cols = p.shape[0], p.numel() // p.shape[0]
            for pack, tr in ((pk, 0), (pkt, 1)):
                if pack is not None:
                    jobs.append((p.data_ptr(), pack.data_ptr(), rows, cols, tr))
                    big = max(big, rows * cols)
        chunks, nch = self._table_chunks(ps, dev)
        lib.ivit_adamw_chunked(len(ps), ptr(tp), ptr(tg), ptr(tm), ptr(tv), ptr(self._table_ptrs(shadows, dev)),
                               ptr(sizes), ptr(chunks), nch, group["lr"], b1, b2, group["eps"],
                               group["weight_decay"], bc1, bc2s, ptr(finite), ptr(sin), ptr(sout), stream())
        if jobs:
            lib.ivit_weight_pack_multi(len(jobs), ptr(self._pack_jobs(jobs, dev)), big, stream())

    def _init_state(self, fresh):
        """Zero moments of the parameters seen for the first time: views into one flat buffer per
        device and moment (a single fill each, not two per parameter)."""
        by_dev = {}
        for p in fresh:
            by_dev.setdefault(p.device, []).append(p)
        for dev, ps in by_dev.items():
            n = sum(p.numel() for p in ps)
            flat = torch.zeros((2, n), dtype=torch.float32, device=dev)
            o = 0
            for p in ps:
                k = p.numel()
                self.state[p].update(step=0, exp_avg=flat[0, o:o + k].view_as(p), exp_avg_sq=flat[1, o:o + k].view_as(p))
                o += k

    def _table_ptrs(self, ptrs, device):
        key = ("ptrs",) + tuple(ptrs)
        tab = self._tables.get(key)
        if tab is None:
            tab = torch.tensor(ptrs, dtype=torch.int64).pin_memory().to(device, non_blocking=True)
            if len(self._tables) > 64:
                self._tables.clear()
            self._tables[key] = tab
        return tab

    def _pack_jobs(self, jobs, device):
        """Device table of ivit_weight_pack_multi records (w, wpack, rows, cols, transposed), 40 B each."""
        key = ("packs",) + tuple(jobs)
        tab = self._tables.get(key)
        if tab is None:
            rec = []
            for w, wp, rows, cols, tr in jobs:
                rec += [w, wp, rows, cols, tr]
            tab = torch.tensor(rec, dtype=torch.int64).pin_memory().to(device, non_blocking=True)
            if len(self._tables) > 64:
                self._tables.clear()
            self._tables[key] = tab
        return tab

    def _table_chunks(self, ps, device):
        """Device int32 [n][2] table of (tensor, chunk) for ivit_adamw_chunked: every
        ivit_adamw_chunk_elems()-element chunk of every tensor of the launch."""
        key = ("chunks",) + tuple(p.numel() for p in ps)
        tab = self._tables.get(key)
        if tab is None:
            ce = lib.ivit_adamw_chunk_elems()
            rec = [(t, c) for t, p in enumerate(ps) for c in range(-(-p.numel() // ce))]
            tab = (torch.tensor(rec, dtype=torch.int32).reshape(-1, 2).pin_memory().to(device, non_blocking=True),
                   len(rec))
            if len(self._tables) > 64:
                self._tables.clear()
            self._tables[key] = tab
        return tab

    def _table_sizes(self, ps, device):
        key = ("sizes",) + tuple(p.numel() for p in ps)
        tab = self._tables.get(key)
        if tab is None:
            tab = torch.tensor([p.numel() for p in ps], dtype=torch.int64).pin_memory().to(device, non_blocking=True)
            self._tables[key] = tab
        return tab
