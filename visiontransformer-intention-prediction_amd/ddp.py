"""Data-parallel gradient exchange for the IntentNetViT train step (BASELINE config 3/5).

One process per GPU (torchrun), ``torch.distributed`` over RCCL (backend "nccl") on MI355X,
gloo for the CPU tests. Samples are independent through fwd/bwd/loss, so the
only exchange is the gradient all-reduce, issued here in buckets while backward is still
running:

* every trainable parameter's ``.grad`` is a persistent view into a flat f32 bucket, so the
  autograd engine accumulates straight into the all-reduce buffer (no copy in or out) and
  FusedAdamW's device pointer tables stay valid across steps;
* buckets are filled in reverse registration order (heads → fusion → ViT blocks 11..0 →
  patch-embed), which is the order backward produces gradients; a bucket's all-reduce is
  launched from the post-accumulate hook of its last parameter, on the collective stream,
  and overlaps the remaining backward kernels;
* ``finish()`` drains the outstanding collectives and applies the 1/world mean in one pass
  per bucket (DDP semantics: the mean of the per-rank gradients; the loss stays normalised
  by the rank-local ``num_pos``, as the reference does per device).

Bucket size: xGMI is point-to-point (7 links x ~153 GB/s); RCCL rings over a few large
buckets amortise the per-collective latency, so the default is 64 MB (≈ 4 buckets for
62.9 M f32 grads) instead of DDP's 25 MB.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_distributed(backend: str | None = None, force_group: bool = False):
    """Read RANK/LOCAL_RANK/WORLD_SIZE from torchrun's env; returns (rank, local_rank, world, device).
    The process group (RCCL — backend "nccl" — on the GPU, bound to this rank's device; gloo on
    the CPU) is created for world > 1, or at world 1 with ``force_group`` (tests: the collective
    path on one GPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        if local >= torch.cuda.device_count():
            raise RuntimeError(f"LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s) visible")
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if (world > 1 or force_group) and not dist.is_initialized():
        be = backend or ("nccl" if dev.type == "cuda" else "gloo")
        if be == "nccl":
            dist.init_process_group(be, device_id=dev)
        else:
            dist.init_process_group(be)
    return rank, local, world, dev


class _Bucket:
    __slots__ = ("params", "flat", "views", "ready", "work", "events", "streams", "pending", "tables")

    def __init__(self, params, flat, views):
        self.params = params
        self.flat = flat
        self.views = views
        self.ready = 0
        self.work = None
        self.events = []
        self.streams = {}  # producing streams of this bucket's gradients (stream_id -> stream)
        self.pending = []  # (param, fresh gradient) to gather into the flat buffer
        self.tables = None  # (key, device pointer / size tables) of the last gather


class GradBuckets:
    """Bucketed, backward-overlapped gradient all-reduce over ``group``.

    Use::

        gb = GradBuckets(model.parameters(), bucket_mb=64)
        gb.zero_grad()            # instead of optimizer.zero_grad()
        loss.backward()           # buckets all-reduce as they fill
        gb.finish()               # wait + average
        optimizer.step()

    Gradients are NOT accumulated into the buckets by autograd: zero_grad() leaves every ``.grad``
    None, so autograd hands each parameter its freshly computed gradient without a copy (the
    AccumulateGrad "steal"), and when a bucket's last gradient arrives its gradients are gathered
    into the flat buffer by ONE multi-tensor copy launch (ivit_copy_multi) on the comm stream, the
    ``.grad`` fields become views of the buffer, and the buffer is all-reduced. (Pre-set bucket views
    made autograd add every fresh gradient into the view: one add kernel per parameter, 327 per
    step, plus the per-step zero fill of the buffers — about 1.5 ms of kernels per step.)
    """

    launched = 0  # collectives issued (tests)

    def __init__(self, params, bucket_mb: float = 64.0, group=None, force_collectives: bool = False):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # world 1: no exchange, unless forced (the collective path exercised on one device)
        self.active = self.world > 1 or (force_collectives and dist.is_initialized())
        ps = [p for p in params if p.requires_grad]
        if len({id(p) for p in ps}) != len(ps):
            raise ValueError("GradBuckets: duplicate parameters")
        cap = max(1, int(bucket_mb * (1 << 20)))
        self.buckets: list[_Bucket] = []
        self._of, self._view, self._done = {}, {}, set()
        cur, cur_bytes = [], 0
        for p in reversed(ps):
            nb = p.numel() * p.element_size()
            if cur and (cur_bytes + nb > cap or p.device != cur[0].device or p.dtype != cur[0].dtype):
                self._add(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nb
        if cur:
            self._add(cur)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in ps]

    def _add(self, params):
        n = sum(p.numel() for p in params)
        flat = torch.zeros(n, dtype=params[0].dtype, device=params[0].device)
        views, off = [], 0
        for p in params:
            v = flat[off:off + p.numel()].view_as(p)
            views.append(v)
            self._view[p] = v
            p.grad = v
            off += p.numel()
        b = _Bucket(params, flat, views)
        for p in params:
            self._of[p] = b
        self.buckets.append(b)

    @property
    def numel(self):
        return sum(b.flat.numel() for b in self.buckets)

    def zero_grad(self):
        """Every ``.grad`` None: the coming backward's gradients are taken over without a copy."""
        for b in self.buckets:
            if b.work is not None:
                raise RuntimeError("GradBuckets.zero_grad() with collectives in flight; call finish() first")
            b.ready = 0
            b.pending = []
            b.streams = {}
            b.events = []
            for p in b.params:
                p.grad = None
        self._done = set()

    def _on_grad(self, p):
        b = self._of[p]
        g = p.grad
        if g is None:
            raise RuntimeError("GradBuckets: post-accumulate hook without a gradient")
        if id(p) in self._done:
            raise RuntimeError("GradBuckets: a parameter received two gradients in one backward "
                               "(call GradBuckets.zero_grad() before each backward)")
        self._done.add(id(p))
        b.ready += 1
        if g.data_ptr() != self._view[p].data_ptr():
            b.pending.append((p, g))
        if not self.active:
            return
        if b.flat.is_cuda:
            # the two ViT streams produce gradients on two HIP streams (model_vit.stream_tokens):
            # the bucket's gather + collective must wait for every producer, not just the last one.
            # The hook runs after its gradient was enqueued, so one event per producing stream
            # recorded when the bucket fills covers all of them
            st = torch.cuda.current_stream(b.flat.device)
            b.streams[st.stream_id] = st
        if b.ready == len(b.params):
            self._launch(b)

    def _gather(self, b):
        """The bucket's fresh gradients into its flat buffer (current stream), ``.grad`` -> views."""
        if not b.pending:
            return
        views = [self._view[p] for p, _ in b.pending]
        srcs = [g if g.is_contiguous() and g.dtype == b.flat.dtype else g.contiguous().to(b.flat.dtype)
                for _, g in b.pending]
        if b.flat.is_cuda:
            from _lib import lib, ptr, stream
            key = tuple(s.data_ptr() for s in srcs) + tuple(v.data_ptr() for v in views)
            if b.tables is None or b.tables[0] != key:
                host = torch.tensor([s.data_ptr() for s in srcs] + [v.data_ptr() for v in views] +
                                    [s.numel() for s in srcs], dtype=torch.int64).pin_memory()
                b.tables = (key, host.to(b.flat.device, non_blocking=True))
            tab, n = b.tables[1], len(srcs)
            lib.ivit_copy_multi(n, ptr(tab[:n]), ptr(tab[n:2 * n]), ptr(tab[2 * n:]),
                                max(s.numel() for s in srcs), stream())
            cur = torch.cuda.current_stream(b.flat.device)
            for s in srcs:
                s.record_stream(cur)  # freed by autograd / below; reused only after this copy
        else:
            for v, s in zip(views, srcs):
                v.copy_(s)
        for (p, _), v in zip(b.pending, views):
            p.grad = v
        b.pending = []

    def _launch(self, b):
        if b.flat.is_cuda:
            comm = self._comm_stream(b.flat.device)
            for st in b.streams.values():
                comm.wait_event(st.record_event())
            for ev in b.events:
                comm.wait_event(ev)
            b.events = []
            b.streams = {}
            with torch.cuda.stream(comm):
                self._gather(b)
                b.work = dist.all_reduce(b.flat, group=self.group, async_op=True)
        else:
            self._gather(b)
            b.work = dist.all_reduce(b.flat, group=self.group, async_op=True)
        GradBuckets.launched += 1

    def _comm_stream(self, device):
        if getattr(self, "_comm", None) is None:
            self._comm = torch.cuda.Stream(device)
        return self._comm

    def finish(self):
        """Launch any bucket that did not fill (parameters without a gradient this step read zero,
        as DistributedDataParallel's buckets), wait, and average."""
        if not self.active:
            for b in self.buckets:
                self._gather(b)
                for p, v in zip(b.params, b.views):
                    if id(p) not in self._done:
                        v.zero_()
                        p.grad = v
                b.ready = 0
            return
        for b in self.buckets:
            if b.work is None:
                missing = [(p, v) for p, v in zip(b.params, b.views) if id(p) not in self._done]
                if b.flat.is_cuda:  # everything queued so far is final
                    b.events = [torch.cuda.current_stream(b.flat.device).record_event()]
                for p, v in missing:
                    v.zero_()
                    p.grad = v
                self._launch(b)
        inv = 1.0 / self.world
        for b in self.buckets:
            b.work.wait()
            b.work = None
            b.ready = 0
            b.events = []
            b.streams = {}
        if getattr(self, "_comm", None) is not None:
            torch.cuda.current_stream(self._comm.device).wait_stream(self._comm)
        if self.world > 1:
            for b in self.buckets:
                b.flat.mul_(inv)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


@torch.no_grad()
def broadcast_state(module, src: int = 0, group=None):
    """Copy rank ``src``'s parameters and buffers (BN running stats included) to every rank,
    as DistributedDataParallel does at construction; a no-op without a process group."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src, group=group)


def all_reduce_sum(values, device, group=None):
    """Sum a list of floats over ranks (f64); returns the list unchanged without a group."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, group=group)
    return t.tolist()


def any_rank(flag: bool, device, group=None) -> bool:
    """Collective OR of a per-rank condition (the train loop's NaN skip must be taken by every
    rank together, or the next bucketed all-reduce would pair different steps)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(int(t.item()))


def min_on_device(t, group=None):
    """Element-wise minimum over ranks of a device tensor, left on the device (no host sync): a
    copy all-reduced with MIN on the current stream."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return t
    out = t.detach().clone()
    dist.all_reduce(out, op=dist.ReduceOp.MIN, group=group)
    return out


def max_over_ranks(value: float, device, group=None) -> float:
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
