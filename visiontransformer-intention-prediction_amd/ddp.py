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


def grad_order(model):
    """The model's trainable parameters in forward order with the two ViT streams interleaved
    block by block (patch embeddings, block 0 of each stream, block 1, ..., the final norms, then
    the rest in registration order), so that the reverse — GradBuckets' fill order — follows the
    order the interleaved backward produces gradients (model_vit.stream_tokens). Models without
    the two-stream backbone: registration order."""
    bb = getattr(model, "backbone", None)
    vl, vm = getattr(bb, "vit_lidar", None), getattr(bb, "vit_map", None)
    if vl is None or vm is None or not hasattr(vl, "blocks") or not hasattr(vm, "blocks"):
        return [p for p in model.parameters()]
    order, seen = [], set()

    def add(mod_or_params):
        ps = mod_or_params.parameters() if isinstance(mod_or_params, torch.nn.Module) else mod_or_params
        for p in ps:
            if id(p) not in seen:
                seen.add(id(p))
                order.append(p)

    for v in (vl, vm):
        add(v.patch_embed)
        add([t for t in (getattr(v, "cls_token", None), getattr(v, "pos_embed", None)) if t is not None])
    for i in range(max(len(vl.blocks), len(vm.blocks))):
        for v in (vl, vm):
            if i < len(v.blocks):
                add(v.blocks[i])
    add(model)  # final norms, adapters, fusion block, heads (registration order)
    return order


# Each parameter's view starts on a 16-byte boundary of its bucket: kernels that write a gradient
# straight into its view (GradSink: the grouped ViT weight gradient's reduce stores 16 B per lane)
# need aligned destinations, and a 35-element bias (the detection head) would otherwise leave every
# later view 4-byte aligned. The padding floats stay zero (all-reduced with the rest, harmless).
_ALIGN = 4  # floats


def _aligned(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


_ON_COMM = object()  # a bucket whose collective was enqueued on the comm stream itself


class _Bucket:
    __slots__ = ("params", "flat", "offs", "ready", "work", "streams")

    def __init__(self, params, flat, offs):
        self.params = params
        self.flat = flat
        self.offs = offs
        self.ready = 0
        self.work = None
        self.streams = {}  # producing streams of this bucket's gradients (stream_id -> stream)


def comm_stream_collectives_ok(version=None, env=None):
    """True when a synchronous-op all-reduce issued on a side stream is enqueued on that stream
    without blocking the host: torch >= 2.8's ProcessGroupNCCL (asyncOp = false runs the collective
    on the current stream), and no TORCH_NCCL_BLOCKING_WAIT / NCCL_BLOCKING_WAIT (wait() would then
    block the autograd thread in every bucket's hook)."""
    version = torch.__version__ if version is None else version
    env = os.environ if env is None else env
    try:
        major, minor = (int(x) for x in version.split("+")[0].split(".")[:2])
    except ValueError:
        return False
    blocking = any(env.get(k, "0") not in ("", "0") for k in ("TORCH_NCCL_BLOCKING_WAIT", "NCCL_BLOCKING_WAIT"))
    return (major, minor) >= (2, 8) and not blocking


class GradSink:
    """A parameter's slot in the gradient buckets, for ops that write the gradient themselves
    (ops.ViTBlockFn: the block's weight / bias / LayerNorm gradients): ``claim()`` -> the bucket view
    to overwrite (None when the view is not freshly zeroed this step, e.g. a second backward
    without zero_grad — the op then returns its gradient to autograd, which adds it), ``done()``
    after the writes are enqueued on the current stream (the bucket bookkeeping of the
    post-accumulate hook, which does not run for a gradient the op returns as None)."""
    __slots__ = ("gb", "p", "view")

    def __init__(self, gb, p, view):
        self.gb, self.p, self.view = gb, p, view

    def claim(self):
        gb = self.gb
        if id(self.p) not in gb._fresh or self.p.grad is None or self.p.grad.data_ptr() != self.view.data_ptr():
            return None
        return self.view

    def done(self):
        self.gb._direct.add(id(self.p))
        self.gb._on_grad(self.p, direct=True)


class GradBuckets:
    """Bucketed, backward-overlapped gradient all-reduce over ``group``.

    Use::

        gb = GradBuckets(model.parameters(), bucket_mb=64)
        gb.zero_grad()            # instead of optimizer.zero_grad()
        loss.backward()           # buckets all-reduce as they fill
        gb.finish()               # wait + average
        optimizer.step()

    Every ``.grad`` is a persistent view into a flat bucket. Autograd accumulates a returned
    gradient into it (one add kernel per parameter); the ViT blocks' gradients (288 of the 327
    IntentNetViT parameters) skip that: their kernels write straight into the views
    (``GradSink``, ``ops.grad_sinks``) and report completion themselves.
    """

    launched = 0  # collectives issued (tests)

    def __init__(self, params, bucket_mb: float = 64.0, group=None, force_collectives: bool = False,
                 last_bucket_mb: float | None = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # world 1: no exchange, unless forced (the collective path exercised on one device)
        self.active = self.world > 1 or (force_collectives and dist.is_initialized())
        ps = [p for p in params if p.requires_grad]
        if len({id(p) for p in ps}) != len(ps):
            raise ValueError("GradBuckets: duplicate parameters")
        cap = max(1, int(bucket_mb * (1 << 20)))
        # last_bucket_mb: the parameters whose gradients arrive last (the end of the reversed list)
        # get a bucket of their own of at most this size, so the collective that cannot overlap
        # the backward is short (IntentNetViT: the LiDAR patch embedding's 28.5-MB weight gradient
        # is the step's last kernel)
        tail = []
        if last_bucket_mb is not None:
            lcap, lbytes = max(1, int(last_bucket_mb * (1 << 20))), 0
            while ps:
                nb = ps[0].numel() * ps[0].element_size()
                if tail and (lbytes + nb > lcap or ps[0].device != tail[0].device or ps[0].dtype != tail[0].dtype):
                    break
                tail.append(ps.pop(0))
                lbytes += nb
        self.buckets: list[_Bucket] = []
        self._of, self._ptr = {}, {}
        self._fresh = set()  # ids of parameters whose bucket view is zeroed and not written yet
        self._seen = set()  # ids of parameters whose gradient arrived in this backward
        self._direct = set()  # ids of parameters written through their GradSink in this backward
        # the comm-stream form (a synchronous-op all-reduce issued inside torch.cuda.stream(comm))
        # relies on torch >= 2.8 ProcessGroupNCCL enqueuing it on the current stream without
        # blocking the host; otherwise (older torch, or TORCH_NCCL_BLOCKING_WAIT making wait()
        # block) the asynchronous form on the process group's own stream keeps the all-reduces
        # overlapping the backward
        self.pg_stream = not comm_stream_collectives_ok()
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
        if tail:
            self._add(list(reversed(tail)))
            ps = tail + ps
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in ps]

    def _add(self, params):
        offs, n = [], 0
        for p in params:
            offs.append(n)
            n += _aligned(p.numel())
        flat = torch.zeros(n, dtype=params[0].dtype, device=params[0].device)
        b = _Bucket(params, flat, offs)
        for p, off in zip(params, offs):
            p.grad = flat[off:off + p.numel()].view_as(p)
            self._of[p] = b
            self._ptr[p] = p.grad.data_ptr()
            p._ivit_sink = GradSink(self, p, p.grad)
        self.buckets.append(b)

    @property
    def numel(self):
        """Gradient elements held (the buckets' alignment padding not counted)."""
        return sum(p.numel() for b in self.buckets for p in b.params)

    def zero_grad(self):
        for b in self.buckets:
            if b.work is not None:
                raise RuntimeError("GradBuckets.zero_grad() with collectives in flight; call finish() first")
            b.flat.zero_()
            b.ready = 0
            b.streams = {}
            for p, off in zip(b.params, b.offs):  # re-attach views if something replaced .grad
                view = b.flat[off:off + p.numel()]
                if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                    p.grad = view.view_as(p)
        self._fresh = {id(p) for b in self.buckets for p in b.params}
        self._seen = set()
        self._direct = set()

    def _on_grad(self, p, direct=False):
        if not direct and id(p) in self._direct:
            # written and counted by its op (GradSink.done); the engine still runs the post-accumulate
            # hook for the None gradient the op returned
            return
        b = self._of[p]
        if p.grad is None or p.grad.data_ptr() != self._ptr[p]:
            raise RuntimeError("GradBuckets: a parameter's .grad was replaced outside the bucket "
                               "(use GradBuckets.zero_grad(), not optimizer.zero_grad(set_to_none=True))")
        self._fresh.discard(id(p))
        if id(p) in self._seen:
            raise RuntimeError(f"GradBuckets: a second gradient for one parameter in one backward "
                               f"({getattr(p, '_dbg_name', tuple(p.shape))})")
        self._seen.add(id(p))
        b.ready += 1
        if not self.active:
            return
        if b.flat.is_cuda:
            # the two ViT streams produce gradients on two HIP streams (model_vit.stream_tokens):
            # the bucket's collective must wait for every producer, not just the last one. A
            # gradient's accumulation is enqueued before its hook runs, so one event per producing
            # stream recorded when the bucket fills covers all of them (a few waits per bucket
            # instead of one event + wait per parameter)
            st = torch.cuda.current_stream(b.flat.device)
            b.streams[st.stream_id] = st
        if b.ready == len(b.params):
            self._launch(b)

    def _launch(self, b):
        if b.flat.is_cuda:
            comm = self._comm_stream(b.flat.device)
            for st in b.streams.values():
                comm.wait_event(st.record_event())
            b.streams = {}
            with torch.cuda.stream(comm):
                if self.pg_stream:
                    b.work = dist.all_reduce(b.flat, group=self.group, async_op=True)
                else:
                    # a synchronous-op collective is enqueued on the CURRENT stream (torch >= 2.8
                    # ProcessGroupNCCL, asyncOp = false): the RCCL kernel runs on `comm` itself, not
                    # on the process group's internal stream, so the step stays at four streams
                    # (default, the two ViT streams, comm) = GPU_MAX_HW_QUEUES. The host does not
                    # block: the op only orders `comm` behind its own end event.
                    dist.all_reduce(b.flat, group=self.group, async_op=False)
                    b.work = _ON_COMM
        else:
            b.work = dist.all_reduce(b.flat, group=self.group, async_op=True)
        GradBuckets.launched += 1

    def _comm_stream(self, device):
        if getattr(self, "_comm", None) is None:
            self._comm = torch.cuda.Stream(device)
        return self._comm

    def finish(self):
        """Launch any bucket that did not fill (unused parameters), wait, and average."""
        self._fresh = set()
        self._seen = set()
        self._direct = set()
        if not self.active:
            for b in self.buckets:
                b.ready = 0
            return
        for b in self.buckets:
            if b.work is None:
                if b.flat.is_cuda:  # unused parameters: everything queued so far is final
                    st = torch.cuda.current_stream(b.flat.device)
                    b.streams[st.stream_id] = st
                self._launch(b)
        inv = 1.0 / self.world
        for b in self.buckets:
            if b.work is not _ON_COMM:
                b.work.wait()
            b.work = None
            b.ready = 0
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
        for b in self.buckets:
            for p in b.params:
                if getattr(p, "_ivit_sink", None) is not None and p._ivit_sink.gb is self:
                    del p._ivit_sink


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
