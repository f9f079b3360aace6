"""N>1 data-parallel path on the CPU: ddp.GradBuckets / ddp.any_rank / trainer.Trainer over
gloo with world_size 2 (the same code runs over RCCL on the GPUs). Checks that the bucketed,
backward-overlapped all-reduce yields exactly the mean of the per-rank gradients (DDP
semantics), across several steps and bucket sizes, with unused parameters,
and that the NaN skip is taken collectively."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)


class Toy(nn.Module):
    """Stand-in with the IntentNetViT forward signature (lidar, map) → (cls, box, intent)."""

    def __init__(self):
        super().__init__()
        self.a = nn.Linear(12, 24)
        self.n = nn.LayerNorm(24)
        self.b = nn.Linear(24, 15)
        self.unused = nn.Linear(3, 3)  # never touched by forward

    def forward(self, lidar, mp):
        h = self.n(torch.relu(self.a(torch.cat([lidar, mp], 1))))
        o = self.b(h)
        return o[:, :1], o[:, 1:7], o[:, 7:]


def _data(rank, step, nan=False, inf_loss=False):
    g = torch.Generator().manual_seed(100 * step + rank)
    x = torch.randn(6, 8, generator=g)
    m = torch.randn(6, 4, generator=g)
    if nan:
        x[0, 0] = float("nan")
    return {"lidar_bev": x, "map_bev": m, "gt_list": ["inf" if inf_loss else None] * 6}


def _loss(c, b, i, anchors, gts):
    loss = c.square().mean() + 0.5 * b.abs().mean() + i.sin().sum() * 0.1
    if gts is not None and gts[0] == "inf":
        loss = loss + float("inf")
    z = loss.detach()
    return {"loss": loss, "cls_loss": z, "box_loss": z, "intent_loss": z, "num_pos_anchors": torch.tensor(0)}


def _ref_grads(world, step, state):
    """Mean over ranks of single-process gradients on each rank's shard."""
    acc = None
    for r in range(world):
        m = Toy()
        m.load_state_dict(state)
        d = _data(r, step)
        c, b, i = m(d["lidar_bev"], d["map_bev"])
        _loss(c, b, i, None, None)["loss"].backward()
        gs = [p.grad if p.grad is not None else torch.zeros_like(p) for p in m.parameters()]
        acc = gs if acc is None else [a + g for a, g in zip(acc, gs)]
    return [a / world for a in acc]


def _bucket_worker(rank, world, port, bucket_mb):
    _init(rank, world, port)
    from ddp import GradBuckets
    torch.manual_seed(0)
    model = Toy()
    gb = GradBuckets(model.parameters(), bucket_mb=bucket_mb)
    assert gb.numel == sum(p.numel() for p in model.parameters())
    # every gradient view starts on a 16-B boundary (kernels store 16 B per lane into them)
    assert all(p.grad.data_ptr() % 16 == 0 for p in model.parameters())
    if bucket_mb < 0.01:
        assert len(gb.buckets) > 2
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    for step in range(3):
        state = {k: v.clone() for k, v in model.state_dict().items()}
        gb.zero_grad()
        d = _data(rank, step)
        c, b, i = model(d["lidar_bev"], d["map_bev"])
        _loss(c, b, i, None, None)["loss"].backward()
        gb.finish()
        ref = _ref_grads(world, step, state)
        for p, r in zip(model.parameters(), ref):
            torch.testing.assert_close(p.grad, r, rtol=1e-5, atol=1e-6)
        assert float(model.unused.weight.grad.abs().sum()) == 0.0
        opt.step()
    # replicas stay identical
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.equal(flat, other)
    dist.destroy_process_group()


def _trainer_worker(rank, world, port):
    _init(rank, world, port)
    from trainer import Trainer
    torch.manual_seed(0)
    model = Toy()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    tr = Trainer(model, _loss, opt, anchors=None, world=world, bucket_mb=0.001, check_nan=True)
    # step 0 normal, step 1 NaN on rank 1 only → skipped on every rank, step 2 normal,
    # step 3 non-finite loss on rank 0 only → no update on any rank (loss.py:190-198)
    outs = []
    for step in range(3):
        outs.append(tr.step(_data(rank, step, nan=(step == 1 and rank == 1))))
    assert outs[0] is not None and outs[1] is None and outs[2] is not None
    assert tr.skipped == 1
    before = [p.detach().clone() for p in model.parameters()]
    st_before = {k: v.clone() if torch.is_tensor(v) else v for k, v in opt.state_dict()["state"][0].items()}
    d = tr.step(_data(rank, 3, inf_loss=(rank == 0)))
    assert d is not None and tr.nonfinite == 1
    assert all(torch.equal(a, p.detach()) for a, p in zip(before, model.parameters()))
    st_after = opt.state_dict()["state"][0]
    assert all(torch.equal(torch.as_tensor(st_before[k]), torch.as_tensor(st_after[k])) for k in st_before)
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.equal(flat, other)
    dist.destroy_process_group()


def _broadcast_sched_worker(rank, world, port):
    """Replicas built from different seeds are made identical by Trainer (broadcast from rank
    0), and ReduceLROnPlateau stepped on the global epoch mean (train_vit.py) keeps the LR,
    and so the replicas, identical although each rank sees different data and losses."""
    _init(rank, world, port)
    from ddp import all_reduce_sum
    from trainer import Trainer
    torch.manual_seed(rank)
    model = Toy()
    model.n.weight.data.add_(rank)  # parameters AND ...
    model.register_buffer("stat", torch.full((3,), float(rank)))  # ... buffers differ per rank
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.1, patience=0)
    tr = Trainer(model, _loss, opt, anchors=None, world=world, bucket_mb=0.001, check_nan=True)
    assert float(model.stat.sum()) == 0.0
    for epoch in range(4):
        acc, n = 0.0, 0
        for step in range(2):
            d = tr.step(_data(rank, 10 * epoch + step))
            acc += float(d["loss"]) * (1 + 5 * rank)  # rank-dependent epoch losses
            n += 1
        tot = all_reduce_sum([acc, n], torch.device("cpu"))
        sched.step(tot[0] / tot[1])
    lrs = torch.tensor([opt.param_groups[0]["lr"]], dtype=torch.float64)
    other = lrs.clone()
    dist.broadcast(other, 0)
    assert torch.equal(lrs, other)
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.equal(flat, other)
    dist.destroy_process_group()


def test_broadcast_and_global_plateau_schedule():
    mp.spawn(_broadcast_sched_worker, args=(2, _port()), nprocs=2, join=True)


def _any_rank_worker(rank, world, port):
    _init(rank, world, port)
    from ddp import any_rank, max_over_ranks
    assert any_rank(rank == 1, torch.device("cpu")) is True
    assert any_rank(False, torch.device("cpu")) is False
    assert max_over_ranks(float(rank) + 0.5, torch.device("cpu")) == world - 0.5
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb", [0.001, 64.0])
def test_grad_buckets_mean_of_ranks(bucket_mb):
    mp.spawn(_bucket_worker, args=(2, _port(), bucket_mb), nprocs=2, join=True)


def test_trainer_collective_nan_skip():
    mp.spawn(_trainer_worker, args=(2, _port()), nprocs=2, join=True)


def test_any_rank_and_max():
    mp.spawn(_any_rank_worker, args=(2, _port()), nprocs=2, join=True)


def test_single_process_buckets_are_views():
    from ddp import GradBuckets
    m = Toy()
    gb = GradBuckets(m.parameters(), bucket_mb=0.001)
    gb.zero_grad()
    d = _data(0, 0)
    c, b, i = m(d["lidar_bev"], d["map_bev"])
    _loss(c, b, i, None, None)["loss"].backward()
    gb.finish()
    ptrs = {b_.flat.data_ptr() for b_ in gb.buckets}
    assert all(any(p.grad.data_ptr() >= q and p.grad.data_ptr() < q + b_.flat.numel() * 4
                   for q, b_ in zip(sorted(ptrs), sorted(gb.buckets, key=lambda x: x.flat.data_ptr())))
               for p in m.parameters())
    m.a.weight.grad = None  # replaced outside the bucket → zero_grad re-attaches the view
    gb.zero_grad()
    assert m.a.weight.grad is not None and float(m.a.weight.grad.abs().sum()) == 0.0


def test_grad_order_interleaves_streams_and_tail_bucket():
    """ddp.grad_order: every IntentNetViT parameter once, the two ViTs' blocks interleaved in
    forward order (so the bucket fill order follows the interleaved backward); GradBuckets'
    last_bucket_mb gives the last-ready parameters (the LiDAR patch embedding) a small bucket."""
    import torch.nn as nn
    from ddp import GradBuckets, grad_order
    from model_vit import IntentNetViT
    m = IntentNetViT()
    order = grad_order(m)
    names = {id(p): n for n, p in m.named_parameters()}
    assert sorted(names[id(p)] for p in order) == sorted(names.values())
    seq = [names[id(p)] for p in order]
    i0 = seq.index("backbone.vit_lidar.blocks.0.attn.qkv.weight")
    i1 = seq.index("backbone.vit_map.blocks.0.attn.qkv.weight")
    i2 = seq.index("backbone.vit_lidar.blocks.1.attn.qkv.weight")
    assert i0 < i1 < i2
    gb = GradBuckets(order, 64.0, last_bucket_mb=32.0)
    last = gb.buckets[-1]
    assert "backbone.vit_lidar.patch_embed.proj.weight" in {names[id(p)] for p in last.params}
    assert last.flat.numel() * 4 <= 32 * (1 << 20)
    assert sum(b.flat.numel() for b in gb.buckets) >= sum(p.numel() for p in m.parameters())
    # a model without the two-stream backbone: registration order
    lin = nn.Linear(3, 4)
    assert grad_order(lin) == list(lin.parameters())


class TwoStream(nn.Module):
    """Two independent branches (the LiDAR / map ViT streams' shape) joined by a fusion layer."""

    def __init__(self):
        super().__init__()
        self.l0, self.l1 = nn.Linear(8, 16), nn.Linear(16, 16)
        self.m0, self.m1 = nn.Linear(4, 16), nn.Linear(16, 16)
        self.fuse = nn.Linear(32, 15)

    def forward(self, lidar, mp):
        hl = self.l1(torch.relu(self.l0(lidar)))
        hm = self.m1(torch.relu(self.m0(mp)))
        o = self.fuse(torch.cat([hl, hm], 1))
        return o[:, :1], o[:, 1:7], o[:, 7:]


def _interleaved_order(m):
    """The order ddp.grad_order builds for IntentNetViT: the two streams' layers interleaved in
    forward order (l0, m0, l1, m1), then the fusion — buckets fill from its end."""
    return [p for mod in (m.l0, m.m0, m.l1, m.m1, m.fuse) for p in mod.parameters()]


def _world4_worker(rank, world, port):
    _init(rank, world, port)
    from ddp import GradBuckets
    torch.manual_seed(0)
    model = TwoStream()
    # tiny buckets (one or two parameters each) + a tail bucket for the first-registered (last-ready)
    # parameters: several collectives per backward, launched from the hooks in fill order
    gb = GradBuckets(_interleaved_order(model), bucket_mb=0.002, last_bucket_mb=0.0006)
    assert len(gb.buckets) >= 4
    assert {id(p) for p in gb.buckets[-1].params} <= {id(p) for p in model.l0.parameters()}
    for step in range(3):
        state = {k: v.clone() for k, v in model.state_dict().items()}
        gb.zero_grad()
        g = torch.Generator().manual_seed(100 * step + rank)
        x, mm = torch.randn(6, 8, generator=g), torch.randn(6, 4, generator=g)
        c, b, i = model(x, mm)
        _loss(c, b, i, None, None)["loss"].backward()
        gb.finish()
        acc = None
        for r in range(world):  # the mean over ranks of single-process gradients
            ref = TwoStream()
            ref.load_state_dict(state)
            g = torch.Generator().manual_seed(100 * step + r)
            xr, mr = torch.randn(6, 8, generator=g), torch.randn(6, 4, generator=g)
            cr, br, ir = ref(xr, mr)
            _loss(cr, br, ir, None, None)["loss"].backward()
            gs = [p.grad for p in ref.parameters()]
            acc = gs if acc is None else [a + q for a, q in zip(acc, gs)]
        for p, r_ in zip(model.parameters(), acc):
            torch.testing.assert_close(p.grad, r_ / world, rtol=1e-5, atol=1e-6)
        with torch.no_grad():
            for p in model.parameters():
                p.add_(p.grad, alpha=-0.1)
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.equal(flat, other)
    dist.destroy_process_group()


def test_grad_buckets_world4_interleaved_order_and_tail():
    """World 4 over gloo: the interleaved two-stream bucket order with a tail bucket — every rank
    launches its bucket all-reduces in the same order from the post-accumulate hooks (gloo pairs
    collectives by issue order: a mismatch gives wrong sums), the result is the mean of the four
    ranks' gradients, and the replicas stay identical."""
    mp.spawn(_world4_worker, args=(4, _port()), nprocs=4, join=True)


def test_comm_stream_collectives_guard():
    """The comm-stream form needs torch >= 2.8 and no blocking wait; otherwise GradBuckets takes the
    asynchronous process-group-stream form."""
    from ddp import GradBuckets, comm_stream_collectives_ok
    assert comm_stream_collectives_ok("2.10.0+rocm7.0", {})
    assert comm_stream_collectives_ok("2.8.0", {"TORCH_NCCL_BLOCKING_WAIT": "0"})
    assert not comm_stream_collectives_ok("2.7.1+rocm6.3", {})
    assert not comm_stream_collectives_ok("2.10.0", {"TORCH_NCCL_BLOCKING_WAIT": "1"})
    assert not comm_stream_collectives_ok("2.10.0", {"NCCL_BLOCKING_WAIT": "1"})
    gb = GradBuckets(nn.Linear(3, 4).parameters(), bucket_mb=1.0)
    assert gb.pg_stream == (not comm_stream_collectives_ok())


def test_tail_bucket_stops_at_dtype_change():
    """last_bucket_mb takes parameters from the front only while device and dtype match the first
    one: every bucket holds one dtype, and a backward through mixed dtypes fills all of them."""
    from ddp import GradBuckets
    a = nn.Parameter(torch.randn(5, dtype=torch.float64))
    b = nn.Parameter(torch.randn(7))
    c = nn.Parameter(torch.randn(3))
    gb = GradBuckets([a, b, c], bucket_mb=1.0, last_bucket_mb=1.0)
    for bk in gb.buckets:
        assert all(p.dtype == bk.flat.dtype for p in bk.params)
    assert [p for p in gb.buckets[-1].params] == [a]
    gb.zero_grad()
    (a.sum() * 2 + b.sum() * 3 + c.sum()).backward()
    gb.finish()
    assert torch.equal(a.grad, torch.full((5,), 2.0, dtype=torch.float64)) and torch.equal(b.grad, torch.full((7,), 3.0))
