"""N = 2 data-parallel train step on the GPU (BASELINE configs 3 / 5 path at a reduced grid): two
ranks share cuda:0 over gloo (RCCL wants one device per rank and the test box has one GPU), each
running the real bf16 IntentNetViT through the HIP kernels with ddp.GradBuckets (per-parameter
producer events of the two ViT streams, the collective on its own stream) and trainer.Trainer
with FusedAdamW. Checks: the bucketed, backward-overlapped all-reduce equals the mean of the two
ranks' single-process gradients (SURVEY.md §8e DDP semantics), and the replicas stay bitwise
identical over optimizer steps. The CPU tests (test_cpu_ddp.py) cover the same code on a toy model."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, H, W, B, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK="0")
        for p in (os.path.join(HERE, ".."), os.path.join(HERE, "..", "visiontransformer-intention-prediction_amd")):
            sys.path.insert(0, p)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import loss as L
        import model_vit
        import utils
        from ddp import GradBuckets
        from optim import FusedAdamW
        from oracle import ivit_oracle as O
        from oracle.weights import make_state_dict, model_cfg
        from trainer import Trainer

        cfg = model_cfg(img_size=(H, W))
        sd = make_state_dict(cfg, seed=0)

        def build():
            m = model_vit.IntentNetViT(backbone_cfg={"img_size": (H, W), "drop_path_rate_lidar": 0.0,
                                                     "drop_path_rate_map": 0.0})
            m.load_state_dict(sd, strict=True)
            return m.cuda().set_compute_dtype(torch.bfloat16).train()

        lidar, mp_, gts = O.synthetic_batch(B, (H, W), seed=100 + rank, grid_scale=H / 400.0)
        lidar, mp_ = lidar.cuda(), mp_.cuda()
        anchors = utils.generate_anchors(H, W, 8, device="cuda")
        keep = (torch.rand((B, anchors.shape[0]), generator=torch.Generator().manual_seed(7 + rank)) < 0.15).float()
        lossf = L.DetectionIntentionLoss()

        def grads(m):
            return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                              for p in m.parameters()])

        # the rank's own gradients, no exchange; their mean over ranks is the reference
        mb = build()
        c, b, i = mb(lidar, mp_)
        lossf(c, b, i, anchors, gts, intent_keep=keep)["loss"].backward()
        ref = grads(mb)
        dist.all_reduce(ref)
        ref /= world
        del mb
        # the same step through the bucketed, backward-overlapped all-reduce (small buckets: many
        # collectives launched from the gradient hooks while backward runs)
        ma = build()
        gb = GradBuckets(ma.parameters(), bucket_mb=8)
        gb.zero_grad()
        c, b, i = ma(lidar, mp_)
        lossf(c, b, i, anchors, gts, intent_keep=keep)["loss"].backward()
        gb.finish()
        got = grads(ma)
        err = float((got - ref).abs().max() / ref.abs().max())
        gb.remove()
        del ma
        # Trainer + FusedAdamW: two steps, every rank on its own data, replicas stay identical
        mt = build()
        opt = FusedAdamW(mt.parameters(), lr=1e-4, weight_decay=1e-4)
        tr = Trainer(mt, lossf, opt, anchors, world=world, bucket_mb=16, check_nan=True)
        init = torch.cat([p.detach().reshape(-1) for p in mt.parameters()]).clone()
        for _ in range(2):
            d = tr.step({"lidar_bev": lidar, "map_bev": mp_, "gt_list": gts})
            assert d is not None
        flat = torch.cat([p.detach().reshape(-1) for p in mt.parameters()])
        other = flat.clone()
        dist.broadcast(other, 0)
        moved = float((flat - init).abs().max())
        q.put((rank, err, bool(torch.equal(flat, other)), moved, None))
        dist.destroy_process_group()
    except Exception as e:  # report to the parent instead of hanging the spawn
        q.put((rank, None, None, None, repr(e)))


@pytest.mark.parametrize("H,W,B", [(64, 96, 2), (400, 720, 2), (800, 1440, 1)])
def test_ddp_two_ranks_bf16_model_on_gpu(H, W, B):
    """(800, 1440, 1) is BASELINE config 5's per-rank workload (2x grid, N = 18 001 tokens per ViT
    stream) through GradBuckets + Trainer."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, H, W, B, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, err, same, moved, exc in res:
        assert exc is None, (rank, exc)
        assert err < 1e-6, (rank, err)  # deterministic kernels: the same two per-rank sums
        assert same, rank
        assert moved > 0.0, rank


def _rccl_worker(port, q):
    """World 1 over RCCL (backend "nccl") on cuda:0: ddp.init_distributed binds the process group to
    the device (device_id), Trainer(force_buckets=True) runs GradBuckets' backward-overlapped bucket
    all-reduce on its comm stream and waits on the work handles — the exact multi-GPU code path,
    with one rank. Two Trainers from the same weights and data, one plain and one through the
    collectives, must end bitwise identical (an all-reduce over one rank is the identity)."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
        for p in (os.path.join(HERE, ".."), os.path.join(HERE, "..", "visiontransformer-intention-prediction_amd")):
            sys.path.insert(0, p)
        import ddp
        rank, local, world, dev = ddp.init_distributed(force_group=True)
        backend = dist.get_backend()
        import loss as L
        import model_vit
        import utils
        from optim import FusedAdamW
        from oracle import ivit_oracle as O
        from oracle.weights import make_state_dict, model_cfg
        from trainer import Trainer
        H, W = 64, 96
        cfg = model_cfg(img_size=(H, W))
        sd = make_state_dict(cfg, seed=0)
        lidar, mp_, gts = O.synthetic_batch(2, (H, W), seed=5, grid_scale=H / 400.0)
        lidar, mp_ = lidar.to(dev), mp_.to(dev)
        anchors = utils.generate_anchors(H, W, 8, device=dev)
        finals = []
        for force in (False, True):
            m = model_vit.IntentNetViT(backbone_cfg={"img_size": (H, W), "drop_path_rate_lidar": 0.0,
                                                     "drop_path_rate_map": 0.0})
            m.load_state_dict(sd, strict=True)
            m = m.to(dev).set_compute_dtype(torch.bfloat16).train()
            lf = L.DetectionIntentionLoss(apply_intention_downsampling=False)
            tr = Trainer(m, lf, FusedAdamW(m.parameters(), lr=1e-4, weight_decay=1e-4), anchors, world=world,
                         bucket_mb=8, check_nan=False, force_buckets=force)
            n0 = ddp.GradBuckets.launched
            for _ in range(2):
                tr.step({"lidar_bev": lidar, "map_bev": mp_, "gt_list": gts})
            torch.cuda.synchronize()
            finals.append((torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone(),
                           ddp.GradBuckets.launched - n0, len(tr.buckets.buckets) if tr.buckets else 0))
        same = bool(torch.equal(finals[0][0], finals[1][0]))
        q.put((backend, world, same, finals[1][1], finals[1][2], None))
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((None, None, None, None, None, traceback.format_exc()))


def test_rccl_world1_bucketed_trainer():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_port(), q))
    p.start()
    backend, world, same, launched, nbuckets, exc = q.get(timeout=240)
    p.join(timeout=60)
    assert exc is None, exc
    assert backend == "nccl" and world == 1
    assert nbuckets > 1 and launched == 2 * nbuckets  # every bucket all-reduced on each of the 2 steps
    assert same
