"""Two processes on one GPU (gloo), each comparing its own plain backward with GradBuckets over a
one-rank subgroup (no exchange): per-parameter gradient differences under two-process contention."""
import os
import sys

import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def worker(rank, world, port, H, W):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    for p in (os.path.join(HERE, ".."), os.path.join(HERE, "..", "visiontransformer-intention-prediction_amd")):
        sys.path.insert(0, p)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    groups = [dist.new_group([r]) for r in range(world)]
    import loss as L
    import model_vit
    import utils
    from ddp import GradBuckets
    from oracle import ivit_oracle as O
    from oracle.weights import make_state_dict, model_cfg
    sd = make_state_dict(model_cfg(img_size=(H, W)), seed=0)

    def build():
        m = model_vit.IntentNetViT(backbone_cfg={"img_size": (H, W), "drop_path_rate_lidar": 0.0,
                                                 "drop_path_rate_map": 0.0})
        m.load_state_dict(sd, strict=True)
        return m.cuda().set_compute_dtype(torch.bfloat16).train()

    lidar, mp_, gts = O.synthetic_batch(2, (H, W), seed=100 + rank, grid_scale=H / 400.0)
    lidar, mp_ = lidar.cuda(), mp_.cuda()
    anchors = utils.generate_anchors(H, W, 8, device="cuda")
    keep = (torch.rand((2, anchors.shape[0]), generator=torch.Generator().manual_seed(7 + rank)) < 0.15).float()
    lossf = L.DetectionIntentionLoss()
    mb = build()
    c, b, i = mb(lidar, mp_)
    lossf(c, b, i, anchors, gts, intent_keep=keep)["loss"].backward()
    if os.environ.get("CAT", "0") == "1":  # test_gpu_ddp's form: one cat right after backward
        names = [n for n, p in mb.named_parameters()]
        flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                          for p in mb.parameters()])
        ref, o = {}, 0
        for n, p in mb.named_parameters():
            ref[n] = flat[o:o + p.numel()].view_as(p).clone()
            o += p.numel()
    else:
        ref = {n: p.grad.detach().clone() for n, p in mb.named_parameters() if p.grad is not None}
    full = os.environ.get("FULL", "0") == "1"  # world-2 exchange: the test_gpu_ddp comparison
    if full:
        for t in ref.values():
            dist.all_reduce(t)
            t /= world
    ma = build()
    gb = GradBuckets(ma.parameters(), bucket_mb=8, group=None if full else groups[rank], force_collectives=True)
    gb.zero_grad()
    c, b, i = ma(lidar, mp_)
    lossf(c, b, i, anchors, gts, intent_keep=keep)["loss"].backward()
    gb.finish()
    torch.cuda.synchronize()
    errs = sorted(((float((p.grad - ref[n]).abs().max() / (ref[n].abs().max() + 1e-30)), n)
                   for n, p in ma.named_parameters() if n in ref), reverse=True)
    print(rank, "bad", sum(1 for e, _ in errs if e > 1e-6), errs[:6], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    H, W = (int(v) for v in os.environ.get("GRID", "64x96").split("x"))
    mp.spawn(worker, args=(2, port, H, W), nprocs=2, join=True)
