"""tests/test_gpu_ddp.py's worker, flow unchanged, printing the worst parameters of part 2."""
import os
import sys

import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))


def worker(rank, world, port, H, W, B):
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
    from oracle import ivit_oracle as O
    from oracle.weights import make_state_dict, model_cfg
    sd = make_state_dict(model_cfg(img_size=(H, W)), seed=0)

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

    mb = build()
    names = [n for n, _ in mb.named_parameters()]
    sizes = [p.numel() for p in mb.parameters()]
    c, b, i = mb(lidar, mp_)
    lossf(c, b, i, anchors, gts, intent_keep=keep)["loss"].backward()
    loc = grads(mb)
    ref = loc.clone()
    dist.all_reduce(ref)
    ref /= world
    del mb
    ma = build()
    gb = GradBuckets(ma.parameters(), bucket_mb=8)
    gb.zero_grad()
    c, b, i = ma(lidar, mp_)
    lossf(c, b, i, anchors, gts, intent_keep=keep)["loss"].backward()
    gb.finish()
    got = grads(ma)
    err = float((got - ref).abs().max() / ref.abs().max())
    torch.cuda.synchronize()
    got2 = grads(ma)
    out, o = [], 0
    for n, k in zip(names, sizes):
        d = float((got[o:o + k] - ref[o:o + k]).abs().max())
        d2 = float((got2[o:o + k] - ref[o:o + k]).abs().max())
        dl = float((got[o:o + k] - loc[o:o + k]).abs().max())
        out.append((d, d2, dl, n))
        o += k
    out.sort(reverse=True)
    print(rank, "err", err, "bad", sum(1 for x in out if x[0] > 0), out[:8], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    H, W = (int(v) for v in os.environ.get("GRID", "64x96").split("x"))
    mp.spawn(worker, args=(2, port, H, W, 2), nprocs=2, join=True)
