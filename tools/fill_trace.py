"""Which host calls launch the small ATen kernels (fills, multiplies, copies) inside one bench
train step: torch.profiler with Python stacks, grouped by (kernel family, op, innermost repo frame).

    python tools/fill_trace.py [--steps 1]
"""
import argparse
import collections
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "visiontransformer-intention-prediction_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1)
    args = ap.parse_args()
    import loss as L
    import model_vit
    import utils
    from optim import FusedAdamW
    from synthetic import synthetic_batch
    from trainer import Trainer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = model_vit.IntentNetViT(backbone_cfg={"img_size": (400, 720)}).to(dev).set_compute_dtype(torch.bfloat16).train()
    batch = synthetic_batch(8, (400, 720), torch.Generator().manual_seed(1234), device=dev)
    anchors = utils.generate_anchors(400, 720, 8, device=dev)
    tr = Trainer(m, L.DetectionIntentionLoss(), FusedAdamW(m.parameters(), lr=1e-4, weight_decay=1e-4), anchors,
                 check_nan=False)
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        for _ in range(args.steps):
            tr.step(batch)
        torch.cuda.synchronize()
    fam = ("Fill", "MulFunctor", "copy", "Copy", "bernoulli", "distribution", "add", "Mul", "Div", "index",
           "cat", "Reduce", "reduce")
    groups = collections.Counter()
    for e in prof.events():
        ks = [k.name for k in getattr(e, "kernels", [])]
        if not ks:
            continue
        for k in ks:
            if k.startswith(("ivit::", "(anonymous")) or not any(f in k for f in fam):
                continue
            frames = [f for f in (e.stack or []) if ROOT in f or "repo" in f]
            where = frames[0].replace(ROOT + "/", "") if frames else "?"
            short = k.split("<")[1].split(",")[0] if "<" in k else k[:60]
            groups[(short[:60], e.name, where)] += 1
    total = sum(groups.values())
    print(f"{total} small ATen kernels in {args.steps} step(s)")
    for (k, op, where), n in groups.most_common(60):
        print(f"{n / args.steps:7.1f}/step  {k:40s} {op:28s} {where}")


if __name__ == "__main__":
    main()
