"""Plain Trainer steps, then Trainer(force_buckets=True) steps on the same model in the same process
(bench.py --force-collectives' order), per-step wall times printed: where the DDP leg's cost sits."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "visiontransformer-intention-prediction_amd"))
import torch  # noqa: E402

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29533"), RANK="0",
                  WORLD_SIZE="1", LOCAL_RANK="0")
from ddp import init_distributed  # noqa: E402
rank, local, world, dev = init_distributed(force_group=True)
import loss as L  # noqa: E402
import model_vit  # noqa: E402
import utils  # noqa: E402
from optim import FusedAdamW  # noqa: E402
from synthetic import synthetic_batch  # noqa: E402
from trainer import Trainer  # noqa: E402

torch.manual_seed(0)
model = model_vit.IntentNetViT(backbone_cfg={"img_size": (400, 720)}).to(dev).set_compute_dtype(torch.bfloat16).train()
anchors = utils.generate_anchors(400, 720, 8, device=dev)
batch = synthetic_batch(8, (400, 720), torch.Generator().manual_seed(1234), device=dev)
opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
lf = L.DetectionIntentionLoss()
order = os.environ.get("ORDER", "plain,force").split(",")
for leg in order:
    tr = Trainer(model, lf, opt, anchors, world=1, bucket_mb=float(os.environ.get("BUCKET_MB", "64")),
                 check_nan=False, force_buckets=(leg == "force"))
    ts = []
    for i in range(12):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step(batch)
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
    print(leg, " ".join(f"{t:.2f}" for t in ts), flush=True)
    if tr.buckets is not None:
        tr.buckets.remove()
print("mem", torch.cuda.memory_stats()["num_alloc_retries"], torch.cuda.memory_reserved() / 2**30, flush=True)
