"""Host issue time of the bench training step vs its GPU time: after warm-up, each phase of
Trainer.step (forward, loss, backward, optimizer) is timed on the host WITHOUT synchronising, then
the GPU is drained; if the host's per-step issue time approaches the GPU time the launch path is
(near) the critical path.   python tools/host_probe.py"""
import os
import sys
import time

PKG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "visiontransformer-intention-prediction_amd")
sys.path.insert(0, PKG)
import torch  # noqa: E402

import loss as L  # noqa: E402
import model_vit  # noqa: E402
import utils  # noqa: E402
from optim import FusedAdamW  # noqa: E402
from synthetic import synthetic_batch  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
H, W, B = 400, 720, 8
model = model_vit.IntentNetViT(backbone_cfg={"img_size": (H, W)}).to(dev).set_compute_dtype(torch.bfloat16)
model.train(True)
anchors = utils.generate_anchors(H, W, 8, device=dev)
batch = synthetic_batch(B, (H, W), torch.Generator().manual_seed(1234), device=dev)
opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
lf = L.DetectionIntentionLoss(use_rotated_iou=False, apply_intention_downsampling=True)


def step(tm):
    t0 = time.perf_counter()
    opt.zero_grad(set_to_none=True)
    cls, box, it = model(batch["lidar_bev"], batch["map_bev"])
    t1 = time.perf_counter()
    d = lf(cls, box, it, anchors, batch["gt_list"])
    t2 = time.perf_counter()
    d["loss"].backward()
    t3 = time.perf_counter()
    opt.step(finite=lf.last_finite)
    t4 = time.perf_counter()
    tm.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3))


for _ in range(3):
    step([])
torch.cuda.synchronize()
tm = []
t0 = time.perf_counter()
for _ in range(10):
    step(tm)
th = time.perf_counter() - t0
torch.cuda.synchronize()
tg = time.perf_counter() - t0
ph = [sum(x[i] for x in tm) / len(tm) * 1e3 for i in range(4)]
print(f"host issue {th / 10 * 1e3:.2f} ms/step (forward {ph[0]:.2f}, loss {ph[1]:.2f}, backward {ph[2]:.2f}, "
      f"optimizer {ph[3]:.2f}); wall incl. GPU drain {tg / 10 * 1e3:.2f} ms/step", flush=True)
