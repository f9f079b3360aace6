"""Micro-benchmark: BEV augmentation passes (ivit_bev_augment) over a batch
of B full-size samples (290 LiDAR + 9 map planes, 400x720 f32), inputs resident in HBM.
Per case: kernel time of one launch over all 2B stacks (pass table prebuilt), the algorithmic
HBM rate (read + write of every plane = 8 B per plane-pixel per pass), and the host API
(utils.augment_bev_batch: draws + table H2D + launches). Yardstick: torch's device copy."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "visiontransformer-intention-prediction_amd"))
import numpy as np
import torch

import utils
from _lib import lib, ptr, stream

B, H, W = int(os.environ.get("AUG_B", "8")), 400, 720
L = torch.rand((B, 290, H, W), device="cuda")
M = (torch.rand((B, 9, H, W), device="cuda") < 0.1).float()
LO, MO = torch.empty_like(L), torch.empty_like(M)
PL = B * 299 * H * W  # planes-pixels per pass over the batch


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def table(p):
    st = utils._stages(p, H, W)
    assert len(st) == 1
    op, f = st[0]
    rows = []
    for b in range(B):
        for src, dst in ((L[b], LO[b]), (M[b], MO[b])):
            e = np.zeros((), utils._BEV_PASS)
            e["src"], e["dst"], e["C"], e["op"], e["flip"] = src.data_ptr(), dst.data_ptr(), src.shape[0], op, p["flip"]
            e["n_rect"] = len(p["rects"])
            if p["rects"]:
                e["rect"][: len(p["rects"])] = p["rects"]
            for k, v in f.items():
                e[k] = v
            rows.append(e)
    return torch.from_numpy(np.stack(rows).view(np.uint8).reshape(-1)).cuda()


res = {"batch": B, "planes_per_sample": 299, "grid": [H, W]}
res["torch_copy_ms"] = timeit(lambda: (LO.copy_(L), MO.copy_(M)))
res["torch_copy_TBps"] = PL * 8 / res["torch_copy_ms"] / 1e9
cases = {"flip_copy": {"flip": True, "angle": None, "scale": None, "rects": [(100, 100, 40, 40)]},
         "rotate": {"flip": True, "angle": -12.5, "scale": None, "rects": []},
         "scale_down": {"flip": False, "angle": None, "scale": 0.957, "rects": []},
         "scale_up": {"flip": False, "angle": None, "scale": 1.043, "rects": [(10, 10, 30, 30)]}}
for name, p in cases.items():
    tab = table(p)
    ms = timeit(lambda: lib.ivit_bev_augment(ptr(tab), 2 * B, H, W, 290, stream()))
    res[name] = {"kernel_ms": round(ms, 4), "TBps_algorithmic": round(PL * 8 / ms / 1e9, 3),
                 "frac_of_8TBps": round(PL * 8 / ms / 1e9 / 8.0, 3)}
gts = [{"boxes_xywha": torch.zeros(20, 5), "intentions": torch.zeros(20, dtype=torch.long)} for _ in range(B)]
import random  # noqa: E402
random.seed(45)
res["augment_bev_batch_ms"] = round(timeit(lambda: utils.augment_bev_batch(L, M, gts, out=(LO, MO)), it=10), 3)
res["augment_bev_batch_samples_per_s"] = round(B / res["augment_bev_batch_ms"] * 1e3, 1)
print(json.dumps(res))
