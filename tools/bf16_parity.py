"""Diagnostic: HIP train step (bf16 or f32) vs the f32 oracle at a given grid; prints output /
loss errors and the per-parameter gradient rel-L2 errors (worst first). GPU only.

    python tools/bf16_parity.py --grid 400x720 --batch 2 --dtype bf16 --dp 0.1
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "visiontransformer-intention-prediction_amd"))

import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", default="400x720")
ap.add_argument("--batch", type=int, default=2)
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--dp", type=float, default=0.1)
ap.add_argument("--attn", default="explicit")
a = ap.parse_args()
H, W = (int(v) for v in a.grid.split("x"))
import test_gpu_model as T  # noqa: E402

if a.dtype == "f32":
    orig = T._model
    T._model = lambda cfg, cd=torch.float32, dp=0.0: orig(cfg, torch.float32, dp)
e, ea, gn = T._bf16_vs_oracle(H, W, a.batch, 1234, a.dp, a.attn, a.attn == "sdpa", 1e9)
for k, (o, am) in sorted(gn.items(), key=lambda kv: -kv[1][0])[:16]:
    print(f"{o:.3e} (autocast {am:.3e}) {k}")
