import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "visiontransformer-intention-prediction_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
import torch
import ops
from oracle import ivit_oracle as O
from oracle.weights import make_state_dict, model_cfg
import model_vit
cfg = model_cfg(img_size=(80, 120))
lidar, mp, gts = O.synthetic_batch(2, (80, 120), seed=5, box_region=(35.0, 60.0, -72.0, -48.0))
orig = ops.bn_backward
def run(l):
    rec = []
    def f(x, y, dy, st, g, relu, od, want_dr=False):
        rec.append((x.clone(), y.clone(), dy.clone(), st.mean.clone(), st.invstd.clone(), g.clone()))
        return orig(x, y, dy, st, g, relu, od, want_dr)
    ops.bn_backward = f
    m = model_vit.IntentNetViT(backbone_cfg={"img_size": (80, 120), "drop_path_rate_lidar": 0.0, "drop_path_rate_map": 0.0})
    m.load_state_dict(make_state_dict(cfg, seed=0)); m = m.cuda().train()
    c, bb, i = m(l.cuda(), mp.cuda())
    g = torch.Generator().manual_seed(9)
    wc, wb, wi = [torch.randn(x.shape, generator=g).cuda() for x in (c, bb, i)]
    ((c * wc).sum() + (bb * wb).sum() + (i * wi).sum()).backward()
    ops.bn_backward = orig
    return rec
a = run(lidar)
b = run(lidar * (1 + 1e-6 * torch.randn(lidar.shape, generator=torch.Generator().manual_seed(3))))
for k, (ra, rb) in enumerate(zip(a, b)):
    xa, ya, da, ma, ia, ga = ra
    xb, yb, db, mb, ib, gb = rb
    flips = ((ya > 0) != (yb > 0)).sum().item()
    print(k, "shape", tuple(xa.shape), "mask flips", flips, "pos frac", (ya > 0).float().mean().item(),
          "near0", ((ya > 0) & (ya < 1e-5)).sum().item(), "invstd max", ia.max().item(), "invstd diff", ((ia - ib).abs() / ia).max().item(),
          "mean diff", (ma - mb).abs().max().item(), "x diff", ((xa - xb).abs().max() / xa.abs().max()).item(),
          "dy diff", ((da - db).abs().max() / da.abs().max()).item(), "gamma", ga.abs().min().item())
