"""End-to-end parity of the HIP IntentNetViT (the product path) against the golden vectors
from the reference's own code and against the CPU oracle. f32 path: within 1e-3 rel
(north_star); bf16 path: bf16-appropriate tolerances; NMS indices bit-exact."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ivit_oracle as O
from oracle.weights import make_state_dict, model_cfg

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(cfg, cd=torch.float32, dp=0.0):
    import model_vit
    m = model_vit.IntentNetViT(backbone_cfg={"img_size": tuple(cfg["img_size"]), "drop_path_rate_lidar": dp,
                                             "drop_path_rate_map": dp})
    m.load_state_dict(make_state_dict(cfg, seed=0), strict=True)
    return m.to(DEV).set_compute_dtype(cd)


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def _gts(z, n):
    return [{"boxes_xywha": torch.from_numpy(z[f"gt{i}_boxes"]), "intentions": torch.from_numpy(z[f"gt{i}_ints"])}
            for i in range(n)]


@pytest.fixture(scope="module")
def small():
    z = golden("model_small.npz")
    cfg = json.loads(str(z["cfg"]))
    cfg["img_size"] = tuple(cfg["img_size"])
    lidar, mp, _ = O.synthetic_batch(2, cfg["img_size"], seed=1234)
    return z, cfg, lidar, mp


def test_small_eval_vs_golden(small):
    z, cfg, lidar, mp = small
    m = _model(cfg).eval()
    with torch.no_grad():
        c, b, i = m(lidar.to(DEV), mp.to(DEV))
    assert _rel(c, z["eval_cls"]) < 1e-3 and _rel(b, z["eval_box"]) < 1e-3 and _rel(i, z["eval_int"]) < 1e-3


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
def test_fusion_stride2_vs_golden(cd):
    """fusion_block_stride=2 (model_vit.py:55,125-128): strided block-0 conv1 / downsample as
    im2col + GEMM, heads at H/16 x W/16, effective_head_stride 16 — eval and train outputs, loss,
    parameter gradients and BN running stats vs the reference's own model (f32: 1e-3 rel; bf16:
    outputs within 6e-2)."""
    import loss as L
    import model_vit
    import utils
    z = golden("model_stride2.npz")
    cfg = json.loads(str(z["cfg"]))
    cfg["img_size"] = tuple(cfg["img_size"])
    m = model_vit.IntentNetViT(backbone_cfg={"img_size": cfg["img_size"], "drop_path_rate_lidar": 0.0,
                                             "drop_path_rate_map": 0.0, "fusion_block_stride": 2})
    assert m.effective_head_stride == 16
    m.load_state_dict(make_state_dict(cfg, seed=0), strict=True)
    m = m.to(DEV).set_compute_dtype(cd)
    lidar, mp, _ = O.synthetic_batch(2, cfg["img_size"], seed=1234)
    tol = 1e-3 if cd == torch.float32 else 6e-2
    m.eval()
    with torch.no_grad():
        c, b, i = m(lidar.to(DEV), mp.to(DEV))
    assert c.shape == (2, 30, 1) and b.shape == (2, 30, 6) and i.shape == (2, 30, 8)
    assert _rel(c, z["eval_cls"]) < tol and _rel(b, z["eval_box"]) < tol and _rel(i, z["eval_int"]) < tol
    m.train()
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    assert _rel(c.detach(), z["train_cls"]) < tol
    anchors = utils.generate_anchors(*cfg["img_size"], 16)
    assert np.array_equal(anchors.cpu().numpy(), z["anchors"])
    d = L.DetectionIntentionLoss(apply_intention_downsampling=False)(c, b, i, anchors, _gts(golden("model_small.npz"), 2))
    got = [float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
           float(d["num_pos_anchors"])]
    np.testing.assert_allclose(got, z["train_loss"], rtol=1e-3 if cd == torch.float32 else 5e-2)
    if cd != torch.float32:
        return
    d["loss"].backward()
    sd = dict(m.named_parameters())
    for name, gas, smp, st in zip(z["grad_names"], z["grad_abssum"], z["grad_samples"], z["grad_strides"]):
        g = sd[str(name)].grad
        assert g is not None, name
        assert float(g.double().abs().sum()) == pytest.approx(gas, rel=1e-3, abs=1e-6), name
    bufs = dict(m.named_buffers())
    for name, val in zip(z["bn_names"], z["bn_values"]):
        np.testing.assert_allclose(bufs[str(name)].cpu().numpy(), val, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
def test_regrid_patch16_map_vs_golden(cd):
    """A patch-16 map ViT (vit_small_patch16_224 at model_vit.py:71): generic patch embedding
    (ivit_patch_im2col_p + linear + ivit_patch_tokens), the map features re-gridded onto the LiDAR
    grid by ivit_bilinear_fwd (model_vit.py:139), the bilinear adjoint in backward — eval and
    train outputs, loss, parameter gradients and BN running stats vs the reference's own model
    (f32: 1e-3 rel; bf16: outputs within 6e-2)."""
    import loss as L
    import model_vit
    import utils
    z = golden("model_regrid.npz")
    cfg = json.loads(str(z["cfg"]))
    cfg["img_size"] = tuple(cfg["img_size"])
    with pytest.warns(UserWarning, match="differ"):
        m = model_vit.IntentNetViT(backbone_cfg={"img_size": cfg["img_size"], "drop_path_rate_lidar": 0.0,
                                                 "drop_path_rate_map": 0.0,
                                                 "vit_model_name_map": "vit_small_patch16_224"})
    assert m.backbone.map_grid_size == (2, 3) and m.backbone.lidar_grid_size == (4, 6)
    assert m.effective_head_stride == 8
    m.load_state_dict(make_state_dict(cfg, seed=0), strict=True)
    m = m.to(DEV).set_compute_dtype(cd)
    lidar, mp, _ = O.synthetic_batch(2, cfg["img_size"], seed=1234)
    tol = 1e-3 if cd == torch.float32 else 6e-2
    m.eval()
    with torch.no_grad():
        c, b, i = m(lidar.to(DEV), mp.to(DEV))
    assert c.shape == (2, 120, 1) and b.shape == (2, 120, 6) and i.shape == (2, 120, 8)
    assert _rel(c, z["eval_cls"]) < tol and _rel(b, z["eval_box"]) < tol and _rel(i, z["eval_int"]) < tol
    m.train()
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    assert _rel(c.detach(), z["train_cls"]) < tol
    anchors = utils.generate_anchors(*cfg["img_size"], 8)
    assert np.array_equal(anchors.cpu().numpy(), z["anchors"])
    d = L.DetectionIntentionLoss(apply_intention_downsampling=False)(c, b, i, anchors, _gts(golden("model_small.npz"), 2))
    got = [float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
           float(d["num_pos_anchors"])]
    np.testing.assert_allclose(got, z["train_loss"], rtol=1e-3 if cd == torch.float32 else 5e-2)
    if cd != torch.float32:
        return
    d["loss"].backward()
    sd = dict(m.named_parameters())
    for name, gas, smp, st in zip(z["grad_names"], z["grad_abssum"], z["grad_samples"], z["grad_strides"]):
        g = sd[str(name)].grad
        assert g is not None, name
        assert float(g.double().abs().sum()) == pytest.approx(gas, rel=1e-3, abs=1e-6), name
    bufs = dict(m.named_buffers())
    for name, val in zip(z["bn_names"], z["bn_values"]):
        np.testing.assert_allclose(bufs[str(name)].cpu().numpy(), val, rtol=1e-4, atol=1e-5)


def test_small_train_loss_grads_vs_golden(small):
    import loss as L
    import utils
    z, cfg, lidar, mp = small
    m = _model(cfg).train()
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    assert _rel(c.detach(), z["train_cls"]) < 1e-3
    anchors = utils.generate_anchors(*cfg["img_size"], 8)
    assert np.array_equal(anchors.cpu().numpy(), z["anchors"])
    lf = L.DetectionIntentionLoss(apply_intention_downsampling=False)
    d = lf(c, b, i, anchors, _gts(z, 2))
    got = [float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
           float(d["num_pos_anchors"])]
    np.testing.assert_allclose(got, z["train_loss"], rtol=1e-3)
    d["loss"].backward()
    sd = dict(m.named_parameters())
    for name, gas, smp, st in zip(z["grad_names"], z["grad_abssum"], z["grad_samples"], z["grad_strides"]):
        g = sd[str(name)].grad
        assert g is not None, name
        assert float(g.double().abs().sum()) == pytest.approx(gas, rel=1e-3, abs=1e-6), name
        s = g.reshape(-1).double()[:: int(st)][:64].cpu().numpy()
        ref = smp[~np.isnan(smp)][: s.size]
        assert np.abs(s - ref).max() <= 1e-3 * max(np.abs(ref).max(), 1e-6) + 1e-7, name
    bufs = dict(m.named_buffers())
    for name, val in zip(z["bn_names"], z["bn_values"]):
        np.testing.assert_allclose(bufs[str(name)].cpu().numpy(), val, rtol=1e-4, atol=1e-5)


def test_loss_full_size_vs_golden():
    import loss as L
    import utils
    z = golden("geometry.npz")
    anchors = utils.generate_anchors(400, 720, 8)
    g = torch.Generator().manual_seed(int(z["logits_seed"][0]))
    NA = anchors.shape[0]
    cls = torch.randn((2, NA, 1), generator=g)
    box = 0.5 * torch.randn((2, NA, 6), generator=g)
    it = torch.randn((2, NA, 8), generator=g)
    gts = _gts(z, 2)
    d = L.DetectionIntentionLoss(apply_intention_downsampling=False)(cls.to(DEV), box.to(DEV), it.to(DEV), anchors,
                                                                      gts)
    got = [float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
           float(d["num_pos_anchors"])]
    np.testing.assert_allclose(got, z["loss_full"], rtol=2e-5)
    empty = [{"boxes_xywha": torch.zeros((0, 5)), "intentions": torch.zeros((0,), dtype=torch.long)}, {}]
    d = L.DetectionIntentionLoss(apply_intention_downsampling=False)(cls.to(DEV), box.to(DEV), it.to(DEV), anchors,
                                                                      empty)
    got = [float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
           float(d["num_pos_anchors"])]
    np.testing.assert_allclose(got, z["loss_empty"], rtol=2e-5)


@pytest.mark.parametrize("downsampling", [False, True])
def test_loss_grads_vs_oracle(downsampling):
    import loss as L
    import utils
    z = golden("geometry.npz")
    anchors = utils.generate_anchors(400, 720, 8)
    NA = anchors.shape[0]
    g = torch.Generator().manual_seed(21)
    cls = torch.randn((2, NA, 1), generator=g)
    box = 0.5 * torch.randn((2, NA, 6), generator=g)
    it = torch.randn((2, NA, 8), generator=g)
    keep = (torch.rand((2, NA), generator=g) < 0.15).float()
    gts = _gts(z, 2)
    ts = [t.clone().to(DEV).requires_grad_(True) for t in (cls, box, it)]
    d = L.DetectionIntentionLoss(apply_intention_downsampling=downsampling)(*ts, anchors, gts, intent_keep=keep)
    d["loss"].backward()
    rs = [t.clone().double().requires_grad_(True) for t in (cls, box, it)]
    ref = O.detection_loss(*rs, anchors.cpu().double(), [{k: v.double() if v.is_floating_point() else v
                                                          for k, v in gg.items()} for gg in gts],
                           downsampling=downsampling, keep=keep)
    ref["loss"].backward()
    assert float(d["loss"]) == pytest.approx(float(ref["loss"]), rel=1e-5)
    for a, r in zip(ts, rs):
        assert _rel(a.grad, r.grad) < 1e-4


def test_medium_grid_fp32_vs_oracle():
    """80x120 grid (N=151 tokens: attention tails, 2 q-blocks) — HIP f32 vs CPU oracle, fwd + grads."""
    cfg = model_cfg(img_size=(80, 120))
    lidar, mp, gts = O.synthetic_batch(2, (80, 120), seed=5, box_region=(35.0, 60.0, -72.0, -48.0))
    m = _model(cfg).train()
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    sd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v.clone())
          for k, v in make_state_dict(cfg, seed=0).items()}
    rc, rb, ri = O.intentnet_forward(sd, lidar, mp, cfg, training=True)
    assert _rel(c.detach(), rc.detach()) < 1e-3 and _rel(i.detach(), ri.detach()) < 1e-3
    g = torch.Generator().manual_seed(9)
    wc, wb, wi = torch.randn(rc.shape, generator=g), torch.randn(rb.shape, generator=g), torch.randn(ri.shape, generator=g)
    ((c * wc.to(DEV)).sum() + (b * wb.to(DEV)).sum() + (i * wi.to(DEV)).sum()).backward()
    ((rc * wc).sum() + (rb * wb).sum() + (ri * wi).sum()).backward()
    # Gradient parity through train-mode BN + ReLU: an activation within f32 rounding of the ReLU
    # kink can land on either side in two correct f32 implementations. tools/fusion_debug2.py
    # found exactly one such element in this input (a 1e-6 input perturbation flips it on the
    # GPU); its O(1) change reaches every upstream gradient through the BN batch-statistic
    # terms at the ~2e-3 level. The bar here is therefore a per-tensor relative L2 error of
    # 5e-3 (an indexing or tail bug shows up at >= 1e-1); the strict 1e-3 max-abs bar on
    # gradients is held by test_small_train_loss_grads_vs_golden, and forward outputs above.
    params = dict(m.named_parameters())
    worst = []
    for k, p in params.items():
        a, r = p.grad.double().cpu(), sd[k].grad.double()
        worst.append((float((a - r).norm() / (r.norm() + 1e-30)), _rel(a, r), k))
    worst.sort(reverse=True)
    print("worst grad (l2 rel, max-abs rel):", worst[:6])
    assert worst[0][0] < 5e-3, worst[:6]


def test_bf16_path_close_to_fp32(small):
    z, cfg, lidar, mp = small
    m32 = _model(cfg).eval()
    m16 = _model(cfg, torch.bfloat16).eval()
    with torch.no_grad():
        a = m32(lidar.to(DEV), mp.to(DEV))
        b = m16(lidar.to(DEV), mp.to(DEV))
    for x, y in zip(a, b):
        assert _rel(y, x) < 6e-2


def _dp_scales(B, depth=12, rate=0.1, seed=0):
    """Per-block (attn_scale[B], mlp_scale[B]) with timm DropPath's values {0, 1/(1-p_i)},
    p_i = linspace(0, rate, depth)[i]; block 0 (p = 0) is the identity. Every sample is
    dropped somewhere, and both branches drop in some block."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for i, p in enumerate(torch.linspace(0, rate, depth).tolist()):
        if p <= 0.0:
            out.append((torch.ones(B), torch.ones(B)))
            continue
        keep = (torch.rand((2, B), generator=g) > 0.3).float()
        keep[i % 2, (i // 2) % B] = 0.0
        s = keep / (1.0 - p)
        out.append((s[0], s[1]))
    return out


def _set_dp(m, dl, dm):
    m.backbone.vit_lidar.set_drop_path_scales(dl)
    m.backbone.vit_map.set_drop_path_scales(dm)


def test_drop_path_injected_vs_oracle():
    """Train mode with the reference's default drop_path_rate 0.1 (model_vit.py:64,71; timm
    DropPath): the same per-sample factors injected into the HIP blocks and into the oracle,
    f32, 80x120 grid — forward and parameter gradients (same bar as the medium-grid test)."""
    cfg = model_cfg(img_size=(80, 120))
    lidar, mp, _ = O.synthetic_batch(2, (80, 120), seed=5, box_region=(35.0, 60.0, -72.0, -48.0))
    m = _model(cfg, dp=0.1).train()
    dl, dm = _dp_scales(2, seed=1), _dp_scales(2, seed=2)
    _set_dp(m, dl, dm)
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    blk = m.backbone.vit_lidar.blocks[5]
    assert torch.equal(blk.last_scales[0].cpu(), dl[5][0]) and torch.equal(blk.last_scales[1].cpu(), dl[5][1])
    sd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v.clone())
          for k, v in make_state_dict(cfg, seed=0).items()}
    rc, rb, ri = O.intentnet_forward(sd, lidar, mp, cfg, training=True, drop_path_scales=(dl, dm))
    assert _rel(c.detach(), rc.detach()) < 1e-3 and _rel(b.detach(), rb.detach()) < 1e-3
    assert _rel(i.detach(), ri.detach()) < 1e-3
    with torch.no_grad():  # the scales matter: without them the oracle differs
        nc, _, _ = O.intentnet_forward({k: v.detach().clone() for k, v in make_state_dict(cfg, seed=0).items()},
                                       lidar, mp, cfg, training=True)
    assert _rel(nc, rc.detach()) > 1e-2
    g = torch.Generator().manual_seed(9)
    wc, wb, wi = torch.randn(rc.shape, generator=g), torch.randn(rb.shape, generator=g), torch.randn(ri.shape, generator=g)
    ((c * wc.to(DEV)).sum() + (b * wb.to(DEV)).sum() + (i * wi.to(DEV)).sum()).backward()
    ((rc * wc).sum() + (rb * wb).sum() + (ri * wi).sum()).backward()
    worst = sorted(((float((p.grad.double().cpu() - sd[k].grad.double()).norm() / (sd[k].grad.double().norm() + 1e-30)), k)
                    for k, p in m.named_parameters()), reverse=True)
    assert worst[0][0] < 5e-3, worst[:6]
    # the drawn (non-injected) masks take timm's values {0, 1/(1-p)}
    _set_dp(m, None, None)
    m(lidar.to(DEV), mp.to(DEV))
    p11 = m.backbone.vit_map.blocks[11].drop_path_rate
    vals = set(torch.cat(m.backbone.vit_map.blocks[11].last_scales).cpu().tolist())
    assert all(v == 0.0 or abs(v - 1.0 / (1.0 - p11)) < 1e-6 for v in vals), vals


def _oracle_step(cfg, lidar, mp, gts, keep, sc, attn, checkpoint, autocast, dtype=torch.float32):
    """The oracle's train step (forward, loss, backward) on the GPU with torch's own kernels:
    f32 (or f64: the conditioning reference of the config-1 test), or under torch.autocast(bf16) —
    the reference's mixed-precision form (timm's fused SDPA + bf16 linears / convs, f32 LayerNorm /
    softmax stats / loss)."""
    fl = lambda v: v.to(dtype) if v.is_floating_point() else v  # noqa: E731
    sd = {k: (fl(v.clone().to(DEV)).requires_grad_(True) if v.is_floating_point() and "running" not in k
              else fl(v.clone().to(DEV))) for k, v in make_state_dict(cfg, seed=0).items()}
    scd = None if sc is None else tuple([(fl(a.to(DEV)), fl(b_.to(DEV))) for a, b_ in s] for s in sc)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        rc, rb, ri = O.intentnet_forward(sd, fl(lidar.to(DEV)), fl(mp.to(DEV)), cfg, training=True,
                                         drop_path_scales=scd, attn=attn, checkpoint=checkpoint)
    if dtype == torch.float32:
        rc, rb, ri = rc.float(), rb.float(), ri.float()
    anchors = fl(O.generate_anchors(*cfg["img_size"]))
    gts_ = [{k: fl(v) for k, v in g.items()} for g in gts]
    rd = O.detection_loss(rc.cpu(), rb.cpu(), ri.cpu(), anchors, gts_, downsampling=True,
                          keep=None if keep is None else fl(keep))
    rd["loss"].backward()
    return (rc.detach(), rb.detach(), ri.detach()), rd, {k: v.grad for k, v in sd.items() if v.grad is not None}


def _bf16_vs_oracle(H, W, B, seed, dp, attn, checkpoint, slack):
    """bf16 HIP train step vs the f32 oracle on the same inputs / weights / DropPath factors
    (outputs, loss terms, every parameter gradient), judged against the error the reference's
    own bf16 mixed precision (the oracle under torch.autocast, torch's kernels) makes vs the
    same f32 oracle: ours must stay within ``slack`` x that error (+ a small floor). The oracle
    (plain PyTorch, pinned to the reference goldens on the CPU) runs on the GPU with torch's
    kernels — independent of this build's — because the full-grid f32 step does not fit a CPU
    test budget. Returns (errors, autocast errors, per-parameter (ours, autocast) grad errors)."""
    import loss as L
    import utils
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    cfg = model_cfg(img_size=(H, W))
    m = _model(cfg, torch.bfloat16, dp=dp).train()
    sc = (_dp_scales(B, seed=3), _dp_scales(B, seed=4)) if dp > 0 else None
    if sc is not None:
        _set_dp(m, *sc)
    lidar, mp, gts = O.synthetic_batch(B, (H, W), seed=seed, grid_scale=H / 400.0)
    anchors = utils.generate_anchors(H, W, 8, device=DEV)
    keep = (torch.rand((B, anchors.shape[0]), generator=torch.Generator().manual_seed(seed)) < 0.15).float()
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    d = L.DetectionIntentionLoss()(c, b, i, anchors, gts, intent_keep=keep)
    d["loss"].backward()
    ours = ((c.detach(), b.detach(), i.detach()), d, {k: p.grad for k, p in m.named_parameters()})
    del m
    ref = _oracle_step(cfg, lidar, mp, gts, keep, sc, attn, checkpoint, autocast=False)
    amp = _oracle_step(cfg, lidar, mp, gts, keep, sc, "sdpa", checkpoint, autocast=True)

    def errs(run):
        e = {k: _rel(x, y) for k, x, y in zip(("cls", "box", "int"), run[0], ref[0])}
        for k in ("loss", "cls_loss", "box_loss", "intent_loss"):
            e[k] = abs(float(run[1][k]) - float(ref[1][k])) / max(abs(float(ref[1][k])), 1e-12)
        return e

    e_ours, e_amp = errs(ours), errs(amp)
    assert int(d["num_pos_anchors"]) == int(ref[1]["num_pos_anchors"])
    gn = {}
    for k, r in ref[2].items():
        rn = r.double().norm() + 1e-30
        gn[k] = (float((ours[2][k].double() - r.double()).norm() / rn), float((amp[2][k].double() - r.double()).norm() / rn))
    worst = sorted(((o / (a + 1e-3), o, a, k) for k, (o, a) in gn.items()), reverse=True)
    print(f"bf16 vs f32 oracle {H}x{W} B={B}: ours", e_ours, "\n  torch autocast bf16", e_amp,
          "\n  worst grad rel-L2 (ratio, ours, autocast, name):", worst[:5],
          "\n  max grad rel-L2 ours", max(o for o, _ in gn.values()), "autocast", max(a for _, a in gn.values()))
    for k in e_ours:
        assert e_ours[k] <= slack * e_amp[k] + 2e-3, (k, e_ours, e_amp)
    for k, (o, a) in gn.items():
        assert o <= slack * a + 1e-2, (k, o, a)
    return e_ours, e_amp, gn


# ours may be at most 1.5x the error of torch's own bf16 autocast path vs the f32 oracle
# (+ 2e-3 on outputs / losses, + 1e-2 on gradient rel-L2): bf16 noise, not a kernel defect.
# Measured (profiles/r02_bf16_parity.txt): ours is below autocast on every output / loss term
# and on nearly every gradient (400x720: outputs 2.0e-2 vs 2.7e-2, worst grad 0.17 vs 0.20).
BF16_SLACK = 1.5


def test_full_grid_bf16_train_step_vs_oracle():
    """BASELINE config 2 shape (400x720, real channels / depth / width), B=2, bf16, DropPath 0.1
    injected: outputs, loss and every parameter gradient vs the f32 oracle. Blocks 0..10 of both
    ViTs take their scaled fc2-dgrad operand from the next block's backward, and each patch
    embedding its bf16 token gradient from block 0's (ops.GradHandoff)."""
    import ops
    before = ops.GradHandoff.used
    _bf16_vs_oracle(400, 720, 2, 1234, 0.1, "explicit", False, BF16_SLACK)
    assert ops.GradHandoff.used - before == 2 * 12


def test_full_grid_bf16_train_step_batch8_vs_oracle():
    """BASELINE config 2 at the benchmarked batch (400x720, B = 8, bf16, DropPath 0.1 injected):
    outputs, loss terms and every parameter gradient vs the f32 oracle (SDPA attention, per-block
    checkpointing for memory), judged as the B = 2 test (train_vit.py:151-187)."""
    _bf16_vs_oracle(400, 720, 8, 4321, 0.1, "sdpa", True, BF16_SLACK)


def test_large_grid_bf16_train_step_vs_oracle():
    """BASELINE config 5 shape (800x1440, N = 18001 tokens, 90000 anchors), B=1, bf16: vs the
    f32 oracle (SDPA attention, per-block checkpointing for memory)."""
    _bf16_vs_oracle(800, 1440, 1, 1234, 0.1, "sdpa", True, BF16_SLACK)


def test_full_grid_bf16_fused_adamw_step():
    """constants.py grid, B=2, bf16 forward + loss + backward + fused AdamW: finite, parameters move."""
    import loss as L
    import utils
    from optim import FusedAdamW
    cfg = model_cfg()
    m = _model(cfg, torch.bfloat16, dp=0.1).train()
    lidar, mp, gts = O.synthetic_batch(2, seed=1234)
    anchors = utils.generate_anchors()
    opt = FusedAdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    lf = L.DetectionIntentionLoss()
    w0 = m.det_head.conv.weight.detach().clone()
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    d = lf(c, b, i, anchors, gts)
    d["loss"].backward()
    opt.step()
    torch.cuda.synchronize()
    assert torch.isfinite(d["loss"]).item()
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all().item(), n
    assert not torch.equal(w0, m.det_head.conv.weight.detach())


def test_fused_adamw_refreshes_packed_weights():
    """FusedAdamW updates parameters through device pointer tables (no version bump), so the bf16
    shadows and the row-panel weight packs the next forward reads are rewritten in the same launch
    (ivit_adamw_chunked). After a large-lr step, the next forward must equal a forward with every
    cached copy rebuilt from the updated f32 weights; the packs must equal freshly built ones; and a
    device finite flag of 0 must leave weights and moments bit-identical."""
    import loss as L
    import ops
    import utils
    from optim import FusedAdamW
    cfg = model_cfg(img_size=(64, 96))
    m = _model(cfg, torch.bfloat16).train()
    lidar, mp, gts = O.synthetic_batch(2, (64, 96), seed=77, grid_scale=64 / 400.0)
    lidar, mp = lidar.to(DEV), mp.to(DEV)
    anchors = utils.generate_anchors(64, 96, 8, device=DEV)
    opt = FusedAdamW(m.parameters(), lr=1e-2, weight_decay=1e-4)
    lf = L.DetectionIntentionLoss()
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        c, b, i = m(lidar, mp)
        lf(c, b, i, anchors, gts)["loss"].backward()
        opt.step()
    n_packs = 0
    for p in m.parameters():
        pk, pkt = ops.packs_of(p)
        if pk is not None:
            fresh = torch.empty_like(pk)
            ops.lib.ivit_patch_weight_pack(ops.ptr(p.detach().contiguous()), p.shape[0], p[0].numel() // 64,
                                           ops.ptr(fresh), ops.stream())
            assert torch.equal(pk, fresh)
            n_packs += 1
        if pkt is not None:
            fresh = torch.empty_like(pkt)
            ops.lib.ivit_weight_pack_t(ops.ptr(p.detach().contiguous()), p.shape[0], p.shape[1], ops.ptr(fresh),
                                       ops.stream())
            assert torch.equal(pkt, fresh)
            n_packs += 1
        sh = ops.shadow_of(p)
        if sh is not None:
            assert torch.equal(sh, p.detach().to(torch.bfloat16))
    assert n_packs >= 2 * 12 * 7 + 2  # per block: 4 packs + 3 transposed packs, + the patch embeddings
    m.eval()
    with torch.no_grad():
        got = m(lidar, mp)
        for cache in (ops._PACKED, ops._PACKED_T, ops._SHADOWS):
            cache.clear()
        want = m(lidar, mp)
    for g_, w_ in zip(got, want):
        assert torch.equal(g_, w_)
    # a 0 finite flag: nothing moves (loss.py:190-198 guard without a host sync)
    m.train()
    c, b, i = m(lidar, mp)
    lf(c, b, i, anchors, gts)["loss"].backward()
    before = [p.detach().clone() for p in m.parameters()]
    mom = [opt.state[p]["exp_avg"].clone() for p in m.parameters()]
    opt.step(finite=torch.zeros((), device=DEV))
    assert all(torch.equal(a, p.detach()) for a, p in zip(before, m.parameters()))
    assert all(torch.equal(a, opt.state[p]["exp_avg"]) for a, p in zip(mom, m.parameters()))
    opt.step(finite=torch.ones((), device=DEV))
    assert not all(torch.equal(a, p.detach()) for a, p in zip(before, m.parameters()))


def test_large_grid_bf16_train_step_finite():
    """BASELINE config 5 (2x BEV resolution, 800x1440: 100x180 patches, N = 18001 tokens,
    90 000 anchors), B=1, bf16 train step: finite loss and gradients, anchors at the 2x grid."""
    import loss as L
    import utils
    import model_vit
    from optim import FusedAdamW
    from synthetic import synthetic_batch
    H, W = 800, 1440
    torch.manual_seed(0)
    m = model_vit.IntentNetViT(backbone_cfg={"img_size": (H, W)}).to(DEV).set_compute_dtype(torch.bfloat16).train()
    batch = synthetic_batch(1, (H, W), torch.Generator().manual_seed(1234), device=DEV)
    anchors = utils.generate_anchors(H, W, 8, device=DEV)
    assert anchors.shape == (90000, 5)
    ra = O.generate_anchors(H, W)
    assert torch.equal(anchors.cpu(), ra)
    opt = FusedAdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    c, b, i = m(batch["lidar_bev"], batch["map_bev"])
    assert c.shape == (1, 90000, 1) and b.shape == (1, 90000, 6) and i.shape == (1, 90000, 8)
    d = L.DetectionIntentionLoss()(c, b, i, anchors, batch["gt_list"])
    d["loss"].backward()
    opt.step()
    torch.cuda.synchronize()
    assert torch.isfinite(d["loss"]).item() and d["num_pos_anchors"] > 0
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all().item(), n


def test_full_grid_fp32_forward_vs_oracle():
    cfg = model_cfg()
    lidar, mp, _ = O.synthetic_batch(1, seed=1234)
    m = _model(cfg).eval()
    with torch.no_grad():
        c, b, i = m(lidar.to(DEV), mp.to(DEV))
        sd = make_state_dict(cfg, seed=0)
        rc, rb, ri = O.intentnet_forward(sd, lidar, mp, cfg, training=False)
    assert _rel(c, rc) < 1e-3 and _rel(b, rb) < 1e-3 and _rel(i, ri) < 1e-3


def test_config1_fp32_full_grid_train_step_vs_oracle():
    """BASELINE config 1's workload on the HIP f32 path: IntentNetViT fp32, B = 1, the constants.py
    grid (400x720, N = 4501 tokens per stream), train mode with the reference's DropPath 0.1
    (factors injected into both), forward + DetectionIntentionLoss (downsampling keep mask
    injected) + backward (train_vit.py:29,151-173) against the oracle's f32 step (plain PyTorch f32,
    explicit attention, run on the GPU with torch's kernels: the CPU oracle step takes minutes).
    Bars: outputs and loss terms 1e-3 relative (north_star). Parameter gradients, per tensor
    (relative L2): within 1e-3 of the f32 oracle, or — where train-mode BatchNorm + ReLU make the
    step ill-conditioned in f32 (an activation within f32 rounding of a ReLU kink lands on either
    side in two correct f32 implementations, and the BN batch-statistic terms carry the O(1) change
    to every upstream gradient) — no further from the same oracle computed in f64 than 2x the f32
    oracle's own distance from it (+1e-4): the HIP f32 step is then as exact as the reference's own
    f32 arithmetic allows. The per-parameter table goes to gpurun_out/config1_grads.txt."""
    import loss as L
    import utils
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    H, W, B, seed = 400, 720, 1, 2024
    cfg = model_cfg(img_size=(H, W))
    m = _model(cfg, torch.float32, dp=0.1).train()
    sc = (_dp_scales(B, seed=5), _dp_scales(B, seed=6))
    _set_dp(m, *sc)
    lidar, mp, gts = O.synthetic_batch(B, (H, W), seed=seed)
    anchors = utils.generate_anchors(H, W, 8, device=DEV)
    keep = (torch.rand((B, anchors.shape[0]), generator=torch.Generator().manual_seed(seed)) < 0.15).float()
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    d = L.DetectionIntentionLoss()(c, b, i, anchors, gts, intent_keep=keep)
    d["loss"].backward()
    ours = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters()}
    outs = (c.detach(), b.detach(), i.detach())
    d = {k: float(v.detach()) for k, v in d.items() if k != "num_pos_anchors"} | {"num_pos_anchors": int(d["num_pos_anchors"])}
    del m, c, b, i
    (rc, rb, ri), rd, rg = _oracle_step(cfg, lidar, mp, gts, keep, sc, "explicit", False, autocast=False)
    rg = {k: v.double().cpu() for k, v in rg.items()}
    e_out = {k: _rel(x, y) for k, x, y in zip(("cls", "box", "int"), outs, (rc, rb, ri))}
    for k in ("loss", "cls_loss", "box_loss", "intent_loss"):
        e_out[k] = abs(d[k] - float(rd[k])) / max(abs(float(rd[k])), 1e-12)
    assert d["num_pos_anchors"] == int(rd["num_pos_anchors"])
    del rc, rb, ri, rd
    torch.cuda.empty_cache()
    _, _, r64 = _oracle_step(cfg, lidar, mp, gts, keep, sc, "explicit", False, autocast=False, dtype=torch.float64)
    r64 = {k: v.double().cpu() for k, v in r64.items()}
    l2 = lambda a, r: float((a - r).norm() / (r.norm() + 1e-30))  # noqa: E731
    rows = sorted(((l2(ours[k], rg[k]), l2(ours[k], r64[k]), l2(rg[k], r64[k]), k) for k in rg), reverse=True)
    n_strict = sum(1 for e, _, _, _ in rows if e < 1e-3)
    bad = [r for r in rows if not (r[0] < 1e-3 or r[1] <= 2 * r[2] + 1e-4)]
    lines = [f"config 1: IntentNetViT fp32, B = 1, 400x720, train mode (DropPath 0.1 injected), loss + backward; "
             f"HIP f32 step vs the oracle's f32 step (o32) and the oracle in f64 (o64), torch kernels on the GPU",
             f"outputs / loss terms (relative; bar 1e-3): " + ", ".join(f"{k} {v:.2e}" for k, v in e_out.items()),
             f"parameter gradients within 1e-3 (relative L2) of o32: {n_strict} of {len(rows)}",
             f"bar for the rest: |ours - o64| <= 2 |o32 - o64| + 1e-4; failing: {len(bad)}",
             f"{'ours-o32':>10} {'ours-o64':>10} {'o32-o64':>10}  parameter"]
    lines += [f"{a:10.3e} {b_:10.3e} {c_:10.3e}  {k}" for a, b_, c_, k in rows]
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "config1_grads.txt"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines[:10]))
    assert len(rows) == len(ours)
    for k, e in e_out.items():
        assert e < 1e-3, (k, e_out)
    assert not bad, bad[:6]


def test_config4_eval_batch32_full_grid_vs_oracle():
    """BASELINE config 4 end to end (eval_vit.py:136-187): B = 32 full-grid bf16 inference, then
    sigmoid >= 0.1, decode, NMS(0.2), intention argmax for all 32 samples through the batched
    device post-processing (ivit_eval_post), against the oracle: decode within 1e-5 rel of the
    oracle's decode, NMS keep indices bit-exact (torchvision CPU semantics) per sample on the same
    boxes / scores, scores and intentions equal."""
    import model_vit
    import utils
    from synthetic import synthetic_batch
    torch.manual_seed(0)
    m = model_vit.IntentNetViT(backbone_cfg={"img_size": (400, 720)}).to(DEV).set_compute_dtype(torch.bfloat16).eval()
    batch = synthetic_batch(32, (400, 720), torch.Generator().manual_seed(1234), device=DEV)
    anchors = utils.generate_anchors(400, 720, 8, device=DEV)
    with torch.inference_mode():
        cls, box, it = m(batch["lidar_bev"], batch["map_bev"])
        preds = utils.postprocess_batch(cls, box, it, anchors, 0.1, 0.2)
    assert len(preds) == 32
    a_cpu = anchors.cpu()
    total = 0
    for b in range(32):
        sc = torch.sigmoid(cls[b].reshape(-1).float())
        idx = torch.nonzero(sc >= 0.1).squeeze(1)
        dec = utils.decode_box_predictions(box[b].reshape(-1, 6)[idx], anchors[idx])
        rdec = O.decode_boxes(box[b].reshape(-1, 6)[idx].float().cpu(), a_cpu[idx.cpu()])
        assert _rel(dec, rdec) < 1e-5
        keep = O.nms_numpy(dec.cpu().numpy(), sc[idx].cpu().numpy(), 0.2)
        p = preds[b]
        assert torch.equal(p["pred_scores"].cpu(), sc[idx].cpu()[keep])
        assert torch.equal(p["pred_boxes_xywha"].cpu(), dec.cpu()[keep])
        ri = torch.argmax(it[b].reshape(-1, 8)[idx].float().cpu()[keep], dim=-1)
        assert torch.equal(p["pred_intentions"].cpu(), ri)
        total += len(keep)
    assert total > 32 * 100  # random init: every anchor passes 0.1, NMS keeps thousands


def test_config4_batch32_forward_samples_vs_small_batch_and_oracle():
    """BASELINE config 4 forward at B = 32 (eval_vit.py:136-151), whose LiDAR raster holds 2.67e9
    elements (> 2^31): the outputs of samples {0, 15, 31} must equal those samples run at B = 3
    (every kernel is row / (batch, head) independent and BatchNorm uses its running statistics, so
    a batch-size-dependent indexing defect in the late samples would show here), and the B = 3
    outputs must match the f32 oracle (torch's kernels on the GPU, eval) within the bf16 bar of the
    train tests: 1.5x the error torch autocast-bf16 makes against the same oracle, + 2e-3."""
    import model_vit
    from synthetic import synthetic_batch
    torch.manual_seed(0)
    m = model_vit.IntentNetViT(backbone_cfg={"img_size": (400, 720)}).to(DEV).set_compute_dtype(torch.bfloat16).eval()
    batch = synthetic_batch(32, (400, 720), torch.Generator().manual_seed(1234), device=DEV)
    assert batch["lidar_bev"].numel() > 2 ** 31
    idx = torch.tensor([0, 15, 31], device=DEV)
    with torch.inference_mode():
        full = m(batch["lidar_bev"], batch["map_bev"])
        full = [t[idx].clone() for t in full]
        lid, mp = batch["lidar_bev"][idx].contiguous(), batch["map_bev"][idx].contiguous()
        del batch
        small = m(lid, mp)
    for f, s in zip(full, small):
        assert _rel(f, s) < 1e-6, _rel(f, s)
    sd = {k: v.detach().float().clone() for k, v in m.state_dict().items()}
    cfg = model_cfg()
    del m
    with torch.no_grad():
        ref = O.intentnet_forward(sd, lid, mp, cfg, training=False, attn="sdpa")
        with torch.autocast("cuda", dtype=torch.bfloat16):
            amp = O.intentnet_forward(sd, lid, mp, cfg, training=False, attn="sdpa")
    for k, s, r, a in zip(("cls", "box", "int"), small, ref, amp):
        e_ours, e_amp = _rel(s.float(), r.float()), _rel(a.float(), r.float())
        print(f"config-4 B=3 {k}: ours {e_ours:.3e} autocast {e_amp:.3e}")
        assert e_ours <= BF16_SLACK * e_amp + 2e-3, (k, e_ours, e_amp)


def test_loss_reference_rng_downsampling_vs_oracle():
    """downsample_rng="reference" reproduces the reference's own draws (loss.py:170-178): after the
    same torch.manual_seed, the keep mask must equal the one the reference's procedure builds on the
    same device — per dominant class in set iteration order, torch.rand(k, device) over its
    positives in flattened order — from the oracle's targets, and the loss / gradients must match
    the oracle fed that mask."""
    import loss as L
    import utils
    z = golden("geometry.npz")
    anchors = utils.generate_anchors(400, 720, 8)
    NA = anchors.shape[0]
    g = torch.Generator().manual_seed(33)
    cls = torch.randn((2, NA, 1), generator=g)
    box = 0.5 * torch.randn((2, NA, 6), generator=g)
    it = torch.randn((2, NA, 8), generator=g)
    gts = _gts(z, 2)
    lf = L.DetectionIntentionLoss(downsample_rng="reference")
    ts = [t.clone().to(DEV).requires_grad_(True) for t in (cls, box, it)]
    torch.manual_seed(2024)
    d = lf(*ts, anchors, gts)
    d["loss"].backward()
    got_keep = lf.last_keep.reshape(-1).cpu()
    # the reference's procedure, replayed from the oracle's targets with the same seed
    cls_t, _, int_t = O.assign_targets(anchors.cpu(), gts)
    ct, itf = cls_t.reshape(-1), int_t.reshape(-1)
    pos_idx = torch.nonzero(ct == 1).squeeze(1)
    itp = itf[pos_idx]
    want = torch.ones(2 * NA)
    torch.manual_seed(2024)
    drawn = 0
    for dcls in set(lf.dominant_intentions):
        sel = itp == dcls
        k = int(sel.sum())
        if k:
            want[pos_idx[sel]] = (torch.rand(k, device=DEV) < lf.intention_downsample_keep_prob).float().cpu()
            drawn += k
    assert drawn > 0
    dom = torch.zeros(2 * NA, dtype=torch.bool)
    dom[pos_idx] = torch.isin(itp, torch.tensor(sorted(lf.dominant_intentions)))
    assert torch.equal(got_keep[dom], want[dom])
    rs = [t.clone().double().requires_grad_(True) for t in (cls, box, it)]
    ref = O.detection_loss(*rs, anchors.cpu().double(), [{k: v.double() if v.is_floating_point() else v
                                                          for k, v in gg.items()} for gg in gts],
                           downsampling=True, keep=want.reshape(2, NA))
    ref["loss"].backward()
    assert float(d["loss"]) == pytest.approx(float(ref["loss"]), rel=1e-5)
    for a, r in zip(ts, rs):
        assert _rel(a.grad, r.grad) < 1e-4


def test_process_stream_method_vs_oracle(small):
    """TwoStreamViTBackbone._process_stream (model_vit.py:116-122) as a method: the LiDAR stream's
    adapted feature map (B, C, Hf, Wf) vs the oracle's restatement (f32, 1e-3), and None (the
    reference's error branch) when the token count does not match the grid."""
    z, cfg, lidar, mp = small
    m = _model(cfg).eval()
    bb = m.backbone
    with torch.no_grad():
        f = bb._process_stream(lidar.to(DEV), bb.vit_lidar, bb.lidar_num_prefix_tokens, bb.lidar_grid_size,
                               bb.adapter_lidar, "LiDAR")
        sd = make_state_dict(cfg, seed=0)
        ref = O._stream(sd, "lidar", lidar, 6, cfg.get("depth") or 12, None)
        bad = bb._process_stream(lidar.to(DEV), bb.vit_lidar, bb.lidar_num_prefix_tokens, (1, 1), bb.adapter_lidar,
                                 "LiDAR")
    assert f.shape == ref.shape
    assert _rel(f, ref) < 1e-3
    assert bad is None
