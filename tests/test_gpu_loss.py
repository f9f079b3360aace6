"""DetectionIntentionLoss option paths on the HIP kernels vs golden vectors from the reference's
own loss.py (oracle/make_golden.py gen_loss_options): intention class weights (loss.py:40-45),
rotated IoU assignment (loss.py:81), and the NaN / Inf guard (loss.py:190-198) — including the
train step, which must leave weights and optimizer state bit-identical when the guard fires."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle.weights import make_state_dict, model_cfg

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gts(z, pre, n=2):
    return [{"boxes_xywha": torch.from_numpy(z[f"{pre}_gt{i}_boxes"]),
             "intentions": torch.from_numpy(z[f"{pre}_gt{i}_ints"])} for i in range(n)]


def _vec(d):
    return np.array([float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
                     float(d["num_pos_anchors"])])


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def test_loss_class_weights_vs_golden():
    import loss as L
    import utils
    z = golden("loss_options.npz")
    anchors = utils.generate_anchors(400, 720, 8)
    g = torch.Generator().manual_seed(int(z["cw_seed"][0]))
    NA = anchors.shape[0]
    ts = [torch.randn((2, NA, 1), generator=g), 0.5 * torch.randn((2, NA, 6), generator=g),
          torch.randn((2, NA, 8), generator=g)]
    ts = [t.to(DEV).requires_grad_(True) for t in ts]
    lf = L.DetectionIntentionLoss(apply_intention_downsampling=False,
                                  intention_class_weights=torch.from_numpy(z["cw_weights"])).to(DEV)
    d = lf(*ts, anchors, _gts(z, "cw"))
    np.testing.assert_allclose(_vec(d), z["cw_loss"], rtol=2e-5)
    d["loss"].backward()
    for t, k in zip(ts, ("cw_gcls", "cw_gbox", "cw_gint")):
        assert _rel(t.grad, z[k]) < 1e-4, k
    # with downsampling on, the weights are ignored (loss.py:41-42): cls / box terms unchanged
    lf2 = L.DetectionIntentionLoss(apply_intention_downsampling=True,
                                   intention_class_weights=torch.from_numpy(z["cw_weights"]))
    assert lf2.final_intention_class_weights is None
    d2 = lf2(*[t.detach() for t in ts], anchors, _gts(z, "cw"))
    np.testing.assert_allclose(_vec(d2)[:3][1:], z["cw_ds_loss_nods_terms"][1:], rtol=2e-5)


def test_loss_rotated_iou_vs_golden():
    import loss as L
    import utils
    z = golden("loss_options.npz")
    H, W = (int(v) for v in z["rot_grid"])
    anchors = utils.generate_anchors(H, W, 8)
    assert np.array_equal(anchors.cpu().numpy(), z["rot_anchors"])
    ts = [torch.from_numpy(z[k]).to(DEV).requires_grad_(True) for k in ("rot_cls", "rot_box", "rot_int")]
    d = L.DetectionIntentionLoss(apply_intention_downsampling=False, use_rotated_iou=True)(*ts, anchors,
                                                                                            _gts(z, "rot"))
    np.testing.assert_allclose(_vec(d), z["rot_loss"], rtol=1e-5)
    d["loss"].backward()
    for t, k in zip(ts, ("rot_gcls", "rot_gbox", "rot_gint")):
        assert _rel(t.grad, z[k]) < 1e-4, k
    d = L.DetectionIntentionLoss(apply_intention_downsampling=False)(*[t.detach() for t in ts], anchors,
                                                                      _gts(z, "rot"))
    np.testing.assert_allclose(_vec(d), z["rot_axis_loss"], rtol=1e-5)


def _poisoned(z, case):
    b, a, k, v = z[f"guard_{case}"]
    ts = [torch.from_numpy(z[n]).clone() for n in ("rot_cls", "rot_box", "rot_int")]
    ts[0 if "cls" in case else 2][int(b), int(a), int(k)] = v
    return ts


@pytest.mark.parametrize("case", ["nan_cls", "inf_cls_neg", "inf_int_pos"])
def test_loss_guard_vs_golden(case):
    """Non-finite total: loss and terms 0, num_pos as the reference, and exact-zero gradients
    (not NaN: a NaN per-anchor gradient x 0 would be NaN)."""
    import loss as L
    import utils
    z = golden("loss_options.npz")
    anchors = utils.generate_anchors(*(int(v) for v in z["rot_grid"]), 8)
    ts = [t.to(DEV).requires_grad_(True) for t in _poisoned(z, case)]
    lf = L.DetectionIntentionLoss(apply_intention_downsampling=False, sync_guard=False)
    d = lf(*ts, anchors, _gts(z, "rot"))
    np.testing.assert_array_equal(_vec(d), z[f"guard_{case}_loss"])
    assert float(lf.last_finite) == 0.0
    d["loss"].backward()
    for t in ts:
        assert t.grad is not None and torch.count_nonzero(t.grad).item() == 0


class _PoisonLoss:
    """DetectionIntentionLoss with one class logit forced to +Inf on a negative anchor."""

    def __init__(self, anchor):
        import loss as L
        self.inner = L.DetectionIntentionLoss()
        self.anchor = anchor

    @property
    def last_finite(self):
        return self.inner.last_finite

    def __call__(self, c, b, i, anchors, gts):
        mask = torch.zeros_like(c)
        mask[0, self.anchor, 0] = float("inf")
        return self.inner(c + mask, b, i, anchors, gts)


def test_train_step_guard_leaves_weights_bit_identical():
    """Trainer + FusedAdamW: a step whose loss is non-finite updates nothing (loss.py:190-198
    returns a disconnected zero leaf → no .grad → torch AdamW skips every parameter)."""
    import model_vit
    import utils
    from optim import FusedAdamW
    from oracle import ivit_oracle as O
    from trainer import Trainer
    cfg = model_cfg(img_size=(32, 48))
    m = model_vit.IntentNetViT(backbone_cfg={"img_size": (32, 48)})
    m.load_state_dict(make_state_dict(cfg, seed=0), strict=True)
    m = m.to(DEV).set_compute_dtype(torch.bfloat16).train()
    lidar, mp, gts = O.synthetic_batch(2, (32, 48), seed=1234, box_region=(54.0, 60.0, -72.0, -62.0))
    batch = {"lidar_bev": lidar.to(DEV), "map_bev": mp.to(DEV), "gt_list": gts}
    anchors = utils.generate_anchors(32, 48, 8, device=DEV)
    opt = FusedAdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    good = Trainer(m, _PoisonLoss(0).inner, opt, anchors, check_nan=True)
    assert good.step(batch) is not None  # a normal step first: Adam state exists
    w0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    s0 = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in opt.state[p].items()}
          for p in m.parameters()}
    bad = Trainer(m, _PoisonLoss(1), opt, anchors, check_nan=True)
    d = bad.step(batch)
    torch.cuda.synchronize()
    assert d is not None and float(d["loss"]) == 0.0 and bad.nonfinite == 1
    for k, v in m.state_dict().items():
        if "num_batches_tracked" in k or "running_" in k:
            continue  # BN statistics move in the forward, as in the reference
        assert torch.equal(v, w0[k]), k
    for p in m.parameters():
        for k, v in opt.state[p].items():
            ref = s0[id(p)][k]
            assert (torch.equal(v, ref) if torch.is_tensor(v) else v == ref), k


@pytest.mark.parametrize("case", ["nan_cls", "inf_int_pos"])
def test_loss_sync_guard_reference_contract(case, capsys):
    """sync_guard (the default outside Trainer): loss.py:190-206 exactly — a disconnected
    requires_grad zero leaf, zero terms, num_pos_anchors a Python int, the reference's message."""
    import loss as L
    import utils
    z = golden("loss_options.npz")
    anchors = utils.generate_anchors(*(int(v) for v in z["rot_grid"]), 8)
    ts = [t.to(DEV).requires_grad_(True) for t in _poisoned(z, case)]
    d = L.DetectionIntentionLoss(apply_intention_downsampling=False)(*ts, anchors, _gts(z, "rot"))
    np.testing.assert_array_equal(_vec(d), z[f"guard_{case}_loss"])
    assert type(d["num_pos_anchors"]) is int
    assert d["loss"].is_leaf and d["loss"].requires_grad and d["loss"].grad_fn is None
    assert "NaN or Inf DETECTED IN LOSS!" in capsys.readouterr().out
    d["loss"].backward()
    for t in ts:
        assert t.grad is None
    # finite inputs: the connected loss, num_pos still an int
    d = L.DetectionIntentionLoss(apply_intention_downsampling=False)(
        *[torch.from_numpy(z[k]).to(DEV) for k in ("rot_cls", "rot_box", "rot_int")], anchors, _gts(z, "rot"))
    assert type(d["num_pos_anchors"]) is int and d["num_pos_anchors"] == int(z["rot_axis_loss"][4])


def test_reference_loop_guard_leaves_weights_and_adamw_bit_identical():
    """The reference's own loop (train_vit.py:151-187: zero_grad(set_to_none) → forward → loss →
    loss.backward() → torch.optim.AdamW.step()) on an injected non-finite loss: the default
    sync_guard returns the disconnected leaf, no parameter gets a .grad, and torch AdamW updates
    nothing — weights, exp_avg / exp_avg_sq and step counts bit-identical."""
    import model_vit
    import utils
    from oracle import ivit_oracle as O
    cfg = model_cfg(img_size=(32, 48))
    m = model_vit.IntentNetViT(backbone_cfg={"img_size": (32, 48)})
    m.load_state_dict(make_state_dict(cfg, seed=0), strict=True)
    m = m.to(DEV).set_compute_dtype(torch.bfloat16).train()
    lidar, mp, gts = O.synthetic_batch(2, (32, 48), seed=1234, box_region=(54.0, 60.0, -72.0, -62.0))
    lidar, mp = lidar.to(DEV), mp.to(DEV)
    anchors = utils.generate_anchors(32, 48, 8, device=DEV)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    lf = _PoisonLoss(1)

    def ref_step(loss_fn):
        opt.zero_grad(set_to_none=True)
        c, b, i = m(lidar, mp)
        d = loss_fn(c, b, i, anchors, gts)
        d["loss"].backward()
        opt.step()
        return d

    d = ref_step(lf.inner)  # a normal step first: Adam state exists
    assert float(d["loss"]) > 0 and type(d["num_pos_anchors"]) is int
    w0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    s0 = {id(p): {k: v.clone() for k, v in opt.state[p].items()} for p in m.parameters()}
    d = ref_step(lf)
    torch.cuda.synchronize()
    assert float(d["loss"]) == 0.0
    assert all(p.grad is None for p in m.parameters())
    for k, v in m.state_dict().items():
        if "num_batches_tracked" in k or "running_" in k:
            continue  # BN statistics move in the forward, as in the reference
        assert torch.equal(v, w0[k]), k
    for p in m.parameters():
        for k, v in opt.state[p].items():
            assert torch.equal(v, s0[id(p)][k]), k
