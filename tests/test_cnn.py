"""IntentNetCNN, the reference's CNN variant (model_cnn.py): strided 5x5 /
3x3 / 1x1 convs as im2col + MFMA GEMM, BN / ReLU / residual kernels, fused heads.

Golden vectors: tests/golden/cnn_small.npz from the reference's OWN IntentNetCNN (default
channels, 32x48 grid) with the seeded filler (oracle/make_golden.py gen_cnn_small). Bar: the f32
path within 1e-3 relative to each output's max (the north_star fp tolerance); bf16 within 6e-2."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ivit_oracle as O
from oracle.weights import fill_state_dict

SMALL = (32, 48)
DEV = "cuda"


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def _gts(z, n):
    return [{"boxes_xywha": torch.from_numpy(z[f"gt{i}_boxes"]), "intentions": torch.from_numpy(z[f"gt{i}_ints"])}
            for i in range(n)]


def _sd(keys_shapes):
    return fill_state_dict(keys_shapes, seed=0)


# ------------------------------------------------------------------ CPU
def test_cnn_oracle_matches_reference_golden():
    import model_cnn
    z = golden("cnn_small.npz")
    m = model_cnn.IntentNetCNN()
    ks = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    assert [k for k, _ in ks] == [str(k) for k in z["keys"]]  # the reference's state_dict order / names
    sd = _sd(ks)
    lidar, mp, _ = O.synthetic_batch(2, SMALL, seed=1234)
    with torch.no_grad():
        c, b, i = O.cnn_forward(dict(sd), lidar, mp, training=False)
    assert _rel(c, z["eval_cls"]) < 1e-5 and _rel(b, z["eval_box"]) < 1e-5 and _rel(i, z["eval_int"]) < 1e-5


def test_cnn_conv_geometry_and_attributes():
    import model_cnn
    bb = model_cnn.CNNBackbone()
    assert (bb.lidar_output_channels, bb.map_output_channels, bb.fusion_inplanes, bb.final_feature_channels) == \
        (224, 96, 320, 512)
    c = bb.lidar_stage1[0].conv1
    assert c.kernel_size == (5, 5) and c.stride == (2, 2) and c.padding == (2, 2) and c.bias is None
    assert bb.fusion_block[0].conv1.kernel_size == (3, 3) and bb.fusion_block[0].downsample[0].stride == (2, 2)
    assert bb.lidar_stage2[0].downsample is not None and bb.lidar_stage2[1].downsample is None


# ------------------------------------------------------------------ GPU
def _model(cd=torch.float32):
    import model_cnn
    m = model_cnn.IntentNetCNN()
    m.load_state_dict(_sd([(k, tuple(v.shape)) for k, v in m.state_dict().items()]), strict=True)
    return m.to(DEV).set_compute_dtype(cd)


@pytest.mark.gpu
def test_cnn_eval_vs_golden():
    z = golden("cnn_small.npz")
    lidar, mp, _ = O.synthetic_batch(2, SMALL, seed=1234)
    m = _model().eval()
    with torch.no_grad():
        c, b, i = m(lidar.to(DEV), mp.to(DEV))
    assert c.shape == (2, 4 * 6 * 5, 1) and b.shape == (2, 120, 6) and i.shape == (2, 120, 8)
    assert _rel(c, z["eval_cls"]) < 1e-3 and _rel(b, z["eval_box"]) < 1e-3 and _rel(i, z["eval_int"]) < 1e-3


@pytest.mark.gpu
def test_cnn_train_loss_grads_bn_vs_golden():
    import loss as L
    import utils
    z = golden("cnn_small.npz")
    lidar, mp, _ = O.synthetic_batch(2, SMALL, seed=1234)
    m = _model().train()
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    assert _rel(c.detach(), z["train_cls"]) < 1e-3 and _rel(i.detach(), z["train_int"]) < 1e-3
    d = L.DetectionIntentionLoss(apply_intention_downsampling=False)(c, b, i, utils.generate_anchors(*SMALL, 8),
                                                                     _gts(z, 2))
    got = [float(d["loss"]), float(d["cls_loss"]), float(d["box_loss"]), float(d["intent_loss"]),
           float(d["num_pos_anchors"])]
    np.testing.assert_allclose(got, z["train_loss"], rtol=1e-3)
    d["loss"].backward()
    ps = dict(m.named_parameters())
    for name, gas, smp, st in zip(z["grad_names"], z["grad_abssum"], z["grad_samples"], z["grad_strides"]):
        g = ps[str(name)].grad
        assert g is not None, name
        assert float(g.double().abs().sum()) == pytest.approx(gas, rel=2e-3, abs=1e-6), name
        s = g.reshape(-1).double()[:: int(st)][:64].cpu().numpy()
        ref = smp[~np.isnan(smp)][: s.size]
        assert np.abs(s - ref).max() <= 2e-3 * max(np.abs(ref).max(), 1e-6) + 1e-7, name
    bufs = dict(m.named_buffers())
    off = 0
    for name, n in zip(z["bn_names"], z["bn_sizes"]):
        np.testing.assert_allclose(bufs[str(name)].cpu().numpy(), z["bn_values"][off:off + n], rtol=1e-4, atol=1e-5)
        off += n


@pytest.mark.gpu
def test_cnn_bf16_close_to_f32_and_module_forwards():
    import model_cnn
    lidar, mp, _ = O.synthetic_batch(2, SMALL, seed=1234)
    m32, m16 = _model().eval(), _model(torch.bfloat16).eval()
    with torch.no_grad():
        a = m32(lidar.to(DEV), mp.to(DEV))
        b = m16(lidar.to(DEV), mp.to(DEV))
        for x, y in zip(a, b):
            assert _rel(y, x) < 6e-2
        f = m32.backbone(lidar.to(DEV), mp.to(DEV))  # NCHW backbone surface (model_cnn.py:110-123)
        assert f.shape == (2, 512, 4, 6)
        blk = m32.backbone.lidar_stage1[0]
        ref = O.cnn_block({f"x.{k}": v for k, v in blk.state_dict().items()}, "x.", lidar.to(DEV), 2, 5, False)
        assert _rel(blk(lidar.to(DEV)), ref) < 1e-3
    assert isinstance(m32.backbone.lidar_stage1[0], model_cnn.BasicBlock)


@pytest.mark.gpu
def test_cnn_full_grid_bf16_train_step_finite():
    """constants.py grid (400x720), B=1, bf16 forward + loss + backward + fused AdamW."""
    import loss as L
    import utils
    from optim import FusedAdamW
    m = _model(torch.bfloat16).train()
    lidar, mp, gts = O.synthetic_batch(1, seed=1234)
    opt = FusedAdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    c, b, i = m(lidar.to(DEV), mp.to(DEV))
    assert c.shape == (1, 50 * 90 * 5, 1)
    d = L.DetectionIntentionLoss()(c, b, i, utils.generate_anchors(), gts)
    d["loss"].backward()
    opt.step()
    torch.cuda.synchronize()
    assert torch.isfinite(d["loss"]).item()
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all().item(), n
