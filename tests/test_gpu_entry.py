"""train_vit.py / eval_vit.py entry points and batched post-processing on the GPU
(small grid so each test takes seconds)."""
import os

import pytest
import torch

from oracle import ivit_oracle as O

pytestmark = pytest.mark.gpu


def test_train_vit_synthetic_epoch_and_checkpoint(tmp_path):
    import train_vit
    rc = train_vit.main(["--synthetic", "--epochs", "2", "--batches-per-epoch", "2", "--batch", "2", "--grid", "32x48",
                         "--dtype", "bf16", "--save-dir", str(tmp_path)])
    assert rc == 0
    ck = tmp_path / "vit_model.pth"
    assert ck.is_file()
    import eval_vit
    d = eval_vit.load_checkpoint(str(ck), torch.device("cuda"))
    assert set(d) == {"epoch", "model_state_dict", "optimizer_state_dict", "backbone_cfg"}
    assert d["epoch"] == 2 and tuple(d["backbone_cfg"]["img_size"]) == (32, 48)
    rc = eval_vit.main_eval_vit(["--synthetic", "--checkpoint", str(ck), "--batch", "2", "--batches", "1",
                                 "--grid", "32x48"])
    assert rc == 0


def test_eval_vit_random_init_rotated():
    import eval_vit
    rc = eval_vit.main_eval_vit(["--synthetic", "--checkpoint", "/nonexistent.pth", "--batch", "2", "--batches", "1",
                                 "--grid", "32x48", "--rotated"])
    assert rc == 0


def test_postprocess_batch_matches_oracle():
    import utils
    g = torch.Generator().manual_seed(5)
    B, NA = 3, 4500
    anchors = O.generate_anchors(240, 600, 8)[:NA]
    cls = torch.randn(B, NA, 1, generator=g) * 2 - 1.0
    box = torch.randn(B, NA, 6, generator=g) * 0.3
    it = torch.randn(B, NA, 8, generator=g)
    got = utils.postprocess_batch(cls.cuda(), box.cuda(), it.cuda(), anchors.cuda(), 0.1, 0.2)
    for b in range(B):
        s = torch.sigmoid(cls[b, :, 0])
        idx = torch.nonzero(s >= 0.1).squeeze(1)
        dec = O.decode_boxes(box[b][idx], anchors[idx])
        dec_dev = utils.decode_box_predictions(box[b][idx].cuda(), anchors[idx].cuda()).cpu()
        assert torch.allclose(dec_dev, dec, rtol=1e-5, atol=1e-5)
        # NMS index selection is bit-exact given the same boxes: feed the device-decoded ones
        keep = torch.as_tensor(O.nms_numpy(dec_dev, s[idx], 0.2), dtype=torch.long)
        dec = dec_dev
        assert got[b]["pred_boxes_xywha"].shape[0] == keep.shape[0] > 0
        assert torch.allclose(got[b]["pred_scores"].cpu(), s[idx][keep])
        assert torch.allclose(got[b]["pred_boxes_xywha"].cpu(), dec[keep], rtol=1e-5, atol=1e-5)
        assert torch.equal(got[b]["pred_intentions"].cpu(), torch.argmax(it[b][idx][keep], -1))


def _post_reference(cls, box, it, anchors, conf=0.1, thr=0.2):
    """The reference's per-sample loop (eval_vit.py:156-176) on the same device tensors: torch's
    GPU sigmoid, torch.where, the device decode, the oracle's torchvision-CPU NMS, CPU argmax."""
    import utils
    out = []
    for b in range(cls.shape[0]):
        s = torch.sigmoid(cls[b].reshape(-1).float())
        idx = torch.where(s >= conf)[0]
        if idx.numel() == 0:
            out.append((torch.empty(0), torch.empty((0, 5)), torch.empty(0, dtype=torch.long)))
            continue
        dec = utils.decode_box_predictions(box[b].reshape(-1, 6)[idx], anchors[idx]).cpu()
        keep = torch.as_tensor(O.nms_numpy(dec.numpy(), s[idx].cpu().numpy(), thr), dtype=torch.long)
        out.append((s[idx].cpu()[keep], dec[keep], torch.argmax(it[b].reshape(cls.shape[1], -1)[idx].cpu()[keep], -1)))
    return out


def test_postprocess_adversarial_vs_reference_loop():
    """ivit_eval_post (one batched pass: sigmoid, threshold compaction, decode, stable score sort,
    NMS, argmax) against the reference's per-sample loop, bit-exact, on a batch holding: random
    logits; every logit equal (22 500 tied scores, all pass); nothing passing; logits at the
    threshold's edge (sigmoid within an ulp of 0.1), NaN / +-inf logits and -0 / +0; quantised
    logits (mass ties) over overlapping boxes; intention rows with tied maxima and NaN."""
    import utils
    g = torch.Generator().manual_seed(11)
    anchors = O.generate_anchors(400, 720, 8)
    NA = anchors.shape[0]
    B = 5
    cls = torch.randn(B, NA, generator=g) * 2.0
    cls[1] = 0.37
    cls[2] = -30.0
    edge = torch.log(torch.tensor(0.1 / 0.9))
    ulps = torch.arange(-64, 64, dtype=torch.float32) * 1.2e-7
    cls[3] = (edge + ulps.repeat(NA // 128 + 1)[:NA]).float()
    cls[3, :50] = float("nan")
    cls[3, 50:60] = float("inf")
    cls[3, 60:70] = float("-inf")
    cls[3, 70:80] = 0.0
    cls[3, 80:90] = -0.0
    cls[4] = torch.round(torch.randn(NA, generator=g) * 2) / 2
    box = torch.randn(B, NA, 6, generator=g) * 0.3
    box[4, :, :4] = 0.05 * torch.randn(NA, 4, generator=g)  # heavy overlaps
    it = torch.round(torch.randn(B, NA, 8, generator=g))  # tied maxima
    it[0, :100, 3] = float("nan")
    it[0, 100:200, 2:4] = float("nan")
    dev_args = (cls.cuda(), box.cuda(), it.cuda(), anchors.cuda())
    got = utils.postprocess_batch(*dev_args, 0.1, 0.2)
    want = _post_reference(*dev_args)
    for b, (p, (ws, wb, wi)) in enumerate(zip(got, want)):
        assert torch.equal(p["pred_scores"].cpu(), ws), b
        assert torch.equal(p["pred_boxes_xywha"].cpu(), wb), b
        assert torch.equal(p["pred_intentions"].cpu(), wi), b
    assert got[2]["pred_scores"].numel() == 0 and got[1]["pred_scores"].numel() > 0


def test_post_pipeline_equals_per_batch_postprocess():
    """utils.PostPipeline (batch k's post-processing on its own stream beside batch k+1's work, counts
    read one batch late) returns, batch by batch, exactly what postprocess_batch returns; the
    producer stream reuses memory between pushes (the inputs are freed after each push), so a missing
    stream hand-off would show as corrupted results. Includes an empty batch and a flush."""
    import utils
    g = torch.Generator().manual_seed(5)
    anchors = O.generate_anchors(400, 720, 8).cuda()
    NA = anchors.shape[0]
    batches = []
    for k in range(4):
        B = 0 if k == 2 else 3
        batches.append((torch.randn(B, NA, generator=g) * 2.0, torch.randn(B, NA, 6, generator=g) * 0.3,
                        torch.round(torch.randn(B, NA, 8, generator=g))))
    want = [utils.postprocess_batch(c.cuda(), b.cuda(), i.cuda(), anchors) for c, b, i in batches]
    want = [[{k: v.cpu() for k, v in p.items()} for p in w] for w in want]
    pipe = utils.PostPipeline(anchors)
    got = []
    for c, b, i in batches:
        cd, bd, idv = c.cuda(), b.cuda(), i.cuda()
        prev = pipe.push(cd, bd, idv)
        del cd, bd, idv  # freed on the producer stream while the pipeline's kernels may still read them
        junk = torch.full((3, NA, 8), float("nan"), device="cuda")  # likely lands in the freed blocks
        if prev is not None:
            got.append([{k: v.cpu() for k, v in p.items()} for p in prev])
        del junk
    got.append([{k: v.cpu() for k, v in p.items()} for p in pipe.flush()])
    assert pipe.flush() is None and len(got) == len(want)
    for k, (gb, wb) in enumerate(zip(got, want)):
        assert len(gb) == len(wb), k
        for p, q in zip(gb, wb):
            for key in q:
                assert torch.equal(p[key], q[key]), (k, key)


def test_postprocess_empty_after_threshold():
    import utils
    anchors = O.generate_anchors(32, 48, 8).cuda()
    NA = anchors.shape[0]
    cls = torch.full((1, NA, 1), -20.0, device="cuda")
    out = utils.postprocess_batch(cls, torch.zeros(1, NA, 6, device="cuda"), torch.zeros(1, NA, 8, device="cuda"),
                                  anchors)
    assert out[0]["pred_scores"].numel() == 0 and out[0]["pred_boxes_xywha"].shape == (0, 5)


def test_train_cnn_synthetic_augmented_epoch_and_checkpoint(tmp_path):
    """train_cnn.py flow (IntentNetCNN, stride 8) with the GPU augment_bev on every batch."""
    import train_cnn
    rc = train_cnn.main(["--synthetic", "--epochs", "1", "--batches-per-epoch", "2", "--batch", "2", "--grid", "32x48",
                         "--dtype", "bf16", "--augment", "--save-dir", str(tmp_path)])
    assert rc == 0
    ck = tmp_path / "cnn_model.pth"
    assert ck.is_file()
    import eval_cnn
    import eval_vit
    d = eval_vit.load_checkpoint(str(ck), torch.device("cuda"))
    assert "backbone.lidar_stage1.0.conv1.weight" in d["model_state_dict"]
    rc = eval_cnn.main_eval_cnn(["--synthetic", "--checkpoint", str(ck), "--batch", "2", "--batches", "1",
                                 "--grid", "32x48"])
    assert rc == 0
