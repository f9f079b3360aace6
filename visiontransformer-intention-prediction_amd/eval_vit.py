"""IntentNetViT evaluation entry point — the flow of the reference's eval_vit.py:27-316 on the
MI355X kernels (BASELINE config 4: batched forward + rotated/axis IoU + NMS on one GPU).

Checkpoint → model (same cfg defaults as eval_vit.py:72-84) → anchors → batched inference with
confidence threshold 0.1, decode, NMS(0.2), argmax intention → detection mAP at
DETECTION_IOU_THRESHOLDS and intention accuracy / F1 on matched detections.

Differences, none in the numerics: ``--synthetic`` evaluates seeded synthetic BEV batches
(random-init weights when no checkpoint exists, which makes every anchor pass the threshold
— the worst case for NMS); checkpoints load with ``torch.load(weights_only=True)`` (the
pickled ``BasicBlock`` class in ``backbone_cfg`` is allow-listed by name); post-processing runs
on the device for the whole batch (utils.postprocess_batch, pipelined by utils.PostPipeline); the mAP / intention matching
walk runs on the device for all samples in one launch (metrics.match_device, ivit_det_match). The reference's undefined names (eval_vit.py:12-13,39,196,219)
come from constants.py / utils.py.
"""
from __future__ import annotations

import argparse
import time
from pathlib import Path

import torch

import model_vit
from constants import (ANCHOR_CONFIGS_PAPER, DETECTION_IOU_THRESHOLDS, EVAL_USE_ROTATED_IOU, GRID_HEIGHT_PX,
                       GRID_WIDTH_PX, INTENTIONS_MAP_REV, IOU_THRESHOLD_FOR_INTENTION_MATCH, LIDAR_TOTAL_CHANNELS,
                       MAP_CHANNELS, NUM_INTENTION_CLASSES)
from metrics import detection_map_device as detection_map, intention_matches_device as intention_matches
from model_vit import IntentNetViT
from synthetic import SyntheticBEVLoader
from utils import PostPipeline, generate_anchors

VAL_DATA_DIR = "./data/argoverse2/sensor/val"
MODEL_SAVE_PATH_VIT = "./trained_models_vit/vit_model.pth"

CONFIDENCE_THRESHOLD = 0.1
NMS_IOU_THRESHOLD = 0.2
INFERENCE_BATCH_SIZE = 8
NUM_WORKERS_EVAL = 0


MODEL_SAVE_PATH_CNN = "./trained_models_cnn/cnn_model.pth"  # eval_cnn.py:19


def load_checkpoint(path, device):
    import model_cnn
    torch.serialization.add_safe_globals([model_vit.BasicBlock, model_cnn.BasicBlock])
    return torch.load(path, map_location=device, weights_only=True)


def default_cfg(cfg: dict, grid):
    cfg.setdefault('img_size', tuple(grid))
    cfg.setdefault('lidar_input_channels', LIDAR_TOTAL_CHANNELS)
    cfg.setdefault('map_input_channels', MAP_CHANNELS)
    cfg.setdefault('vit_model_name_lidar', 'vit_small_patch8_224')
    cfg.setdefault('vit_model_name_map', 'vit_tiny_patch8_224')
    cfg.setdefault('pretrained_lidar', False)
    cfg.setdefault('pretrained_map', False)
    cfg.setdefault('drop_path_rate_lidar', 0.1)
    cfg.setdefault('drop_path_rate_map', 0.1)
    cfg.setdefault('lidar_adapter_out_channels', 192)
    cfg.setdefault('map_adapter_out_channels', 128)
    return cfg


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--checkpoint", type=str, default=None)
    ap.add_argument("--batch", type=int, default=INFERENCE_BATCH_SIZE)
    ap.add_argument("--batches", type=int, default=4, help="synthetic batches")
    ap.add_argument("--grid", type=str, default=f"{GRID_HEIGHT_PX}x{GRID_WIDTH_PX}")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="fp32")
    ap.add_argument("--rotated", action="store_true", default=EVAL_USE_ROTATED_IOU,
                    help="rotated IoU for mAP / matching (device kernel; no shapely needed)")
    return ap.parse_args(argv)


def run_inference(model, loader, anchors, conf=CONFIDENCE_THRESHOLD, nms=NMS_IOU_THRESHOLD):
    """eval_vit.py:136-180: forward + post-processing per batch, in loader order. The
    post-processing of a batch (utils.PostPipeline) runs beside the next batch's forward; results
    are the per-batch postprocess_batch ones, appended in the same order."""
    results = []
    pipe = PostPipeline(anchors, conf, nms)
    gts = []

    def emit(preds):
        for p, gt in zip(preds, gts.pop(0)):
            results.append({**{k: v.cpu() for k, v in p.items()},
                            "gt_boxes_xywha": gt.get("boxes_xywha", torch.empty((0, 5))),
                            "gt_intentions": gt.get("intentions", torch.empty(0, dtype=torch.long))})

    with torch.inference_mode():
        for batch in loader:
            dev = anchors.device
            cls, box, it = model(batch["lidar_bev"].to(dev, non_blocking=True),
                                 batch["map_bev"].to(dev, non_blocking=True))
            gts.append(batch["gt_list"])
            prev = pipe.push(cls, box, it)
            if prev is not None:
                emit(prev)
        last = pipe.flush()
        if last is not None:
            emit(last)
    return results


def main_eval_vit(argv=None, variant="vit"):
    """variant "vit" (eval_vit.py) or "cnn" (eval_cnn.py: IntentNetCNN, stride 8)."""
    args = parse_args(argv)
    tag = "ViT" if variant == "vit" else "CNN"
    if args.checkpoint is None:
        args.checkpoint = MODEL_SAVE_PATH_VIT if variant == "vit" else MODEL_SAVE_PATH_CNN
    if not torch.cuda.is_available():
        raise RuntimeError("eval_vit.py runs on the MI355X kernels: no ROCm GPU visible")
    device = torch.device("cuda")
    H, W = (int(v) for v in args.grid.lower().split("x"))
    print(f"--- {tag} Model Evaluation ---")
    print(f"Torch version: {torch.__version__}, device: {torch.cuda.get_device_name(0)}")
    print(f"Evaluation using Rotated IoU for mAP/matching: {args.rotated}")

    ckpt = None
    if Path(args.checkpoint).is_file():
        print(f"\nLoading TRAINED {tag} Model from: {args.checkpoint}")
        ckpt = load_checkpoint(args.checkpoint, device)
        cfg = ckpt.get('backbone_cfg')
        if not cfg:
            print(f"ERROR: 'backbone_cfg' not found in {tag} checkpoint.")
            return 1
    elif args.synthetic:
        print(f"No checkpoint at {args.checkpoint}: random-init weights (synthetic run)")
        from train_vit import backbone_cfg, cnn_backbone_cfg
        cfg = backbone_cfg((H, W)) if variant == "vit" else cnn_backbone_cfg()
    else:
        print(f"ERROR: {tag} Model checkpoint not found at {args.checkpoint}")
        return 1
    if variant == "vit":
        cfg = default_cfg(dict(cfg), (H, W))
        model = IntentNetViT(backbone_cfg=cfg).to(device)
        img_size = tuple(cfg['img_size'])
    else:
        from model_cnn import IntentNetCNN
        model = IntentNetCNN(backbone_cfg=dict(cfg)).to(device)
        img_size = (H, W)
    if ckpt is not None:
        model.load_state_dict(ckpt['model_state_dict'])
    model.set_compute_dtype(torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    model.eval()

    if args.synthetic:
        loader = SyntheticBEVLoader(args.batch, args.batches, img_size, rank=0, device=device,
                                    resident=False)
    else:
        if not Path(VAL_DATA_DIR).is_dir():
            print(f"ERROR: Evaluation data directory not found: {VAL_DATA_DIR} (use --synthetic)")
            return 1
        raise SystemExit("The Argoverse-2 dataset loader is outside this build's scope; use --synthetic")

    if variant == "vit":
        stride = int(cfg.get('vit_model_name_lidar', 'vit_small_patch8_224').split('_patch')[-1].split('_')[0]) \
            * cfg.get('fusion_block_stride', 1)
    else:
        stride = 8  # eval_cnn.py: FEATURE_MAP_STRIDE_CNN
    Hc, Wc = img_size
    anchors = generate_anchors(Hc, Wc, stride, ANCHOR_CONFIGS_PAPER, device=device)
    print(f"Anchors for {tag} evaluation generated (stride {stride}), shape: {tuple(anchors.shape)}")

    t0 = time.perf_counter()
    results = run_inference(model, loader, anchors)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"Collected results for {len(results)} samples ({len(results) / dt:.2f} samples/s incl. host transfer)")

    print(f"\n--- {tag} Detection Results (mAP) ---")
    maps = detection_map(results, DETECTION_IOU_THRESHOLDS, args.rotated)
    for t, v in maps.items():
        print(f"{tag} mAP @ IoU={t:.1f}: {v:.4f}")

    mp, mg = intention_matches(results, IOU_THRESHOLD_FOR_INTENTION_MATCH, args.rotated)
    if mp:
        from sklearn.metrics import accuracy_score, f1_score
        labels = list(range(NUM_INTENTION_CLASSES))
        print(f"\n--- {tag} Intention Prediction Results (on TP detections @ IoU>={IOU_THRESHOLD_FOR_INTENTION_MATCH}) ---")
        print(f"{tag} Overall Accuracy: {accuracy_score(mg, mp):.4f}")
        print(f"{tag} F1 (Macro):   {f1_score(mg, mp, labels=labels, average='macro', zero_division=0):.4f}")
        print(f"{tag} F1 (Weighted): {f1_score(mg, mp, labels=labels, average='weighted', zero_division=0):.4f}")
        per = f1_score(mg, mp, labels=labels, average=None, zero_division=0)
        print(f"{tag} F1 (Per Class):")
        for i in labels:
            print(f"  {INTENTIONS_MAP_REV.get(i, f'Class_{i}'):<20}: {per[i]:.4f}")
    else:
        print(f"\nNo True Positive detections found for {tag} model at IoU >= {IOU_THRESHOLD_FOR_INTENTION_MATCH} "
              "to evaluate intention.")
    print(f"\n--- Evaluation Script for {tag} Finished ---")
    return 0


if __name__ == '__main__':
    raise SystemExit(main_eval_vit())
