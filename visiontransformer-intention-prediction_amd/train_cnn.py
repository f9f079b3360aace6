"""IntentNetCNN training entry point — the flow of the reference's train_cnn.py (same
configuration: CNN_BACKBONE_CFG, FEATURE_MAP_STRIDE_CNN = 8, MODEL_SAVE_DIR_CNN) on the MI355X
kernels; it shares train_vit.py's loop (same loss / AdamW / scheduler / NaN skips / checkpoint
dict, --synthetic, --augment, torchrun data parallel)."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import train_vit  # noqa: E402


def main(argv=None):
    return train_vit.main(argv, variant="cnn")


if __name__ == '__main__':
    raise SystemExit(main())
