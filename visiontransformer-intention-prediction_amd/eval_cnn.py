"""IntentNetCNN evaluation entry point — the flow of the reference's eval_cnn.py (checkpoint
MODEL_SAVE_PATH_CNN, stride-8 anchors) on the MI355X kernels; it shares eval_vit.py's loop
(inference, sigmoid >= 0.1, decode, batched NMS 0.2, device mAP / intention matching)."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import eval_vit  # noqa: E402


def main_eval_cnn(argv=None):
    return eval_vit.main_eval_vit(argv, variant="cnn")


if __name__ == '__main__':
    raise SystemExit(main_eval_cnn())
