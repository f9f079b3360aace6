"""DetectionHead / IntentionHead (heads.py:1-42 of the reference): 3x3 conv heads whose
output is viewed per anchor as (B, Hf, Wf, A, k). In the fused model path both heads run
as ONE implicit GEMM (A*7 + A*K output channels) inside ``ops.NeckFn``."""
import torch.nn as nn

from constants import NUM_ANCHORS_PER_LOC, NUM_INTENTION_CLASSES
from layers import Conv2d


class DetectionHead(nn.Module):
    def __init__(self, in_channels: int, num_anchors: int = NUM_ANCHORS_PER_LOC):
        super().__init__()
        self.num_anchors = num_anchors
        self.conv = Conv2d(in_channels, num_anchors * 7, kernel_size=3, padding=1)

    def forward(self, x):
        out = self.conv(x)
        B, _, Hf, Wf = out.shape
        out = out.view(B, self.num_anchors, 7, Hf, Wf).permute(0, 3, 4, 1, 2).contiguous()
        return out[..., 0], out[..., 1:]


class IntentionHead(nn.Module):
    def __init__(self, in_channels: int, num_anchors: int = NUM_ANCHORS_PER_LOC,
                 num_classes: int = NUM_INTENTION_CLASSES):
        super().__init__()
        self.num_anchors, self.num_classes = num_anchors, num_classes
        self.conv = Conv2d(in_channels, num_anchors * num_classes, kernel_size=3, padding=1)

    def forward(self, x):
        out = self.conv(x)
        B, _, Hf, Wf = out.shape
        return out.view(B, self.num_anchors, self.num_classes, Hf, Wf).permute(0, 3, 4, 1, 2).contiguous()
