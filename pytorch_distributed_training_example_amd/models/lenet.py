"""LeNet (reference model) and the 2-layer MLP plumbing model.

LeNet parity: /root/reference/cnn.py:4-30 — bilinear upsample 28→32 (align_corners=True),
three 5×5 convs with LeakyReLU(0.2) and 2×2 max-pools, FC 120→84→10, softmax output.
state_dict keys are identical (``ConvNet.{1,4,7}.{weight,bias}``, ``FC.{0,2}.{weight,bias}``),
so ``mnist_cnn.pt`` files are interchangeable with the reference's.

``output='probs'`` reproduces the reference's softmax output (which it then feeds to
``nll_loss``, cnn.py:23 + train.py:48); ``output='logits'`` drops the final Softmax so a
proper cross-entropy can be used (the default training path here).

On MI355X the conv stack runs through the fused LeNet kernels (ops/lenet.py,
csrc/kernels/lenet.hip): upsample+conv1+LeakyReLU+pool in one kernel, conv2 on MIOpen
followed by a fused LeakyReLU+pool, conv3 on MIOpen. ``fused=False`` keeps the plain
``nn.Sequential`` path (same parameters, same results up to fp32 rounding).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from ..ops._native import disabled as _native_disabled


class LeNet(nn.Module):
    def __init__(self, output: str = "probs", fused: bool = True):
        super().__init__()
        if output not in ("probs", "logits", "log_probs"):
            raise ValueError(output)
        self.output = output
        self.fused = fused
        self.ConvNet = nn.Sequential(
            nn.UpsamplingBilinear2d(size=32),
            nn.Conv2d(1, 6, 5, padding=0, stride=1),
            nn.LeakyReLU(0.2),
            nn.MaxPool2d(2, stride=2, padding=0),
            nn.Conv2d(6, 16, 5, padding=0, stride=1),
            nn.LeakyReLU(0.2),
            nn.MaxPool2d(2, stride=2, padding=0),
            nn.Conv2d(16, 120, 5, padding=0, stride=1),
            nn.LeakyReLU(0.2),
        )
        self.FC = nn.Sequential(nn.Linear(120, 84), nn.LeakyReLU(0.2), nn.Linear(84, 10))

    def _features_fused(self, img: torch.Tensor) -> torch.Tensor:
        from ..ops.lenet import leaky_pool, lenet_stem
        c = self.ConvNet
        y = lenet_stem(img, c[1].weight, c[1].bias, c[2].negative_slope)
        y = leaky_pool(F.conv2d(y, c[4].weight, c[4].bias), c[5].negative_slope)
        return F.leaky_relu(F.conv2d(y, c[7].weight, c[7].bias), c[8].negative_slope)

    def _can_fuse(self, img: torch.Tensor) -> bool:
        if not (self.fused and img.is_cuda) or _native_disabled():
            return False
        from ..ops.lenet import stem_native_ok
        return stem_native_ok(img, self.ConvNet[1].weight)

    def forward(self, img: torch.Tensor) -> torch.Tensor:
        out = self._features_fused(img) if self._can_fuse(img) else self.ConvNet(img)
        out = out.reshape(out.shape[0], -1)
        logits = self.FC(out)
        if self.output == "probs":
            return torch.softmax(logits, dim=-1)
        if self.output == "log_probs":
            return torch.log_softmax(logits, dim=-1)
        return logits


class MLP(nn.Module):
    """2-layer MLP on random tensors (BASELINE.json config 1: DDP plumbing on CPU/gloo)."""

    def __init__(self, in_features: int = 32, hidden: int = 64, out_features: int = 8):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden)
        self.act = nn.ReLU()
        self.fc2 = nn.Linear(hidden, out_features)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.fc2(self.act(self.fc1(x)))
