"""LeNet (reference model) and the 2-layer MLP plumbing model.

LeNet parity: /root/reference/cnn.py:4-30 — bilinear upsample 28→32 (align_corners=True),
three 5×5 convs with LeakyReLU(0.2) and 2×2 max-pools, FC 120→84→10, softmax output.
state_dict keys are identical (``ConvNet.{1,4,7}.{weight,bias}``, ``FC.{0,2}.{weight,bias}``),
so ``mnist_cnn.pt`` files are interchangeable with the reference's.

``output='probs'`` reproduces the reference's softmax output (which it then feeds to
``nll_loss``, cnn.py:23 + train.py:48); ``output='logits'`` drops the final Softmax so a
proper cross-entropy can be used (the default training path here).
"""
from __future__ import annotations

import torch
from torch import nn


class LeNet(nn.Module):
    def __init__(self, output: str = "probs"):
        super().__init__()
        if output not in ("probs", "logits", "log_probs"):
            raise ValueError(output)
        self.output = output
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

    def forward(self, img: torch.Tensor) -> torch.Tensor:
        out = self.ConvNet(img)
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
