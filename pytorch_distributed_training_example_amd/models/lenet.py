"""LeNet (reference model) and the 2-layer MLP plumbing model.

LeNet parity: /root/reference/cnn.py:4-30 — bilinear upsample 28→32 (align_corners=True),
three 5×5 convs with LeakyReLU(0.2) and 2×2 max-pools, FC 120→84→10, softmax output.
state_dict keys are identical (``ConvNet.{1,4,7}.{weight,bias}``, ``FC.{0,2}.{weight,bias}``),
so ``mnist_cnn.pt`` files are interchangeable with the reference's.

``output='probs'`` reproduces the reference's softmax output (which it then feeds to
``nll_loss``, cnn.py:23 + train.py:48); ``output='logits'`` drops the final Softmax so a
proper cross-entropy can be used (the default training path here).

On MI355X the whole network runs on our LeNet kernels (ops/lenet.py): upsample + conv1 + LeakyReLU
+ pool in one kernel (csrc/kernels/lenet.hip), then conv2 + LeakyReLU + pool + conv3 + LeakyReLU +
fc1 + LeakyReLU + fc2 in ONE more kernel (csrc/kernels/lenet_tail.hip); backward is the tail's two
kernels + the stem's weight-gradient kernel — no MIOpen, no hipBLASLt, no aten elementwise ops.
``fused=False`` keeps the plain ``nn.Sequential`` path (same parameters, same results up to fp32
rounding).
"""
from __future__ import annotations

import torch
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

    def _tail_params(self):
        c, f = self.ConvNet, self.FC
        return (c[4].weight, c[4].bias, c[7].weight, c[7].bias, f[0].weight, f[0].bias, f[2].weight, f[2].bias)

    def _logits_fused(self, img: torch.Tensor) -> torch.Tensor:
        from ..ops.lenet import lenet_stem, lenet_tail
        c = self.ConvNet
        y = lenet_stem(img, c[1].weight, c[1].bias, c[2].negative_slope)
        return lenet_tail(y, self._tail_params(), c[5].negative_slope)

    def _can_fuse(self, img: torch.Tensor) -> bool:
        if not (self.fused and img.is_cuda) or _native_disabled():
            return False
        from torch.nn.modules import module as _m
        if _m._global_forward_hooks or _m._global_forward_pre_hooks or any(
                m._forward_hooks or m._forward_pre_hooks for m in self.modules() if m is not self):
            return False  # submodule hooks must see their modules run
        slopes = {self.ConvNet[i].negative_slope for i in (2, 5, 8)} | {self.FC[1].negative_slope}
        from ..ops.lenet import stem_native_ok
        # the fused tail max-pools the raw conv outputs and activates the winner: equal to the
        # reference's MaxPool(LeakyReLU(z)) (cnn.py:14-15) only for a strictly increasing activation
        return len(slopes) == 1 and next(iter(slopes)) > 0 and stem_native_ok(img, self.ConvNet[1].weight)

    def forward(self, img: torch.Tensor) -> torch.Tensor:
        if self._can_fuse(img):
            logits = self._logits_fused(img)
        else:
            out = self.ConvNet(img)
            logits = self.FC(out.reshape(out.shape[0], -1))
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
