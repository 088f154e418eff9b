"""LR schedules. ``step`` = the reference's StepLR(step_size=1, gamma) per epoch
(/root/reference/train.py:101,105); ``cosine`` = linear warmup + cosine decay (ViT/GPT-2)."""
from __future__ import annotations

import math

from torch.optim.lr_scheduler import LambdaLR, StepLR


def warmup_cosine(optimizer, warmup_steps: int, total_steps: int, min_ratio: float = 0.1):
    def f(step):
        if step < warmup_steps:
            return (step + 1) / max(1, warmup_steps)
        t = (step - warmup_steps) / max(1, total_steps - warmup_steps)
        return min_ratio + (1 - min_ratio) * 0.5 * (1 + math.cos(math.pi * min(1.0, t)))
    return LambdaLR(optimizer, f)


def build_scheduler(name: str, optimizer, gamma: float = 0.9, step_size: int = 1, warmup_steps: int = 0,
                    total_steps: int = 1):
    if name == "step":
        return StepLR(optimizer, step_size=step_size, gamma=gamma)
    if name == "cosine":
        return warmup_cosine(optimizer, warmup_steps, total_steps)
    if name in ("none", "constant"):
        return LambdaLR(optimizer, lambda s: 1.0)
    raise ValueError(name)
