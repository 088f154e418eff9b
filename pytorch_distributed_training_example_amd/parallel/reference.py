"""The reference's gradient-averaging algorithm, kept as a baseline ("B1" in BASELINE.md).

/root/reference/train.py:34-39: after ``backward()``, for every parameter in registration
order, a blocking SUM all-reduce followed by ``grad /= world_size``. Re-implemented so the
MI355X bench can price it against the bucketed, overlapped reducer (parallel/ddp.py).
"""
from __future__ import annotations

import torch.distributed as dist
import torch.nn as nn


def average_gradients(model: nn.Module, group=None) -> None:
    if not dist.is_initialized():
        return
    size = float(dist.get_world_size(group))
    for param in model.parameters():
        if param.grad is None:
            continue
        dist.all_reduce(param.grad.data, op=dist.ReduceOp.SUM, group=group)
        param.grad.data /= size


def broadcast_parameters(model: nn.Module, src: int = 0, group=None) -> None:
    """What the reference lacks: make replicas identical without relying on equal seeds."""
    if not dist.is_initialized():
        return
    for t in list(model.parameters()) + list(model.buffers()):
        dist.broadcast(t.data, src=src, group=group)
