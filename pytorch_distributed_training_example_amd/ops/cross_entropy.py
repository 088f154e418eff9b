"""Fused softmax cross-entropy (csrc/kernels/softmax_ce.hip) and the reference's loss.

``cross_entropy`` is the training loss of every model here (one pass over the logits,
label smoothing, ignore_index, mean/sum/none reductions). ``nll_on_probs`` reproduces the
reference's loss exactly: the LeNet ends in Softmax (/root/reference/cnn.py:23) and the
loop applies ``F.nll_loss`` to those probabilities (train.py:48, 68), i.e. ``-mean(p[y])``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._native import native, use_native


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, smoothing, ignore_index, reduction):
        loss, lse = native().ce_fwd(logits, target, smoothing, ignore_index)
        ctx.save_for_backward(logits, target, lse)
        ctx.smoothing, ctx.ignore_index, ctx.reduction = smoothing, ignore_index, reduction
        if reduction == "none":
            return loss
        if reduction == "sum":
            return loss.sum()
        count = (target != ignore_index).sum().clamp_min(1)
        ctx.count = count
        return loss.sum() / count

    @staticmethod
    def backward(ctx, dloss):
        logits, target, lse = ctx.saved_tensors
        if ctx.reduction == "none":
            d, scale = dloss, 1.0
        elif ctx.reduction == "sum":
            d, scale = dloss.reshape(1), 1.0
        else:
            d, scale = (dloss / ctx.count).reshape(1), 1.0
        dl = native().ce_bwd(logits, target, lse, d, scale, ctx.smoothing, ctx.ignore_index)
        return dl, None, None, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, label_smoothing: float = 0.0,
                  ignore_index: int = -100, reduction: str = "mean") -> torch.Tensor:
    if logits.dim() > 2:
        logits = logits.reshape(-1, logits.shape[-1])
        target = target.reshape(-1)
    if use_native(logits) and logits.dtype in (torch.float32, torch.bfloat16):
        return _CEFn.apply(logits.contiguous(), target.contiguous().long(), float(label_smoothing),
                           int(ignore_index), reduction)
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index, reduction=reduction,
                           label_smoothing=label_smoothing)


def nll_on_probs(probs: torch.Tensor, target: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    """The reference's loss: nll_loss applied to softmax probabilities (train.py:48)."""
    return F.nll_loss(probs, target, reduction=reduction)
