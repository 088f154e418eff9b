"""Multi-tensor helpers (csrc/kernels/amp.hip): one launch over many tensors.

Used by the AMP grad scaler (unscale + inf check), gradient clipping (L2 norm + scale, all on
device), and DDP bucket packing (copy with dtype conversion and folded averaging factor).
CPU tensors take a ``torch._foreach_*`` reference path.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from ._native import native, use_native


def _groups(tensors: Sequence[torch.Tensor]):
    by = {}
    for i, t in enumerate(tensors):
        by.setdefault(t.dtype, []).append(i)
    return by


def unscale_(grads: List[torch.Tensor], inv_scale: torch.Tensor, found_inf: torch.Tensor) -> None:
    """grads *= inv_scale in place; found_inf := 1 if any grad is non-finite (found_inf not reset)."""
    grads = [g for g in grads if g is not None]
    if not grads:
        return
    if use_native(*grads):
        for _, idx in _groups(grads).items():
            native().amp_unscale([grads[i] for i in idx], inv_scale, found_inf)
        return
    for g in grads:
        if not torch.isfinite(g).all():
            found_inf.fill_(1.0)
        g.mul_(inv_scale.to(g.dtype))


def scale_(tensors: List[torch.Tensor], scale: Optional[torch.Tensor] = None, factor: float = 1.0) -> None:
    tensors = [t for t in tensors if t is not None]
    if not tensors:
        return
    if use_native(*tensors):
        for _, idx in _groups(tensors).items():
            native().mt_scale([tensors[i] for i in idx], scale, factor)
        return
    k = factor if scale is None else scale * factor
    for t in tensors:
        t.mul_(k if not torch.is_tensor(k) else k.to(t.dtype))


def copy_(src: List[torch.Tensor], dst: List[torch.Tensor], scale: Optional[torch.Tensor] = None,
          factor: float = 1.0) -> None:
    """dst[i] = src[i] * factor (* scale) with dtype conversion, one launch per dtype pair."""
    if not src:
        return
    if use_native(*src, *dst):
        pairs = {}
        for i, (s, d) in enumerate(zip(src, dst)):
            pairs.setdefault((s.dtype, d.dtype), []).append(i)
        for _, idx in pairs.items():
            native().mt_copy([src[i] for i in idx], [dst[i] for i in idx], scale, factor)
        return
    for s, d in zip(src, dst):
        v = s.float() * factor
        if scale is not None:
            v = v * scale
        d.copy_(v)


def l2_norm_sq(tensors: List[torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    tensors = [t for t in tensors if t is not None]
    dev = tensors[0].device if tensors else torch.device("cpu")
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=dev)
    if tensors and use_native(*tensors):
        groups = list(_groups(tensors).items())
        tmp = torch.empty(len(groups), dtype=torch.float32, device=dev)
        for k, (_, idx) in enumerate(groups):
            native().l2norm_sq([tensors[i] for i in idx], tmp[k:k + 1])
        out.copy_(tmp.sum().reshape(out.shape))
        return out
    out.zero_()
    for t in tensors:
        out += t.float().pow(2).sum()
    return out


def clip_grad_norm_(grads: List[torch.Tensor], max_norm: float) -> torch.Tensor:
    """Device-side global-norm clipping (no host sync). Returns the total norm tensor."""
    grads = [g for g in grads if g is not None]
    if not grads:
        return torch.zeros(())
    sumsq = l2_norm_sq(grads)
    if use_native(*grads):
        coef = torch.empty(1, dtype=torch.float32, device=sumsq.device)
        norm = torch.empty(1, dtype=torch.float32, device=sumsq.device)
        native().clip_coef(sumsq, float(max_norm), coef, norm)
        scale_(grads, coef)
        return norm
    norm = sumsq.sqrt()
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef.to(g.dtype))
    return norm
