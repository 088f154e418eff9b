"""LayerNorm backed by the wave-per-row HIP kernel (csrc/kernels/layernorm.hip).

``LayerNorm`` subclasses ``torch.nn.LayerNorm`` (same state_dict). Parameters are kept in
fp32 while activations may be bf16; the kernel reads bf16 rows, normalises in fp32 and
writes bf16. Falls back to ``F.layer_norm`` for CPU tensors or unsupported widths.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from ._native import native, use_native

_SUPPORTED_K = {1, 2, 3, 4, 5, 6, 8}


class _LNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        y, mean, rstd, _ = native().ln_fwd(x, weight, bias, eps)
        ctx.save_for_backward(x, weight, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, mean, rstd = ctx.saved_tensors
        dx, dw, db = native().ln_bwd(dy.contiguous(), x, weight, mean, rstd)
        return dx, dw, db, None


def layer_norm(x, normalized_shape, weight, bias, eps=1e-5):
    if _ln_native_ok(x, weight, bias, normalized_shape):
        return _LNFn.apply(x.contiguous(), weight, bias, float(eps))
    if weight is not None and x.dtype != weight.dtype:
        return F.layer_norm(x.float(), normalized_shape, weight.float(),
                            bias.float() if bias is not None else None, eps).to(x.dtype)
    return F.layer_norm(x, normalized_shape, weight, bias, eps)


class _AddLNFn(torch.autograd.Function):
    """(s, y) = (x + h, LayerNorm(x + h)) in one kernel; backward dx = dh = LN'(dy) + ds."""

    @staticmethod
    def forward(ctx, x, h, weight, bias, eps):
        y, mean, rstd, s = native().ln_fwd(x, weight, bias, eps, h)
        ctx.save_for_backward(s, weight, mean, rstd)
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        s, weight, mean, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(s)
        dres = ds.contiguous() if ds is not None else None
        dx, dw, db = native().ln_bwd(dy.contiguous(), s, weight, mean, rstd, dres)
        return dx, dx, dw, db, None


def _ln_native_ok(x, weight, bias, normalized_shape) -> bool:
    D = x.shape[-1]
    return (use_native(x) and weight is not None and bias is not None and len(normalized_shape) == 1
            and D % 256 == 0 and D // 256 in _SUPPORTED_K and x.dtype in (torch.float32, torch.bfloat16)
            and weight.dtype == torch.float32 and bias.dtype == torch.float32)


def add_layer_norm(x: torch.Tensor, h: torch.Tensor, ln: nn.LayerNorm):
    """Pre-norm residual step: returns ``(s, ln(s))`` with ``s = x + h``. On the native path the
    add, the LayerNorm and (in backward) the two gradients of ``s`` are one kernel each way,
    instead of an add kernel + LayerNorm forward and LayerNorm backward + an add kernel."""
    if (_ln_native_ok(x, ln.weight, ln.bias, ln.normalized_shape) and h.shape == x.shape
            and h.dtype == x.dtype):
        return _AddLNFn.apply(x.contiguous(), h.contiguous(), ln.weight, ln.bias, float(ln.eps))
    s = x + h
    return s, ln(s)


class LayerNorm(nn.LayerNorm):
    def forward(self, x):
        return layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)
