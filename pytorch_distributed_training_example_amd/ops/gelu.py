"""Bias + GELU (csrc/kernels/gelu.hip): ``gelu(x + bias)`` with the bias gradient fused."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from ._native import native, use_native


class _BiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, tanh_form):
        y = native().bias_gelu_fwd(x, bias, tanh_form)
        ctx.save_for_backward(x, bias)
        ctx.tanh_form = tanh_form
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        dx, db = native().bias_gelu_bwd(dy.contiguous(), x, bias, ctx.tanh_form)
        return dx, (db if bias is not None else None), None


def bias_gelu(x: torch.Tensor, bias: Optional[torch.Tensor] = None, approximate: str = "none") -> torch.Tensor:
    tanh_form = approximate == "tanh"
    if bias is not None and bias.dtype == torch.bfloat16 and (not bias.is_contiguous() or bias.data_ptr() % 16):
        bias = bias.float()  # the kernel reads 8 bf16 bias values per 16-B load
    if (use_native(x) and x.dtype in (torch.float32, torch.bfloat16) and x.shape[-1] % 8 == 0
            and (bias is None or bias.dtype == torch.float32 or (bias.dtype == torch.bfloat16 and bias.is_contiguous()))):
        # (a bf16 bias is read as is and gets a bf16 gradient: no fp32 copy and no cast back)
        return _BiasGeluFn.apply(x.contiguous(), bias, tanh_form)
    if bias is not None:
        x = x + bias.to(x.dtype)
    return F.gelu(x, approximate=approximate)
