"""Scaled-dot-product attention entry point.

``attention(q, k, v, causal)`` on [B, H, T, Dh] tensors. On GPU it dispatches to the
hand-written flash-attention HIP kernel (csrc/kernels/attention.hip) when that kernel covers
the shape, otherwise to PyTorch's fused SDPA. CPU tensors use the math reference.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ._native import native, use_native

_HAS_KERNEL = None


def _kernel_ok(q: torch.Tensor, dropout_p: float) -> bool:
    global _HAS_KERNEL
    if _HAS_KERNEL is None:
        _HAS_KERNEL = hasattr(native(), "attn_fwd")
    return (_HAS_KERNEL and dropout_p == 0.0 and q.dtype == torch.bfloat16 and q.shape[-1] in (64, 128))


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = native().attn_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = native().attn_bwd(do.contiguous(), q, k, v, o, lse, ctx.causal, ctx.scale)
        return dq, dk, dv, None, None


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False,
              dropout_p: float = 0.0, scale: float | None = None) -> torch.Tensor:
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if use_native(q) and _kernel_ok(q, dropout_p):
        return _FlashAttnFn.apply(q.contiguous(), k.contiguous(), v.contiguous(), causal, scale)
    return F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=causal, scale=scale)


def attention_reference(q, k, v, causal=False, scale=None):
    """fp32 math reference (tests)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if causal:
        T, S = s.shape[-2], s.shape[-1]
        mask = torch.ones(T, S, dtype=torch.bool, device=q.device).tril(S - T)
        s = s.masked_fill(~mask, float("-inf"))
    return torch.softmax(s, dim=-1) @ v.float()
