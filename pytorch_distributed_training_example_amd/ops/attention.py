"""Scaled-dot-product attention backed by the flash-attention HIP kernels (csrc/kernels/attention.hip).

``attention_qkv(qkv, heads, causal)`` takes the packed QKV projection output [B, T, 3·H·Dh]
(bf16, the c_attn GEMM result) and returns [B, T, H·Dh] ready for the output projection:
the kernels read Q/K/V through strided views of the packed tensor and write O token-major,
and the backward writes dQ/dK/dV straight into one packed [B, T, 3·H·Dh] gradient — no
permute/contiguous/cat copies around attention (PyTorch SDPA needs three of them).

Head dim 64 (ViT-B/16, GPT-2-medium) runs on the HIP kernels; anything else falls back to
``F.scaled_dot_product_attention``. CPU tensors use the math reference.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ._native import native, use_native

KERNEL_HEAD_DIMS = (64,)


def _views(qkv: torch.Tensor, heads: int):
    B, T, C3 = qkv.shape
    dh = C3 // (3 * heads)
    v5 = qkv.view(B, T, 3, heads, dh)
    return [v5[:, :, i].permute(0, 2, 1, 3) for i in range(3)], dh  # each [B, H, T, Dh] strided


class _FlashQKVFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads, causal, scale):
        B, T, _ = qkv.shape
        (q, k, v), dh = _views(qkv, heads)
        out = torch.empty(B, T, heads, dh, device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty(B, heads, T, device=qkv.device, dtype=torch.float32)
        native().attn_fwd_out(q, k, v, out.permute(0, 2, 1, 3), lse, causal, scale)
        ctx.save_for_backward(qkv, out, lse)
        ctx.heads, ctx.causal, ctx.scale = heads, causal, scale
        return out.view(B, T, heads * dh)

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        B, T, _ = qkv.shape
        heads = ctx.heads
        (q, k, v), dh = _views(qkv, heads)
        dout = dout.contiguous().view(B, T, heads, dh).permute(0, 2, 1, 3)
        dqkv = torch.empty_like(qkv)
        (dq, dk, dv), _ = _views(dqkv, heads)
        native().attn_bwd_out(dout, q, k, v, out.permute(0, 2, 1, 3), lse, dq, dk, dv, ctx.causal, ctx.scale)
        return dqkv, None, None, None


def attention_qkv(qkv: torch.Tensor, heads: int, causal: bool = False, dropout_p: float = 0.0,
                  scale: float | None = None) -> torch.Tensor:
    """Packed-QKV attention: [B, T, 3·H·Dh] -> [B, T, H·Dh]."""
    B, T, C3 = qkv.shape
    dh = C3 // (3 * heads)
    scale = scale if scale is not None else 1.0 / math.sqrt(dh)
    if (use_native(qkv) and qkv.dtype == torch.bfloat16 and dh in KERNEL_HEAD_DIMS and dropout_p == 0.0
            and qkv.stride(-1) == 1 and hasattr(native(), "attn_fwd_out")):
        return _FlashQKVFn.apply(qkv.contiguous(), heads, causal, scale)
    (q, k, v), _ = _views(qkv, heads)
    if qkv.is_cuda:
        y = F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=causal, scale=scale)
    else:
        y = attention_reference(q, k, v, causal, scale).to(qkv.dtype)
    return y.transpose(1, 2).reshape(B, T, heads * dh)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False,
              dropout_p: float = 0.0, scale: float | None = None) -> torch.Tensor:
    """Unpacked [B, H, T, Dh] interface (SDPA-compatible)."""
    return F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=causal, scale=scale)


def attention_reference(q, k, v, causal=False, scale=None):
    """fp32 math reference (tests, CPU)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if causal:
        T, S = s.shape[-2], s.shape[-1]
        mask = torch.ones(T, S, dtype=torch.bool, device=q.device).tril(S - T)
        s = s.masked_fill(~mask, float("-inf"))
    return torch.softmax(s, dim=-1) @ v.float()
