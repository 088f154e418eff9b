"""GPT-2 token + position embedding on our HIP kernels (csrc/kernels/embedding.hip).

Forward: ``wte[idx] + wpe[arange(T)]`` in ONE pass (aten: two gathers and an add). Backward:
a deterministic scatter — counting sort of the token ids, then each vocabulary row sums its
tokens' gradient rows in increasing token order and is written exactly once (no zero-fill pass,
no atomics on the gradient values, no sort-based aten path), and the position gradient sums the
batch in order. Reruns and replicas give bit-identical ``wte``/``wpe`` gradients.

Not in the reference (its only model is LeNet, /root/reference/cnn.py); SURVEY.md §2.3 lists the
embedding among the kernels the GPT-2 north-star config needs. CPU / fp32 / disabled-native inputs
take the PyTorch reference path (same math).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..config import SW
from ._native import native, use_native


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe):
        ctx.save_for_backward(idx)
        ctx.V, ctx.P = wte.shape[0], wpe.shape[0]
        return native().embedding_fwd(idx, wte, wpe)

    @staticmethod
    def backward(ctx, dout):
        (idx,) = ctx.saved_tensors
        dwte, dwpe = native().embedding_bwd(idx, dout, ctx.V, ctx.P)
        return None, dwte, dwpe


def token_position_embedding(idx: torch.Tensor, wte: torch.Tensor, wpe: torch.Tensor) -> torch.Tensor:
    """``wte[idx] + wpe[arange(T)]`` for idx [B, T]."""
    if (use_native(idx, wte) and SW.embedding_native and wte.dtype == torch.bfloat16 and wpe.dtype == torch.bfloat16
            and idx.dtype == torch.long and idx.dim() == 2 and wte.shape[1] % 8 == 0 and wte.is_contiguous()
            and wpe.is_contiguous() and idx.shape[1] <= wpe.shape[0]):
        return _EmbeddingFn.apply(idx.contiguous(), wte, wpe)
    pos = torch.arange(idx.shape[1], device=idx.device)
    return F.embedding(idx, wte) + F.embedding(pos, wpe)
