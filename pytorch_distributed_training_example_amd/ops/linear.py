"""Linear layer with the bias gradient on the column-strip HIP kernel (csrc/kernels/gelu.hip).

Forward is one hipBLASLt GEMM with the bias fused in its epilogue (``F.linear``). Backward is the
two library GEMMs (dX = dY·W, dW = dYᵀ·X) plus ``colsum`` for dbias — aten would reduce dY with a
generic ``sum(0)`` reduction kernel, which streams a [tokens, D] bf16 gradient at a fraction of
HBM rate (profiles/r1_steady_gpt2_medium_ours.md: 73 ``reduce_kernel`` calls, 1.6 ms/step).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from ..config import SW
from ._native import native, use_native

# weight gradient dW = dY^T X sums over all tokens (K = 6K-25K): one hipBLASLt GEMM leaves most of
# the chip idle on the ViT/GPT-2 shapes (27-36 output tiles of 256x256); split-K batched GEMMs
# over token slices + an fp32-accumulated sum measured 0.5-0.9x of its time
# (tools/linear_wgrad_bench.py). The slice count is timed once per shape (eager steps; a shape
# first seen under hipGraph capture keeps the single GEMM). PDT_LINEAR_SPLITK=0: single GEMM.
_WG_CHOICE: Dict[Tuple, int] = {}


def _wgrad(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    from .conv import _wgrad_splitk
    T = dy2.shape[0]
    if not SW.linear_splitk or not dy2.is_cuda:
        return dy2.t() @ x2
    key = (T, dy2.shape[1], x2.shape[1], dy2.dtype)
    sk = _WG_CHOICE.get(key)
    if sk is None:
        if torch.cuda.is_current_stream_capturing():
            return dy2.t() @ x2
        cands = {1: lambda: dy2.t() @ x2}
        for s in (2, 4, 8, 16):
            if T % s == 0 and T // s >= 256:
                cands[s] = (lambda s=s: _wgrad_splitk(dy2, x2, s))
        from .conv import _time
        times = {s: _time(fn) for s, fn in cands.items()}
        sk = _WG_CHOICE[key] = min(times, key=times.get)
    return dy2.t() @ x2 if sk == 1 else _wgrad_splitk(dy2, x2, sk)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        d = dy.shape[-1]
        dy2 = dy.reshape(-1, d)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = (dy2 @ w).reshape(*dy.shape[:-1], w.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _wgrad(dy2, x.reshape(-1, x.shape[-1]))
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = native().colsum(dy2, w.dtype)
        return dx, dw, db


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    if (use_native(x) and x.dtype in (torch.float32, torch.bfloat16) and weight.dtype == x.dtype
            and (bias is None or bias.dtype == x.dtype) and weight.shape[0] % 8 == 0):
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)
