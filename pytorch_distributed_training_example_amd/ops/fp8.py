"""FP8 (OCP e4m3fn) Linear layers with delayed per-tensor scaling — BASELINE.json config 3
("ViT-B/16 DDP + AMP (bf16/fp8)").

Every Linear inside the transformer blocks runs its three GEMMs on fp8 operands through
hipBLASLt (``torch._scaled_mm``; 1.4-2.3x the bf16 rate on these shapes on gfx950,
tools/fp8_bench.py) with fp32 accumulation and bf16 outputs:

    fwd    Y  = Xq · Wqᵀ              (+ bias in the GEMM epilogue)
    dgrad  dX = dYq · Wq
    wgrad  dW = dYqᵀ · Xq             (dbias on the column-strip kernel)

The casts (csrc/kernels/fp8.hip) write each operand once row-major and once transposed — the
layouts the three GEMMs need — in one pass, scaled by the tensor's *delayed* scale (derived from
the max |x| over the last ``history`` steps) and folding this step's max |x| into the tensor's
amax slot. All scaling state lives in one device tensor per model (``Fp8State``); one kernel per
forward refreshes every scale. No host synchronisation anywhere: the step stays capturable.

Master weights stay fp32 in the optimizer and parameters bf16 (models/precision.py); only GEMM
operands are fp8.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from ._native import native, use_native


class Fp8State(nn.Module):
    """Scaling state of ``n`` fp8 tensors: rows (amax, scale, scale_inv, history[L])."""

    def __init__(self, n: int, history: int = 16, margin: float = 0.0):
        super().__init__()
        self.history, self.margin = history, margin
        st = torch.zeros(n, 3 + history)
        st[:, 1:3] = 1.0
        self.register_buffer("state", st, persistent=False)
        self.next_slot = 0

    def alloc(self, k: int) -> int:
        i = self.next_slot
        if i + k > self.state.shape[0]:
            raise RuntimeError("Fp8State: out of slots")
        self.next_slot += k
        return i

    @torch.no_grad()
    def update(self) -> None:
        if self.state.is_cuda:
            native().fp8_update_scales(self.state, self.history, self.margin)


class _Fp8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, state, slot):
        C = native()
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        xq, xqt = C.fp8_cast_transpose(x2, state[slot], True)
        wq, wqt = C.fp8_cast_transpose(w, state[slot + 1], True)
        y = torch._scaled_mm(xq, wq.t(), scale_a=state[slot, 2], scale_b=state[slot + 1, 2], bias=b,
                             out_dtype=torch.bfloat16)
        ctx.save_for_backward(xqt, wqt, state)
        ctx.slot, ctx.has_b, ctx.xshape = slot, b is not None, x.shape
        return y.reshape(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        xqt, wqt, state = ctx.saved_tensors
        s = ctx.slot
        C = native()
        n = dy.shape[-1]
        dy2 = dy.reshape(-1, n)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dyq, dyqt = C.fp8_cast_transpose(dy2, state[s + 2], True)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch._scaled_mm(dyq, wqt.t(), scale_a=state[s + 2, 2], scale_b=state[s + 1, 2],
                                  out_dtype=torch.bfloat16).reshape(ctx.xshape)
        if ctx.needs_input_grad[1]:
            dw = torch._scaled_mm(dyqt, xqt.t(), scale_a=state[s + 2, 2], scale_b=state[s, 2],
                                  out_dtype=torch.bfloat16)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = C.colsum(dy2, torch.bfloat16)
        return dx, dw, db, None, None


def fp8_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    m = x.numel() // max(x.shape[-1], 1)
    return (use_native(x) and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.shape[-1] % 16 == 0 and w.shape[0] % 16 == 0 and m % 16 == 0 and m > 0)


def fp8_linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], state: Fp8State,
               slot: int) -> torch.Tensor:
    if fp8_ok(x, weight):
        return _Fp8LinearFn.apply(x, weight, bias, state.state, slot)
    return torch.nn.functional.linear(x, weight, bias)


def enable_fp8(model: nn.Module, history: int = 16, margin: float = 0.0, blocks_only: bool = True) -> Fp8State:
    """Route ``nn.Linear`` layers through fp8 GEMMs (3 scaling slots each: input, weight,
    output-gradient) — by default those inside transformer ``Block``s (the classifier / LM heads
    stay bf16). Registers the state on the model and a forward pre-hook that refreshes all scales
    once per training forward. Returns the state."""
    from ..models.transformer import Block
    roots = [m for m in model.modules() if isinstance(m, Block)] if blocks_only else [model]
    lins = [m for r in roots for m in r.modules() if isinstance(m, nn.Linear)]
    state = Fp8State(3 * len(lins), history, margin)
    p = next(model.parameters(), None)
    if p is not None:
        state.to(p.device)
    for m in lins:
        m._fp8 = (state, state.alloc(3))
    model.fp8_state = state

    def _refresh(mod, args):
        if mod.training:
            state.update()
    model._fp8_hook = model.register_forward_pre_hook(_refresh)
    return state
