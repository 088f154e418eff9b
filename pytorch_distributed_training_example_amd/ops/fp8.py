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

from ..config import SW
from ._native import native, use_native


class Fp8State(nn.Module):
    """Scaling state of ``n`` fp8 tensors: rows (amax, scale, scale_inv, pad, 16 amax stripes 16
    floats apart, history[L]) — csrc/fp8_pack.h. The producing kernels fold each workgroup's |x|max
    into stripe (workgroup % 16) instead of one word (one contended L2 line cost 8.6 us of a 23 us
    cast); ``update`` reduces the stripes into the history."""

    STRIPED = 260  # history offset of a striped row

    def __init__(self, n: int, history: int = 16, margin: float = 0.0):
        super().__init__()
        self.history, self.margin = history, margin
        st = torch.zeros(n, self.STRIPED + history)
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

    @torch.no_grad()
    def cast_weights(self, lins) -> None:
        """fp8 copies (row-major + transposed) of every tagged Linear's weight in ONE launch
        (``fp8_cast_multi``), cached for this forward: the per-Linear cast launches are gone."""
        self.wcache = {}
        ws = [m.weight for m in lins if fp8_ok_weight(m.weight)]
        if not ws or not ws[0].is_cuda:
            return
        rows = [self.state[m._fp8[1] + 1] for m in lins if fp8_ok_weight(m.weight)]
        out = native().fp8_cast_multi(ws, rows)
        for i, w in enumerate(ws):
            self.wcache[id(w)] = (w, out[2 * i], out[2 * i + 1], w._version)

    def weight_fp8(self, w: torch.Tensor, slot: int):
        """(wq, wqt) of ``w``: this forward's cached cast, or a cast now (eval / untagged calls, or a weight
        modified in place since the cast — e.g. a submodule called right after optimizer.step: the version
        counter tells, so a GEMM never reads a stale fp8 copy)."""
        e = self.wcache.get(id(w)) if getattr(self, "wcache", None) else None
        if e is not None and e[0] is w and e[3] == w._version:
            return e[1], e[2]
        return native().fp8_cast_transpose(w, self.state[slot + 1], True)

    def clear_weight_cache(self) -> None:
        """Drop this forward's fp8 weight copies (they are otherwise kept until the next forward recasts)."""
        self.wcache = {}


class _Fp8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, state, slot, st=None, xq=None, xqt=None):
        C = native()
        K = x.shape[-1]
        if xq is None:
            x2 = x.reshape(-1, K)
            if not x2.is_contiguous():
                x2 = x2.contiguous()
            xq, xqt = C.fp8_cast_transpose(x2, state[slot], True)
        wq, wqt = st.weight_fp8(w, slot) if st is not None else C.fp8_cast_transpose(w, state[slot + 1], True)
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
        dx = dw = db = None
        if ctx.has_b and ctx.needs_input_grad[2] and _colsum_ok(dy2):
            dyq, dyqt, db = C.fp8_cast_colsum(dy2, state[s + 2], torch.bfloat16)  # cast + bias grad, one pass
        else:
            dyq, dyqt = C.fp8_cast_transpose(dy2, state[s + 2], True)
        if ctx.needs_input_grad[0]:
            dx = torch._scaled_mm(dyq, wqt.t(), scale_a=state[s + 2, 2], scale_b=state[s + 1, 2],
                                  out_dtype=torch.bfloat16).reshape(ctx.xshape)
        if ctx.needs_input_grad[1]:
            dw = torch._scaled_mm(dyqt, xqt.t(), scale_a=state[s + 2, 2], scale_b=state[s, 2],
                                  out_dtype=torch.bfloat16)
        if ctx.has_b and ctx.needs_input_grad[2] and db is None:
            db = C.colsum(dy2, torch.bfloat16)
        return dx, dw, db, None, None, None, None, None


def _colsum_ok(dy2: torch.Tensor) -> bool:
    return SW.fp8_cast_colsum and dy2.shape[1] % 64 == 0


def fp8_ok_weight(w: torch.Tensor) -> bool:
    return (w.dim() == 2 and w.dtype == torch.bfloat16 and w.is_contiguous() and w.shape[0] % 16 == 0
            and w.shape[1] % 16 == 0)


def fp8_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    m = x.numel() // max(x.shape[-1], 1)
    return (use_native(x) and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.shape[-1] % 16 == 0 and w.shape[0] % 16 == 0 and m % 16 == 0 and m > 0)


class Fp8Act:
    """An activation its producer already wrote in e4m3 for the fp8 GEMM that consumes it
    (``add_layer_norm_fp8``): the row-major and transposed copies, plus ``token`` — a
    zero-storage bf16 tensor of the activation's shape that carries the autograd edge (the
    consumer returns the bf16 gradient of the activation as the token's gradient)."""
    __slots__ = ("token", "q", "qt")

    def __init__(self, token, q, qt):
        self.token, self.q, self.qt = token, q, qt

    @property
    def shape(self):
        return self.token.shape


def fp8_linear(x, weight: torch.Tensor, bias: Optional[torch.Tensor], state: Fp8State,
               slot: int) -> torch.Tensor:
    if isinstance(x, Fp8Act):  # the producer emitted fp8 for exactly this GEMM (fp8_input_slot)
        return _Fp8LinearFn.apply(x.token, weight, bias, state.state, slot, state, x.q, x.qt)
    if fp8_ok(x, weight):
        return _Fp8LinearFn.apply(x, weight, bias, state.state, slot, state)
    return torch.nn.functional.linear(x, weight, bias)


class _Fp8MlpFn(torch.autograd.Function):
    """fc1 -> bias + GELU -> fc2 with the activation produced in fp8 where it is computed:
    ``fp8_gelu_cast`` turns fc1's bf16 output h into gelu(h + b1) as e4m3 (+ transpose) in one
    pass, and its backward form turns (dg, h) into dh = dg gelu'(h + b1) as e4m3 (+ transpose,
    + the b1 gradient). The bf16 activation and its gradient are never written (unfused: a strip
    kernel writing them + a cast-transpose reading them back, twice per block)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, state, s1, s2, st, tanh_form, xq=None, xqt=None):
        C = native()
        D = x.shape[-1]
        if xq is None:
            x2 = x.reshape(-1, D)
            if not x2.is_contiguous():
                x2 = x2.contiguous()
            xq, xqt = C.fp8_cast_transpose(x2, state[s1], True)
        w1q, w1qt = st.weight_fp8(w1, s1)
        h = torch._scaled_mm(xq, w1q.t(), scale_a=state[s1, 2], scale_b=state[s1 + 1, 2], out_dtype=torch.bfloat16)
        b1f = None if b1 is None else b1.float()
        gq, gqt, _ = C.fp8_gelu_cast(h, None, b1f, state[s2], tanh_form)
        w2q, w2qt = st.weight_fp8(w2, s2)
        y = torch._scaled_mm(gq, w2q.t(), scale_a=state[s2, 2], scale_b=state[s2 + 1, 2], bias=b2,
                             out_dtype=torch.bfloat16)
        ctx.save_for_backward(xqt, w1qt, h, gqt, w2qt, b1f, state)
        ctx.s1, ctx.s2, ctx.tanh_form, ctx.xshape = s1, s2, tanh_form, x.shape
        ctx.b1_dtype = None if b1 is None else b1.dtype
        ctx.has_b2 = b2 is not None
        return y.reshape(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        xqt, w1qt, h, gqt, w2qt, b1f, state = ctx.saved_tensors
        s1, s2 = ctx.s1, ctx.s2
        C = native()
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        db2 = None
        if ctx.has_b2 and _colsum_ok(dy2):
            dyq, dyqt, db2 = C.fp8_cast_colsum(dy2, state[s2 + 2], torch.bfloat16)
        else:
            dyq, dyqt = C.fp8_cast_transpose(dy2, state[s2 + 2], True)
        dg = torch._scaled_mm(dyq, w2qt.t(), scale_a=state[s2 + 2, 2], scale_b=state[s2 + 1, 2],
                              out_dtype=torch.bfloat16)
        dw2 = torch._scaled_mm(dyqt, gqt.t(), scale_a=state[s2 + 2, 2], scale_b=state[s2, 2], out_dtype=torch.bfloat16)
        if ctx.has_b2 and db2 is None:
            db2 = C.colsum(dy2, torch.bfloat16)
        dbt = ctx.b1_dtype if ctx.b1_dtype in (torch.float32, torch.bfloat16) else torch.float32
        dhq, dhqt, db1 = C.fp8_gelu_cast(h, dg, b1f, state[s1 + 2], ctx.tanh_form, dbt)
        dx = torch._scaled_mm(dhq, w1qt.t(), scale_a=state[s1 + 2, 2], scale_b=state[s1 + 1, 2],
                              out_dtype=torch.bfloat16).reshape(ctx.xshape)
        dw1 = torch._scaled_mm(dhqt, xqt.t(), scale_a=state[s1 + 2, 2], scale_b=state[s1, 2], out_dtype=torch.bfloat16)
        if db1 is not None and ctx.b1_dtype is not None and db1.dtype != ctx.b1_dtype:
            db1 = db1.to(ctx.b1_dtype)
        return dx, dw1, db1, dw2, db2, None, None, None, None, None, None, None


def _mlp_ok(x: torch.Tensor, fc1: nn.Linear, fc2: nn.Linear) -> bool:
    a, b = getattr(fc1, "_fp8", None), getattr(fc2, "_fp8", None)
    if a is None or b is None or a[0] is not b[0] or not SW.fp8_fused_gelu:
        return False
    m = x.numel() // max(x.shape[-1], 1)
    return (fp8_ok(x, fc1.weight) and fc2.weight.dtype == torch.bfloat16 and fc1.weight.shape[0] % 64 == 0
            and fc2.weight.shape[0] % 16 == 0 and fc1.weight.is_contiguous() and fc2.weight.is_contiguous()
            and m % 16 == 0 and (fc1.bias is None or fc1.bias.dtype in (torch.float32, torch.bfloat16)))


def fp8_mlp(x, fc1: nn.Linear, fc2: nn.Linear, approximate: str) -> Optional[torch.Tensor]:
    """The MLP on fp8 with the fused GELU casts, or None when a shape / dtype is not served (the
    caller then runs the per-Linear path). ``x`` may be an ``Fp8Act`` (then it is always served)."""
    a, b = getattr(fc1, "_fp8", None), getattr(fc2, "_fp8", None)
    pre = isinstance(x, Fp8Act)
    xt = x.token if pre else x
    if not pre and not _mlp_ok(x, fc1, fc2):
        return None
    st = a[0]
    return _Fp8MlpFn.apply(xt, fc1.weight, fc1.bias, fc2.weight, fc2.bias, st.state, a[1], b[1], st,
                           approximate == "tanh", x.q if pre else None, x.qt if pre else None)


def fp8_input_slot(consumer: nn.Module, x: torch.Tensor):
    """(state, slot) when ``consumer`` — an fp8-tagged Linear, or an MLP whose fused fp8 path
    will run — takes ``x`` as an fp8 GEMM operand and can be handed an ``Fp8Act``; else None."""
    if not SW.fp8_ln:
        return None
    if isinstance(consumer, nn.Linear):
        t = getattr(consumer, "_fp8", None)
        return (t[0], t[1]) if t is not None and fp8_ok(x, consumer.weight) else None
    fc1, fc2 = getattr(consumer, "c_fc", None), getattr(consumer, "c_proj", None)
    if isinstance(fc1, nn.Linear) and isinstance(fc2, nn.Linear) and _mlp_ok(x, fc1, fc2):
        return fc1._fp8[0], fc1._fp8[1]
    return None


class _AddLNFp8Fn(torch.autograd.Function):
    """(s, y) = (x + h, LayerNorm(x + h)) with y emitted as e4m3 (+ transpose) for the consumer's
    fp8 GEMM (layernorm.hip ln_fwd_fp8_kernel): returns s, the zero-storage token standing for
    y, and the fp8 copies. Backward: the token's gradient is dy; dx = dh = LN'(dy) + ds, as the
    bf16 add+LayerNorm Function."""

    @staticmethod
    def forward(ctx, x, h, weight, bias, eps, state_row):
        D = x.shape[-1]
        yq, yqt, mean, rstd, s = native().ln_fwd_fp8(x.reshape(-1, D), weight, bias, eps, h.reshape(-1, D), state_row)
        s = s.view(x.shape)
        token = torch.empty((), dtype=x.dtype, device=x.device).expand(x.shape)  # never read
        ctx.mark_non_differentiable(yq, yqt)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the fp8 copies
        ctx.save_for_backward(s, weight, mean, rstd)
        return s, token, yq, yqt

    @staticmethod
    def backward(ctx, ds, dy, _dq, _dqt):
        s, weight, mean, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(s)
        dres = ds.contiguous() if ds is not None else None
        dx, dw, db = native().ln_bwd(dy.contiguous(), s, weight, mean, rstd, dres)
        return dx, dx, dw, db, None, None


def add_layer_norm_fp8(x: torch.Tensor, h: torch.Tensor, ln: nn.Module, state: "Fp8State", slot: int):
    """``(s, Fp8Act(ln(s)))`` with ``s = x + h``; the caller checked ``fp8_input_slot``."""
    s, token, q, qt = _AddLNFp8Fn.apply(x.contiguous(), h.contiguous(), ln.weight, ln.bias, float(ln.eps),
                                        state.state[slot])
    return s, Fp8Act(token, q, qt)


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
            if SW.fp8_weight_multi:
                state.cast_weights(lins)
        else:
            state.wcache = {}
    model._fp8_hook = model.register_forward_pre_hook(_refresh)
    return state
