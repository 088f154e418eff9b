"""Linear layer with the bias gradient on the column-strip HIP kernel (csrc/kernels/gelu.hip).

Forward is one hipBLASLt GEMM with the bias fused in its epilogue (``F.linear``). Backward is the
two library GEMMs (dX = dY·W, dW = dYᵀ·X) plus ``colsum`` for dbias — aten would reduce dY with a
generic ``sum(0)`` reduction kernel, which streams a [tokens, D] bf16 gradient at a fraction of
HBM rate (profiles/r1_steady_gpt2_medium_ours.md: 73 ``reduce_kernel`` calls, 1.6 ms/step).

Forward GEMMs on our MFMA kernel (csrc/kernels/gemm.hip: bias epilogue, and the MLP's fc1 + bias + GELU in
one pass, ``linear_gelu``) are chosen PER SHAPE by measurement, as the 1x1 convs are (ops/conv.py _pick):
``PDT_LINEAR_EPILOGUE=auto`` (default) looks the (kind, M, N, K) up in ``tuning/linear_gfx950.json`` (decided by
whole-step A/B); a shape not in the table runs the library. ``=time`` times an unlisted shape once (eager steps
only) against hipBLASLt (+ our bias+GELU kernel for the fused kind) and caches the winner — isolated timings
mispredict the step (GPT-2-medium lost 3 % on them), hence not the default. Our kernel wins on
some shapes only (vit_qkv 1.08x, vit_fc2 1.03x, gpt2_proj + bias 1.05x; 0.61-0.94x on the others:
profiles/r5/gemm_bn128.txt, profiles/r3/gemm_vs_hipblaslt.md), so all-or-nothing would lose. ``=1``: ours
on every shape it serves, ``=0``: never. ``PDT_LINEAR_DUMP=path`` writes the decisions at exit.
"""
from __future__ import annotations

import atexit
import json
import os
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


def gemm_nt_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes our GEMM kernel serves: bf16, out features % 128, in features % 64."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.dim() == 2
            and w.shape[0] % 128 == 0 and w.shape[1] % 64 == 0 and x.shape[-1] == w.shape[1] and x.numel() > 0)


_LIN_CHOICE: Dict[str, str] = {}
_LIN_TABLE = [False]
TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tuning",
                     "linear_gfx950.json")


def _lin_table() -> None:
    if _LIN_TABLE[0]:
        return
    _LIN_TABLE[0] = True
    try:
        with open(TABLE) as f:
            d = json.load(f)
        if d.get("arch") in (None, _arch()):
            _LIN_CHOICE.update({k: v for k, v in d.get("choices", {}).items() if v in ("ours", "lib")})
    except (OSError, ValueError):
        pass
    out = os.environ.get("PDT_LINEAR_DUMP")
    if out:
        atexit.register(lambda: json.dump({"arch": _arch(), "choices": dict(sorted(_LIN_CHOICE.items()))},
                                          open(out, "w"), indent=1))


def _arch() -> str:
    try:
        return torch.cuda.get_device_properties(0).gcnArchName.split(":")[0]
    except Exception:  # pragma: no cover - no GPU
        return "cpu"


def _ours(x: torch.Tensor, w: torch.Tensor, kind: str = "bias", b: Optional[torch.Tensor] = None,
          tanh_form: bool = False) -> bool:
    """Run this forward GEMM (``kind``: "bias" | "nobias" | "gelu") on our kernel? See the module docstring."""
    mode = SW.linear_epilogue
    if mode == "0" or not gemm_nt_ok(x, w):
        return False
    if mode == "1":
        return True
    M, K, N = x.numel() // x.shape[-1], x.shape[-1], w.shape[0]
    key = f"{kind},{M},{N},{K}"
    c = _LIN_CHOICE.get(key)
    if c is None:
        _lin_table()
        c = _LIN_CHOICE.get(key)
    if c is None and mode != "time":
        # a shape the table does not list runs the library: isolated forward timings picked ours for GPT-2-medium's
        # qkv / fc1 / fused GELU and the whole step lost 3 % (tuning/linear_gfx950.json _note); "time" re-enables it
        c = _LIN_CHOICE[key] = "lib"
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return False
        from .conv import _time
        x2, wc = x.reshape(-1, K).contiguous(), w.contiguous()
        if kind == "gelu":
            bf = b.float() if b is not None else None
            ours = lambda: native().gemm_nt(x2, wc, bf, 2, tanh_form)  # noqa: E731
            from .gelu import bias_gelu
            lib = lambda: bias_gelu(F.linear(x2, wc), bf, "tanh" if tanh_form else "none")  # noqa: E731
        else:
            bb = b if kind == "bias" else None
            ours = lambda: native().gemm_nt(x2, wc, bb, 1 if bb is not None else 0, False)  # noqa: E731
            lib = lambda: F.linear(x2, wc, bb)  # noqa: E731
        with torch.no_grad():
            c = "ours" if _time(ours) < _time(lib) else "lib"
        _LIN_CHOICE[key] = c
    return c == "ours"


def linear_choices() -> Dict[str, str]:
    """Decisions taken so far: {"kind,M,N,K": "ours" | "lib"}."""
    return dict(_LIN_CHOICE)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        if _ours(x, w, "bias" if b is not None else "nobias", b):
            x2 = x.reshape(-1, x.shape[-1]).contiguous()
            y = native().gemm_nt(x2, w.contiguous(), b, 1 if b is not None else 0, False)[0]
            return y.view(*x.shape[:-1], w.shape[0])
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
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        # autocast does not reach into an autograd.Function: cast the operands the way autocast casts
        # F.linear's, then run (and later backpropagate) the Function with autocast off, so its saved
        # tensors and the incoming gradient share one dtype (amp_bf16: our bf16 path; amp_fp16: aten)
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return linear(x.to(dt), weight.to(dt), bias.to(dt) if bias is not None else None)
    if (use_native(x) and x.dtype in (torch.float32, torch.bfloat16) and weight.dtype == x.dtype
            and (bias is None or bias.dtype == x.dtype) and weight.shape[0] % 8 == 0):
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class Linear(torch.nn.Linear):
    """``nn.Linear`` (same parameters and state-dict keys) on :func:`linear`: dbias on the ``colsum``
    kernel. Besides speed this keeps the step hipGraph-safe: aten's ``sum(0)`` over a [1024, 1000]
    gradient takes its multi-block path, whose staging workspace does not survive a captured
    backward — a replay after any later allocation returns a wrong bias gradient (the ResNet head at
    1024/GPU trained to NaN; tools/diag_graph_colsum_bwd.py, profiles/r6/graph_colsum_bwd.txt)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.weight, self.bias)


class _LinearGeluFn(torch.autograd.Function):
    """g = gelu(x·Wᵀ + b) with the GEMM, bias and GELU in one kernel (EPI_GELU); h = x·Wᵀ is kept for
    the backward, which is the column-strip GELU-backward + bias-gradient kernel and two GEMMs."""

    @staticmethod
    def forward(ctx, x, w, b, tanh_form):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        bf = b.float() if b is not None else None
        h, g = native().gemm_nt(x2, w.contiguous(), bf, 2, tanh_form)
        ctx.save_for_backward(x2, w, h, bf)
        ctx.tanh_form, ctx.xshape, ctx.has_b, ctx.bdtype = tanh_form, x.shape, b is not None, (
            b.dtype if b is not None else None)
        return g.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dg):
        x2, w, h, bf = ctx.saved_tensors
        dh, db = native().bias_gelu_bwd(dg.reshape(h.shape).contiguous(), h, bf, ctx.tanh_form)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = (dh @ w).view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            dw = _wgrad(dh, x2)
        dbias = db.to(ctx.bdtype) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dw, dbias, None


def linear_gelu(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], approximate: str) -> Optional[torch.Tensor]:
    """gelu(linear(x, weight, bias)) on the fused-epilogue kernel, or None when it does not apply
    (switch off, unsupported shape/dtype): the caller then runs linear + bias_gelu."""
    if (bias is not None and bias.dtype not in (torch.bfloat16, torch.float32)) or not use_native(x) \
            or not _ours(x, weight, "gelu", bias, approximate == "tanh"):
        return None
    return _LinearGeluFn.apply(x, weight, bias, approximate == "tanh")
