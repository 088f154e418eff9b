"""GPT-2 token + position embedding on our HIP kernels (csrc/kernels/embedding.hip).

Forward: ``wte[idx] + wpe[arange(T)]`` in ONE pass (aten: two gathers and an add). Backward:
a deterministic scatter — counting sort of the token ids, then each vocabulary row sums its
tokens' gradient rows in increasing token order and is written exactly once (no zero-fill pass,
no atomics on the gradient values, no sort-based aten path), and the position gradient sums the
batch in order. Reruns and replicas give bit-identical ``wte``/``wpe`` gradients.

Not in the reference (its only model is LeNet, /root/reference/cnn.py); SURVEY.md §2.3 lists the
embedding among the kernels the GPT-2 north-star config needs. CPU / fp32 / disabled-native inputs
take the PyTorch reference path (same math).

Token ids are range-checked on the device: an id outside [0, V) reads nothing (zero output row, no
gradient) and sets an error word. Without a host sync, that word is copied to pinned memory behind
every forward and checked at the next call (``IndexError``, one step late, like an asynchronous
device assert; raised once, then cleared); ``check_ids()`` syncs and checks now. ``PDT_EMBEDDING_CHECK=1`` checks every call.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

import os

from ..config import SW
from ._native import native, use_native

_ERR = {"host": None, "event": None}
_SYNC_CHECK = os.environ.get("PDT_EMBEDDING_CHECK", "0") == "1"


def _raise_if_bad(err_value: int) -> None:
    if err_value:
        raise IndexError("token_position_embedding: a token id is outside [0, vocab size) "
                         "(its rows were zeroed; the error word stays set: see check_ids)")


def _poll_previous(device) -> None:
    """Raise (once) for an out-of-range id seen by the PREVIOUS call. The error is cleared before
    raising — the device word is zeroed stream-ordered, ahead of this call's kernel — so a caller
    that catches the IndexError is not poisoned on every later step (nn.Embedding raises once)."""
    ev = _ERR["event"]
    if ev is not None and not torch.cuda.is_current_stream_capturing() and ev.query():
        bad = int(_ERR["host"][0])
        if bad:
            _ERR["event"] = None
            _ERR["host"].zero_()
            native().embedding_err(torch.empty(0, device=device)).zero_()
            raise IndexError("token_position_embedding: a token id of the PREVIOUS call was outside "
                             "[0, vocab size) (its rows were zeroed; set PDT_EMBEDDING_CHECK=1 to "
                             "raise on the offending call itself)")


def check_ids(device=None) -> None:
    """Host sync: raise IndexError if any embedding call so far saw an out-of-range id."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    _raise_if_bad(int(native().embedding_err(torch.empty(0, device=dev)).item()))


def reset_id_errors(device=None) -> None:
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    native().embedding_err(torch.empty(0, device=dev)).zero_()
    _ERR["event"] = None


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe):
        ctx.save_for_backward(idx)
        ctx.V, ctx.P = wte.shape[0], wpe.shape[0]
        _poll_previous(idx.device)
        out = native().embedding_fwd(idx, wte, wpe)
        if _SYNC_CHECK:
            check_ids(idx.device)
        elif not torch.cuda.is_current_stream_capturing():
            if _ERR["host"] is None:
                _ERR["host"] = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            _ERR["host"].copy_(native().embedding_err(idx), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            _ERR["event"] = ev
        return out

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
