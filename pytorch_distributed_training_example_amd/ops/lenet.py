"""LeNet (reference model) fused ops — csrc/kernels/lenet.hip.

  * ``lenet_stem``      upsample 28→32 (align_corners) + conv1 5×5 + bias + LeakyReLU + 2×2 max-pool
                        (/root/reference/cnn.py:9-12) in one kernel; backward gives conv1's dW/db only
                        (the input is data, it needs no gradient).
  * ``leaky_pool``      LeakyReLU + 2×2 max-pool with a 1-byte argmax/sign code (cnn.py:14-15).
  * ``lenet_tail``      everything after the stem — conv2 + LeakyReLU + pool, conv3 + LeakyReLU, fc1 +
                        LeakyReLU, fc2 (cnn.py:13-22) — as one forward kernel and two backward kernels
                        (csrc/kernels/lenet_tail.hip); returns the logits.
  * ``softmax_nll``     fused softmax loss for small class counts: ``mode='ce'`` cross-entropy, or
                        ``mode='prob_nll'`` — the reference's ``nll_loss`` on softmax probabilities
                        (cnn.py:23 + train.py:48, loss = −mean p_y) computed from logits. Forward
                        also produces the gradient of the mean loss (one pass over the logits).
  * ``eval_metrics_``   loss sum / correct / count accumulated on device for a batch of logits
                        (replaces train.py:68-70's per-batch ``.item()`` syncs).

CPU tensors (tests) run PyTorch reference implementations of the same math.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._native import native, use_native

SLOPE = 0.2  # LeakyReLU(0.2) throughout the reference LeNet (cnn.py:11,14,17,21)


# ---------------------------------------------------------------- references (CPU / oracle)
def stem_reference(x, w, b, slope=SLOPE):
    up = F.interpolate(x, size=(32, 32), mode="bilinear", align_corners=True)
    return F.max_pool2d(F.leaky_relu(F.conv2d(up, w, b), slope), 2)


def leaky_pool_reference(x, slope=SLOPE):
    return F.max_pool2d(F.leaky_relu(x, slope), 2)


def softmax_nll_reference(logits, target, mode="ce", label_smoothing=0.0):
    if mode == "ce":
        return F.cross_entropy(logits.float(), target, label_smoothing=label_smoothing)
    return F.nll_loss(torch.softmax(logits.float(), dim=-1), target)


# ---------------------------------------------------------------- autograd wrappers
class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, slope):
        y, code = native().lenet_stem_fwd(x, w, b, slope)
        ctx.save_for_backward(x, code)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, dy):
        x, code = ctx.saved_tensors
        dw, db = native().lenet_stem_bwd(dy, code, x, ctx.slope)
        return None, dw, db, None


class _LeakyPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slope):
        y, code = native().leaky_pool_fwd(x, slope)
        ctx.save_for_backward(code)
        ctx.shape, ctx.slope = x.shape, slope
        return y

    @staticmethod
    def backward(ctx, dy):
        (code,) = ctx.saved_tensors
        return native().leaky_pool_bwd(dy, code, ctx.shape[2], ctx.shape[3], ctx.slope), None


class _TailFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p1, slope, *params):
        logits, code2, p2, h3, h4 = native().lenet_tail_fwd(p1, list(params), slope)
        ctx.save_for_backward(p1, code2, p2, h3, h4, *params)
        ctx.slope = slope
        return logits

    @staticmethod
    def backward(ctx, dl):
        p1, code2, p2, h3, h4, *params = ctx.saved_tensors
        dp1, *g = native().lenet_tail_bwd(dl, p1, list(params), ctx.slope, code2, p2, h3, h4)
        return (dp1, None, *g)


def tail_reference(p1, params, slope=SLOPE):
    w2, b2, w3, b3, fw1, fb1, fw2, fb2 = params
    y = F.max_pool2d(F.leaky_relu(F.conv2d(p1, w2, b2), slope), 2)
    y = F.leaky_relu(F.conv2d(y, w3, b3), slope).reshape(p1.shape[0], -1)
    return F.linear(F.leaky_relu(F.linear(y, fw1, fb1), slope), fw2, fb2)


_TAIL_SHAPES = ((16, 6, 5, 5), (16,), (120, 16, 5, 5), (120,), (84, 120), (84,), (10, 84), (10,))


def tail_native_ok(p1, params) -> bool:
    return (p1.dim() == 4 and tuple(p1.shape[1:]) == (6, 14, 14) and p1.dtype == torch.float32
            and len(params) == 8 and all(tuple(p.shape) == s and p.dtype == torch.float32
                                         for p, s in zip(params, _TAIL_SHAPES)))


def lenet_tail(p1, params, slope=SLOPE):
    """Logits of the reference LeNet from the stem's pooled output p1 [N,6,14,14]; ``params`` = (conv2
    weight, bias, conv3 weight, bias, fc1 weight, bias, fc2 weight, bias)."""
    if use_native(p1) and tail_native_ok(p1, params):
        return _TailFn.apply(p1.contiguous(), float(slope), *[p.contiguous() for p in params])
    return tail_reference(p1, params, slope)


_MODES = {"ce": 0, "prob_nll": 1}


class _SoftmaxNLLFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, mode, smoothing):
        n = logits.shape[0]
        if n == 0:
            ctx.save_for_backward(torch.empty_like(logits))
            return logits.new_zeros((), dtype=torch.float32)
        _, dl, mean = native().softmax_nll_small(logits, target, _MODES[mode], smoothing, True, True, 1.0 / n, None,
                                                 mean_scale=1.0 / n)
        ctx.save_for_backward(dl)
        return mean

    @staticmethod
    def backward(ctx, dloss):
        (dl,) = ctx.saved_tensors
        return dl * dloss.to(dl.dtype), None, None, None


# ---------------------------------------------------------------- public API
def stem_native_ok(x, w) -> bool:
    return (x.dim() == 4 and tuple(x.shape[1:]) == (1, 28, 28) and x.dtype == torch.float32
            and w.dtype == torch.float32 and tuple(w.shape) == (6, 1, 5, 5) and not x.requires_grad)


def lenet_stem(x, w, b, slope=SLOPE):
    if use_native(x) and stem_native_ok(x, w):
        return _StemFn.apply(x.contiguous(), w.contiguous(), b.contiguous(), float(slope))
    return stem_reference(x, w, b, slope)


def leaky_pool(x, slope=SLOPE):
    if use_native(x) and x.dtype == torch.float32 and x.dim() == 4:
        return _LeakyPoolFn.apply(x.contiguous(), float(slope))
    return leaky_pool_reference(x, slope)


def softmax_nll(logits, target, mode="ce", label_smoothing=0.0):
    """Mean loss over rows; ``mode`` 'ce' (cross-entropy) or 'prob_nll' (reference: −mean p_y)."""
    if mode not in _MODES:
        raise ValueError(mode)
    if use_native(logits) and logits.dim() == 2 and logits.shape[1] <= 1024 and \
            logits.dtype in (torch.float32, torch.bfloat16):
        return _SoftmaxNLLFn.apply(logits.contiguous(), target.contiguous().long(), mode, float(label_smoothing))
    return softmax_nll_reference(logits, target, mode, label_smoothing)


def eval_metrics_(acc: torch.Tensor, logits: torch.Tensor, target: torch.Tensor, mode: str = "ce") -> None:
    """acc[0] += Σ loss, acc[1] += #correct (argmax), acc[2] += #rows — on device, no host sync."""
    with torch.no_grad():
        if use_native(logits) and logits.dim() == 2 and logits.shape[1] <= 1024 and \
                logits.dtype in (torch.float32, torch.bfloat16) and acc.dtype == torch.float64:
            native().softmax_nll_small(logits.contiguous(), target.contiguous().long(), _MODES[mode], 0.0,
                                       False, False, 1.0, acc)
            return
        lf = logits.float()
        if mode == "ce":
            l = F.cross_entropy(lf, target, reduction="sum")
        else:
            l = F.nll_loss(torch.softmax(lf, dim=-1), target, reduction="sum")
        acc[0] += l.double()
        acc[1] += (lf.argmax(dim=1) == target).sum().double()
        acc[2] += target.numel()
