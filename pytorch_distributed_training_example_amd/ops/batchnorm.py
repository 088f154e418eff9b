"""BatchNorm2d with fused ReLU and fused residual add, backed by NHWC bf16 HIP kernels.

``BatchNorm2d`` subclasses ``torch.nn.BatchNorm2d`` (same parameters, buffers and state_dict
keys, so torchvision-style ResNet checkpoints load unchanged) and adds
``forward(x, residual=None, relu=None)``:

    y = relu?( batchnorm(x) + residual? )

On a channels_last bf16 GPU tensor this is 3 kernels forward (reduce, finalize, apply) and 3
backward, instead of BN + add + ReLU as separate passes (csrc/kernels/batchnorm.hip). Other
inputs (CPU, fp32, NCHW) take the PyTorch reference path — identical math, used by the
CPU tests and as the numerics oracle.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn

from ..config import SW
from ._native import native, use_native


def bn_reference(x, residual, weight, bias, running_mean, running_var, training, momentum, eps, relu):
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    if relu:
        y = F.relu(y)
    return y


class ResidualGradLink:
    """Meeting point of the two branch gradients of one tensor (a ResNet block input feeds the
    main branch's conv1 and the shortcut): the first branch to finish backward deposits its
    gradient here and returns None to autograd; the second accumulates into it — conv1's
    data-gradient GEMM with beta = 1 — and returns the sum, so autograd never runs a separate
    add kernel (a full read-read-write pass per block). Identity blocks: the fused
    ``relu(bn3(x) + identity)`` backward deposits (it always runs first: the main branch is
    upstream of it); downsample blocks: the shortcut conv deposits (ops/conv.py linked_conv)."""

    __slots__ = ("grad", "lazy", "consumer_last")

    def __init__(self, lazy: bool = False, consumer_last: bool = False):
        self.grad = None
        # lazy: the depositing BatchNorm hands over (dy, relu mask) instead of writing dres = dy*mask;
        # the consumer (our 1x1 dgrad GEMM) applies the mask in its accumulate epilogue
        self.lazy = lazy
        # consumer_last: the accumulating conv's backward always runs after the depositor's (identity
        # blocks: bn3 is downstream of conv1). Finding the link empty then means the depositor took a
        # path that returned its gradient through autograd (e.g. a BatchNorm in eval mode): the consumer
        # must return its own dx instead of parking it for a partner that never comes.
        self.consumer_last = consumer_last

    def take(self):
        g, self.grad = self.grad, None
        return g


class GradStatsSource:
    """A BatchNorm output's link to the kernel that will produce its gradient: the consumer (our
    1x1-conv data-gradient GEMM, ops/conv.py) computes this BatchNorm's backward reduction —
    sum(dz), sum(dz * (x - mean)), dz = dy * ReLU mask — in its epilogue from the saved input /
    mask / mean held here, and deposits the per-tile partials together with the identity of the
    gradient tensor it wrote. The BatchNorm's backward uses them only if the dy it receives IS that
    tensor, unmodified (same storage, same version counter) — e.g. not when autograd summed
    another branch's gradient into it — and otherwise falls back to its own reduce pass.
    ``PDT_BN_BWD_STATS=0`` turns the hand-off off."""

    __slots__ = ("x", "mask", "mean", "out_version", "part", "grad_ptr", "grad_version", "masked", "sum_only",
                 "part_sum_only")

    def __init__(self):
        self.x = self.mask = self.mean = self.part = None
        self.out_version = self.grad_ptr = self.grad_version = None
        self.masked = False  # the depositing kernel stored the gradient already multiplied by the ReLU mask
        # sum_only (set by the BatchNorm's forward, PDT_BWD_ALG=2): the consumer computes sum(dz) only and never
        # reads x; the BatchNorm's backward completes sum(dz (x - mean)) through the ALG pass (part_sum_only)
        self.sum_only = self.part_sum_only = False

    def ready(self) -> bool:
        return self.x is not None and self.part is None

    def deposit(self, part: torch.Tensor, grad: torch.Tensor, masked: bool = False, sum_only: bool = False) -> None:
        """``masked``: ``grad`` was stored as dy * relu mask (our 1x1 GEMM's BSTATS epilogue does);
        ``sum_only``: ``part``'s centred sums are NOT valid (the producer did not read x)."""
        self.part, self.grad_ptr, self.grad_version = part, grad.data_ptr(), grad._version
        self.masked = bool(masked)
        self.part_sum_only = bool(sum_only)

    def bn_kwargs(self) -> dict:
        """conv1x1_gemm / gap_bwd keyword arguments of this BatchNorm's backward reduction."""
        if self.sum_only:
            return dict(bn_x=None, bn_mask=self.mask, bn_mean=self.mean, bn_sum_only=True)
        return dict(bn_x=self.x, bn_mask=self.mask, bn_mean=self.mean)

    def take(self, dy: torch.Tensor):
        part, self.part = self.part, None
        self.x = self.mask = self.mean = None  # the BatchNorm's backward is the last user
        if part is not None and dy.data_ptr() == self.grad_ptr and dy._version == self.grad_version:
            return part
        return None


def bwd_stats_enabled() -> bool:
    return SW.bn_bwd_stats


def grad_stats_source_of(x: torch.Tensor):
    """The ``GradStatsSource`` of a BatchNorm output ``x`` (unmodified since), else None."""
    g = getattr(x, "_pdt_gsrc", None)
    if g is not None and g.out_version == x._version and g.ready():
        return g
    return None


class MaskedGrad:
    """A ReLU'd residual gradient not yet materialised: ``dy * mask`` (mask = the BatchNorm's
    1-bit ReLU mask, bit j of byte k covers element 8k + j). ``masked``: dy already equals dy * mask (its
    producer stored it masked); ``s1``: sum(dy * mask) per channel (fp32) when the depositing BatchNorm's backward
    already has it (its bias gradient) — the downsample ALG backward (_alg_ds_prelude) takes both."""

    __slots__ = ("dy", "mask", "masked", "s1")

    def __init__(self, dy: torch.Tensor, mask: torch.Tensor, masked: bool = False, s1=None):
        self.dy, self.mask, self.masked, self.s1 = dy, mask, masked, s1

    def dense(self) -> torch.Tensor:
        bits = (self.mask.view(-1, 1) >> torch.arange(8, device=self.mask.device, dtype=torch.uint8)) & 1
        return self.dy * bits.view(self.dy.permute(0, 2, 3, 1).shape).permute(0, 3, 1, 2).to(self.dy.dtype)


class DeferredBNGrad:
    """The gradient at a BatchNorm's INPUT, not materialised: ``dx = A dy m + B (x - mean) + D`` per
    channel (``coef`` = [3, C] fp32 = A, B, D; ``m`` = the 1-bit ReLU mask, or none). Handed by the
    BatchNorm's backward to the conv that produced ``x`` through a ``BNGradLink``: that conv's fused
    backward (csrc/kernels/conv1x1_bwd_fused.hip) forms dx while loading it, so the BatchNorm's apply
    pass — a read of (dy, x, mask) and a write of dx, then two re-reads of dx — never runs."""

    __slots__ = ("dy", "x", "mask", "mean", "coef", "dy_masked", "wg", "virt")

    def __init__(self, dy, x, mask, mean, coef, dy_masked: bool = False, wg=None, virt=None):
        self.dy, self.x, self.mask, self.mean, self.coef = dy, x, mask, mean, coef
        self.virt = virt  # (conv input, weight) when x was never written (PDT_Z3_VIRTUAL, ops/conv.py)
        # dy_masked: dy already equals dy * m (no mask, or the producing kernel stored it masked): the ALG
        # backward (ops/conv.py _bwd_alg) then uses dy directly as the GEMM operand g
        self.dy_masked = dy_masked
        self.wg = wg  # the ALG weight-gradient pass, when the BatchNorm's backward already ran it

    def materialize(self) -> torch.Tensor:
        """dx as a tensor (fallback when the consumer cannot take the deferred form)."""
        sh = (1, -1, 1, 1) if self.x.dim() == 4 else (1, -1)
        g = self.dy.float()
        if self.mask is not None:
            g = g * MaskedGrad(torch.ones_like(self.dy), self.mask).dense().float()
        a, b, d = (c.view(sh) for c in self.coef)
        dx = a * g + b * (self.x.float() - self.mean.view(sh)) + d
        fmt = torch.channels_last if self.x.dim() == 4 else torch.contiguous_format
        return dx.to(self.x.dtype).contiguous(memory_format=fmt)


class BNGradLink:
    """One-way hand-off of a ``DeferredBNGrad`` from a BatchNorm's backward (which then returns None
    as its input gradient) to the backward of the conv that produced the BatchNorm's input (which
    runs next, with its output gradient None: ``set_materialize_grads(False)``)."""

    __slots__ = ("grad", "needs_masked", "alg_src")

    def __init__(self, needs_masked: bool = False):
        self.grad = None
        # needs_masked: the receiving conv takes the deferred form only with dy already masked (the ALG backward,
        # ops/conv.py _bwd_alg); otherwise the BatchNorm's backward runs its own apply and returns dx to autograd
        self.needs_masked = needs_masked
        self.alg_src = None  # (a, W): the receiving conv's input and weight (set by its forward)

    def take(self):
        g, self.grad = self.grad, None
        return g


class _BNTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, momentum, eps, relu, link=None,
                part=None, gsrc=None, glink=None, res_ab=None, defer=None, out_link=None, defer_relu=None,
                gemm=None, sub=None):
        C = native()
        ctx.defer_relu = defer_relu
        # x may be a statistics-only conv output (never written, PDT_Z3_VIRTUAL): only the APPLY GEMM path below and
        # the ALG backward may leave it unwritten; any other use recomputes it first (ops/conv.py materialize_virtual)
        virt = getattr(x, "_pdt_virtual", None)
        if virt is not None and not (defer_relu is None and defer is None and gemm is not None and part is not None
                                     and residual is not None and relu):
            from .conv import materialize_virtual
            materialize_virtual(x, virt)
            x._pdt_virtual = virt = None
        if defer_relu is not None:  # stats only; the consumer conv applies relu(a x + b) (DeferredReLUBN)
            if part is not None:
                _, _, mean, invstd, ab = C.bn_fwd_train_tiles(x, part, None, weight, bias, running_mean,
                                                              running_var, momentum, eps, False, apply=False)
            else:
                _, _, mean, invstd, ab = C.bn_fwd_train(x, None, weight, bias, running_mean, running_var,
                                                        momentum, eps, False, apply=False)
            M = x.numel() // x.shape[1]
            dmask = torch.empty(M * x.shape[1] // 8, dtype=torch.uint8, device=x.device)  # filled in backward
            defer_relu.extend([ab, dmask, mean])
            y, mask = x.view_as(x), None
        elif defer is not None:  # statistics only: the consumer applies y = a x + b itself (deferred apply)
            if part is not None:
                _, _, mean, invstd, ab = C.bn_fwd_train_tiles(x, part, None, weight, bias, running_mean,
                                                              running_var, momentum, eps, False, apply=False)
            else:
                _, _, mean, invstd, ab = C.bn_fwd_train(x, None, weight, bias, running_mean, running_var,
                                                        momentum, eps, False, apply=False)
            defer.append(ab)
            y, mask = x.view_as(x), None
        elif gemm is not None and part is not None and residual is not None and relu:
            # x came from our 1x1-conv GEMM (ops/conv.py GemmSource): the apply runs as that GEMM again with
            # the apply epilogue, reading the conv's input instead of x (conv1x1.hip APPLY)
            _, _, mean, invstd, ab = C.bn_fwd_train_tiles(x, part, None, weight, bias, running_mean, running_var,
                                                          momentum, eps, False, apply=False)
            a2, w2 = gemm.operands()
            y, mask = C.conv1x1_gemm_apply(a2, w2, residual, ab, res_ab, gemm.acoef)
        elif part is not None:  # statistics from the producing conv's epilogue: no reduce pass over x
            r = C.bn_fwd_train_tiles(x, part, residual, weight, bias, running_mean, running_var, momentum, eps, relu,
                                     res_ab=res_ab, sub=sub[0] if sub else 0) if sub else ()
            if len(r) == 5:  # + the stride-s subsample of y (the next stage's strided shortcut input)
                y, mask, mean, invstd, ys = r
                sub.append(ys)
            else:
                y, mask, mean, invstd = C.bn_fwd_train_tiles(x, part, residual, weight, bias, running_mean,
                                                             running_var, momentum, eps, relu, res_ab=res_ab)
        else:
            y, mask, mean, invstd = C.bn_fwd_train(x, residual, weight, bias, running_mean, running_var,
                                                   momentum, eps, relu, res_ab=res_ab)
        ctx.relu = relu
        if defer_relu is not None:
            ctx.dmask = defer_relu[1]  # NOT saved_tensors: the consumer's backward writes it (raw pointer)
        ctx.has_res = residual is not None
        ctx.has_weight = weight is not None
        ctx.link = link
        ctx.gsrc = gsrc
        # out_link: the conv that produced x takes this BatchNorm's input gradient in deferred form
        # (DeferredBNGrad) when the residual gradient needs no dense tensor either
        # — or, for a statistics-only shortcut BN whose gradient arrives through glink as (dy, mask)
        ctx.out_link = out_link if ((defer is None and (residual is None or (link is not None and link.lazy)))
                                    or (defer is not None and glink is not None)) else None
        # glink: this output's only consumer (a residual BatchNorm) may hand its gradient over as
        # (dy, ReLU mask) and give autograd None — backward then runs with dy = None
        ctx.glink = glink
        if glink is not None:
            ctx.set_materialize_grads(False)
        if gsrc is not None:  # what the consumer's dgrad GEMM needs for this BN's backward reduction
            gsrc.x, gsrc.mask, gsrc.mean = x, (mask if relu else None), mean
            # PDT_BWD_ALG=2: the consumer takes sum(dz) only; this backward completes the reduction (ALG prelude)
            gsrc.sum_only = bool(SW.bwd_alg >= 2 and ctx.out_link is not None and ctx.out_link.needs_masked
                                 and relu)
        if virt is not None and not (gsrc is not None and gsrc.sum_only):
            # the consumer's backward epilogue would read x for this BN's reduction: write it after all
            from .conv import materialize_virtual
            materialize_virtual(x, virt)
            x._pdt_virtual = virt = None
        ctx.virt = virt
        # backward needs the BN input and a 1-bit ReLU mask, never the output y
        ctx.save_for_backward(x, mask if (relu and defer_relu is None) else None, weight, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, mean, invstd = ctx.saved_tensors
        if ctx.defer_relu is not None:  # the mask was written by the consumer's backward
            mask = ctx.dmask
        tail = (None,) * 15
        need_w = ctx.has_weight and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        if dy is None:  # gradient handed over through glink as (dy, mask): a ReLU'd dy of the consumer
            g = ctx.glink.take() if ctx.glink is not None else None
            if g is None:
                return (None,) * 4 + tail
            if isinstance(g, MaskedGrad) and ctx.out_link is not None and ctx.out_link.needs_masked and not ctx.relu:
                # the shortcut conv runs the ALG backward: no reduce pass over (g, x), no apply (_alg_ds_prelude)
                r = _alg_ds_prelude(ctx, g, x, weight, mean, invstd, need_w)
                if r is not None:
                    coef, dg, db, wg = r
                    ctx.out_link.grad = DeferredBNGrad(g.dy, x, None, mean, coef, True, wg)
                    return (None, None, dg if need_w else None, db if need_w else None) + tail
            if isinstance(g, MaskedGrad) and ctx.out_link is not None:
                # coefficients only: the shortcut conv's fused backward forms dx on load (DeferredBNGrad)
                coef, dg, db = native().bn_bwd_coef(g.dy, x, None, g.mask, weight, mean, invstd, True, need_w)
                ctx.out_link.grad = DeferredBNGrad(g.dy, x, g.mask, mean, coef)
                return (None, None, dg if need_w else None, db if need_w else None) + tail
            if isinstance(g, MaskedGrad):
                dx, _, dg, db = native().bn_bwd_train(g.dy, x, g.mask, weight, mean, invstd, True, False, need_w)
            else:
                dx, _, dg, db = native().bn_bwd_train(g, x, None, weight, mean, invstd, False, False, need_w)
            return (dx, None, dg if need_w else None, db if need_w else None) + tail
        fmt = torch.channels_last if x.dim() == 4 else torch.contiguous_format
        dy = dy.contiguous(memory_format=fmt)
        # the reduction over (dy, x), if the kernel that wrote dy already took it (GradStatsSource)
        part = ctx.gsrc.take(dy) if ctx.gsrc is not None else None
        alg_wg = None
        if part is not None and ctx.gsrc.part_sum_only:
            # the producer summed dz only: complete sum(dz (x - mean)) from the ALG weight-gradient pass of the
            # conv that produced x (z = a W^T: sum_m dz (z - mean) = rowsum(P * W) - mean sum(dz), bn_alg.hip)
            alg_wg = _alg_prelude(ctx, dy, part)
            if alg_wg is None:
                part = None  # not completable: the finalize below reduces over (dy, x) itself

        def bwd(relu, has_res):
            if part is not None:
                return native().bn_bwd_train_tiles(dy, x, part, mask, weight, mean, invstd, relu, has_res, need_w)
            return native().bn_bwd_train(dy, x, mask, weight, mean, invstd, relu, has_res, need_w)

        dy_masked = not ctx.relu or (part is not None and ctx.gsrc.masked)
        defer_out = (ctx.out_link is not None and (not ctx.relu or mask is not None)
                     and (dy_masked or not ctx.out_link.needs_masked))
        if ctx.virt is not None and not (defer_out and part is not None):
            # every remaining path reads x (its reduce pass or apply): recompute the unwritten conv output
            from .conv import materialize_virtual
            materialize_virtual(x, ctx.virt)
            ctx.virt = None
        if defer_out:
            # coefficients only: the producing conv's fused backward forms dx = A dy m + B (x - mean) + D
            coef, dg, db = native().bn_bwd_coef(dy, x, part, mask if ctx.relu else None, weight, mean, invstd,
                                                ctx.relu, need_w)
            ctx.out_link.grad = DeferredBNGrad(dy, x, mask if ctx.relu else None, mean, coef, dy_masked, alg_wg,
                                               ctx.virt)
            if ctx.has_res:  # lazy link (checked in forward): the shortcut gets (dy, mask) as before
                # (+ sum(dy * mask) = this BN's bias gradient, for a downsample BN on the ALG backward)
                ctx.link.grad = MaskedGrad(dy, mask, dy_masked, db if (need_w and dy_masked) else None) \
                    if ctx.relu else dy
            return (None, None, dg if need_w else None, db if need_w else None) + tail
        if ctx.has_res and ctx.link is not None and ctx.link.lazy and ctx.relu:
            # the shortcut gradient dy*mask is never written: the consumer's GEMM masks dy itself
            dx, _, dg, db = bwd(True, False)
            ctx.link.grad = MaskedGrad(dy, mask)
            return (dx, None, dg if need_w else None, db if need_w else None) + tail
        dx, dres, dg, db = bwd(ctx.relu, ctx.has_res)
        if ctx.has_res and ctx.link is not None:
            ctx.link.grad = dres  # the main-branch consumer adds its gradient into this buffer
            dres = None
        return (dx, dres if ctx.has_res else None, dg if need_w else None, db if need_w else None) + tail


def _alg_prelude(ctx, dy, part):
    """The ALG weight-gradient pass [g | a | 1]^T a (ops/conv.py _bwd_alg) run from the BatchNorm's backward, and
    ``part``'s centred sums completed from it in place; returns that pass's fp32 output (handed to the conv's
    backward in the DeferredBNGrad), or None when it cannot run (no conv source, unmasked dy)."""
    link = ctx.out_link
    src = link.alg_src if link is not None else None
    if src is None or not ctx.gsrc.masked:
        return None
    a, w = src
    from .conv import _nhwc2d
    C4, CW = w.shape[0], w.shape[1]
    wg = native().conv1x1_wgrad_seg(_nhwc2d(a), _nhwc2d(dy), _nhwc2d(a))
    if wg is None:
        return None
    native().bn_alg_fix_s2(part, wg, w.reshape(C4, CW).contiguous())
    return wg


def _alg_ds_prelude(ctx, g, x, weight, mean, invstd, need_w):
    """A downsample block's shortcut BatchNorm backward for the ALG path of its conv (ops/conv.py _bwd_alg): the
    BN's output gradient g is bn3's (same block output, same ReLU mask), so sum(g) is bn3's bias gradient
    (``g.s1``), and sum(g (x - mean)) = rowsum(P * W) - mean sum(g) with P = g^T a from the ALG weight-gradient
    pass over the conv's input a. No pass over (g, x) and no apply: (coef, dgamma, dbeta, wg), or None when the
    path does not apply (g not stored masked, no sum, no conv source)."""
    link = ctx.out_link
    src = link.alg_src
    if src is None or not g.masked or g.s1 is None:
        return None
    a, w = src
    from .conv import _nhwc2d
    C4, CW = w.shape[0], w.shape[1]
    dy = g.dy.contiguous(memory_format=torch.channels_last)
    if dy.shape != x.shape:
        return None
    wg = native().conv1x1_wgrad_seg(_nhwc2d(a), _nhwc2d(dy), _nhwc2d(a))
    if wg is None:
        return None
    # one "tile": sum(g), then -mean sum(g) + rowsum(P * W)
    part = native().bn_alg_ds_part(g.s1.float().contiguous(), mean.contiguous(), wg, w.reshape(C4, CW).contiguous())
    coef, dg, db = native().bn_bwd_coef(dy, x, part, None, weight, mean, invstd, False, need_w)
    return coef, dg, db, wg


class _BNEvalFn(torch.autograd.Function):
    """Inference-statistics BatchNorm (+residual)(+ReLU): native forward; backward in PyTorch ops
    (not a hot path) including the affine gradients — a BN frozen in eval mode inside a training
    model (fine-tuning) still trains gamma / beta, as in torch."""

    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, eps, relu):
        y = native().bn_fwd_eval(x, residual, weight, bias, running_mean, running_var, eps, relu)
        ctx.relu, ctx.has_res, ctx.eps = relu, residual is not None, eps
        ctx.save_for_backward(x, y if relu else None, weight, running_mean, running_var)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, weight, rm, rv = ctx.saved_tensors
        dz = (dy * (y > 0) if ctx.relu else dy).float()
        shape = (1, -1, 1, 1) if dz.dim() == 4 else (1, -1)
        dims = (0, 2, 3) if dz.dim() == 4 else (0,)
        invstd = torch.rsqrt(rv.float() + ctx.eps)
        a = invstd * weight.float() if weight is not None else invstd
        dx = (dz * a.view(shape)).to(dy.dtype)
        dw = db = None
        if weight is not None and ctx.needs_input_grad[2]:
            dw = (dz * ((x.float() - rm.float().view(shape)) * invstd.view(shape))).sum(dims).to(weight.dtype)
        if ctx.needs_input_grad[3]:
            db = dz.sum(dims).to(weight.dtype if weight is not None else dz.dtype)
        return dx, (dz.to(dy.dtype) if ctx.has_res else None), dw, db, None, None, None, None


class _MaterializeFn(torch.autograd.Function):
    """y = a*t + b per channel, where ``t`` is a deferred BatchNorm's autograd output (its storage
    holds the BN INPUT): the gradient passes through UNCHANGED, because ``_BNTrainFn.backward``
    already applies the BN chain rule (gamma * invstd and the mean/var terms) to the gradient it
    receives as the gradient of its output."""

    @staticmethod
    def forward(ctx, t, ab):
        shape = (1, -1, 1, 1) if t.dim() == 4 else (1, -1)
        return (t.float() * ab[0].view(shape) + ab[1].view(shape)).to(t.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None


class DeferredBNOutput:
    """Internal handle for a BatchNorm output whose apply pass was deferred (statistics only; the
    value is ``a*raw + b`` per channel with ``ab`` = [2, C] fp32). It is NOT a tensor, so nothing
    can read it as the BN output by accident: the only consumer that takes it as-is is the native
    fused ``relu(bn3(x) + a*raw + b)`` apply (``batch_norm_act`` with it as ``residual``); every
    other use must call ``materialize()``. Only ``Bottleneck`` creates one, through
    ``BatchNorm2d._forward_stats_only`` (never through the public module call, so forward hooks
    on the BN always see a real output)."""

    __slots__ = ("raw", "ab")

    def __init__(self, raw: torch.Tensor, ab: torch.Tensor):
        self.raw, self.ab = raw, ab

    def materialize(self) -> torch.Tensor:
        return _MaterializeFn.apply(self.raw, self.ab)


class DeferredReLUBN:
    """Internal handle for ``relu(bn(x))`` whose apply was deferred INTO THE CONSUMER CONV (ResNet
    bottleneck bn2 -> conv3): statistics only in the forward; conv3's GEMM reads ``relu(a x + b)`` on
    load (conv1x1.hip ATR) and its fused backward recomputes that operand and WRITES this BatchNorm's
    ReLU bits into ``mask`` (conv1x1_bwd_fused.hip RECOMP), which the BatchNorm's backward then reads.
    ``raw`` is the BatchNorm's autograd output (its storage holds the BN INPUT x); ``ab`` = [2, C]
    fp32 (a, b); ``gsrc`` receives the BatchNorm's backward reduction from conv3's backward.
    Only ``Bottleneck`` creates one, and only together with conv3's fused backward (``bwd_link``)."""

    __slots__ = ("raw", "ab", "mask", "gsrc")

    def __init__(self, raw, ab, mask, gsrc):
        self.raw, self.ab, self.mask, self.gsrc = raw, ab, mask, gsrc

    def materialize_parts(self):
        """(relu(a x + b) as bf16, its ReLU bits) computed with PyTorch ops (fallback path)."""
        sh = (1, -1, 1, 1)
        t = self.raw.float() * self.ab[0].view(sh) + self.ab[1].view(sh)
        y = t.clamp_min(0).to(self.raw.dtype).contiguous(memory_format=torch.channels_last)
        pos = (t > 0).permute(0, 2, 3, 1).reshape(-1, 8).to(torch.int32)
        bits = (pos << torch.arange(8, device=pos.device, dtype=torch.int32)).sum(1).to(torch.uint8)
        return y, bits


def materialize(t):
    """The value of a possibly apply-deferred BatchNorm output (a tensor passes through)."""
    return t.materialize() if isinstance(t, DeferredBNOutput) else t


def batch_norm_act(x, residual, weight, bias, running_mean, running_var, training, momentum, eps, relu,
                   res_link: Optional[ResidualGradLink] = None, grad_link: Optional[ResidualGradLink] = None,
                   defer_apply: bool = False, out_link: Optional[BNGradLink] = None,
                   defer_relu_apply: bool = False, sub_stride: int = 0):
    """Functional fused BN(+add)(+ReLU). Native when x is a channels_last bf16 GPU tensor.
    ``res_link``: route the residual gradient through it instead of returning it (see
    ``ResidualGradLink``); only honoured on the native training path — callers check
    ``res_link.grad`` is set before relying on it. ``grad_link``: the output's gradient may arrive
    through this link instead of autograd (the output is the ``residual`` of a BatchNorm given
    the same link as ``res_link``: a ResNet downsample shortcut's BN). ``defer_apply`` (internal):
    compute the statistics only and return a ``DeferredBNOutput`` handle (when the native path
    applies; a plain tensor otherwise); the consumer BN (the handle as its ``residual``) adds
    a*x + b in its own apply pass, so this output is never written. ``sub_stride`` (internal, >= 2): the apply also
    writes the output's stride-s subsample, attached to the output as ``_pdt_sub`` for the next stage's strided
    1x1 shortcut (ops/conv.py ``subsample_of``), whose gather pass then never runs."""
    ab = None
    if isinstance(residual, DeferredBNOutput):
        residual, ab = residual.raw, residual.ab
    nhwc = x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) or \
        (x.dim() == 2 and x.is_contiguous())
    native_ok = (use_native(x) and x.dtype == torch.bfloat16 and nhwc and x.shape[1] % 64 == 0
                 and (residual is None or (residual.shape == x.shape and residual.dtype == x.dtype)))
    if ab is not None and not (native_ok and training and relu):
        # only the native relu+residual apply takes (a, b)
        residual, ab = DeferredBNOutput(residual, ab).materialize(), None
    if native_ok:
        if residual is not None:
            residual = residual.contiguous(memory_format=torch.channels_last if x.dim() == 4
                                           else torch.contiguous_format)
        if training:
            from .conv import bn_stats_of
            part = bn_stats_of(x) if x.dim() == 4 else None
            gsrc = (GradStatsSource() if x.dim() == 4 and torch.is_grad_enabled() and bwd_stats_enabled()
                    and (x.requires_grad or (weight is not None and weight.requires_grad)) else None)
            defer = [] if (defer_apply and residual is None and not relu and x.dim() == 4) else None
            if defer is not None:
                gsrc = None
            dre = [] if (defer_relu_apply and residual is None and relu and x.dim() == 4 and gsrc is not None) else None
            from .conv import gemm_source_of
            gemm = gemm_source_of(x) if (relu and residual is not None and part is not None) else None
            sub = [int(sub_stride)] if (sub_stride >= 2 and x.dim() == 4 and defer is None and dre is None
                                         and SW.subsample_native and SW.sub_out) else None
            y = _BNTrainFn.apply(x, residual, weight, bias, running_mean, running_var,
                                 float(momentum), float(eps), bool(relu), res_link, part, gsrc, grad_link, ab, defer,
                                 out_link, dre, gemm, sub)
            if sub is not None and len(sub) > 1:
                y._pdt_sub = (sub[0], sub[1], y._version)
            if defer:
                return DeferredBNOutput(y, defer[0])
            if dre:
                ab2, dmask, mean = dre
                gsrc.x, gsrc.mask, gsrc.mean = x, dmask, mean
                gsrc.out_version = y._version
                return DeferredReLUBN(y, ab2, dmask, gsrc)
            if gsrc is not None:  # a consumer conv may take this BN's backward reduction (ops/conv.py)
                gsrc.out_version = y._version
                y._pdt_gsrc = gsrc
            return y
        return _BNEvalFn.apply(x, residual, weight, bias, running_mean, running_var, float(eps), bool(relu))
    return bn_reference(x, residual, weight, bias, running_mean, running_var, training, momentum, eps, relu)


class _BNReluMaxPoolFn(torch.autograd.Function):
    """ResNet stem tail (train): BN → ReLU → MaxPool2d(3, 2, 1) with the BN output never stored."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps):
        y, code, mean, invstd = native().bn_relu_maxpool_fwd(x, weight, bias, running_mean, running_var,
                                                             momentum, eps)
        ctx.has_weight = weight is not None
        ctx.hw = (x.shape[2], x.shape[3])
        ctx.save_for_backward(x, code, weight, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, code, weight, mean, invstd = ctx.saved_tensors
        need_w = ctx.has_weight and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        dy = dy.contiguous(memory_format=torch.channels_last)
        if x.shape[1] == 64 and SW.stem_bwd_fused:
            # the pool gradient kernel also takes the BN's backward reduction: no pass over (dz, x)
            dx, dg, db = native().maxpool3s2_bwd_bn(dy, code, x, weight, mean, invstd, need_w)
            return dx, (dg if need_w else None), (db if need_w else None), None, None, None, None
        dz = native().maxpool3s2_bwd(dy, code, ctx.hw[0], ctx.hw[1])
        dx, _, dg, db = native().bn_bwd_train(dz, x, None, weight, mean, invstd, False, False, need_w)
        return dx, (dg if need_w else None), (db if need_w else None), None, None, None, None


def batch_norm_relu_maxpool(x, weight, bias, running_mean, running_var, training, momentum, eps):
    """relu(batchnorm(x)) followed by max_pool2d(kernel 3, stride 2, padding 1) — one fused
    apply+pool pass on the native path (training, channels_last bf16, C % 64 == 0)."""
    if (training and use_native(x) and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 64 == 0):
        return _BNReluMaxPoolFn.apply(x, weight, bias, running_mean, running_var, float(momentum), float(eps))
    y = batch_norm_act(x, None, weight, bias, running_mean, running_var, training, momentum, eps, True)
    return F.max_pool2d(y, 3, 2, 1)


class BatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` + fused ReLU / residual (state_dict-compatible)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True,
                 fused_relu: bool = False, device=None, dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, device, dtype)
        self.fused_relu = fused_relu
        self._nbt = 0  # host-side num_batches_tracked (synced into the buffer on save)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                relu: Optional[bool] = None, res_link: Optional[ResidualGradLink] = None,
                grad_link: Optional[ResidualGradLink] = None, out_link: Optional[BNGradLink] = None,
                sub_stride: int = 0) -> torch.Tensor:
        relu = self.fused_relu if relu is None else relu
        training = self.training or not self.track_running_stats
        momentum = self.momentum
        if self.training and self.track_running_stats:
            self._nbt += 1
            if momentum is None:  # cumulative moving average
                momentum = 1.0 / float(self._nbt + int(self.num_batches_tracked.item()))
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        w = self.weight if self.affine else None
        b = self.bias if self.affine else None
        return batch_norm_act(x, residual, w, b, rm, rv, training, momentum if momentum is not None else 0.0,
                              self.eps, relu, res_link, grad_link, out_link=out_link, sub_stride=sub_stride)

    def has_hooks(self) -> bool:
        """Forward (pre-)hooks registered on this module or globally: they must see real outputs."""
        from torch.nn.modules import module as _m
        return bool(self._forward_hooks or self._forward_pre_hooks or _m._global_forward_hooks
                    or _m._global_forward_pre_hooks)

    def _forward_stats_only(self, x: torch.Tensor, grad_link: Optional[ResidualGradLink] = None,
                            out_link: Optional[BNGradLink] = None):
        """Internal (``Bottleneck``'s shortcut BN): statistics + running-stat update only, returned
        as a ``DeferredBNOutput`` on the native training path (a normal output tensor otherwise).
        ``out_link``: the shortcut conv (``fused_bwd_ok``) takes this BN's input gradient in deferred
        form. Bypasses the module call, so callers use it only when ``has_hooks()`` is False."""
        training = self.training or not self.track_running_stats
        momentum = self.momentum
        if self.training and self.track_running_stats:
            self._nbt += 1
            if momentum is None:
                momentum = 1.0 / float(self._nbt + int(self.num_batches_tracked.item()))
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        w = self.weight if self.affine else None
        b = self.bias if self.affine else None
        return batch_norm_act(x, None, w, b, rm, rv, training, momentum if momentum is not None else 0.0,
                              self.eps, False, None, grad_link, defer_apply=True, out_link=out_link)

    def _forward_deferred_relu(self, x: torch.Tensor):
        """Internal (``Bottleneck``'s bn2 when conv3 runs the fused backward): ``relu(bn(x))`` as a
        ``DeferredReLUBN`` (statistics only; conv3 applies it on load) on the native training path, a
        normal output tensor otherwise. Bypasses the module call: callers check ``has_hooks()``."""
        training, w, b, rm, rv, momentum, eps = self._step_args()
        return batch_norm_act(x, None, w, b, rm, rv, training, momentum, eps, True, defer_relu_apply=True)

    def _step_args(self):
        """Per-call arguments of a training / eval forward (counts the batch, as ``forward`` does):
        (training, weight, bias, running_mean, running_var, momentum, eps)."""
        training = self.training or not self.track_running_stats
        momentum = self.momentum
        if self.training and self.track_running_stats:
            self._nbt += 1
            if momentum is None:
                momentum = 1.0 / float(self._nbt + int(self.num_batches_tracked.item()))
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        w = self.weight if self.affine else None
        b = self.bias if self.affine else None
        return training, w, b, rm, rv, float(momentum if momentum is not None else 0.0), float(self.eps)

    def forward_relu_maxpool(self, x: torch.Tensor) -> torch.Tensor:
        """``max_pool2d(relu(bn(x)), 3, 2, 1)`` (ResNet stem) with the pool fused into the BN apply."""
        training, w, b, rm, rv, momentum, eps = self._step_args()
        return batch_norm_relu_maxpool(x, w, b, rm, rv, training, momentum, eps)

    def stem_params(self):
        """(weight, bias, running_mean, running_var, momentum, eps) of one training forward of the
        stem's fused conv + BN + ReLU + pool node (``ops.conv.stem_block``); counts the batch."""
        _, w, b, rm, rv, momentum, eps = self._step_args()
        return w, b, rm, rv, momentum, eps

    def sync_num_batches_tracked(self) -> None:
        if self.track_running_stats and self._nbt:
            self.num_batches_tracked.add_(self._nbt)
            self._nbt = 0

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        self.sync_num_batches_tracked()
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def _load_from_state_dict(self, *args, **kwargs):
        self._nbt = 0
        super()._load_from_state_dict(*args, **kwargs)
