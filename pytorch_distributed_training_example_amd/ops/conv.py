"""1x1 convolutions as GEMMs, with per-shape algorithm selection (MIOpen vs hipBLASLt).

Not in the reference (LeNet's convs are 5x5, /root/reference/cnn.py:10-16); this serves the
ResNet-50 north-star config, where 36 of 53 convolutions are 1x1. In channels_last (NHWC) a
stride-1 1x1 convolution IS a GEMM on views, no copies:

    X [N,H,W,Ci] -> [M, Ci],  W [Co,Ci,1,1] -> [Co, Ci],  Y = X W^T -> [M, Co] = [N,H,W,Co]
    dX = dY W,  dW = dY^T X

These shapes are HBM-bound (K = Ci is 64..2048 while M = N*H*W is 12K..800K), and which
library streams them best depends on the shape: MIOpen's implicit-GEMM kernels win for narrow
K/N (and need a zero-fill + fp32->bf16 cast pass for their atomic split-K outputs), hipBLASLt
wins for wide ones (tools/conv_bench.py: 1.2 ms/step of ResNet-50 difference). So each
direction (forward, data-grad, weight-grad) of each shape is timed once with both back ends on
its first eager call — like ``cudnn.benchmark`` — and the faster one is used from then on
(``PDT_CONV1X1=miopen|gemm|auto``). Never timed under hipGraph capture (capture falls back to
MIOpen for an unseen shape), so the warm-up steps before ``StaticStep.capture`` settle it.

Decisions measured on an MI355X are committed in ``tuning/conv1x1_gfx950.json`` (keyed by direction,
dtype and GEMM shape; loaded only on a gfx950 device, measured for bf16) and used without
timing: a shape decided for GEMM then never calls MIOpen at all, which matters on a fresh box,
where timing the MIOpen candidate costs its full algorithm search (ResNet-50 at 1024/GPU: most
of a 237 s first step). ``PDT_CONV1X1_TABLE=0`` ignores the table; ``PDT_CONV1X1_DUMP=<path>``
writes table + new decisions at exit (to extend the table).
"""
from __future__ import annotations

import atexit
import json
import os
from typing import Dict, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from ..config import SW
from ._native import disabled

_CHOICE: Dict[Tuple, str] = {}
_TABLE_LOADED = [False]
TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                     "tuning", "conv1x1_gfx950.json")


def _key_str(key: Tuple) -> str:
    return ",".join(str(k) for k in key)


def load_table(path: str | None = None) -> int:
    """Seed the decisions from a measured table; returns the number of entries loaded."""
    path = path or TABLE
    if not os.path.exists(path):
        return 0
    with open(path) as f:
        tab = json.load(f)
    for k, v in tab.items():
        d, dt, *dims = k.split(",")
        if (v in ("miopen", "gemm", "ours") or v.startswith("splitk")) and len(dims) == 3:
            _CHOICE.setdefault((d, dt, *map(int, dims)), v)
    return len(tab)


def _dtype_name(t: torch.Tensor) -> str:
    return {torch.bfloat16: "bf16", torch.float16: "fp16", torch.float32: "fp32"}.get(t.dtype, str(t.dtype))


def _table_arch_ok() -> bool:
    """The committed decisions were measured on gfx950: any other device times its own."""
    if not torch.cuda.is_available():
        return False
    return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.startswith("gfx950")


def dump_table(path: str) -> None:
    """Write every decision (table + measured this run) as a table file."""
    with open(path, "w") as f:
        json.dump({_key_str(k): v for k, v in sorted(_CHOICE.items())}, f, indent=0, sort_keys=True)


def _ensure_table() -> None:
    if _TABLE_LOADED[0]:
        return
    _TABLE_LOADED[0] = True
    if SW.conv1x1_table and _table_arch_ok():
        load_table()
    if SW.conv1x1_dump:
        atexit.register(dump_table, SW.conv1x1_dump)

# Weight gradients run in-stream by default: a side stream for them measured 4 % SLOWER on ResNet-50 at
# 1024 images (10,212 vs 10,617 img/s, round 2) — both streams' kernels already fill the chip. At small
# per-GPU batches (128 / rank: layer 3-4 grids of 200-400 workgroups on 256 CUs) the data and weight
# gradient of one conv can share the chip: PDT_WGRAD_STREAM_M (SW.wgrad_stream_m) sends the weight
# gradients of convs with at most that many output pixels to a side stream.
_SIDE = {}


class _WgradFork:
    """Fork point of one conv backward: created BEFORE the data gradient is queued (an event on the current
    stream), ``run(fn)`` launches the weight gradient on the side stream after that event — so it overlaps
    the data gradient — and joins the current stream to it before returning (the gradient is consumed on
    the current stream right after the backward returns). Inside hipGraph capture the event fork / join
    become graph edges. Off (plain call) unless SW.wgrad_stream_m >= M."""

    __slots__ = ("cur", "ev")

    def __init__(self, t: torch.Tensor, M: int):
        self.cur = self.ev = None
        if SW.wgrad_stream_m and M <= SW.wgrad_stream_m and t.is_cuda:
            self.cur = torch.cuda.current_stream(t.device)
            self.ev = torch.cuda.Event()
            self.ev.record(self.cur)

    def run(self, fn):
        # Allocator safety of the operands fn reads on the side stream (gy, x and their 2-D views, allocated on the
        # current stream, NOT record_stream'ed): the join below (current stream waits for the side stream) is
        # enqueued before this returns, and the caller holds the operands until after — so any free of them, and
        # any reuse of that memory by a later kernel on the current stream, is stream-ordered after fn's kernels.
        if self.cur is None:
            return fn()
        dev = self.cur.device
        s = _SIDE.get(dev)
        if s is None:
            s = _SIDE[dev] = torch.cuda.Stream(device=dev)
        s.wait_event(self.ev)
        with torch.cuda.stream(s):
            dw = fn()
        if dw is not None:
            dw.record_stream(self.cur)  # allocated on the side stream, read on the current one
        self.cur.wait_stream(s)
        return dw


def _ours_ok(direction: str, M: int, K: int, N: int) -> bool:
    """Stride-1 1x1 conv direction on our MFMA kernels: ``fwd`` (csrc/kernels/conv1x1.hip, with the
    consuming BatchNorm's statistics in the epilogue), ``dgrad`` (same GEMM, shortcut gradient
    accumulated in place) or ``wgrad`` (conv1x1_wgrad.hip; K = Ci, N = Co), if listed in
    ``PDT_CONV1X1_OURS`` (config.SW)."""
    return (direction in SW.conv1x1_ours and K % 32 == 0 and N % 64 == 0
            and M * max(K, N) < 2 ** 31 and SW.conv1x1 in ("auto", "ours"))


# ---- per-step weight transforms (csrc/kernels/weight_prep.hip): the data gradients of our 1x1 GEMM and 3x3
# kernels read W^T [Ci, Co] / the flipped transposed 3x3 weights. ``prepare_weights`` (called by the model at
# the start of a training forward) makes all of them in ONE launch; a backward takes its conv's copy only
# if it was made by the latest prepare call (``prepared``), else transforms on its own as before.
_PREP = {"stamp": 0, "map": {}}


def prepare_weights(convs) -> None:
    """W^T of every 1x1 and the flipped weights of every 3x3 conv in ``convs``, one kernel launch. The copies
    are keyed by the weight OBJECT (a weakref, checked with ``is``) and its storage pointer, so a freed weight
    whose address is reused by another never matches."""
    import weakref
    _PREP["stamp"] += 1
    stamp = _PREP["stamp"]
    mp = {}
    srcs, dsts = [], []
    for m in convs:
        w = m.weight
        k = w.shape[-1]
        if not (w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 4 and k in (1, 3) and w.shape[-2] == k):
            continue
        if k == 3 and not w.is_contiguous(memory_format=torch.channels_last):
            continue
        Co, Ci = w.shape[:2]
        # the copy is OWNED by the weight (attribute), not by this module-global map: a captured hipGraph
        # holds its address, and another model's training forward replaces the map — the buffer must
        # live as long as the weight, not until the next prepare call of any model
        dst = getattr(w, "_pdt_wprep", None)
        want = (Ci, Co) if k == 1 else (Ci, Co, 3, 3)
        if dst is None or tuple(dst.shape) != want or dst.device != w.device:
            dst = (torch.empty(want, dtype=w.dtype, device=w.device) if k == 1 else
                   torch.empty(want, dtype=w.dtype, device=w.device).contiguous(memory_format=torch.channels_last))
            w._pdt_wprep = dst
        mp[id(w)] = (stamp, weakref.ref(w), w.data_ptr(), dst)
        srcs.append(w.detach())
        dsts.append(dst)
    _PREP["map"] = mp
    if srcs:
        from ._native import native
        native().weight_prep(srcs, dsts)


def prepared(weight: torch.Tensor):
    """This step's transformed copy of ``weight`` (see prepare_weights), or None."""
    e = _PREP["map"].get(id(weight))
    if e is None or e[0] != _PREP["stamp"] or e[1]() is not weight or e[2] != weight.data_ptr():
        return None
    return e[3]


def _wt_of(weight: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """W^T [Ci, Co] of a 1x1 conv weight (w2 = its [Co, Ci] view)."""
    wt = prepared(weight)
    return wt if wt is not None else w2.t().contiguous()


def _flip_of(weight: torch.Tensor) -> torch.Tensor:
    from ._native import native
    wf = prepared(weight)
    return wf if wf is not None else native().conv3x3_flip(weight)


class GemmSource:
    """How a 1x1 conv output z was computed by our GEMM (input, weight, ATR coefficients): the consuming
    BatchNorm's apply can run as that GEMM again with the apply epilogue (conv1x1.hip APPLY), reading the
    conv input instead of z. Valid while z is unmodified (``version``)."""

    __slots__ = ("x", "weight", "acoef", "version")

    def __init__(self, x, weight, acoef, version):
        self.x, self.weight, self.acoef, self.version = x, weight, acoef, version

    def operands(self):
        Co, Ci = self.weight.shape[:2]
        return _nhwc2d(self.x), self.weight.reshape(Co, Ci).contiguous()


def gemm_source_of(z: torch.Tensor):
    g = getattr(z, "_pdt_gemm_src", None)
    return g if (g is not None and g.version == z._version) else None


def materialize_virtual(z: torch.Tensor, src) -> torch.Tensor:
    """Write a statistics-only conv output z (PDT_Z3_VIRTUAL: never stored) by running its GEMM; ``src`` =
    (input, weight). Every consumer that reads z's values outside the APPLY GEMM calls this first."""
    from ._native import native
    a, w = src
    Co, Ci = w.shape[:2]
    native().conv1x1_gemm(_nhwc2d(a), w.reshape(Co, Ci).contiguous(), _nhwc2d(z), False, False)
    return z


def _attach_gemm_source(y, x, weight, acoef):
    if 0 < weight.shape[1] <= SW.bn_apply_gemm_k:
        y._pdt_gemm_src = GemmSource(x, weight, acoef, y._version)


class BNStats:
    """Per-tile BatchNorm statistics of a conv output, computed in the conv's epilogue
    (conv1x1_gemm ``stats``), attached to the output tensor as ``_pdt_bn_stats``; the BatchNorm
    that consumes the tensor uses them instead of a reduce pass if the tensor is unmodified
    (same version counter)."""

    __slots__ = ("part", "version")

    def __init__(self, part: torch.Tensor, version: int):
        self.part, self.version = part, version


def bn_stats_of(x: torch.Tensor):
    st = getattr(x, "_pdt_bn_stats", None)
    if st is not None and st.version == x._version:
        return st.part
    return None


def _time(fn, reps: int = 3) -> float:
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1)


def _pick(key: Tuple, cands: Dict[str, callable], fused: bool = False) -> str:
    """Backend for one (direction, dtype, M, Ci, Co): forced mode > per-shape override >
    ``PDT_CONV1X1_PREFER`` > measured table > ``fused`` (our GEMM would also take the consuming
    BatchNorm's statistics / backward reduction in its epilogue, removing a whole reduce pass that
    a conv-only timing cannot see: take it untimed) > time the candidates once."""
    mode = SW.conv1x1
    if mode in cands:
        return mode
    o = SW.conv1x1_override.get(_key_str(key)) if SW.conv1x1_override else None
    if o is not None and o in cands:
        return o
    if "ours" in cands and key[0] in SW.conv1x1_prefer:
        return "ours"
    _ensure_table()
    c = _CHOICE.get(key)
    if c is not None:  # a decided back end that is switched off here: the GEMM library, untimed
        return c if c in cands else "gemm"
    if fused and "ours" in cands:
        _CHOICE[key] = "ours"
        return "ours"
    if torch.cuda.is_current_stream_capturing():
        return "miopen"
    times = {name: _time(fn) for name, fn in cands.items()}
    c = min(times, key=times.get)
    _CHOICE[key] = c
    return c


def choices() -> Dict[Tuple, str]:
    """Decisions taken so far: {(direction, dtype, M, Ci, Co): 'miopen' | 'gemm'}."""
    return dict(_CHOICE)


_SPLITK = (8, 16, 32, 64)


def _wgrad_splitk(g2: torch.Tensor, x2: torch.Tensor, sk: int) -> torch.Tensor:
    """1x1-conv weight gradient dW[Co, Ci] = dY^T X over K = M pixels as ``sk`` batched GEMMs of
    M/sk pixels each (hipBLASLt) summed in fp32: with K ~1e5 and both operands pixel-major, one
    GEMM (or MIOpen's kernel) keeps too few tiles busy — ResNet-50 layer2-4 shapes measured
    0.5-0.75x of MIOpen's time (tools/wgrad_split_bench.py)."""
    M, Co = g2.shape
    Ci = x2.shape[1]
    part = torch.bmm(g2.view(sk, M // sk, Co).transpose(1, 2), x2.view(sk, M // sk, Ci))
    if part.is_cuda and part.dtype == torch.bfloat16 and (Co * Ci) % 8 == 0 and SW.slice_sum:
        from ._native import native
        return native().slice_sum(part)  # csrc/kernels/slice_sum.hip: bf16 out, fp32 accumulation
    return part.sum(0)


def _nhwc2d(t: torch.Tensor) -> torch.Tensor:
    """[N,C,H,W] channels_last -> [N*H*W, C] view."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, link=None, stats_out=None, gsrc=None, bwd_link=None, dre=None, nostore=False):
        """``dre``: x is the INPUT of a BatchNorm + ReLU whose apply is deferred to here
        (ops/batchnorm.py DeferredReLUBN): the GEMM reads relu(a x + b) (our kernel, ATR). ``nostore``: with
        ``stats_out``, our GEMM takes the statistics only and y stays unwritten ("virtual": ``stats_out``
        then gets a second entry, True)."""
        N, Ci, H, W = x.shape
        Co = weight.shape[0]
        x2 = _nhwc2d(x)
        w2 = weight.reshape(Co, Ci)
        M = x2.shape[0]
        ctx.link = link
        ctx.gsrc = gsrc  # x is a BatchNorm output: our dgrad GEMM can take that BN's backward reduction
        # bwd_link: the BatchNorm consuming y may hand its input gradient over in deferred form
        # (ops/batchnorm.py DeferredBNGrad) and give autograd None: backward then runs with gy = None
        ctx.bwd_link = bwd_link
        if bwd_link is not None:
            ctx.set_materialize_grads(False)
            if bwd_link.needs_masked:  # the consuming BatchNorm's backward may run the ALG pass (batchnorm.py)
                bwd_link.alg_src = (x, weight)
        ctx.save_for_backward(x, weight)
        ctx.dre = dre
        if dre is not None:  # always our GEMM: no library takes the deferred operand
            from ._native import native
            y = torch.empty((N, Co, H, W), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
            part = native().conv1x1_gemm(x2, w2.contiguous(), _nhwc2d(y), False, stats_out is not None,
                                         a_coef=dre.ab)
            if stats_out is not None:
                stats_out.append(part)
            return y
        cands = {"miopen": lambda: F.conv2d(x, weight), "gemm": lambda: torch.mm(x2, w2.t())}
        if x.dtype == torch.bfloat16 and _ours_ok("fwd", M, Ci, Co):
            from ._native import native

            def ours(stats=False, no_store=False):
                y = torch.empty((N, Co, H, W), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
                return y, native().conv1x1_gemm(x2, w2.contiguous(), _nhwc2d(y), False, stats, no_store=no_store)
            cands["ours"] = ours
        algo = _pick(("fwd", _dtype_name(x), M, Ci, Co), cands, fused=stats_out is not None)
        if algo == "ours":  # with the consuming BatchNorm's statistics in the epilogue
            nostore = bool(nostore and stats_out is not None)
            y, part = cands["ours"](stats_out is not None, nostore)
            if stats_out is not None:
                stats_out.append(part)
                if nostore:
                    stats_out.append(True)
            return y
        if algo == "gemm":
            y = torch.mm(x2, w2.t()).view(N, H, W, Co).permute(0, 3, 1, 2)
        else:
            y = F.conv2d(x, weight)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        N, Ci, H, W = x.shape
        Co = weight.shape[0]
        none7 = (None,) * 6
        if gy is None:  # the consuming BatchNorm handed its input gradient over (or there is none)
            d = ctx.bwd_link.take() if ctx.bwd_link is not None else None
            if d is None and ctx.link is not None:  # the partner branch still expects this one's gradient
                gy = torch.zeros((N, Co, H, W), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
                return _Conv1x1Fn._backward_dense(ctx, gy, x, weight) + (None,) * 6
            if d is None:
                return (None, None) + none7
            r = _bwd_fused(ctx, d, x, weight)
            if r is None:
                r = _bwd_alg(ctx, d, x, weight)
                if r is not None and ctx.link is not None:  # first of the two branches: conv1's GEMM adds to it
                    ctx.link.grad, r = r[0], (None, r[1])
            if r is not None:
                return (r[0], r[1]) + none7
            if d.virt is not None:  # the BatchNorm input was never written (PDT_Z3_VIRTUAL): recompute it
                materialize_virtual(d.x, d.virt)
            gy = d.materialize()
        if ctx.dre is not None:  # fallback: materialise the deferred operand and its ReLU bits
            xa, bits = ctx.dre.materialize_parts()
            ctx.dre.mask.copy_(bits)
            r = _Conv1x1Fn._backward_dense(ctx, gy, xa, weight)
            return r + (None,) * 6
        return _Conv1x1Fn._backward_dense(ctx, gy, x, weight) + (None,) * 6

    @staticmethod
    def _backward_dense(ctx, gy, x, weight):
        """(dx, dw) from a dense output gradient (the library / our GEMM paths)."""
        N, Ci, H, W = x.shape
        Co = weight.shape[0]
        gy = gy.contiguous(memory_format=torch.channels_last)
        x2, g2, w2 = _nhwc2d(x), _nhwc2d(gy), weight.reshape(Co, Ci)
        M = x2.shape[0]
        fork = _WgradFork(gy, M)
        dx = None

        def conv_bwd(mask):
            return torch.ops.aten.convolution_backward(gy, x, weight, None, [1, 1], [0, 0], [1, 1], False, [0, 0],
                                                       1, mask)

        # the other branch's gradient of x, if it already arrived (ResidualGradLink)
        acc = ctx.link.take() if ctx.link is not None else None
        first = ctx.link is not None and acc is None and not ctx.link.consumer_last
        strided = None
        if isinstance(acc, StridedGrad):  # a stride-2 shortcut's compact gradient: added below
            strided, acc = acc, None
        from .batchnorm import MaskedGrad
        # (the stride-2 shortcut's compact gradient added in our GEMM's epilogue instead of the
        # strided add pass below measured 0.4 % slower on ResNet-50 — hipBLASLt dgrad + add wins on
        # those three shapes — so it is taken only where the same epilogue also takes the producing
        # BatchNorm's backward reduction, which saves that BatchNorm a reduce pass: PDT_STRIDED_BSTATS)
        if (strided is not None and SW.strided_bstats and not first and acc is None and ctx.needs_input_grad[0]
                and ctx.gsrc is not None and ctx.gsrc.ready() and gy.dtype == torch.bfloat16
                and _subsample_native(strided.t) and _ours_ok("dgrad", M, Co, Ci)):
            from ._native import native
            gs = ctx.gsrc
            dx = torch.empty_like(x)
            gpart = native().conv1x1_gemm(g2, _wt_of(weight, w2), _nhwc2d(dx), True, False, strided.t,
                                          c_stride=strided.s, c_H=H, c_W=W, **gs.bn_kwargs())
            gs.deposit(gpart, dx, masked=gs.mask is not None, sum_only=gs.sum_only)
            strided = None
            return dx, _Conv1x1Fn._wgrad(ctx, g2, x2, x, gy, weight, M, Ci, Co, fork)
        # dx is final (nothing is added to it after the GEMM) unless this is the first of two linked
        # branches or a strided shortcut's gradient is added below: only then can the GEMM's epilogue
        # take the producing BatchNorm's backward reduction (GradStatsSource)
        gs = ctx.gsrc if (ctx.gsrc is not None and ctx.gsrc.ready() and not first and strided is None) else None
        bn_kw = gs.bn_kwargs() if gs is not None else {}
        gpart = None
        if isinstance(acc, MaskedGrad) and ctx.needs_input_grad[0] and _ours_ok("dgrad", M, Co, Ci):
            # dx = dy*mask + dY W: the shortcut's ReLU-masked gradient applied in the GEMM epilogue
            from ._native import native
            dx = torch.empty_like(x)
            gpart = native().conv1x1_gemm(g2, _wt_of(weight, w2), _nhwc2d(dx), True, False, acc.dy, acc.mask,
                                          **bn_kw)
            acc = None
        elif isinstance(acc, MaskedGrad):
            acc = acc.dense()
        if dx is not None:
            pass
        elif ctx.needs_input_grad[0]:
            cands = {"miopen": lambda: conv_bwd([True, False, False]), "gemm": lambda: torch.mm(g2, w2)}
            if gy.dtype == torch.bfloat16 and _ours_ok("dgrad", M, Co, Ci):
                from ._native import native
                wt = _wt_of(weight, w2)  # [Ci, Co]: the B operand rows of dX = dY W

                def ours_d():
                    d = torch.empty_like(x)
                    native().conv1x1_gemm(g2, wt, _nhwc2d(d), False, False)
                    return d
                cands["ours"] = ours_d
            algo = _pick(("bwd_data", _dtype_name(x), M, Ci, Co), cands, fused=gs is not None)
            if algo == "ours" and acc is not None and acc.is_contiguous(memory_format=torch.channels_last):
                # dx = dres + dY W, in place
                gpart = native().conv1x1_gemm(g2, wt, _nhwc2d(acc), True, False, **bn_kw)
                dx, acc = acc, None
            elif algo == "ours" and acc is None:
                dx = torch.empty_like(x)
                gpart = native().conv1x1_gemm(g2, wt, _nhwc2d(dx), False, False, **bn_kw)
            elif algo == "ours":
                dx = ours_d()
            elif algo == "gemm" and acc is not None and acc.is_contiguous(memory_format=torch.channels_last):
                _nhwc2d(acc).addmm_(g2, w2)  # dx = dres + dY W in one GEMM (beta = 1)
                dx, acc = acc, None
            elif algo == "gemm":
                dx = torch.mm(g2, w2).view(N, H, W, Ci).permute(0, 3, 1, 2)
            else:
                dx = conv_bwd([True, False, False])[0]
            if acc is not None:
                dx = dx.add_(acc)
        elif acc is not None:
            dx = acc
        if strided is not None and dx is not None:
            strided.add_into(dx)
        if gpart is not None and dx is not None:
            gs.deposit(gpart, dx, masked=gs.mask is not None, sum_only=gs.sum_only)  # stored masked (conv1x1.hip)
        if first and dx is not None:  # first of the two branches: leave dx for the partner to add to
            ctx.link.grad, dx = dx, None
        return dx, _Conv1x1Fn._wgrad(ctx, g2, x2, x, gy, weight, M, Ci, Co, fork)

    @staticmethod
    def _wgrad(ctx, g2, x2, x, gy, weight, M, Ci, Co, fork=None):
        """dW of a 1x1 conv (None when not needed): the fastest of MIOpen / one GEMM / split-K GEMMs /
        our one-pass kernel for the shape (on the side stream when ``fork`` is active, see _WgradFork)."""
        dw = None

        def conv_bwd(mask):
            return torch.ops.aten.convolution_backward(gy, x, weight, None, [1, 1], [0, 0], [1, 1], False, [0, 0],
                                                       1, mask)
        if ctx.needs_input_grad[1]:
            cands = {"miopen": lambda: conv_bwd([False, True, False]), "gemm": lambda: torch.mm(g2.t(), x2)}
            splitk_on = SW.wgrad_splitk
            for sk in _SPLITK if splitk_on else ():
                if M % sk == 0 and M // sk >= 256:
                    cands[f"splitk{sk}"] = (lambda sk=sk: _wgrad_splitk(g2, x2, sk))
            if x.dtype == torch.bfloat16 and _ours_ok("wgrad", M, Ci, Co) and Ci % 64 == 0:
                from ._native import native
                # csrc/kernels/conv1x1_wgrad.hip: one HBM pass over dY and X (split-K over pixels)
                cands["ours"] = lambda: native().conv1x1_wgrad(x2, g2)
            key = ("bwd_weight", _dtype_name(x), M, Ci, Co)
            algo = "miopen" if not splitk_on and str(_CHOICE.get(key, "")).startswith("splitk") else _pick(key, cands)
            # a 1x1 kernel has the same element order in NCHW and NHWC: keep weight's strides
            if algo == "gemm":
                wfn = lambda: torch.mm(g2.t(), x2).as_strided(weight.shape, weight.stride())  # noqa: E731
            elif algo == "ours":
                wfn = lambda: cands["ours"]().as_strided(weight.shape, weight.stride())  # noqa: E731
            elif algo.startswith("splitk"):
                sk = int(algo[6:])
                wfn = lambda: _wgrad_splitk(g2, x2, sk).as_strided(weight.shape, weight.stride())  # noqa: E731
            else:
                wfn = lambda: conv_bwd([False, True, False])[1]  # noqa: E731
            dw = fork.run(wfn) if fork is not None else wfn()
        return dw


def _bwd_fused(ctx, d, x, weight):
    """conv3 + bn3 backward of a bottleneck as ONE kernel (csrc/kernels/conv1x1_bwd_fused.hip): from the
    BatchNorm's deferred input gradient ``d`` (DeferredBNGrad) -> (dx, dw), with the producing BatchNorm's
    backward reduction deposited in its GradStatsSource. None when the kernel does not take the shape
    (the caller materialises d and runs the unfused path)."""
    # linked (a downsample shortcut conv): only as the FIRST of the two branches — dx is deposited for
    # conv1's dgrad GEMM to accumulate into, so it is not final and takes no BatchNorm reduction
    linked = ctx.link is not None
    if ctx.bwd_link is not None and ctx.bwd_link.needs_masked:
        return None  # planned for the ALG backward (models/resnet.py)
    if not (SW.bwd_fused and (not linked or ctx.link.grad is None) and ctx.needs_input_grad[0]
            and ctx.needs_input_grad[1] and d.mask is not None and fused_bwd_shape_ok(weight)):
        return None
    from ._native import native
    gs = ctx.gsrc if (ctx.gsrc is not None and ctx.gsrc.ready() and not linked) else None
    dre = ctx.dre
    if dre is not None and gs is None:
        return None  # the recompute mode needs bn2's input / mean (its GradStatsSource)
    r = native().conv1x1_bwd_fused(d.dy.contiguous(memory_format=torch.channels_last), d.x, d.mask, d.mean, d.coef,
                                   weight, x, gs.x if gs else None, gs.mask if gs else None, gs.mean if gs else None,
                                   dre.ab if dre is not None else None, prepared(weight))
    if not r:
        return None
    dx, dw, part = r
    if gs is not None and part is not None:
        gs.deposit(part, dx)
    if linked:
        ctx.link.grad, dx = dx, None
    return dx, dw


def alg_bwd_shape_ok(weight: torch.Tensor) -> bool:
    """(Co, Ci) of a bottleneck conv3 whose backward ``_bwd_alg`` takes: Co (bn3's channels) a multiple of 128, Ci 64
    or a multiple of 128 (the segment blocks of conv1x1_wgrad.hip / the GEMM tiles), bf16 1x1 weights. (Layer 1's
    256x64 conv3 takes the fused kernel first where PDT_BWD_FUSED_SHAPES lists it.)"""
    return (weight.dim() == 4 and tuple(weight.shape[2:]) == (1, 1) and weight.dtype == torch.bfloat16
            and weight.shape[0] % 128 == 0 and (weight.shape[1] == 64 or weight.shape[1] % 128 == 0)
            and weight.shape[0] > weight.shape[1])


def _bwd_alg(ctx, d, x, weight):
    """conv3 + bn3 backward of a bottleneck WITHOUT bn3's apply pass (csrc/kernels/bn_alg.hip header): with
    z = a W^T (this conv's forward) substituted into bn3's backward dz = A g + B (z - mean) + D,

        dW = diag(A) P + diag(B) W Gram + E (x) S,    da = [g | a | a | 1] [diag(A) W | G_hi | G_lo | c]^T

    where P = g^T a, Gram = a^T a, S = sum(a) come from ONE weight-gradient pass over (g, a)
    (conv1x1_wgrad_seg), G = W^T diag(B) W, c = E W, E = D - B mean. The data-gradient GEMM
    (conv1x1_gemm_seg) also takes bn2's backward reduction in its epilogue. Neither dz nor z is read: per
    block the 4C-channel tensor is read twice (g) instead of five times (dy, z, dz x 2 + the apply's write).
    Needs g = dy * mask as a plain tensor (``d.dy_masked``: the producer stored it masked). None when the
    path does not apply (the caller materialises dz)."""
    # linked (a downsample block's shortcut conv, PDT_DS_ALG): only as the FIRST of the two branches — dx is handed
    # to conv1's dgrad GEMM to accumulate into (or, strided, added at the sampled pixels), so it takes no reduction
    linked = ctx.link is not None
    if not (SW.bwd_alg and (not linked or ctx.link.grad is None) and getattr(ctx, "dre", None) is None
            and ctx.needs_input_grad[0] and ctx.needs_input_grad[1] and d.dy_masked and alg_bwd_shape_ok(weight)
            and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)):
        return None
    from ._native import native
    C4, CW = weight.shape[0], weight.shape[1]
    g2 = _nhwc2d(d.dy.contiguous(memory_format=torch.channels_last))  # [M, C4] gradient at bn3's output, masked
    a2 = _nhwc2d(x)  # [M, CW] this conv's input (bn2's output)
    wg = d.wg  # run by bn3's backward already (PDT_BWD_ALG=2, batchnorm.py _alg_prelude)
    if wg is None:
        wg = native().conv1x1_wgrad_seg(a2, g2, a2)  # [C4 + CW + ones, CW] fp32: P, Gram, column sums of a
    if wg is None:
        return None
    w2 = weight.reshape(C4, CW).contiguous()
    coef = d.coef.contiguous()
    # W^T diag(B) W [CW, CW], diag(B) W Gram [C4, CW] (fp32), on the matrix cores from W^T (the dgrad's prepared copy)
    G, bwg = native().bn_alg_small_gemm(w2, coef, wg, _wt_of(weight, w2))
    rep = 2 if SW.alg_glo else 1  # G as a bf16 hi + lo pair (a repeated in K), or its hi half only
    bcat, dw2 = native().bn_alg_assemble(w2, coef, d.mean.contiguous(), G, wg, bwg, rep)
    gsrc = getattr(ctx, "gsrc", None)
    gs = gsrc if (gsrc is not None and gsrc.ready() and not linked) else None
    dx = torch.empty_like(x, memory_format=torch.channels_last)
    part = native().conv1x1_gemm_seg(g2, a2, rep, bcat, _nhwc2d(dx), bn_x=gs.x if gs else None,
                                     bn_mask=gs.mask if gs else None, bn_mean=gs.mean if gs else None)
    if gs is not None and part is not None:
        gs.deposit(part, dx, masked=gs.mask is not None)
    return dx, dw2.as_strided(weight.shape, weight.stride())


def fused_bwd_shape_ok(weight: torch.Tensor) -> bool:
    """(Co, Ci) of a 1x1 conv whose backward conv1x1_bwd_fused takes (ResNet-50 layer-1 / layer-2 conv3;
    ``PDT_BWD_FUSED_SHAPES``, e.g. "256x64", restricts the set)."""
    return weight.dim() == 4 and tuple(weight.shape[:2]) in SW.bwd_fused_shapes and weight.dtype == torch.bfloat16


def _subsample_native(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 4 and t.shape[1] % 8 == 0
            and t.is_contiguous(memory_format=torch.channels_last) and not disabled() and SW.subsample_native)


def subsample_of(x: torch.Tensor, s: int):
    """``x[:, :, ::s, ::s]`` as a compact channels_last tensor when the kernel that wrote x also wrote it (a ResNet
    stage's last BatchNorm apply, ops/batchnorm.py ``sub_stride``) and x is unmodified since; else None."""
    t = getattr(x, "_pdt_sub", None)
    if t is not None and t[0] == s and t[2] == x._version:
        return t[1]
    return None


class StridedGrad:
    """Gradient of a strided subsampling ``x[:, :, ::s, ::s]`` kept compact (only the sampled
    positions are non-zero) until it is added into a full-size gradient of ``x``."""

    __slots__ = ("t", "s")

    def __init__(self, t: torch.Tensor, s: int):
        self.t, self.s = t, s

    def add_into(self, full: torch.Tensor) -> torch.Tensor:
        if _subsample_native(full) and _subsample_native(self.t):
            from ._native import native
            native().subsample_scatter_add(self.t, full, self.s)  # csrc/kernels/subsample.hip
        else:
            full[:, :, ::self.s, ::self.s].add_(self.t)
        return full

    def dense(self, shape) -> torch.Tensor:
        full = torch.zeros(shape, dtype=self.t.dtype, device=self.t.device).contiguous(
            memory_format=torch.channels_last)
        return self.add_into(full)


class _Conv1x1StridedFn(torch.autograd.Function):
    """Stride-s 1x1 convolution (the ResNet downsample shortcut) as a gather of the sampled pixels
    + GEMMs, instead of MIOpen's strided implicit-GEMM kernels (which need zero-fill passes). The
    data gradient is non-zero only at the sampled positions: with a ``ResidualGradLink`` it is
    handed over compact (``StridedGrad``) and added into conv1's full-size gradient at those
    positions, so no full-size zero tensor is ever written."""

    @staticmethod
    def forward(ctx, x, weight, s, link, stats_out=None, bwd_link=None):
        """``bwd_link``: the shortcut BatchNorm may hand its input gradient over in deferred form for the ALG
        backward (``_bwd_alg`` on the gathered input; PDT_DS_ALG)."""
        N, Ci, H, W = x.shape
        Co = weight.shape[0]
        xs = subsample_of(x, s)  # written by the producing BatchNorm apply (its _pdt_sub), or None
        if xs is not None:
            pass
        elif _subsample_native(x):
            from ._native import native
            xs = native().subsample_gather(x, s)  # csrc/kernels/subsample.hip
        else:
            xs = x[:, :, ::s, ::s].contiguous(memory_format=torch.channels_last)
        Hs, Ws = xs.shape[2], xs.shape[3]
        M = N * Hs * Ws
        ctx.save_for_backward(xs, weight)
        ctx.s, ctx.link, ctx.xshape = s, link, x.shape
        ctx.bwd_link = bwd_link
        if bwd_link is not None:
            ctx.set_materialize_grads(False)
            bwd_link.alg_src = (xs, weight)
        if x.dtype == torch.bfloat16 and _ours_ok("fwd", M, Ci, Co):
            # our GEMM, with the consuming (downsample) BatchNorm's statistics in the epilogue
            from ._native import native
            y = torch.empty((N, Co, Hs, Ws), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
            part = native().conv1x1_gemm(_nhwc2d(xs), weight.reshape(Co, Ci).contiguous(), _nhwc2d(y), False,
                                         stats_out is not None)
            if stats_out is not None:
                stats_out.append(part)
            return y
        return torch.mm(_nhwc2d(xs), weight.reshape(Co, Ci).t()).view(N, Hs, Ws, Co).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        xs, weight = ctx.saved_tensors
        N, Ci, Hs, Ws = xs.shape
        Co = weight.shape[0]
        if gy is None:  # the shortcut BatchNorm handed its input gradient over (or there is none)
            d = ctx.bwd_link.take() if ctx.bwd_link is not None else None
            r = _bwd_alg(ctx, d, xs, weight) if d is not None else None
            if r is not None:
                return _Conv1x1StridedFn._deliver(ctx, r[0]), r[1], None, None, None, None
            if d is None and ctx.link is None:
                return (None,) * 6
            gy = d.materialize() if d is not None else torch.zeros(
                (N, Co, Hs, Ws), dtype=xs.dtype, device=xs.device, memory_format=torch.channels_last)
        gy = gy.contiguous(memory_format=torch.channels_last)
        g2, w2 = _nhwc2d(gy), weight.reshape(Co, Ci)
        M = g2.shape[0]
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if gy.dtype == torch.bfloat16 and _ours_ok("dgrad", M, Co, Ci):
                from ._native import native
                d = torch.empty((N, Ci, Hs, Ws), dtype=gy.dtype, device=gy.device, memory_format=torch.channels_last)
                native().conv1x1_gemm(g2, _wt_of(weight, w2), _nhwc2d(d), False, False)
            else:
                d = torch.mm(g2, w2).view(N, Hs, Ws, Ci).permute(0, 3, 1, 2)
            dx = _Conv1x1StridedFn._deliver(ctx, d)
        if ctx.needs_input_grad[1]:
            sk = max(8, min(64, 1 << max(0, (M // 3136).bit_length() - 1)))  # ~3-6K pixels per slice
            if M % sk == 0 and M // sk >= 256:
                dw = _wgrad_splitk(g2, _nhwc2d(xs), sk).as_strided(weight.shape, weight.stride())
            else:
                dw = torch.mm(g2.t(), _nhwc2d(xs)).as_strided(weight.shape, weight.stride())
        return dx, dw, None, None, None, None

    @staticmethod
    def _deliver(ctx, d):
        """The compact data gradient ``d`` (sampled pixels only) to the input: handed to conv1's backward through
        the link when this branch is first, else added into the partner's gradient / a zero tensor (returned)."""
        compact = StridedGrad(d, ctx.s)
        acc = ctx.link.take() if ctx.link is not None else None
        if ctx.link is not None and acc is None:
            ctx.link.grad = compact  # first: conv1's backward adds it into its full gradient
            return None
        if acc is not None:
            return compact.add_into(acc)
        return compact.dense(ctx.xshape)


class _LinkedConvFn(torch.autograd.Function):
    """Plain (MIOpen) convolution whose input gradient meets the other branch's gradient of the
    same input through a ``ResidualGradLink``: the first branch to finish backward stashes its
    gradient and returns None, the second adds into it and returns the sum — correct in either
    execution order, no autograd add node."""

    @staticmethod
    def forward(ctx, x, weight, stride, padding, link):
        ctx.save_for_backward(x, weight)
        ctx.stride, ctx.padding, ctx.link = stride, padding, link
        return F.conv2d(x, weight, None, stride, padding)

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        args = (gy, x, weight, None, list(ctx.stride), list(ctx.padding), [1, 1], False, [0, 0], 1)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(*args, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            dw = torch.ops.aten.convolution_backward(*args, [False, True, False])[1]
        if dx is not None:
            acc = ctx.link.take()
            if acc is None:
                ctx.link.grad, dx = dx, None
            else:
                dx = acc.add_(dx)
        return dx, dw, None, None, None


class _Conv3x3Fn(torch.autograd.Function):
    """Stride-1 pad-1 3x3 convolution on our MFMA kernels: forward = conv3x3s1(x, w)
    (csrc/kernels/conv3x3.hip); data gradient = the SAME kernel on dY with the weights flipped and
    transposed (conv3x3_flip); weight gradient = the halo-tiled split-K MFMA kernel
    (csrc/kernels/conv3x3_wgrad.hip; ``PDT_CONV3X3_WGRAD=miopen`` or an unsupported shape: MIOpen)."""

    @staticmethod
    def forward(ctx, x, weight, stats_out=None, gsrc=None):
        from ._native import native
        ctx.save_for_backward(x, weight)
        ctx.gsrc = gsrc  # x is a BatchNorm output: the dgrad kernel can take that BN's backward reduction
        if stats_out is not None:  # BatchNorm statistics in the epilogue (halo kernel shapes)
            r = native().conv3x3s1_fwd_stats(x, weight)
            if len(r) == 2:
                stats_out.append(r[1])
            return r[0]
        return native().conv3x3s1_fwd(x, weight)

    @staticmethod
    def backward(ctx, gy):
        from ._native import native
        x, weight = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        fork = _WgradFork(gy, gy.shape[0] * gy.shape[2] * gy.shape[3])
        dx = dw = None
        if ctx.needs_input_grad[0]:
            gs = ctx.gsrc if ctx.gsrc is not None and ctx.gsrc.ready() else None
            if gs is not None:  # dx is the gradient at a BatchNorm's output: its reduction in the epilogue
                r = native().conv3x3s1_fwd_bnbwd(gy, _flip_of(weight), gs.x, gs.mask, gs.mean)
                dx = r[0]
                if len(r) == 2:
                    gs.deposit(r[1], dx)
            else:
                dx = native().conv3x3s1_fwd(gy, _flip_of(weight))
        if ctx.needs_input_grad[1]:
            if SW.conv3x3_wgrad == "ours":
                dw = fork.run(lambda: native().conv3x3s1_wgrad(x, gy))
            if dw is None:
                args = (gy, x, weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1)
                dw = torch.ops.aten.convolution_backward(*args, [False, True, False])[1]
        return dx, dw, None, None


class _Conv3x3S2Fn(torch.autograd.Function):
    """Stride-2 pad-1 3x3 convolution on our MFMA kernels (csrc/kernels/conv3x3_s2.hip): forward =
    gathered implicit GEMM with the consuming BatchNorm's statistics in the epilogue; data gradient =
    the four output-parity phases of the transposed conv in one launch (with the producing BatchNorm's
    backward reduction in the epilogue); weight gradient = the halo-tiled split-K kernel at stride 2
    (conv3x3_wgrad.hip). Replaces MIOpen's ck grouped_conv_fwd / igemm_bwd / igemm_wrw on ResNet-50's
    layer2-4 block-0 conv2."""

    @staticmethod
    def forward(ctx, x, weight, stats_out=None, gsrc=None):
        from ._native import native
        ctx.save_for_backward(x, weight)
        ctx.gsrc = gsrc
        r = native().conv3x3s2_fwd(x, weight, stats_out is not None)
        if not r:  # shape the kernel does not take
            return F.conv2d(x, weight, None, 2, 1)
        if stats_out is not None:
            stats_out.append(r[1])
        return r[0]

    @staticmethod
    def backward(ctx, gy):
        from ._native import native
        x, weight = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        fork = _WgradFork(gy, gy.shape[0] * gy.shape[2] * gy.shape[3])
        args = (gy, x, weight, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            H, W = x.shape[2], x.shape[3]
            gs = ctx.gsrc if ctx.gsrc is not None and ctx.gsrc.ready() else None
            kw = dict(bn_x=gs.x, bn_mask=gs.mask, bn_mean=gs.mean) if gs is not None else {}
            r = native().conv3x3s2_dgrad(gy, _flip_of(weight), H, W, **kw)
            if r:
                dx = r[0]
                if len(r) == 2:
                    gs.deposit(r[1], dx)
            else:
                dx = torch.ops.aten.convolution_backward(*args, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            if SW.conv3x3_wgrad == "ours":
                dw = fork.run(lambda: native().conv3x3s2_wgrad(x, gy))
            if dw is None:
                dw = torch.ops.aten.convolution_backward(*args, [False, True, False])[1]
        return dx, dw, None, None


def conv3x3s2_eligible(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Our stride-2 3x3 kernels apply: stride 2, padding 1, no bias/groups/dilation, channels_last
    bf16 GPU input with Ci % 64 == 0 and Co % 64 == 0 (ResNet-50: layer2-4 block-0 conv2; ResNet-18/34:
    layer2-4 block-0 conv1; 64-channel GEMM N dimensions take the kernel's 64-wide tile)."""
    return (conv.kernel_size == (3, 3) and conv.stride == (2, 2) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None and conv.padding_mode == "zeros"
            and x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 64 == 0
            and conv.out_channels % 64 == 0 and x.shape[2] >= 2 and x.shape[3] >= 2
            and SW.conv3x3_s2 == "ours" and not disabled())


def conv3x3_eligible(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Our 3x3 kernel applies: stride 1, padding 1, no bias/groups/dilation, channels_last bf16 GPU
    input with Ci % 64 == 0 and Co % 64 == 0 (the data gradient swaps them; ResNet-50: 13 of 16 3x3 convs)."""
    return (conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None and conv.padding_mode == "zeros"
            and x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 64 == 0
            and conv.out_channels % 64 == 0 and SW.conv3x3 == "ours" and not disabled())


class _StemConvFn(torch.autograd.Function):
    """ResNet stem (7x7 / stride 2 / pad 3, 3 -> 64) on our MFMA kernels (csrc/kernels/conv_stem.hip):
    forward and weight gradient (W <= 224; MIOpen beyond); the input gradient — which training
    never asks for (the images need none) — on MIOpen."""

    @staticmethod
    def forward(ctx, x, weight):
        from ._native import native
        ctx.save_for_backward(x, weight)
        return native().stem_conv_fwd(x, weight)

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        args = (gy, x, weight, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(*args, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            if x.shape[3] <= 224:
                from ._native import native
                dw = native().stem_conv_wgrad(x, gy)
            else:
                dw = torch.ops.aten.convolution_backward(*args, [False, True, False])[1]
        return dx, dw


def stem_eligible(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Our stem kernel applies: 7x7 / stride 2 / pad 3, 3 -> 64 channels, no bias, channels_last
    bf16 GPU input with W % 32 == 0 (``PDT_CONV_STEM=miopen`` switches back)."""
    return (conv.kernel_size == (7, 7) and conv.stride == (2, 2) and conv.padding == (3, 3)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None and conv.padding_mode == "zeros"
            and conv.in_channels == 3 and conv.out_channels == 64 and x.is_cuda and x.dim() == 4
            and x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[3] % 32 == 0
            and SW.conv_stem == "ours" and not disabled())


class _StemBlockFn(torch.autograd.Function):
    """ResNet stem in training: conv 7x7/s2 -> BatchNorm -> ReLU -> MaxPool2d(3, 2, 1) as ONE autograd
    node, so its backward can hand the BatchNorm's backward apply to the stem weight-gradient kernel:
    the pool-gradient kernel takes the BN reduction and yields dz (the gradient at the BN output) and
    the dx coefficients, and ``stem_conv_wgrad_bn`` forms dx = A dz + B (x - mean) + D while loading
    its operand — the BN's dx (1.6 GB at batch 1024) is never written or read back. Forward: the stem
    conv with the BN statistics in its epilogue (``PDT_STEM_BN_STATS``, 224-wide images), then the BN
    finalize + ReLU + pool kernel — or the unfused modules' kernels (stem conv; BN reduce, ReLU, pool)."""

    @staticmethod
    def forward(ctx, img, weight, gamma, beta, running_mean, running_var, momentum, eps):
        from ._native import native
        n = native()
        r = n.stem_conv_fwd_stats(img, weight) if SW.stem_bn_stats else []
        if r:  # the statistics come from the conv's epilogue partials: no reduce pass over xb
            xb, part = r
            y, code, mean, invstd = n.bn_relu_maxpool_fwd_parts(xb, part, gamma, beta, running_mean, running_var,
                                                                momentum, eps)
        else:
            xb = n.stem_conv_fwd(img, weight)
            y, code, mean, invstd = n.bn_relu_maxpool_fwd(xb, gamma, beta, running_mean, running_var, momentum, eps)
        ctx.save_for_backward(img, weight, xb, code, gamma, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        from ._native import native
        n = native()
        img, weight, xb, code, gamma, mean, invstd = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        need_bn = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        dimg = dw = None
        if ctx.needs_input_grad[0]:  # training never asks for the image gradient: the unfused chain
            dx, dg, db = n.maxpool3s2_bwd_bn(dy, code, xb, gamma, mean, invstd, need_bn)
            args = (dx, img, weight, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1)
            dimg = torch.ops.aten.convolution_backward(*args, [True, False, False])[0]
            if ctx.needs_input_grad[1]:
                dw = n.stem_conv_wgrad(img, dx)
        elif SW.stem_pool_wgrad and ctx.needs_input_grad[1]:
            # the pool gradient's BN reduction only (no dz written); the weight gradient re-forms dz per tile
            _, coef, dg, db = n.maxpool3s2_bwd_bn_coef(dy, code, xb, gamma, mean, invstd, need_bn, False)
            dw = n.stem_conv_wgrad_bn_pool(img, dy, code, xb, coef, mean)
        else:
            dz, coef, dg, db = n.maxpool3s2_bwd_bn_coef(dy, code, xb, gamma, mean, invstd, need_bn)
            if ctx.needs_input_grad[1]:
                dw = n.stem_conv_wgrad_bn(img, dz, xb, coef, mean)
        return dimg, dw, (dg if need_bn else None), (db if need_bn else None), None, None, None, None


def _has_hooks(m: nn.Module) -> bool:
    from torch.nn.modules import module as _m
    return bool(m._forward_hooks or m._forward_pre_hooks or _m._global_forward_hooks
                or _m._global_forward_pre_hooks)


def stem_block(conv: nn.Conv2d, bn: nn.Module, x: torch.Tensor):
    """``max_pool2d(relu(bn(conv(x))), 3, 2, 1)`` as one ``_StemBlockFn`` node when our stem kernels
    and the fused BN + pool path both apply in training (affine BN with running statistics, images
    of width <= 224, no module hooks, ``PDT_STEM_BN_WGRAD=1``); None otherwise (the caller runs the
    modules)."""
    if not (SW.stem_bn_wgrad and SW.stem_bwd_fused and bn.training and torch.is_grad_enabled()
            and isinstance(conv, SplitConv2d) and stem_eligible(conv, x) and x.shape[3] <= 224
            and getattr(bn, "affine", False) and getattr(bn, "track_running_stats", False)
            and hasattr(bn, "stem_params") and not _has_hooks(conv) and not bn.has_hooks()):
        return None
    w, b, rm, rv, momentum, eps = bn.stem_params()
    return _StemBlockFn.apply(x, conv.weight, w, b, rm, rv, momentum, eps)


class SplitConv2d(nn.Conv2d):
    """``nn.Conv2d`` (same parameters / state_dict). On the GPU, stride-1 and stride-2 3x3
    convolutions and the ResNet stem run on our MFMA kernels (``_Conv3x3Fn`` / ``_Conv3x3S2Fn`` /
    ``_StemConvFn``; ``PDT_CONV3X3=miopen`` / ``PDT_CONV3X3_S2=miopen`` / ``PDT_CONV_STEM=miopen``
    switch back)."""

    emit_bn_stats = True  # output feeds a BatchNorm: fuse its statistics where our kernel runs

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        s1 = conv3x3_eligible(self, x)
        if s1 or conv3x3s2_eligible(self, x):
            holder = [] if (self.emit_bn_stats and self.training and torch.is_grad_enabled()
                            and SW.conv_bn_stats) else None
            from .batchnorm import grad_stats_source_of
            fn = _Conv3x3Fn if s1 else _Conv3x3S2Fn
            y = fn.apply(x, self.weight, holder,
                         grad_stats_source_of(x) if self.training and torch.is_grad_enabled() else None)
            if holder:
                y._pdt_bn_stats = BNStats(holder[0], y._version)
            return y
        if stem_eligible(self, x):
            return _StemConvFn.apply(x, self.weight)
        return super().forward(x)


class PatchConv2d(nn.Conv2d):
    """``nn.Conv2d`` (same parameters / state_dict) for a non-overlapping patch embedding — kernel ==
    stride, no padding, no dilation, groups 1 (ViT's ``conv_proj``). On the GPU it runs as patchify
    (one reshape copy of the input into [B * gh * gw, C * p * p] rows, the weight's (c, kh, kw)
    order) + ONE GEMM through ``ops.linear`` (hipBLASLt forward with the bias in its epilogue,
    split-K weight gradient, column-strip bias gradient), instead of MIOpen's strided implicit-GEMM
    forward / weight-gradient kernels, their transposes and their run-time compile on a fresh box.
    The output is returned as the [B, D, gh, gw] view of the GEMM's [B, gh, gw, D] rows, so
    ``flatten(2).transpose(1, 2)`` (the token sequence) is contiguous again without a copy."""

    def _patch_ok(self, x: torch.Tensor) -> bool:
        k = self.kernel_size
        return (x.is_cuda and x.dim() == 4 and k == self.stride and self.padding == (0, 0)
                and self.dilation == (1, 1) and self.groups == 1 and self.padding_mode == "zeros"
                and x.dtype == self.weight.dtype and not disabled())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self._patch_ok(x):
            return super().forward(x)
        from .linear import linear
        ph, pw = self.kernel_size
        B, C, H, W = x.shape
        gh, gw = H // ph, W // pw
        xp = (x[:, :, :gh * ph, :gw * pw].reshape(B, C, gh, ph, gw, pw).permute(0, 2, 4, 1, 3, 5)
              .reshape(B * gh * gw, C * ph * pw))
        y = linear(xp, self.weight.reshape(self.out_channels, -1), self.bias)
        return y.view(B, gh, gw, self.out_channels).permute(0, 3, 1, 2)


def linked_conv(conv: nn.Conv2d, x: torch.Tensor, link, bwd_link=None) -> torch.Tensor:
    """``conv(x)`` whose input gradient is summed with the partner branch's through ``link``
    (``bwd_link``: see ``Conv1x1.forward``; the caller checked ``fused_bwd_ok``)."""
    if isinstance(conv, Conv1x1) and (conv.gemm_eligible(x) or conv.strided_gemm_eligible(x)):
        return conv(x, res_link=link, bwd_link=bwd_link)
    assert bwd_link is None, "bwd_link needs the stride-1 GEMM path"
    return _LinkedConvFn.apply(x, conv.weight, conv.stride, conv.padding, link)


class Conv1x1(nn.Conv2d):
    """``nn.Conv2d(Ci, Co, 1, bias=False)`` (same parameters and state_dict) whose stride-1 GPU
    channels_last path runs as autotuned GEMMs; everything else is plain ``nn.Conv2d``."""

    def __init__(self, inp: int, out: int, stride: int = 1, emit_bn_stats: bool = True):
        super().__init__(inp, out, 1, stride=stride, bias=False)
        self.emit_bn_stats = emit_bn_stats  # output feeds a BatchNorm: fuse its statistics (our GEMM)

    def _gemm_ok(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dim() == 4 and x.dtype == self.weight.dtype and self.padding == (0, 0)
                and x.is_contiguous(memory_format=torch.channels_last) and SW.conv1x1 != "off" and not disabled())

    def gemm_eligible(self, x: torch.Tensor) -> bool:
        return self.stride == (1, 1) and self._gemm_ok(x)

    def masked_residual_ok(self, x: torch.Tensor) -> bool:
        """Our dgrad GEMM can take the shortcut gradient as (dy, ReLU mask) (``MaskedGrad``):
        ``PDT_RES_MASKED=0`` turns the hand-off off."""
        N, Ci, H, W = x.shape
        return (SW.res_masked and x.dtype == torch.bfloat16
                and self.gemm_eligible(x) and _ours_ok("dgrad", N * H * W, self.out_channels, Ci))

    def strided_gemm_eligible(self, x: torch.Tensor) -> bool:
        s = self.stride[0]
        # gather + our GEMM (BN statistics fused) + split-K weight gradient: ResNet-50 +1.7% over
        # MIOpen's strided kernels (12,318 vs 12,118 img/s, tools/gpu_s2b.sh; PDT_CONV1X1_S2=0 = MIOpen)
        return s > 1 and self.stride == (s, s) and self._gemm_ok(x) and SW.conv1x1_s2

    def forward(self, x: torch.Tensor, res_link=None, bwd_link=None) -> torch.Tensor:
        """``res_link``: a ``ResidualGradLink`` whose gradient (the other branch's gradient of
        ``x``) meets this conv's input gradient; requires one of the GEMM paths. ``bwd_link``: a
        ``BNGradLink`` through which the BatchNorm consuming the output may hand over its input
        gradient in deferred form (stride-1 GEMM path only; check ``fused_bwd_ok``). ``x`` may be a
        ``DeferredReLUBN`` (bn2 -> conv3 with the fused backward): relu(a x + b) read on load."""
        from .batchnorm import DeferredReLUBN
        if isinstance(x, DeferredReLUBN):
            assert bwd_link is not None and res_link is None and self.gemm_eligible(x.raw), \
                "a deferred BatchNorm input needs the fused-backward GEMM path"
            holder = [] if (self.emit_bn_stats and SW.conv_bn_stats) else None
            y = _Conv1x1Fn.apply(x.raw, self.weight, None, holder, x.gsrc, bwd_link, x)
            if holder:
                y._pdt_bn_stats = BNStats(holder[0], y._version)
                _attach_gemm_source(y, x.raw, self.weight, x.ab)
            return y
        if self.gemm_eligible(x):
            holder = [] if (self.emit_bn_stats and self.training and torch.is_grad_enabled()
                            and SW.conv_bn_stats) else None
            from .batchnorm import grad_stats_source_of
            # a bottleneck conv3 on the ALG backward (PDT_BWD_ALG=2): its output z is needed only for the consuming
            # BatchNorm's statistics (this GEMM's epilogue) and its apply, which runs as this GEMM again (APPLY
            # epilogue) — so z is never written (PDT_Z3_VIRTUAL; materialize_virtual recomputes it on a fallback)
            virt = (holder is not None and bwd_link is not None and bwd_link.needs_masked and SW.bwd_alg >= 2
                    and x.dtype == torch.bfloat16
                    and (SW.z3_virtual == 1 or (SW.z3_virtual == 2 and 0 < self.in_channels <= SW.bn_apply_gemm_k)))
            y = _Conv1x1Fn.apply(x, self.weight, res_link, holder,
                                 grad_stats_source_of(x) if self.training and torch.is_grad_enabled() else None,
                                 bwd_link, None, virt)
            if holder:  # (our GEMM ran: the statistics came from its epilogue)
                y._pdt_bn_stats = BNStats(holder[0], y._version)
                if virt and len(holder) > 1:  # the store was skipped: only the APPLY GEMM may consume z
                    y._pdt_virtual = (x, self.weight)
                    y._pdt_gemm_src = GemmSource(x, self.weight, None, y._version)
                else:
                    _attach_gemm_source(y, x, self.weight, None)
            return y
        if self.strided_gemm_eligible(x):
            holder = [] if (self.emit_bn_stats and self.training and torch.is_grad_enabled()
                            and SW.conv_bn_stats) else None
            y = _Conv1x1StridedFn.apply(x, self.weight, self.stride[0], res_link, holder, bwd_link)
            if holder:
                y._pdt_bn_stats = BNStats(holder[0], y._version)
            return y
        assert res_link is None and bwd_link is None, "res_link / bwd_link need a GEMM path"
        return super().forward(x)

    def alg_bwd_ok(self, x: torch.Tensor) -> bool:
        """This conv's backward can take its consuming BatchNorm's input gradient in deferred form and run the
        ALG backward (``_bwd_alg``; ``PDT_BWD_ALG=0`` turns it off)."""
        return (SW.bwd_alg and self.training and torch.is_grad_enabled() and x.dtype == torch.bfloat16
                and x.numel() // max(1, x.shape[1]) >= SW.bwd_alg_min_m
                and self.gemm_eligible(x) and alg_bwd_shape_ok(self.weight) and not _has_hooks(self)
                and not self._backward_hooks and not self._backward_pre_hooks)

    def ds_alg_ok(self, x: torch.Tensor) -> bool:
        """As a downsample block's shortcut conv (stride 1 or strided GEMM path): its backward can run the ALG
        backward with the shortcut BatchNorm's input gradient in deferred form (``PDT_DS_ALG``: input channels up
        to that many; ResNet-50 layer 4's 1024 -> 2048 shortcut would double its GEMM for a 180 us pass)."""
        s = self.stride[0]
        m_out = x.shape[0] * (-(-x.shape[2] // s)) * (-(-x.shape[3] // s)) if x.dim() == 4 else 0
        return (SW.bwd_alg >= 2 and 0 < self.in_channels <= SW.ds_alg and self.training and torch.is_grad_enabled()
                and x.dtype == torch.bfloat16 and m_out >= SW.bwd_alg_min_m
                and (self.gemm_eligible(x) or self.strided_gemm_eligible(x))
                and alg_bwd_shape_ok(self.weight) and not _has_hooks(self)
                and not self._backward_hooks and not self._backward_pre_hooks)

    def fused_bwd_ok(self, x: torch.Tensor) -> bool:
        """This conv's backward can take its consuming BatchNorm's input gradient in deferred form
        (``bwd_link``) and run it as one fused kernel (``PDT_BWD_FUSED=0`` turns it off)."""
        return (SW.bwd_fused and self.training and torch.is_grad_enabled() and x.dtype == torch.bfloat16
                and self.gemm_eligible(x) and fused_bwd_shape_ok(self.weight) and not _has_hooks(self)
                and not self._backward_hooks and not self._backward_pre_hooks)
