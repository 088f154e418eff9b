"""Fused multi-tensor optimizers: SGD, Adam/AdamW, Adadelta (csrc/kernels/optim.hip).

Reference parity: the reference trains with ``torch.optim.Adadelta(lr=args.lr)`` + ``StepLR``
(/root/reference/train.py:99,101). These classes are drop-in ``torch.optim.Optimizer``s with the
same hyper-parameters, the same update math and the same per-parameter state keys
(``momentum_buffer``; ``step``/``exp_avg``/``exp_avg_sq``; ``step``/``square_avg``/``acc_delta``)
so torch optimizer checkpoints load into them and vice versa.

MI355X-first differences:
  * one kernel per (param dtype, grad dtype) group and ≤320 chunks of 32 Ki elements —
    param, grad and state are read once and written once;
  * ``master_weights=True``: bf16 parameters get an fp32 master copy in
    ``state['master_param']``; the kernel updates the master and writes the bf16 parameter
    in the same pass (no separate cast kernel, no autocast weight casts in forward);
  * lr (and Adam's step) live in device tensors, so a hipGraph-captured step replays with
    the current schedule value (``sync_lr()`` refreshes them outside the graph);
  * AMP: ``step(inv_scale=..., found_inf=...)`` unscales in-kernel and skips the update on
    device when an overflow was found — no host readback.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
from torch.optim import Optimizer

from ..ops._native import cuda_available, native, use_native


def _capturing() -> bool:
    return cuda_available() and torch.cuda.is_current_stream_capturing()


class _FusedOptimizer(Optimizer):
    _state_keys: Tuple[str, ...] = ()

    def __init__(self, params, defaults, master_weights: bool = True):
        super().__init__(params, defaults)
        self.master_weights = master_weights
        self._lr_dev: Dict[int, torch.Tensor] = {}
        self._lr_host: Dict[int, float] = {}

    # -- helpers -------------------------------------------------------------
    def _lr_tensor(self, gi: int, group: dict, device: torch.device) -> torch.Tensor:
        t = self._lr_dev.get(gi)
        lr = float(group["lr"])
        if t is None or t.device != device:
            t = torch.full((1,), lr, dtype=torch.float32, device=device)
            self._lr_dev[gi] = t
            self._lr_host[gi] = lr
        elif not _capturing() and self._lr_host.get(gi) != lr:
            t.fill_(lr)
            self._lr_host[gi] = lr
        return t

    def sync_lr(self) -> None:
        """Push host-side ``group['lr']`` into the device lr tensors (call outside graph replay)."""
        for gi, group in enumerate(self.param_groups):
            if gi in self._lr_dev and self._lr_host.get(gi) != float(group["lr"]):
                self._lr_dev[gi].fill_(float(group["lr"]))
                self._lr_host[gi] = float(group["lr"])

    def _master(self, p: torch.Tensor) -> Optional[torch.Tensor]:
        if not (self.master_weights and p.dtype in (torch.bfloat16, torch.float16)):
            return None
        st = self.state[p]
        m = st.get("master_param")
        if m is None:
            m = torch.empty_like(p, dtype=torch.float32)
            m.copy_(p.detach())
            st["master_param"] = m
        return m

    def _buckets(self, group) -> Dict[tuple, List[torch.Tensor]]:
        out: Dict[tuple, List[torch.Tensor]] = {}
        for p in group["params"]:
            if p.grad is None:
                continue
            if p.grad.is_sparse:
                raise RuntimeError("fused optimizers do not support sparse gradients")
            m = self._master(p)
            key = ((m if m is not None else p).dtype, p.grad.dtype, m is not None, p.device)
            out.setdefault(key, []).append(p)
        return out

    @torch.no_grad()
    def step(self, closure=None, inv_scale: Optional[torch.Tensor] = None,
             found_inf: Optional[torch.Tensor] = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            for key, ps in self._buckets(group).items():
                self._init_state(group, ps)
                masters = [self.state[p]["master_param"] for p in ps] if key[2] else []
                kparams = masters if key[2] else ps
                copies = ps if key[2] else []
                grads = [p.grad for p in ps]
                if use_native(*kparams):
                    self._native_step(gi, group, ps, kparams, grads, copies, inv_scale, found_inf)
                else:
                    if found_inf is not None and float(found_inf.item()) != 0.0:
                        continue
                    if inv_scale is not None:
                        grads = [g * inv_scale.to(g.dtype) for g in grads]
                    self._ref_step(group, ps, kparams, grads)
                    for p, m in zip(copies, masters):
                        p.copy_(m)
        return loss

    def _init_state(self, group, ps):
        raise NotImplementedError

    def _native_step(self, gi, group, ps, kparams, grads, copies, inv_scale, found_inf):
        raise NotImplementedError

    def _ref_step(self, group, ps, kparams, grads):
        raise NotImplementedError


class FusedSGD(_FusedOptimizer):
    """``torch.optim.SGD`` semantics (momentum, dampening, nesterov, weight_decay, maximize)."""

    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, maximize: bool = False,
                 master_weights: bool = True):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                      weight_decay=weight_decay, nesterov=nesterov, maximize=maximize),
                         master_weights)

    def _init_state(self, group, ps):
        if group["momentum"] == 0:
            return
        for p in ps:
            st = self.state[p]
            if st.get("momentum_buffer") is None:
                ref = st.get("master_param", p)
                st["momentum_buffer"] = torch.zeros_like(ref, dtype=torch.float32)
                st["_first"] = True

    def _native_step(self, gi, group, ps, kparams, grads, copies, inv_scale, found_inf):
        bufs = [self.state[p]["momentum_buffer"] for p in ps] if group["momentum"] != 0 else []
        first = bool(bufs) and bool(self.state[ps[0]].get("_first", False))
        native().sgd(kparams, grads, bufs, copies, float(group["lr"]),
                     self._lr_tensor(gi, group, kparams[0].device), float(group["momentum"]),
                     float(group["dampening"]), float(group["weight_decay"]), bool(group["nesterov"]),
                     first, bool(group["maximize"]), inv_scale, found_inf)
        for p in ps:
            self.state[p]["_first"] = False

    def _ref_step(self, group, ps, kparams, grads):
        for p, kp, g in zip(ps, kparams, grads):
            g = g.float()
            if group["maximize"]:
                g = -g
            if group["weight_decay"]:
                g = g + group["weight_decay"] * kp.float()
            if group["momentum"]:
                st = self.state[p]
                b = st["momentum_buffer"]
                if st.get("_first", False):
                    b.copy_(g)
                    st["_first"] = False
                else:
                    b.mul_(group["momentum"]).add_(g, alpha=1 - group["dampening"])
                g = g + group["momentum"] * b if group["nesterov"] else b
            kp.add_(g.to(kp.dtype), alpha=-group["lr"])

    def state_dict(self):
        sd = super().state_dict()
        for st in sd["state"].values():
            st.pop("_first", None)
        return sd


class FusedAdam(_FusedOptimizer):
    """``torch.optim.Adam`` / ``AdamW`` semantics (``adam_w_mode`` selects decoupled decay)."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False, maximize: bool = False,
                 adam_w_mode: bool = False, master_weights: bool = True):
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported by the fused kernel")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                                      maximize=maximize, adam_w_mode=adam_w_mode), master_weights)
        self._step_dev: Dict[int, torch.Tensor] = {}

    def _init_state(self, group, ps):
        shared = None
        for p in ps:
            st = self.state[p]
            if "exp_avg" not in st:
                ref = st.get("master_param", p)
                st["exp_avg"] = torch.zeros_like(ref, dtype=torch.float32)
                st["exp_avg_sq"] = torch.zeros_like(ref, dtype=torch.float32)
                if shared is None:
                    shared = torch.zeros((), dtype=torch.float32, device=p.device)
                st["step"] = shared

    def _native_step(self, gi, group, ps, kparams, grads, copies, inv_scale, found_inf):
        # every param of the group shares one device step counter (equal by construction)
        step_t = self.state[ps[0]]["step"]
        if step_t.device != kparams[0].device:
            step_t = step_t.to(kparams[0].device)
            self.state[ps[0]]["step"] = step_t
        if found_inf is None:
            step_t.add_(1)
        else:
            step_t.add_((found_inf.reshape(()) == 0).to(step_t.dtype))
        for p in ps[1:]:
            if self.state[p]["step"] is not step_t:  # e.g. after load_state_dict: alias once
                self.state[p]["step"] = step_t
        b1, b2 = group["betas"]
        native().adam(kparams, grads, [self.state[p]["exp_avg"] for p in ps],
                      [self.state[p]["exp_avg_sq"] for p in ps], copies, float(group["lr"]),
                      self._lr_tensor(gi, group, kparams[0].device), float(b1), float(b2), float(group["eps"]),
                      float(group["weight_decay"]), bool(group["adam_w_mode"]), step_t.reshape(1), 0.0,
                      bool(group["maximize"]), inv_scale, found_inf)

    def _ref_step(self, group, ps, kparams, grads):
        b1, b2 = group["betas"]
        bumped = set()
        for p, kp, g in zip(ps, kparams, grads):
            st = self.state[p]
            if id(st["step"]) not in bumped:  # step tensors may be shared across the group
                st["step"] += 1
                bumped.add(id(st["step"]))
            t = float(st["step"])
            g = g.float()
            if group["maximize"]:
                g = -g
            lr, wd = group["lr"], group["weight_decay"]
            if group["adam_w_mode"]:
                kp.mul_(1 - lr * wd)
            elif wd:
                g = g + wd * kp.float()
            st["exp_avg"].lerp_(g, 1 - b1)
            st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
            bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
            denom = (st["exp_avg_sq"].sqrt() / math.sqrt(bc2)).add_(group["eps"])
            kp.addcdiv_(st["exp_avg"], denom, value=-lr / bc1)


class FusedAdamW(FusedAdam):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, amsgrad: bool = False, maximize: bool = False,
                 master_weights: bool = True):
        super().__init__(params, lr, betas, eps, weight_decay, amsgrad, maximize, adam_w_mode=True,
                         master_weights=master_weights)


class FusedAdadelta(_FusedOptimizer):
    """``torch.optim.Adadelta`` semantics — the reference's optimizer (train.py:99)."""

    def __init__(self, params, lr: float = 1.0, rho: float = 0.9, eps: float = 1e-6,
                 weight_decay: float = 0.0, maximize: bool = False, master_weights: bool = True):
        super().__init__(params, dict(lr=lr, rho=rho, eps=eps, weight_decay=weight_decay, maximize=maximize),
                         master_weights)

    def _init_state(self, group, ps):
        for p in ps:
            st = self.state[p]
            if "square_avg" not in st:
                ref = st.get("master_param", p)
                st["step"] = torch.zeros((), dtype=torch.float32)
                st["square_avg"] = torch.zeros_like(ref, dtype=torch.float32)
                st["acc_delta"] = torch.zeros_like(ref, dtype=torch.float32)

    def _native_step(self, gi, group, ps, kparams, grads, copies, inv_scale, found_inf):
        if not _capturing():
            for p in ps:
                self.state[p]["step"] += 1
        native().adadelta(kparams, grads, [self.state[p]["square_avg"] for p in ps],
                          [self.state[p]["acc_delta"] for p in ps], copies, float(group["lr"]),
                          self._lr_tensor(gi, group, kparams[0].device), float(group["rho"]), float(group["eps"]),
                          float(group["weight_decay"]), bool(group["maximize"]), inv_scale, found_inf)

    def _ref_step(self, group, ps, kparams, grads):
        rho, eps, lr, wd = group["rho"], group["eps"], group["lr"], group["weight_decay"]
        for p, kp, g in zip(ps, kparams, grads):
            st = self.state[p]
            st["step"] += 1
            g = g.float()
            if group["maximize"]:
                g = -g
            if wd:
                g = g + wd * kp.float()
            sa, ad = st["square_avg"], st["acc_delta"]
            sa.mul_(rho).addcmul_(g, g, value=1 - rho)
            std = sa.add(eps).sqrt_()
            delta = ad.add(eps).sqrt_().div_(std).mul_(g)
            ad.mul_(rho).addcmul_(delta, delta, value=1 - rho)
            kp.add_(delta, alpha=-lr)


def build_optimizer(name: str, params, lr: float, **kw) -> Optimizer:
    name = name.lower()
    if name == "sgd":
        return FusedSGD(params, lr=lr, **kw)
    if name == "adamw":
        return FusedAdamW(params, lr=lr, **kw)
    if name == "adam":
        return FusedAdam(params, lr=lr, **kw)
    if name == "adadelta":
        return FusedAdadelta(params, lr=lr, **kw)
    raise ValueError(f"unknown optimizer {name}")
