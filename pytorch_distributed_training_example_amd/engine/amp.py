"""Mixed precision: autocast policy + a device-resident dynamic loss scaler.

Not in the reference (fp32 only). bf16 (the default here) needs no loss scaling; fp16 does.
``GradScaler`` keeps scale, growth tracker and the overflow flag in device tensors and
updates them with HIP kernels (csrc/kernels/amp.hip): unscale + inf-check is ONE multi-tensor
launch, the optimizer skips its update on device when the flag is set, and the scale update
is a 1-thread kernel — no ``.item()`` per step, so the whole step stays graph-capturable.
``state_dict`` uses torch.amp.GradScaler's keys.
"""
from __future__ import annotations

from contextlib import nullcontext
from typing import Optional

import torch

from ..ops import multi_tensor as mt
from ..ops._native import native, use_native


def autocast_ctx(precision: str, device_type: str = "cuda"):
    if precision == "amp_bf16":
        return torch.autocast(device_type, dtype=torch.bfloat16)
    if precision == "amp_fp16":
        return torch.autocast(device_type, dtype=torch.float16)
    return nullcontext()


class GradScaler:
    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000, enabled: bool = True, device: str = "cuda"):
        self.enabled = enabled
        self.growth_factor = growth_factor
        self.backoff_factor = backoff_factor
        self.growth_interval = growth_interval
        dev = torch.device(device) if torch.cuda.is_available() or device == "cpu" else torch.device("cpu")
        self._scale = torch.full((1,), init_scale, dtype=torch.float32, device=dev)
        self._inv_scale = torch.full((1,), 1.0 / init_scale, dtype=torch.float32, device=dev)
        self._growth_tracker = torch.zeros((1,), dtype=torch.int32, device=dev)
        self._found_inf = torch.zeros((1,), dtype=torch.float32, device=dev)
        self._unscaled = False

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        if not self.enabled:
            return loss
        return loss * self._scale.to(loss.dtype).reshape(())

    def _grads(self, optimizer):
        return [p.grad for g in optimizer.param_groups for p in g["params"] if p.grad is not None]

    def unscale_(self, optimizer) -> None:
        if not self.enabled or self._unscaled:
            return
        torch.reciprocal(self._scale, out=self._inv_scale)
        mt.unscale_(self._grads(optimizer), self._inv_scale, self._found_inf)
        self._unscaled = True

    def step(self, optimizer, *args, **kwargs):
        if not self.enabled:
            return optimizer.step(*args, **kwargs)
        self.unscale_(optimizer)
        if hasattr(optimizer, "_native_step"):  # fused optimizers: skip on device
            return optimizer.step(*args, found_inf=self._found_inf, **kwargs)
        if float(self._found_inf.item()) == 0.0:  # stock optimizers need a host decision
            return optimizer.step(*args, **kwargs)
        return None

    def update(self) -> None:
        if not self.enabled:
            return
        if use_native(self._scale):
            native().amp_update(self._scale, self._growth_tracker, self._found_inf, self.growth_factor,
                                self.backoff_factor, self.growth_interval)
        else:
            if float(self._found_inf.item()) != 0.0:
                self._scale.mul_(self.backoff_factor)
                self._growth_tracker.zero_()
            else:
                self._growth_tracker.add_(1)
                if int(self._growth_tracker.item()) == self.growth_interval:
                    self._scale.mul_(self.growth_factor)
                    self._growth_tracker.zero_()
        self._found_inf.zero_()
        self._unscaled = False

    def get_scale(self) -> float:
        return float(self._scale.item())

    def found_inf(self) -> torch.Tensor:
        return self._found_inf

    def state_dict(self) -> dict:
        return {"scale": self.get_scale(), "growth_factor": self.growth_factor,
                "backoff_factor": self.backoff_factor, "growth_interval": self.growth_interval,
                "_growth_tracker": int(self._growth_tracker.item())}

    def load_state_dict(self, sd: dict) -> None:
        self._scale.fill_(float(sd["scale"]))
        self.growth_factor = float(sd["growth_factor"])
        self.backoff_factor = float(sd["backoff_factor"])
        self.growth_interval = int(sd["growth_interval"])
        self._growth_tracker.fill_(int(sd["_growth_tracker"]))
