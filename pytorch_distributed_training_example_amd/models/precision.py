"""Model precision policies.

``bf16_mixed``: every parameter and floating buffer in bf16 EXCEPT normalisation layers
(BatchNorm / LayerNorm weights, biases and running statistics stay fp32, which the fused
norm kernels consume directly). The fused optimizers keep an fp32 master copy of each bf16
parameter and write the bf16 copy in the update kernel, so the forward pass needs no
per-step weight casts (what autocast would add) and DDP reduces half the bytes.
"""
from __future__ import annotations

import torch
from torch import nn

NORM_TYPES = (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d, nn.LayerNorm, nn.GroupNorm)


def to_bf16_mixed(model: nn.Module) -> nn.Module:
    for mod in model.modules():
        if isinstance(mod, NORM_TYPES):
            continue
        for name, p in list(mod.named_parameters(recurse=False)):
            if p.is_floating_point():
                p.data = p.data.to(torch.bfloat16)
        for name, b in list(mod.named_buffers(recurse=False)):
            if b is not None and b.is_floating_point():
                setattr(mod, name, b.to(torch.bfloat16))
    return model


def apply_precision(model: nn.Module, precision: str) -> nn.Module:
    if precision in ("fp32", "amp_bf16", "amp_fp16"):
        return model
    if precision == "bf16":
        return to_bf16_mixed(model)
    if precision == "fp8":
        # bf16 params + fp32 master weights, and every transformer-block GEMM on OCP e4m3 operands
        # with delayed per-tensor scaling (ops/fp8.py)
        from ..ops.fp8 import enable_fp8
        model = to_bf16_mixed(model)
        enable_fp8(model)
        return model
    raise ValueError(f"unknown precision {precision}")
