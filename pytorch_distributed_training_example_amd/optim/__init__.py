"""Fused multi-tensor optimizers and LR schedules."""
from .fused import FusedAdadelta, FusedAdam, FusedAdamW, FusedSGD, build_optimizer
from .schedules import build_scheduler, warmup_cosine

__all__ = ["FusedAdadelta", "FusedAdam", "FusedAdamW", "FusedSGD", "build_optimizer", "build_scheduler",
           "warmup_cosine"]
