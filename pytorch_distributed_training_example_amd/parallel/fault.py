"""Failure injection and elastic-restart support (absent in the reference).

The reference's ``spawn(join=True)`` turns a child exception into ``ProcessExitedException``
and kills the siblings; there is no timeout, restart or resume (/root/reference/train.py:147).
Here:
  * ``FaultInjector`` — kills (``os._exit``) or raises on a chosen rank at a chosen step,
    configured by ``PDT_FAULT="rank:step[:mode]"``; used by the CPU/gloo resume test;
  * ``restart_count()`` — torchrun's ``TORCHELASTIC_RESTART_COUNT`` so a restarted job knows
    to resume from the last checkpoint;
  * the launcher sets a bounded process-group timeout so a dead peer surfaces as an error
    instead of a hang (launcher.init_distributed(timeout_s=...)).
"""
from __future__ import annotations

import os
from typing import Optional


class InjectedFault(RuntimeError):
    pass


class FaultInjector:
    def __init__(self, spec: Optional[str] = None, rank: int = 0):
        spec = spec if spec is not None else os.environ.get("PDT_FAULT", "")
        self.rank = rank
        self.target_rank: Optional[int] = None
        self.step: Optional[int] = None
        self.mode = "exit"
        if spec:
            parts = spec.split(":")
            self.target_rank, self.step = int(parts[0]), int(parts[1])
            if len(parts) > 2:
                self.mode = parts[2]
        # only fire on the first attempt of an elastic job
        if restart_count() > 0 and os.environ.get("PDT_FAULT_EVERY_RESTART", "0") != "1":
            self.target_rank = None

    def maybe_fail(self, step: int) -> None:
        if self.target_rank is None or self.rank != self.target_rank or step != self.step:
            return
        if self.mode == "raise":
            raise InjectedFault(f"injected fault on rank {self.rank} at step {step}")
        os._exit(17)


def restart_count() -> int:
    return int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
