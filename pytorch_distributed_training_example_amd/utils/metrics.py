"""Observability: rank-aware logging, JSONL metrics, HIP-event step timers, throughput meter.

The reference only ``print``s on rank 0 (/root/reference/train.py:52-55,73-76). Here rank 0 also
writes structured JSONL records (loss, lr, throughput, step time, comm time, loss scale), and
``StepTimer`` measures device time per step with HIP events (no host sync until ``read``).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from typing import Optional

import torch


def get_logger(name: str = "pdt", rank: Optional[int] = None, level=logging.INFO) -> logging.Logger:
    from ..parallel import launcher
    rank = launcher.get_rank() if rank is None else rank
    log = logging.getLogger(f"{name}.r{rank}")
    if not log.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter(f"[%(asctime)s r{rank}] %(levelname)s %(message)s", "%H:%M:%S"))
        log.addHandler(h)
    log.setLevel(level if rank == 0 else max(level, logging.WARNING))
    return log


class MetricsWriter:
    """Append-only JSONL on rank 0 (no-op elsewhere)."""

    def __init__(self, path: Optional[str], rank: int = 0):
        self.path = path if (path and rank == 0) else None
        self._f = None
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            self._f = open(self.path, "a", buffering=1)

    def log(self, rec: dict) -> None:
        if self._f is None:
            return
        rec = dict(rec)
        rec.setdefault("time", time.time())
        self._f.write(json.dumps(rec) + "\n")

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None


class StepTimer:
    """Device-side step timing with HIP events; host reads once at the end."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._events = []

    def mark(self) -> None:
        if self.enabled:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events.append(e)

    def read_ms(self) -> list:
        if not self.enabled or len(self._events) < 2:
            return []
        self._events[-1].synchronize()
        return [a.elapsed_time(b) for a, b in zip(self._events[:-1], self._events[1:])]

    def reset(self) -> None:
        self._events = []


class Throughput:
    def __init__(self):
        self.samples = 0
        self.t0 = time.perf_counter()

    def add(self, n: int) -> None:
        self.samples += n

    def rate(self) -> float:
        return self.samples / max(time.perf_counter() - self.t0, 1e-9)
