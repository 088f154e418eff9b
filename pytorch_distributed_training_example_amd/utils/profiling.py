"""Tracing/profiling hooks (absent in the reference).

  * ``range(name)`` — a roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm builds) so
    rocprofv3 ``--marker-trace`` / ``--kernel-trace`` timelines show fwd / bwd / comm / optim;
  * ``torch_profiler(...)`` — torch.profiler with a schedule, exporting a Chrome trace;
  * ``summarize_kernel_stats(csv)`` — top-N kernels from a rocprofv3 ``*_kernel_stats.csv``
    (used to produce the committed summaries under ``profiles/``).
"""
from __future__ import annotations

import contextlib
import csv
import os
from typing import Iterator, Optional

import torch


_RANGES = [os.environ.get("PDT_ROCTX", "0") == "1"]


def enable_ranges(on: bool = True) -> None:
    """Turn the step-phase roctx ranges (forward / backward / optimizer) on or off."""
    _RANGES[0] = on


@contextlib.contextmanager
def range(name: str) -> Iterator[None]:  # noqa: A001 - mirrors nvtx.range
    if _RANGES[0] and torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


def torch_profiler(out_dir: str, wait: int = 1, warmup: int = 1, active: int = 3):
    from torch.profiler import ProfilerActivity, profile, schedule, tensorboard_trace_handler
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    os.makedirs(out_dir, exist_ok=True)
    return profile(activities=acts, schedule=schedule(wait=wait, warmup=warmup, active=active),
                   on_trace_ready=tensorboard_trace_handler(out_dir), record_shapes=True)


def summarize_kernel_stats(path: str, top: int = 30, total_steps: Optional[int] = None) -> str:
    """Markdown table of the top kernels by total time from a rocprofv3 kernel_stats.csv."""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    tot = sum(float(r.get("TotalDurationNs", 0)) for r in rows) or 1.0
    rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0)))
    lines = ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:top]:
        t = float(r["TotalDurationNs"])
        name = r["Name"][:90].replace("|", "/")
        lines.append(f"| `{name}` | {r['Calls']} | {t / 1e6:.2f} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{100 * t / tot:.1f} |")
    lines.append(f"\nTotal GPU kernel time: {tot / 1e6:.1f} ms over {len(rows)} distinct kernels"
                 + (f" ({tot / 1e6 / total_steps:.2f} ms/step)" if total_steps else ""))
    return "\n".join(lines)
