"""Race / desync detection for data parallelism (absent in the reference).

  * ``replica_fingerprint`` / ``check_replicas_in_sync`` — all-gather a cheap fingerprint
    (fp64 sum and sum of squares per tensor, one collective) of parameters or gradients and
    raise if any rank disagrees: catches replicas that silently diverged (e.g. the
    reference's reliance on equal seeds, train.py:80-81) or a broken reduction;
  * ``CollectiveLog`` — records the sequence of (op, shape, dtype) a rank issues; comparing
    the per-rank logs pinpoints the first mismatching collective (the classic hang cause);
  * ``stream_check`` — asserts a tensor produced on a side stream has been waited on by the
    current stream (debug mode for the overlap logic).
"""
from __future__ import annotations

import hashlib
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist


def replica_fingerprint(tensors: Iterable[torch.Tensor]) -> torch.Tensor:
    """[2 * n] fp64: (sum, sum of squares) of every tensor (zeros for None)."""
    tensors = list(tensors)
    dev = next((t.device for t in tensors if t is not None), torch.device("cpu"))
    out = torch.zeros(2 * len(tensors), dtype=torch.float64, device=dev)
    for i, t in enumerate(tensors):
        if t is None:
            continue
        d = t.detach().double()
        out[2 * i] = d.sum()
        out[2 * i + 1] = (d * d).sum()
    return out


def check_replicas_in_sync(tensors: List[torch.Tensor], what: str = "parameters", rtol: float = 0.0,
                           group=None) -> None:
    """Raise RuntimeError naming the first tensor index whose fingerprint differs across ranks."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    fp = replica_fingerprint(list(tensors))
    world = dist.get_world_size(group)
    out = [torch.empty_like(fp) for _ in range(world)]
    dist.all_gather(out, fp, group=group)
    ref = out[0]
    for r, o in enumerate(out[1:], 1):
        diff = (o - ref).abs()
        tol = rtol * ref.abs()
        bad = (diff > tol).nonzero()
        if bad.numel():
            i = int(bad[0, 0]) // 2
            raise RuntimeError(f"replica desync: {what}[{i}] differs between rank 0 and rank {r} "
                               f"(fingerprint {ref[2 * i].item():.6g} vs {o[2 * i].item():.6g})")


class CollectiveLog:
    """Per-rank record of issued collectives, comparable across ranks."""

    def __init__(self):
        self.entries: List[str] = []

    def record(self, op: str, t: Optional[torch.Tensor] = None) -> None:
        self.entries.append(f"{op}:{tuple(t.shape) if t is not None else ()}:{t.dtype if t is not None else ''}")

    def digest(self) -> str:
        return hashlib.sha1("\n".join(self.entries).encode()).hexdigest()

    def check(self, group=None) -> None:
        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return
        objs: List[Optional[object]] = [None] * dist.get_world_size(group)
        dist.all_gather_object(objs, (self.digest(), len(self.entries), self.entries[-50:]), group=group)
        base = objs[0]
        for r, o in enumerate(objs):
            if o[0] != base[0]:
                first = next((i for i, (a, b) in enumerate(zip(base[2], o[2])) if a != b), None)
                raise RuntimeError(f"collective sequence mismatch rank0 vs rank{r}: counts {base[1]} vs {o[1]}, "
                                   f"first differing recent entry: {first}")


def stream_check(t: torch.Tensor, producer: "torch.cuda.Stream") -> None:
    """Make the current stream wait on ``producer`` and remember the use (record_stream)."""
    if t.is_cuda:
        cur = torch.cuda.current_stream(t.device)
        if producer != cur:
            cur.wait_stream(producer)
            t.record_stream(cur)
