"""Race / desync detection for data parallelism (absent in the reference).

The reference keeps replicas identical only by giving every rank the same seed
(/root/reference/train.py:80-81) and averages with unchecked per-parameter all-reduces
(train.py:34-39). Nothing detects a rank that diverged or issued a different collective.

  * ``replica_fingerprint`` / ``check_replicas_in_sync`` — all-gather a cheap fingerprint
    (fp64 sum and sum of squares per tensor, one collective) of parameters or gradients and
    raise if any rank disagrees (``cli.py --check-sync``);
  * ``ReducerDebug`` — the DDP reducer's debug mode (``PDT_DDP_DEBUG=1`` or
    ``DistributedDataParallel(debug=True)``, parallel/ddp.py). Per backward it
      1. logs every bucket collective in a ``CollectiveLog`` and compares the logs across ranks
         (names the first differing collective: the classic hang / mismatch cause);
      2. asserts stream safety before the optimizer may read the bucket views: the compute
         stream's position after the reducer's waits is synchronised and every collective must
         then report completion (``assert_collective_done``) — a missing or misplaced
         stream-ordered wait fails here instead of letting the optimizer read a half-reduced bucket;
      3. all-gathers a per-bucket checksum of the reduced buffers and raises naming the first
         bucket (and its parameters) that differs between ranks (``check_bucket_checksums``).
    Every check synchronises the host: debug mode is for finding bugs, not for timing.
"""
from __future__ import annotations

import hashlib
from typing import Any, Iterable, List, Optional, Sequence

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


def _first_mismatch(fps: Sequence[torch.Tensor], rtol: float) -> Optional[tuple]:
    """(rank, tensor index, ref value, value) of the first fingerprint entry that differs from rank 0's."""
    ref = fps[0]
    for r, o in enumerate(fps[1:], 1):
        bad = ((o - ref).abs() > rtol * ref.abs()).nonzero()
        if bad.numel():
            e = int(bad[0, 0])
            return r, e // 2, ref[e].item(), o[e].item()
    return None


def _gather(t: torch.Tensor, group) -> List[torch.Tensor]:
    out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return out


def check_replicas_in_sync(tensors: List[torch.Tensor], what: str = "parameters", rtol: float = 0.0,
                           group=None) -> None:
    """Raise RuntimeError naming the first tensor index whose fingerprint differs across ranks."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    bad = _first_mismatch(_gather(replica_fingerprint(list(tensors)), group), rtol)
    if bad is not None:
        r, i, a, b = bad
        raise RuntimeError(f"replica desync: {what}[{i}] differs between rank 0 and rank {r} "
                           f"(fingerprint {a:.6g} vs {b:.6g})")


class CollectiveLog:
    """Per-rank record of issued collectives, comparable across ranks."""

    def __init__(self):
        self.entries: List[str] = []

    def record(self, op: str, t: Optional[torch.Tensor] = None) -> None:
        self.entries.append(f"{op}:{tuple(t.shape) if t is not None else ()}:{t.dtype if t is not None else ''}")

    def clear(self) -> None:
        self.entries = []

    def digest(self) -> str:
        return hashlib.sha1("\n".join(self.entries).encode()).hexdigest()

    def check(self, group=None) -> None:
        """Raise naming the first entry where any rank's log differs from rank 0's."""
        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return
        objs: List[Optional[object]] = [None] * dist.get_world_size(group)
        dist.all_gather_object(objs, (self.digest(), self.entries), group=group)
        base = objs[0][1]
        for r, o in enumerate(objs):
            if o[0] == objs[0][0]:
                continue
            ent = o[1]
            i = next((k for k, (a, b) in enumerate(zip(base, ent)) if a != b), min(len(base), len(ent)))
            a = base[i] if i < len(base) else "<none>"
            b = ent[i] if i < len(ent) else "<none>"
            raise RuntimeError(f"collective sequence mismatch rank 0 vs rank {r} at collective #{i}: "
                               f"{a!r} vs {b!r} (counts {len(base)} vs {len(ent)})")


def assert_collective_done(works: Sequence[Any], what: str = "bucket") -> None:
    """Stream-safety assert: the current stream has reached this point (synchronised by an event on
    it), so every collective it is ordered after must be complete. A collective that is still running
    means the consumer (optimizer / unpack) is NOT ordered after it: a race."""
    if torch.cuda.is_available() and torch.cuda.is_initialized() and not torch.cuda.is_current_stream_capturing():
        ev = torch.cuda.Event()
        ev.record()
        ev.synchronize()
    for i, w in works:
        if w is None:
            continue
        done = w.is_completed() if hasattr(w, "is_completed") else w.done()
        if not done:
            raise RuntimeError(f"stream-safety violation: {what} {i}'s collective is not complete when the "
                               f"compute stream reaches the optimizer (missing stream-ordered wait)")


def bucket_checksums(buffers: Sequence[torch.Tensor]) -> torch.Tensor:
    """[2 * n] fp64 (sum, sum of squares) of every bucket buffer."""
    return replica_fingerprint(buffers)


def check_bucket_checksums(buffers: Sequence[torch.Tensor], names: Sequence[Sequence[str]], group=None,
                           step: Optional[int] = None) -> None:
    """All-gather the per-bucket checksums of the REDUCED buffers (identical on every rank after an
    all-reduce) and raise naming the first bucket that differs, with the parameters it holds."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    bad = _first_mismatch(_gather(bucket_checksums(buffers), group), 0.0)
    if bad is not None:
        r, b, x, y = bad
        ps = ", ".join(list(names[b])[:4]) + (", ..." if len(names[b]) > 4 else "")
        at = f" at step {step}" if step is not None else ""
        raise RuntimeError(f"gradient desync{at}: bucket {b} ({ps}) differs between rank 0 and rank {r} "
                           f"after the all-reduce (checksum {x:.9g} vs {y:.9g})")


class ReducerDebug:
    """The DDP reducer's per-backward debug checks (see the module docstring)."""

    def __init__(self, group=None):
        self.group = group
        self.log = CollectiveLog()
        self.step = 0

    def on_launch(self, index: int, buffer: torch.Tensor, op: str = "all_reduce") -> None:
        self.log.record(f"{op}[bucket {index}]", buffer)

    def after_backward(self, works: Sequence[Any], buffers: Sequence[torch.Tensor],
                       names: Sequence[Sequence[str]]) -> None:
        assert_collective_done(works)
        self.log.check(self.group)
        check_bucket_checksums(buffers, names, self.group, self.step)
        self.log.clear()
        self.step += 1
