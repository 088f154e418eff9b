"""Gradient bucket assignment.

The reference issues one blocking all-reduce per parameter after backward
(/root/reference/train.py:34-39: 10 un-bucketed fp32 collectives per LeNet step). Here
gradients are packed into flat buckets so the collective count per step is
``ceil(bytes / cap)`` and each bucket can be reduced as soon as its last gradient is
produced, overlapping backward.

Assignment rules (compatible with torch DDP's so bucket boundaries line up):
  * parameters are visited in *reverse* registration order (≈ the order backward
    produces their gradients);
  * a bucket holds a single (dtype, device);
  * the first bucket is capped at ``first_bucket_bytes`` (small, so the first
    collective starts early), the rest at ``bucket_cap_bytes``;
  * buckets are ordered by the position at which they FILL (their last member in the
    ready order), i.e. the order the reducer can launch them. Sorting by the *first*
    member instead lets a small bucket of another dtype that opens early but fills last
    (the fp32 norm parameters of a bf16-mixed model: ResNet-50's BN bucket fills at
    position 159 of 161, GPT-2's LayerNorm bucket at 289 of 292) sit in front of every
    bf16 bucket; launches are strictly in bucket order (ranks must agree), so it would
    hold all of them until the end of backward. torch's reducer likewise keeps buckets
    in fill order after its rebuild.

MI355X sizing note: ring all-reduce over xGMI is bound by one ≈153 GB/s link per ring;
RCCL runs several rings to use the 7 links. A 25 MiB bucket costs ≈0.04–0.3 ms at n=8
(SURVEY.md §5.1), i.e. well under one layer's backward for ResNet-50 at batch 256, so
mid-backward buckets can be large. What is NOT hidden is the bucket that fills last: its
collective starts when backward's compute ends. ``plan_auto`` (``bucket_cap_mb="auto"``) is
a comm-model plan built backwards from the end of backward: the last-filling bucket is capped at
``tail_bytes`` (2 MiB: α-dominated, ≈15 µs of wire time on one xGMI link at n = 8), the one
before at ``growth`` × that, and so on up to the 25 MiB cap, so each bucket's all-reduce is
no longer than the (growing) stretch of backward compute still ahead of it. The sweep tool
(tools/bucket_sweep.py) tunes the fixed caps per model.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import torch

DEFAULT_FIRST_BUCKET_BYTES = 1 * 1024 * 1024
DEFAULT_BUCKET_CAP_MB = 25.0
AUTO_TAIL_BYTES = 2 * 1024 * 1024
AUTO_GROWTH = 4


@dataclass
class BucketSpec:
    indices: List[int]                 # parameter indices (registration order numbering)
    dtype: torch.dtype
    device: torch.device
    offsets: List[int] = field(default_factory=list)
    numels: List[int] = field(default_factory=list)
    total: int = 0

    @property
    def nbytes(self) -> int:
        return self.total * torch.empty((), dtype=self.dtype).element_size()


def _align(n: int, a: int) -> int:
    return (n + a - 1) // a * a


def compute_bucket_assignment(
    params: Sequence[torch.Tensor],
    bucket_cap_bytes: int,
    first_bucket_bytes: int = DEFAULT_FIRST_BUCKET_BYTES,
    order: Sequence[int] | None = None,
    align_elems: int = 8,
) -> List[BucketSpec]:
    """Assign ``params`` to buckets.

    ``order``: the order gradients are expected to become ready (defaults to reverse
    registration order). ``align_elems``: every parameter slot starts at a multiple of
    this many elements so the HIP kernels can use 16-byte vector accesses per slot.
    """
    n = len(params)
    if order is None:
        order = list(range(n - 1, -1, -1))
    pos = {idx: i for i, idx in enumerate(order)}
    open_buckets: Dict[Tuple[torch.dtype, torch.device], Tuple[List[int], int]] = {}
    limits_used: Dict[Tuple[torch.dtype, torch.device], int] = {}
    done: List[Tuple[List[int], torch.dtype, torch.device]] = []
    for idx in order:
        p = params[idx]
        key = (p.dtype, p.device)
        members, size = open_buckets.get(key, ([], 0))
        members.append(idx)
        size += p.numel() * p.element_size()
        limit = first_bucket_bytes if limits_used.get(key, 0) == 0 else bucket_cap_bytes
        if size >= limit:
            done.append((members, p.dtype, p.device))
            limits_used[key] = limits_used.get(key, 0) + 1
            open_buckets.pop(key, None)
        else:
            open_buckets[key] = (members, size)
    for key, (members, _) in open_buckets.items():
        if members:
            done.append((members, key[0], key[1]))
    done.sort(key=lambda b: (max(pos[i] for i in b[0]), min(pos[i] for i in b[0])))
    specs: List[BucketSpec] = []
    for members, dtype, device in done:
        spec = BucketSpec(indices=list(members), dtype=dtype, device=device)
        off = 0
        for i in members:
            spec.offsets.append(off)
            spec.numels.append(params[i].numel())
            off = _align(off + params[i].numel(), align_elems)
        spec.total = max(off, 1)
        specs.append(spec)
    return specs


def plan_auto(
    params: Sequence[torch.Tensor],
    bucket_cap_bytes: int = int(DEFAULT_BUCKET_CAP_MB * 1024 * 1024),
    tail_bytes: int = AUTO_TAIL_BYTES,
    growth: int = AUTO_GROWTH,
    order: Sequence[int] | None = None,
    align_elems: int = 8,
) -> List[BucketSpec]:
    """The comm-model bucket plan (module docstring): walk the ready order BACKWARDS per
    (dtype, device); the first bucket met (the one that fills last) is capped at ``tail_bytes``,
    each earlier one at ``growth`` × the previous cap, up to ``bucket_cap_bytes``. A single
    parameter larger than its cap gets a bucket of its own. Buckets are returned in fill order."""
    n = len(params)
    if order is None:
        order = list(range(n - 1, -1, -1))
    pos = {idx: i for i, idx in enumerate(order)}
    cur: Dict[Tuple[torch.dtype, torch.device], Tuple[List[int], int]] = {}
    cap: Dict[Tuple[torch.dtype, torch.device], int] = {}
    done: List[Tuple[List[int], torch.dtype, torch.device]] = []
    for idx in reversed(list(order)):
        p = params[idx]
        key = (p.dtype, p.device)
        nb = p.numel() * p.element_size()
        members, size = cur.get(key, ([], 0))
        limit = cap.setdefault(key, min(tail_bytes, bucket_cap_bytes))
        if members and size + nb > limit:  # close it: the next (earlier-filling) bucket may be larger
            done.append((members, key[0], key[1]))
            cap[key] = min(limit * growth, bucket_cap_bytes)
            members, size = [], 0
        members.append(idx)
        cur[key] = (members, size + nb)
    for key, (members, _) in cur.items():
        if members:
            done.append((members, key[0], key[1]))
    specs: List[BucketSpec] = []
    for members, dtype, device in sorted(done, key=lambda b: (max(pos[i] for i in b[0]),
                                                              min(pos[i] for i in b[0]))):
        members = sorted(members, key=lambda i: pos[i])  # slots in ready order, as the greedy plan
        spec = BucketSpec(indices=members, dtype=dtype, device=device)
        off = 0
        for i in members:
            spec.offsets.append(off)
            spec.numels.append(params[i].numel())
            off = _align(off + params[i].numel(), align_elems)
        spec.total = max(off, 1)
        specs.append(spec)
    return specs
