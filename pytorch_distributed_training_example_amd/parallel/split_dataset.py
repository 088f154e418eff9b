"""Contiguous dataset partitioning (``SplitDataset``), bug-fixed.

Parity target: /root/reference/splitdataset.py:5-87 (vendored from torchnet). Same API:
``SplitDataset(dataset, partitions, initial_partition=None)``, ``.select(name)``,
``__len__``, ``__getitem__`` and the same contiguous, unshuffled layout with partition
names sorted lexicographically (splitdataset.py:44-46).

Fixes (each one a reference defect):
  * ``len(partitions) == 1`` is allowed (reference asserts >= 2, splitdataset.py:38) so a
    single-GPU run works.
  * Fractional weights are detected by ``sum <= 1 + 1e-9`` instead of ``<= 1`` — for 9 or
    11 ranks ``sum([1/n]*n) == 1.0000000000000002`` and the reference falls into the
    integer branch and asserts (splitdataset.py:51-57).
  * Fractional sizes use largest-remainder apportionment, so sizes always sum to at most
    ``len(dataset)`` (reference ``round()`` reads past the end for 6/7/14 ranks).
  * ``natural_order=True`` sorts ``'2' < '10'`` (reference sorts lexicographically, which
    permutes shards for >= 11 ranks; kept as default for parity).
"""
from __future__ import annotations

import math
import re
from typing import Dict, Optional

import numpy as np
from torch.utils.data import Dataset


def _natural_key(s: str):
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", s)]


def apportion(weights, total: int) -> list[int]:
    """Largest-remainder apportionment of ``total`` items to fractional ``weights``.

    If ``sum(weights) < 1`` the remainder is left unassigned (reference semantics: the
    partitions cover only the requested fraction of the dataset).
    """
    w = [float(x) for x in weights]
    s = sum(w)
    target = int(math.floor(min(s, 1.0) * total + 1e-9)) if s < 1.0 - 1e-9 else total
    raw = [x * total / max(s, 1.0) for x in w] if s > 1.0 else [x * total for x in w]
    base = [int(math.floor(r + 1e-9)) for r in raw]
    rem = target - sum(base)
    order = sorted(range(len(w)), key=lambda i: (-(raw[i] - base[i]), i))
    for i in order[: max(rem, 0)]:
        base[i] += 1
    return base


class SplitDataset(Dataset):
    """Partition ``dataset`` into named contiguous partitions; ``select`` one."""

    def __init__(self, dataset, partitions: Dict[str, float], initial_partition: Optional[str] = None,
                 natural_order: bool = False):
        super().__init__()
        if not isinstance(partitions, dict):
            raise TypeError("partitions must be a dict")
        if len(partitions) < 1:
            raise ValueError("SplitDataset needs at least one partition")
        if min(partitions.values()) < 0:
            raise ValueError("partition sizes cannot be negative")
        if max(partitions.values()) <= 0:
            raise ValueError("all partitions cannot be empty")
        self.dataset = dataset
        self.partitions = partitions
        key = _natural_key if natural_order else None
        self.partition_names = sorted(partitions.keys(), key=key)
        self.partition_index = {p: i for i, p in enumerate(self.partition_names)}
        sizes = [partitions[p] for p in self.partition_names]
        if sum(sizes) <= 1.0 + 1e-9:
            sizes = apportion(sizes, len(dataset))
        else:
            for x in sizes:
                if x != int(x):
                    raise ValueError("partition sizes should be integer numbers, or sum up to <= 1")
            sizes = [int(x) for x in sizes]
            if sum(sizes) > len(dataset):
                raise ValueError(f"partition sizes sum to {sum(sizes)} > len(dataset)={len(dataset)}")
        self.partition_sizes = sizes
        self.partition_cum_sizes = np.cumsum(sizes)
        self.current_partition_idx: Optional[int] = None
        if initial_partition is not None:
            self.select(initial_partition)

    def select(self, partition: str) -> None:
        self.current_partition_idx = self.partition_index[partition]

    def _check(self) -> int:
        if self.current_partition_idx is None:
            raise ValueError("Select a partition before accessing data.")
        return self.current_partition_idx

    def offset(self) -> int:
        p = self._check()
        return 0 if p == 0 else int(self.partition_cum_sizes[p - 1])

    def __len__(self) -> int:
        return self.partition_sizes[self._check()]

    def __getitem__(self, idx: int):
        n = len(self)
        if idx < 0:
            idx += n
        if not 0 <= idx < n:
            raise IndexError(idx)
        return self.dataset[self.offset() + idx]


def rank_partition(dataset, rank: int, world_size: int, natural_order: bool = True) -> SplitDataset:
    """The reference's per-rank sharding (train.py:86-93) as one call."""
    parts = {str(i): 1.0 / world_size for i in range(world_size)}
    ds = SplitDataset(dataset, parts, natural_order=natural_order)
    ds.select(str(rank))
    return ds
