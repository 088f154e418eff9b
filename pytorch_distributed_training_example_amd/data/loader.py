"""Loaders.

Reference: per rank ``DataLoader(batch_size=ceil(B/world), num_workers=4, pin_memory=True,
shuffle=True)`` over a ``SplitDataset`` shard, with a synchronous ``.cuda()`` copy per batch
(/root/reference/train.py:82-83,95-96,45).

MI355X-first replacements:
  * ``ResidentLoader`` — a dataset that fits in HBM (MNIST: 188 MB fp32 vs 288 GB per GPU)
    is copied to the device ONCE; each epoch shuffles indices on the device and batches are
    gathered on the device: no worker processes, no per-step H2D copy, no host sync.
  * ``PrefetchLoader`` — for datasets that do not fit, wraps a ``DataLoader`` (pinned memory)
    and issues the H2D copy of batch i+1 on a side HIP stream while batch i computes.
  * ``SyntheticBatches`` — device-generated batches of a fixed shape (benchmarks).
"""
from __future__ import annotations

import math
from typing import Iterator, Optional, Sequence, Tuple

import torch
from torch.utils.data import DataLoader, Dataset


class ResidentLoader:
    """Whole (x, y) shard resident on ``device``; shuffled per epoch on device."""

    def __init__(self, x: torch.Tensor, y: torch.Tensor, batch_size: int, device, shuffle: bool = True,
                 drop_last: bool = False, seed: int = 0, dtype: Optional[torch.dtype] = None,
                 channels_last: bool = False):
        self.x = x.to(device, non_blocking=False)
        if dtype is not None:
            self.x = self.x.to(dtype)
        if channels_last and self.x.dim() == 4:
            self.x = self.x.contiguous(memory_format=torch.channels_last)
        self.y = y.to(device)
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.device = torch.device(device)
        self.seed = seed
        self.epoch = 0
        self.dataset = _LenOnly(self.x.shape[0])

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __len__(self) -> int:
        n = self.x.shape[0]
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        n = self.x.shape[0]
        if self.shuffle:
            g = torch.Generator(device=self.device)
            g.manual_seed(self.seed + self.epoch)
            perm = torch.randperm(n, device=self.device, generator=g)
        else:
            perm = None
        self.epoch += 1
        for i in range(len(self)):
            s = i * self.batch_size
            e = min(n, s + self.batch_size)
            if perm is None:
                yield self.x[s:e], self.y[s:e]
            else:
                idx = perm[s:e]
                yield self.x.index_select(0, idx), self.y.index_select(0, idx)


class _LenOnly:
    def __init__(self, n: int):
        self.n = n

    def __len__(self) -> int:
        return self.n


class PrefetchLoader:
    """Overlap the H2D copy of the next batch with compute (side stream + events)."""

    def __init__(self, loader: DataLoader, device, channels_last: bool = False,
                 dtype: Optional[torch.dtype] = None):
        self.loader = loader
        self.device = torch.device(device)
        self.channels_last = channels_last
        self.dtype = dtype
        self.dataset = loader.dataset

    def __len__(self) -> int:
        return len(self.loader)

    def _to(self, batch):
        x, y = batch
        x = x.to(self.device, non_blocking=True)
        if self.dtype is not None:
            x = x.to(self.dtype)
        if self.channels_last and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
        return x, y.to(self.device, non_blocking=True)

    def __iter__(self):
        if self.device.type != "cuda":
            for b in self.loader:
                yield self._to(b)
            return
        stream = torch.cuda.Stream(device=self.device)
        nxt = None
        for b in self.loader:
            with torch.cuda.stream(stream):
                cur = self._to(b)
            if nxt is not None:
                yield nxt
            torch.cuda.current_stream().wait_stream(stream)
            for t in cur:
                t.record_stream(torch.cuda.current_stream())
            nxt = cur
        if nxt is not None:
            yield nxt


class SyntheticBatches:
    """Fixed-shape random batches generated on the device (benchmark input)."""

    def __init__(self, shape: Sequence[int], num_classes: int, steps: int, device, dtype=torch.float32,
                 channels_last: bool = False, seed: int = 0, pool: int = 2, int_inputs: bool = False):
        g = torch.Generator(device=device).manual_seed(seed)
        self.steps = steps
        self.pool = []
        for _ in range(pool):
            if int_inputs:
                x = torch.randint(0, num_classes, tuple(shape), device=device, generator=g)
                y = torch.randint(0, num_classes, tuple(shape), device=device, generator=g)
            else:
                x = torch.randn(*shape, device=device, generator=g).to(dtype)
                if channels_last and x.dim() == 4:
                    x = x.contiguous(memory_format=torch.channels_last)
                y = torch.randint(0, num_classes, (shape[0],), device=device, generator=g)
            self.pool.append((x, y))
        self.dataset = _LenOnly(steps * shape[0])

    def __len__(self) -> int:
        return self.steps

    def __iter__(self):
        for i in range(self.steps):
            yield self.pool[i % len(self.pool)]


def reference_loader(dataset: Dataset, batch_size: int, shuffle: bool = True, num_workers: int = 4,
                     pin_memory: bool = True, sampler=None) -> DataLoader:
    """The reference's DataLoader configuration (train.py:83)."""
    return DataLoader(dataset, batch_size=batch_size, shuffle=shuffle if sampler is None else False,
                      num_workers=num_workers, pin_memory=pin_memory, sampler=sampler,
                      persistent_workers=num_workers > 0)
