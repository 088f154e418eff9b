"""``DistributedSampler``: API- and order-compatible with ``torch.utils.data.DistributedSampler``.

The reference shards by contiguous ``SplitDataset`` partitions (/root/reference/train.py:86-93)
and has no sampler; the north star (BASELINE.json) asks for a DistributedSampler that is
API-compatible. Index order matches torch's exactly (same ``seed + epoch`` generator,
padding by wrap-around, ``rank::num_replicas`` striding) so a job can switch between the
two samplers and resume mid-epoch without changing which samples each rank sees.

Extra over torch: ``set_start_index`` to resume inside an epoch (skip already-consumed
samples after a checkpoint restore).
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch
from torch.utils.data import Sampler

from . import launcher


class DistributedSampler(Sampler[int]):
    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False) -> None:
        if num_replicas is None:
            num_replicas = launcher.get_world_size()
        if rank is None:
            rank = launcher.get_rank()
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if self.drop_last and n % self.num_replicas != 0:
            self.num_samples = math.ceil((n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas
        self.shuffle = shuffle
        self.seed = seed
        self.start_index = 0

    def global_indices(self) -> list[int]:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(n, generator=g).tolist()
        else:
            indices = list(range(n))
        if not self.drop_last:
            padding_size = self.total_size - len(indices)
            if padding_size <= len(indices):
                indices += indices[:padding_size]
            else:
                indices += (indices * math.ceil(padding_size / len(indices)))[:padding_size]
        else:
            indices = indices[: self.total_size]
        assert len(indices) == self.total_size
        return indices

    def __iter__(self) -> Iterator[int]:
        indices = self.global_indices()[self.rank:self.total_size:self.num_replicas]
        assert len(indices) == self.num_samples
        return iter(indices[self.start_index:])

    def __len__(self) -> int:
        return self.num_samples - self.start_index

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
        self.start_index = 0

    def set_start_index(self, start: int) -> None:
        """Resume inside an epoch: skip the first ``start`` samples of this rank's order."""
        self.start_index = max(0, min(int(start), self.num_samples))

    def state_dict(self) -> dict:
        return {"epoch": self.epoch, "start_index": self.start_index, "seed": self.seed}

    def load_state_dict(self, sd: dict) -> None:
        self.epoch = int(sd["epoch"])
        self.seed = int(sd.get("seed", self.seed))
        self.start_index = int(sd.get("start_index", 0))
