"""Distributed runtime: launch/init, DDP reducer, samplers, dataset partitioning."""
from .launcher import (DistContext, barrier, context, destroy, find_free_port, get_rank,
                       get_world_size, init_distributed, spawn)
from .ddp import DistributedDataParallel, GradBucket, unwrap
from .buckets import compute_bucket_assignment, BucketSpec
from .sampler import DistributedSampler
from .split_dataset import SplitDataset, rank_partition
from .reference import average_gradients, broadcast_parameters
from . import comm_hooks

__all__ = [
    "DistContext", "barrier", "context", "destroy", "find_free_port", "get_rank",
    "get_world_size", "init_distributed", "spawn", "DistributedDataParallel", "GradBucket",
    "unwrap", "compute_bucket_assignment", "BucketSpec", "DistributedSampler", "SplitDataset",
    "rank_partition", "average_gradients", "broadcast_parameters", "comm_hooks",
]
