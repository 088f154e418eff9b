"""DDP communication hooks (``hook(state, bucket) -> Future[Tensor]``).

Same contract as ``torch.distributed.algorithms.ddp_comm_hooks``; used with
``DistributedDataParallel.register_comm_hook``. Not present in the reference (which has a
single hard-coded per-parameter all-reduce, /root/reference/train.py:34-39).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _avg_allreduce_fut(tensor: torch.Tensor, group=None):
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        return dist.all_reduce(tensor, op=dist.ReduceOp.AVG, group=group, async_op=True).get_future()
    work = dist.all_reduce(tensor, op=dist.ReduceOp.SUM, group=group, async_op=True)
    fut = work.get_future()
    return fut.then(lambda f: [f.value()[0].div_(world)])


def allreduce_hook(process_group, bucket):
    """Plain averaged all-reduce of the whole bucket."""
    return _avg_allreduce_fut(bucket.buffer(), process_group)


def _compress_hook(dtype):
    def hook(process_group, bucket):
        buf = bucket.buffer()
        compressed = buf.to(dtype)
        fut = _avg_allreduce_fut(compressed, process_group)

        def decompress(f):
            out = f.value()
            out = out[0] if isinstance(out, (list, tuple)) else out
            buf.copy_(out)
            return buf
        return fut.then(decompress)
    return hook


bf16_compress_hook = _compress_hook(torch.bfloat16)
fp16_compress_hook = _compress_hook(torch.float16)


def noop_hook(process_group, bucket):
    """No communication (for measuring compute-only step time)."""
    fut = torch.futures.Future()
    fut.set_result(bucket.buffer())
    return fut
