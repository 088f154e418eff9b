"""Intra-node P2P all-reduce over xGMI and a DDP comm hook that uses it for
small buckets.

The reference reduces 10 tiny fp32 tensors per step with one NCCL call each
(/root/reference/train.py:34-39, 247 KB in total): pure collective latency. On an 8-GPU MI355X
node every GPU has a direct xGMI link to every other one, so a small bucket is reduced fastest
by letting each GPU read all 7 peers' copies at once (one-shot) instead of walking a ring:

  * ``P2PAllReduce(group)`` allocates an uncached IPC-exportable staging + flag region per rank
    (csrc/kernels/p2p.hip, C++ ``P2PComm``), exchanges the ``hipIpcMemHandle``s through the
    process group (``all_gather_object``), maps every peer's region, and then all-reduces with
    ONE kernel on the caller's stream — no host involvement, no RCCL channels;
  * every rank sums the peers in rank order with fp32 accumulation: bit-identical replicas;
  * ``p2p_allreduce_hook`` (``DistributedDataParallel.register_comm_hook``) sends buckets up to
    ``max_bytes`` through it on a side HIP stream (overlapping backward like RCCL does) and
    larger ones through RCCL (``ReduceOp.AVG``).

All ranks of the group must be on one node (IPC). Ranks may share a GPU (tests do this).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..ops._native import native


class P2PAllReduce:
    def __init__(self, group=None, capacity_bytes: int = 8 << 20, max_blocks: int = 64,
                 device: Optional[torch.device] = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.comm = native().P2PComm(self.rank, self.world, int(capacity_bytes), int(max_blocks), dev.index)
        blobs = [None] * self.world
        dist.all_gather_object(blobs, self.comm.handles(), group=group)
        self.comm.open(blobs)
        dist.barrier(group=group)  # every rank mapped every peer before the first kernel

    @property
    def capacity(self) -> int:
        return self.comm.capacity()

    def fits(self, t: torch.Tensor) -> bool:
        return t.is_cuda and t.numel() % 8 == 0 and t.numel() * t.element_size() <= self.capacity \
            and t.dtype in (torch.float32, torch.bfloat16)

    def all_reduce(self, t: torch.Tensor, average: bool = True, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """In-place (or into ``out``) sum / mean over the group, enqueued on the current stream."""
        out = t if out is None else out
        self.comm.allreduce(t, out, 1.0 / self.world if average else 1.0)
        return out

    def check(self) -> None:
        """Raise if any peer failed to arrive (host sync; call outside the hot loop)."""
        if self.comm.error():
            raise RuntimeError("P2P all-reduce: a peer did not arrive within the spin limit")


class _StreamFuture:
    """Minimal future for our DDP reducer: ``wait()`` makes the current stream wait on the side
    stream that ran the P2P kernel, then returns the reduced buffer."""

    def __init__(self, value: torch.Tensor, event: torch.cuda.Event):
        self._value, self._event = value, event

    def wait(self):
        torch.cuda.current_stream().wait_event(self._event)
        return self._value

    def value(self):
        return self._value


class P2PHookState:
    def __init__(self, p2p: P2PAllReduce, max_bytes: int = 1 << 20, process_group=None):
        self.p2p, self.max_bytes, self.process_group = p2p, max_bytes, process_group
        self.stream = torch.cuda.Stream(device=p2p.device)
        self.p2p_calls = 0
        self.rccl_calls = 0


def p2p_allreduce_hook(state: P2PHookState, bucket):
    """Averaged all-reduce: one-shot P2P kernel for buckets <= ``state.max_bytes``, RCCL above."""
    buf = bucket.buffer()
    nbytes = buf.numel() * buf.element_size()
    if nbytes <= state.max_bytes and state.p2p.fits(buf):
        state.p2p_calls += 1
        cur = torch.cuda.current_stream()
        state.stream.wait_stream(cur)
        with torch.cuda.stream(state.stream):
            state.p2p.all_reduce(buf, average=True)
            ev = torch.cuda.Event()
            ev.record(state.stream)
        buf.record_stream(state.stream)
        return _StreamFuture(buf, ev)
    state.rccl_calls += 1
    from .comm_hooks import _avg_allreduce_fut
    return _avg_allreduce_fut(buf, state.process_group)
