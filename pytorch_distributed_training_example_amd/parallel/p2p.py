"""Intra-node P2P all-reduce over xGMI, a DDP comm hook that uses it for small and
mid-size buckets, and a registered ``torch.distributed`` backend (``"pdt_p2p"``) built on it.

The reference reduces 10 tiny fp32 tensors per step with one NCCL call each
(/root/reference/train.py:34-39, 247 KB in total): pure collective latency. On an 8-GPU MI355X
node every GPU has a direct xGMI link to every other one, so:

  * ``P2PAllReduce(group)`` allocates an uncached IPC-exportable staging + flag region per rank
    (csrc/kernels/p2p.hip, C++ ``P2PComm``), exchanges the ``hipIpcMemHandle``s through the
    process group (``all_gather_object``) or the c10d store, maps every peer's region, and then
    all-reduces with ONE kernel on the caller's stream — no host involvement, no RCCL channels;
  * one-shot (every rank reads all peers' copies: (n-1)·S in per GPU over all links at once) up
    to ``oneshot_max_bytes``; two-shot (reduce-scatter + all-gather through peer reads: 2(n-1)/n·S
    in per GPU, still over all links) above it, up to the staging capacity;
  * every chunk is summed in rank order with fp32 accumulation: bit-identical replicas;
  * the call counter lives in device memory and is advanced by the kernel, so the kernel can be
    captured in a hipGraph and replayed (round 2's host-side epoch could not);
  * a peer that has not arrived within ``timeout_s`` of WALL-CLOCK time (default: the process
    group's timeout, capped at ``MAX_TIMEOUT_S``; the kernel bounds its wait by s_memrealtime) sets a
    sticky device error word and the output slice becomes NaN — never a partial sum; ``check()``
    raises, and the DDP hook raises on its next call (the error word is copied to pinned memory
    behind each kernel, read without a sync); ``reset_error()`` clears it.
  * calls are serialised on ONE internal stream per group (joined to the caller's stream both
    ways), as RCCL serialises its work: the device epoch and the staging parity assume stream-ordered
    calls, so two all-reduces issued from different caller streams must never overlap.

All ranks of the group must be on one node (IPC). Ranks may share a GPU (tests do this).
"""
from __future__ import annotations

import datetime
import pickle
import time
from typing import Optional

import torch
import torch.distributed as dist

from ..ops._native import native

# one-shot below, two-shot above (latency vs bytes moved per GPU). An estimate, not a measurement: the crossover
# needs >= 2 GPUs of one node (tools/p2p_crossover.py measures it, and the hook's RCCL crossover, under torchrun);
# the P2P hook stays opt-in (--comm-hook p2p) until it is measured.
ONESHOT_MAX_BYTES = 256 << 10
DEFAULT_TIMEOUT_S = 300.0  # a peer may be this late (wall clock) before the call poisons its output
MAX_TIMEOUT_S = 1800.0


class P2PAllReduce:
    def __init__(self, group=None, capacity_bytes: int = 8 << 20, max_blocks: int = 64,
                 device: Optional[torch.device] = None, oneshot_max_bytes: int = ONESHOT_MAX_BYTES,
                 rank: Optional[int] = None, world: Optional[int] = None, store=None,
                 timeout_s: Optional[float] = None):
        """``store`` (with ``rank``/``world``): exchange the IPC handles through a c10d store instead
        of a process group (used by the registered backend, which IS the group being built).
        ``timeout_s``: how long (wall clock) a call waits for a late peer; default the group's
        timeout (``DEFAULT_TIMEOUT_S`` when unknown), at most ``MAX_TIMEOUT_S``."""
        self.group = group
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world = dist.get_world_size(group) if world is None else world
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.oneshot_max_bytes = int(oneshot_max_bytes)
        if timeout_s is None:
            timeout_s = _group_timeout_s(group)
        self.timeout_s = float(min(max(timeout_s, 1e-3), MAX_TIMEOUT_S))
        self.stream = torch.cuda.Stream(device=dev)
        self.comm = native().P2PComm(self.rank, self.world, int(capacity_bytes), int(max_blocks), dev.index)
        # [0] epoch, [1] finished-block counter, [2] sticky error: advanced by the kernel itself
        self.state = torch.zeros(4, dtype=torch.int32, device=dev)
        if store is None:
            blobs = [None] * self.world
            dist.all_gather_object(blobs, self.comm.handles(), group=group)
            self.comm.open(blobs)
            dist.barrier(group=group)  # every rank mapped every peer before the first kernel
        else:
            store.set(f"p2p_handles_{self.rank}", pickle.dumps(self.comm.handles()))
            blobs = [pickle.loads(store.get(f"p2p_handles_{r}")) for r in range(self.world)]
            self.comm.open(blobs)
            store.add("p2p_opened", 1)
            deadline = datetime.datetime.now() + datetime.timedelta(seconds=120)
            while int(store.add("p2p_opened", 0)) < self.world:
                if datetime.datetime.now() > deadline:
                    raise RuntimeError("P2P all-reduce: peers did not map the staging buffers in 120 s")
                time.sleep(0.002)

    @property
    def capacity(self) -> int:
        return self.comm.capacity()

    def fits(self, t: torch.Tensor) -> bool:
        return t.is_cuda and t.numel() % 8 == 0 and t.numel() * t.element_size() <= self.capacity \
            and t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous()

    def algo_for(self, nbytes: int) -> int:
        return 0 if nbytes <= self.oneshot_max_bytes or self.world <= 2 else 1

    def all_reduce(self, t: torch.Tensor, average: bool = True, out: Optional[torch.Tensor] = None,
                   algo: Optional[int] = None) -> torch.Tensor:
        """In-place (or into ``out``) sum / mean over the group, enqueued on the current stream."""
        out = t if out is None else out
        if algo is None:
            algo = self.algo_for(t.numel() * t.element_size())
        cur = torch.cuda.current_stream(self.device)
        if cur == self.stream:  # already on the group's stream (e.g. the DDP hook's)
            self.comm.allreduce(t, out, 1.0 / self.world if average else 1.0, self.state, int(algo), self.timeout_s)
            return out
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.comm.allreduce(t, out, 1.0 / self.world if average else 1.0, self.state, int(algo), self.timeout_s)
        cur.wait_stream(self.stream)
        t.record_stream(self.stream)
        if out is not t:
            out.record_stream(self.stream)
        return out

    def reset_error(self) -> None:
        """Clear the sticky error word after a handled failure (stream-ordered, no sync)."""
        self.state[2].zero_()

    def error(self) -> bool:
        """Host sync: True if a peer failed to arrive in any call so far."""
        return bool(self.state[2].item())

    def check(self) -> None:
        """Raise if any peer failed to arrive (host sync; call outside the hot loop)."""
        if self.error():
            raise RuntimeError(f"P2P all-reduce: a peer did not arrive within {self.timeout_s:g} s "
                               "(the affected outputs were set to NaN)")


def _group_timeout_s(group) -> float:
    """The process group's timeout in seconds (its backend's ``options._timeout``; for our own
    registered backend the timeout it was built with); ``DEFAULT_TIMEOUT_S`` when it cannot be read."""
    try:
        pg = group if group is not None else dist.distributed_c10d._get_default_group()
        for dev in ("cuda", "cpu"):
            try:
                b = pg._get_backend(torch.device(dev))
            except Exception:  # noqa: BLE001 — no backend for this device type
                continue
            t = getattr(b, "_timeout_s", None)
            if t is None and hasattr(b, "options"):
                t = b.options._timeout.total_seconds()
            if t:
                return float(t)
    except Exception:  # noqa: BLE001 — no group: the default
        pass
    return DEFAULT_TIMEOUT_S


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
    def __init__(self, p2p: P2PAllReduce, max_bytes: Optional[int] = None, process_group=None):
        """Buckets up to ``max_bytes`` (default: the staging capacity) go through the P2P kernels,
        larger ones through RCCL."""
        self.p2p = p2p
        self.max_bytes = p2p.capacity if max_bytes is None else max_bytes
        self.process_group = process_group
        self.stream = p2p.stream  # the group's one stream: every P2P call is ordered on it
        self.p2p_calls = 0
        self.rccl_calls = 0
        # the device error word, copied behind every P2P kernel: read (no sync) on the next call
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._err_event: Optional[torch.cuda.Event] = None

    def raise_if_failed(self) -> None:
        ev = self._err_event
        if ev is not None and not torch.cuda.is_current_stream_capturing() and ev.query() \
                and int(self._err_host[0]) != 0:
            raise RuntimeError(f"P2P all-reduce: a peer did not arrive within {self.p2p.timeout_s:g} s in "
                               "an earlier bucket; its gradients were poisoned with NaN")


def p2p_allreduce_hook(state: P2PHookState, bucket):
    """Averaged all-reduce: P2P kernels (one-/two-shot by size) for buckets <= ``state.max_bytes``,
    RCCL above. Raises if a previous P2P call lost a peer."""
    state.raise_if_failed()
    buf = bucket.buffer()
    nbytes = buf.numel() * buf.element_size()
    if nbytes <= state.max_bytes and state.p2p.fits(buf):
        state.p2p_calls += 1
        cur = torch.cuda.current_stream()
        state.stream.wait_stream(cur)
        with torch.cuda.stream(state.stream):
            state.p2p.all_reduce(buf, average=True)
            state._err_host.copy_(state.p2p.state[2:3], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(state.stream)
        state._err_event = ev
        buf.record_stream(state.stream)
        return _StreamFuture(buf, ev)
    state.rccl_calls += 1
    from .comm_hooks import _avg_allreduce_fut
    return _avg_allreduce_fut(buf, state.process_group)


# ---------------------------------------------------------------- registered c10d backend
class _DoneWork(dist._Work if hasattr(dist, "_Work") else torch._C._distributed_c10d.Work):
    """Work of a collective already enqueued on the caller's stream (stream-ordered: wait() is a
    no-op for the host, like an RCCL work's wait on the current stream)."""

    def __init__(self, result):
        super().__init__()
        self._fut = torch.futures.Future()
        self._fut.set_result(result)

    def wait(self, timeout=None):
        return True

    def get_future(self):
        return self._fut


class P2PProcessGroup(dist.ProcessGroup):
    """``dist.init_process_group("pdt_p2p")``: all-reduce of one contiguous bf16/fp32 GPU tensor
    (SUM or AVG) that fits the staging buffer runs on the xGMI P2P kernels; every other collective
    (and CPU tensors) goes to an inner RCCL (``nccl``) or gloo group built from the same store.
    Intra-node only (IPC); one rank per GPU (or ranks sharing a GPU with the gloo inner group)."""

    def __init__(self, store, rank: int, world: int, timeout, capacity_bytes: int = 8 << 20,
                 inner_backend: Optional[str] = None):
        super().__init__(rank, world)
        self._store, self._rank, self._world = store, rank, world
        self._capacity = capacity_bytes
        self._timeout_s = timeout.total_seconds() if hasattr(timeout, "total_seconds") else DEFAULT_TIMEOUT_S
        if inner_backend is None:
            inner_backend = "nccl" if torch.cuda.is_available() else "gloo"
        self.inner_backend = inner_backend
        prefix = dist.PrefixStore("pdt_p2p_inner", store)
        if inner_backend == "nccl":
            opts = dist.ProcessGroupNCCL.Options()
            opts._timeout = timeout
            self.inner = dist.ProcessGroupNCCL(prefix, rank, world, opts)
        else:
            self.inner = dist.ProcessGroupGloo(prefix, rank, world, timeout)
        self._p2p: Optional[P2PAllReduce] = None
        self.p2p_calls = 0

    def getBackendName(self) -> str:
        return "pdt_p2p"

    def _p2p_for(self, t: torch.Tensor) -> Optional[P2PAllReduce]:
        if not t.is_cuda:
            return None
        if self._p2p is None:  # lazily: the device is bound by now
            self._p2p = P2PAllReduce(capacity_bytes=self._capacity, device=t.device, rank=self._rank,
                                     world=self._world, store=dist.PrefixStore("pdt_p2p_ipc", self._store),
                                     timeout_s=self._timeout_s)
        return self._p2p if self._p2p.fits(t) and t.device == self._p2p.device else None

    def allreduce(self, tensors, opts=None):
        if opts is None:
            opts = dist.AllreduceOptions()
        op = opts.reduceOp
        # (ReduceOp == RedOpType works, ``op in (SUM, AVG)`` does not)
        if len(tensors) == 1 and (op == dist.ReduceOp.SUM or op == dist.ReduceOp.AVG):
            p2p = self._p2p_for(tensors[0])
            if p2p is not None:
                self.p2p_calls += 1
                p2p.all_reduce(tensors[0], average=op == dist.ReduceOp.AVG)
                return _DoneWork(tensors)
        if self._avg_needs_divide(op):
            # gloo has no AVG (this path: CPU tensors, or buckets the staging buffer cannot take,
            # e.g. past its capacity or numel % 8 != 0)
            self.inner.allreduce(tensors, self._sum_opts(dist.AllreduceOptions())).wait()
            return self._divided(tensors)
        return self.inner.allreduce(tensors, opts)

    # gloo has no ReduceOp.AVG: every AVG reduction that goes to a gloo inner group runs as SUM and
    # then one true division per output (floating tensors only: an integer average is not exact)
    def _avg_needs_divide(self, op) -> bool:
        return op == dist.ReduceOp.AVG and self.inner_backend != "nccl"

    @staticmethod
    def _sum_opts(opts):
        opts.reduceOp = dist.ReduceOp.SUM
        return opts

    def _divided(self, tensors):
        for t in tensors:
            if not t.is_floating_point():
                raise TypeError(f"pdt_p2p: ReduceOp.AVG of a {t.dtype} tensor (integer average is not exact)")
            t.div_(self._world)
        return _DoneWork(tensors)

    def allreduce_coalesced(self, tensors, opts=None):
        opts = opts or dist.AllreduceCoalescedOptions()
        if self._avg_needs_divide(opts.reduceOp):
            self.inner.allreduce_coalesced(tensors, self._sum_opts(dist.AllreduceCoalescedOptions())).wait()
            return self._divided(tensors)
        return self.inner.allreduce_coalesced(tensors, opts)

    def broadcast(self, tensors, opts=None):
        return self.inner.broadcast(tensors, opts or dist.BroadcastOptions())

    def allgather(self, output_tensors, input_tensors, opts=None):
        return self.inner.allgather(output_tensors, input_tensors, opts or dist.AllgatherOptions())

    def _allgather_base(self, output, input, opts=None):
        return self.inner._allgather_base(output, input, opts or dist.AllgatherOptions())

    def reduce_scatter(self, output_tensors, input_tensors, opts=None):
        return self.inner.reduce_scatter(output_tensors, input_tensors, opts or dist.ReduceScatterOptions())

    def _reduce_scatter_base(self, output, input, opts=None):
        return self.inner._reduce_scatter_base(output, input, opts or dist.ReduceScatterOptions())

    def reduce(self, tensors, opts=None):
        opts = opts or dist.ReduceOptions()
        if self._avg_needs_divide(opts.reduceOp):
            sum_opts = dist.ReduceOptions()
            sum_opts.rootRank, sum_opts.rootTensor = opts.rootRank, opts.rootTensor
            self.inner.reduce(tensors, self._sum_opts(sum_opts)).wait()
            return self._divided(tensors) if self._rank == opts.rootRank else _DoneWork(tensors)
        return self.inner.reduce(tensors, opts)

    def alltoall_base(self, output, input, output_split_sizes, input_split_sizes, opts=None):
        return self.inner.alltoall_base(output, input, output_split_sizes, input_split_sizes,
                                        opts or dist.AllToAllOptions())

    def barrier(self, opts=None):
        return self.inner.barrier(opts or dist.BarrierOptions())

    def send(self, tensors, dst, tag=0):
        return self.inner.send(tensors, dst, tag)

    def recv(self, tensors, src, tag=0):
        return self.inner.recv(tensors, src, tag)

    def check(self) -> None:
        if self._p2p is not None:
            self._p2p.check()


def _create_pg(store, rank, world, timeout):
    import os
    # PDT_P2P_INNER=gloo: the non-P2P collectives on gloo (tests: ranks sharing one GPU, which RCCL
    # refuses); default RCCL on GPU machines
    return P2PProcessGroup(store, rank, world, timeout, inner_backend=os.environ.get("PDT_P2P_INNER") or None)


def register_backend(name: str = "pdt_p2p") -> str:
    """Register the P2P process group as a c10d backend (idempotent); returns its name."""
    if name.upper() not in dist.Backend.backend_list and name not in dist.Backend.backend_list:
        dist.Backend.register_backend(name, _create_pg, devices=["cuda", "cpu"])
    return name
