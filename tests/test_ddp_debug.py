"""Reducer debug mode (PDT_DDP_DEBUG / DistributedDataParallel(debug=True)) on gloo, 2 ranks.

SURVEY.md §5 race / desync: the reference keeps replicas equal only through equal seeds
(/root/reference/train.py:80-81); the debug mode must catch a rank whose reduced gradients or
collective sequence diverge, and name the first differing bucket / collective.
"""
import pytest
import torch
import torch.nn as nn

from dist_utils import run_ranks


def _model(extra: bool = False):
    from pytorch_distributed_training_example_amd.models.lenet import MLP
    torch.manual_seed(0)
    m = MLP(16, 32, 4)
    if extra:  # a rank with a different architecture: its bucket layout differs
        m.extra = nn.Linear(4, 4)
    return m


def _steps(ddp, n=2):
    x = torch.randn(8, 16, generator=torch.Generator().manual_seed(3))
    for _ in range(n):
        ddp.zero_grad()
        ddp(x).square().mean().backward()


def _clean(rank, world):
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    ddp = DistributedDataParallel(_model(), bucket_cap_mb=1e-6, first_bucket_mb=1e-6, debug=True)
    _steps(ddp, 3)
    return ddp._debug.step


def test_debug_mode_passes_when_in_sync():
    assert run_ranks(_clean, world=2) == [3, 3]


def _perturb_hook(state, bucket):
    """all-reduce, then rank 1 perturbs bucket 2 (a corrupted reduction on one rank)."""
    import torch.distributed as dist
    buf = bucket.buffer()
    dist.all_reduce(buf)
    buf.div_(dist.get_world_size())
    if dist.get_rank() == 1 and bucket.index() == 2:
        buf[0] += 1e-3
    fut = torch.futures.Future()
    fut.set_result(buf)
    return fut


def _perturbed(rank, world):
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    ddp = DistributedDataParallel(_model(), bucket_cap_mb=1e-6, first_bucket_mb=1e-6, debug=True)
    ddp.register_comm_hook(None, _perturb_hook)
    try:
        _steps(ddp, 1)
    except RuntimeError as e:
        return str(e)
    return None


def test_debug_mode_names_first_differing_bucket():
    msgs = run_ranks(_perturbed, world=2)
    for m in msgs:
        assert m is not None and "bucket 2" in m and "rank 1" in m, m
    # the message names the parameters the bucket holds
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    names = [n for n, _ in _model().named_parameters()]
    assert any(n in msgs[0] for n in names), msgs[0]


def _mismatched(rank, world):
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    # rank 1 has an extra layer; rebuild off so the bucket plans (and collective sequences) differ
    ddp = DistributedDataParallel(_model(extra=(rank == 1)), bucket_cap_mb=1e-6, first_bucket_mb=1e-6,
                                  debug=True, init_sync=False, rebuild_buckets=False)
    ddp.register_comm_hook(None, _noop_hook)
    try:
        _steps(ddp, 1)
    except RuntimeError as e:
        return str(e)
    return None


def _noop_hook(state, bucket):
    fut = torch.futures.Future()
    fut.set_result(bucket.buffer())
    return fut


def test_debug_mode_names_first_differing_collective():
    msgs = run_ranks(_mismatched, world=2)
    for m in msgs:
        assert m is not None and "collective sequence mismatch" in m and "collective #1" in m, m


def test_stream_safety_assert_catches_incomplete_work():
    from pytorch_distributed_training_example_amd.parallel.debug import assert_collective_done

    class Pending:
        def is_completed(self):
            return False

    class Done:
        def is_completed(self):
            return True

    assert_collective_done([(0, Done()), (1, None)])
    with pytest.raises(RuntimeError, match="bucket 1"):
        assert_collective_done([(0, Done()), (1, Pending())])


def test_debug_env_switch(monkeypatch):
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    monkeypatch.setenv("PDT_DDP_DEBUG", "1")
    assert DistributedDataParallel(_model())._debug is not None
    monkeypatch.setenv("PDT_DDP_DEBUG", "0")
    assert DistributedDataParallel(_model())._debug is None
