"""The registered ``pdt_p2p`` c10d backend (parallel/p2p.py P2PProcessGroup): on CPU tensors every
collective is delegated to its inner gloo group, so the group is a drop-in default process group;
the P2P kernel path itself is covered on the GPU by tests/test_p2p_gpu.py."""
import torch
import torch.distributed as dist

from dist_utils import run_ranks


def _worker(rank, world):
    import os
    from pytorch_distributed_training_example_amd.parallel import launcher
    from pytorch_distributed_training_example_amd.parallel.p2p import P2PProcessGroup, register_backend
    launcher.destroy()  # run_ranks initialised gloo; re-init the default group on pdt_p2p
    os.environ["MASTER_PORT"] = str(int(os.environ["MASTER_PORT"]) + 1)
    assert register_backend() == "pdt_p2p"
    ctx = launcher.init_distributed(backend="pdt_p2p", use_gpu=False, timeout_s=60)
    assert dist.get_backend() == "pdt_p2p" and ctx.world_size == world
    t = torch.arange(8, dtype=torch.float32) * (rank + 1)
    dist.all_reduce(t)
    avg = torch.arange(8, dtype=torch.float32) * (rank + 1)
    dist.all_reduce(avg, op=dist.ReduceOp.AVG)  # gloo has no AVG: the backend sums and divides
    # every AVG that reaches the gloo inner group goes through SUM + divide (not just all_reduce)
    co = [torch.full((4,), float(rank + 1)), torch.full((2,), 2.0 * (rank + 1))]
    dist.all_reduce_coalesced(co, op=dist.ReduceOp.AVG)
    red = torch.full((4,), float(rank + 1))
    dist.reduce(red, dst=0, op=dist.ReduceOp.AVG)
    iavg_err = None
    try:
        dist.all_reduce(torch.ones(4, dtype=torch.int32), op=dist.ReduceOp.AVG)
    except Exception as e:  # integer average is not exact: refused, not truncated
        iavg_err = type(e).__name__
    b = torch.full((3,), float(rank))
    dist.broadcast(b, src=1)
    outs = [torch.zeros(2) for _ in range(world)]
    dist.all_gather(outs, torch.full((2,), float(rank)))
    dist.barrier()
    # our DDP on top of it: gloo inner group -> SUM + divide
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    torch.manual_seed(0)
    m = torch.nn.Linear(4, 2)
    ddp = DistributedDataParallel(m)
    x = torch.ones(3, 4) * (rank + 1)
    ddp(x).sum().backward()
    pg = dist.distributed_c10d._get_default_group()
    return (t, b, torch.stack(outs), m.weight.grad.clone(), isinstance(pg, P2PProcessGroup) or "pdt_p2p", avg,
            co, red, iavg_err)


def test_pdt_p2p_backend_delegates_on_cpu():
    out = run_ranks(_worker, 2)
    for r in range(2):
        t, b, g, wg, kind, avg, co, red, iavg_err = out[r]
        assert torch.equal(co[0], torch.full((4,), 1.5)) and torch.equal(co[1], torch.full((2,), 3.0))
        if r == 0:
            assert torch.equal(red, torch.full((4,), 1.5))
        assert iavg_err is not None
        assert torch.equal(t, torch.arange(8, dtype=torch.float32) * 3)
        assert torch.equal(avg, torch.arange(8, dtype=torch.float32) * 1.5)
        assert torch.equal(b, torch.ones(3))
        assert torch.equal(g, torch.tensor([[0., 0.], [1., 1.]]))
        # mean over ranks of sum_batch(x) = 3 * mean(1, 2) = 4.5 per weight entry
        assert torch.allclose(wg, torch.full((2, 4), 4.5))
