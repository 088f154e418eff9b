"""Intra-node P2P all-reduce (csrc/kernels/p2p.hip, parallel/p2p.py): two ranks sharing the one
GPU of the test box, peer buffers mapped through hipIpc handles exchanged over a gloo group."""
import pytest
import torch

from dist_utils import run_ranks

pytestmark = pytest.mark.gpu


def _inputs(rank, n, dtype):
    g = torch.Generator().manual_seed(1000 + rank)
    return torch.randn(n, generator=g).to(dtype)


def _allreduce_worker(rank, world, sizes):
    from pytorch_distributed_training_example_amd.parallel.p2p import P2PAllReduce
    p2p = P2PAllReduce(capacity_bytes=4 << 20)
    res = []
    for rep in range(3):  # cycles the staging parity and the device epoch counter
        for algo in (0, 1):  # one-shot, two-shot (interleaved: shared epoch sequence)
            for dtype in (torch.float32, torch.bfloat16):
                for n in sizes:
                    x = _inputs(rank, n, dtype).cuda() * (rep + 1)
                    y = torch.empty_like(x)
                    p2p.all_reduce(x, average=False, out=y, algo=algo)
                    x2 = x.clone()
                    p2p.all_reduce(x2, average=True, algo=algo)  # in place
                    torch.cuda.synchronize()
                    res.append((rep, algo, str(dtype), n, y.cpu(), x2.cpu()))
    p2p.check()
    return res, int(p2p.state[0].item())


@pytest.mark.parametrize("world", [2, 3])
def test_p2p_allreduce_exact(world):
    """One-shot and two-shot (uneven chunks at world 3) sums and means equal the fp32 sum of the
    ranks' inputs (rounded once), bit-identical on every rank; the device epoch counts every call."""
    sizes = [8, 4096, 100000 - 8, 1 << 20]
    out = run_ranks(_allreduce_worker, world, (sizes,), use_gpu=True)
    calls = 3 * 2 * 2 * len(sizes) * 2
    for r in range(world):
        assert out[r][1] == calls, (r, out[r][1])
    for rows in zip(*[o[0] for o in out]):
        rep, algo, dt, n, y0, a0 = rows[0]
        dtype = torch.float32 if "float32" in dt else torch.bfloat16
        xs = [_inputs(r, n, dtype) * (rep + 1) for r in range(world)]
        ref = sum(x.float() for x in xs)
        for row in rows[1:]:
            assert torch.equal(row[4], y0) and torch.equal(row[5], a0), "replicas must be bit-identical"
        assert torch.equal(y0, ref.to(dtype)), (algo, dt, n)
        assert torch.equal(a0, (ref * (1.0 / world)).to(dtype)), (algo, dt, n)


def _graph_worker(rank, world, n, replays):
    """The P2P all-reduce captured in a hipGraph and replayed: the epoch advances on the device, so
    each replay synchronises with the peers' matching replay (a host-side epoch baked into the
    captured node would let replays read peers' half-written staging)."""
    from pytorch_distributed_training_example_amd.parallel.p2p import P2PAllReduce
    p2p = P2PAllReduce(capacity_bytes=4 << 20)
    static_in = torch.zeros(n, device="cuda")
    static_out = torch.zeros(n, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up (eager) call
        p2p.all_reduce(static_in, average=False, out=static_out)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        p2p.all_reduce(static_in, average=False, out=static_out, algo=1 if n >= 4096 else 0)
    outs = []
    for i in range(replays):
        static_in.copy_(_inputs(rank, n, torch.float32).cuda() * (i + 2))
        g.replay()
        outs.append(static_out.cpu())
    torch.cuda.synchronize()
    p2p.check()
    return outs, int(p2p.state[0].item())


@pytest.mark.parametrize("n", [1024, 262144])
def test_p2p_allreduce_graph_replay_exact(n):
    replays = 6
    out = run_ranks(_graph_worker, 2, (n, replays), use_gpu=True)
    for r in range(2):
        assert out[r][1] == 1 + replays  # warm-up + every replay advanced the device epoch
    for i in range(replays):
        ref = sum(_inputs(r, n, torch.float32) * (i + 2) for r in range(2))
        assert torch.equal(out[0][0][i], ref) and torch.equal(out[1][0][i], ref), i


def _timeout_worker(rank, world):
    """Rank 1 never joins the collective: rank 0's kernel gives up after its (wall-clock) timeout, sets
    the error word and writes NaN instead of a partial sum; check() raises; reset_error() clears it."""
    from pytorch_distributed_training_example_amd.parallel.p2p import P2PAllReduce
    p2p = P2PAllReduce(capacity_bytes=1 << 20, timeout_s=1.0)
    x = torch.ones(4096, device="cuda")
    raised = None
    if rank == 0:
        p2p.all_reduce(x, average=False)
        torch.cuda.synchronize()
        try:
            p2p.check()
        except RuntimeError as e:
            raised = str(e)
        p2p.reset_error()
        assert not p2p.error()
    torch.distributed.barrier()
    return raised, bool(torch.isnan(x).all().item()) if rank == 0 else None


def test_p2p_lost_peer_raises_and_poisons():
    out = run_ranks(_timeout_worker, 2, use_gpu=True)
    raised, all_nan = out[0]
    assert raised is not None and "did not arrive within 1 s" in raised
    assert all_nan, "a lost peer must never produce a partial sum"


def _late_worker(rank, world, delay_s):
    """Rank 1 joins ``delay_s`` late (first-step skew): rank 0's kernel waits for it — the wait is
    bounded by the group's timeout (120 s here), not by an iteration count — and the sum is exact."""
    import time
    from pytorch_distributed_training_example_amd.parallel.p2p import P2PAllReduce
    p2p = P2PAllReduce(capacity_bytes=1 << 20)
    x = torch.full((8192,), float(rank + 1), device="cuda")
    torch.distributed.barrier()
    if rank == 1:
        time.sleep(delay_s)
    t0 = time.time()
    p2p.all_reduce(x, average=False)
    torch.cuda.synchronize()
    waited = time.time() - t0
    p2p.check()
    return x.cpu(), waited, p2p.timeout_s


def test_p2p_late_peer_still_exact():
    out = run_ranks(_late_worker, 2, (3.0,), use_gpu=True)
    for x, _, tmo in out:
        assert torch.equal(x, torch.full((8192,), 3.0)) and tmo == 120.0
    assert out[0][1] > 2.0, "rank 0 should have waited for the late peer"


def _ddp_worker(rank, world):
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    from pytorch_distributed_training_example_amd.parallel.p2p import (P2PAllReduce, P2PHookState,
                                                                        p2p_allreduce_hook)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 8)).cuda()
    ddp = DistributedDataParallel(model, bucket_cap_mb=0.004, first_bucket_mb=0.002)
    state = P2PHookState(P2PAllReduce(capacity_bytes=1 << 20))
    ddp.register_comm_hook(state, p2p_allreduce_hook)
    g = torch.Generator().manual_seed(rank)
    x, t = torch.randn(16, 32, generator=g).cuda(), torch.randn(16, 8, generator=g).cuda()
    for _ in range(3):
        ddp.zero_grad(set_to_none=True)
        torch.nn.functional.mse_loss(ddp(x), t).backward()
    torch.cuda.synchronize()
    state.p2p.check()
    return [p.grad.cpu() for p in model.parameters()], state.p2p_calls, len(ddp._buckets), x.cpu(), t.cpu()


def test_ddp_p2p_hook_matches_full_batch_grads():
    out = run_ranks(_ddp_worker, 2, use_gpu=True)
    (g0, calls, nb, x0, t0), (g1, _, _, x1, t1) = out
    assert nb > 1 and calls >= 3 * nb
    for a, b in zip(g0, g1):
        assert torch.equal(a, b)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 8))
    loss = 0.5 * (torch.nn.functional.mse_loss(model(x0), t0) + torch.nn.functional.mse_loss(model(x1), t1))
    loss.backward()
    for a, p in zip(g0, model.parameters()):
        torch.testing.assert_close(a, p.grad, rtol=1e-5, atol=1e-6)


def _backend_worker(rank, world):
    """dist.init_process_group("pdt_p2p") as the default group: GPU all-reduces take the P2P kernels
    (counted), the rest goes to the inner group (gloo here: two ranks share the one GPU)."""
    import os
    import torch.distributed as dist
    from pytorch_distributed_training_example_amd.parallel import launcher
    launcher.destroy()
    os.environ["MASTER_PORT"] = str(int(os.environ["MASTER_PORT"]) + 1)
    os.environ["PDT_P2P_INNER"] = "gloo"
    launcher.init_distributed(backend="pdt_p2p", use_gpu=True, timeout_s=60)
    pg = dist.distributed_c10d._get_default_group()
    t = torch.full((4096,), float(rank + 1), device="cuda", dtype=torch.bfloat16)
    dist.all_reduce(t)
    a = torch.full((1024,), float(rank + 1), device="cuda")
    dist.all_reduce(a, op=dist.ReduceOp.AVG)
    c = torch.full((16,), float(rank))
    dist.all_reduce(c)  # CPU: inner group
    torch.cuda.synchronize()
    pg.check()
    return t.float().cpu(), a.cpu(), c, pg.p2p_calls


def _backend_ddp_worker(rank, world):
    """Our DDP on ``pdt_p2p`` with a gloo inner group and a bucket past the 8 MiB staging capacity: that
    bucket takes the inner group with AVG, which gloo lacks (the backend sums and divides)."""
    import os
    import torch.distributed as dist
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel, launcher
    launcher.destroy()
    os.environ["MASTER_PORT"] = str(int(os.environ["MASTER_PORT"]) + 1)
    os.environ["PDT_P2P_INNER"] = "gloo"
    launcher.init_distributed(backend="pdt_p2p", use_gpu=True, timeout_s=60)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(1536, 1536), torch.nn.ReLU(), torch.nn.Linear(1536, 8)).cuda()
    ddp = DistributedDataParallel(model, bucket_cap_mb=25)
    g = torch.Generator().manual_seed(rank)
    x, t = torch.randn(4, 1536, generator=g).cuda(), torch.randn(4, 8, generator=g).cuda()
    torch.nn.functional.mse_loss(ddp(x), t).backward()
    torch.cuda.synchronize()
    return [p.grad.cpu() for p in model.parameters()], x.cpu(), t.cpu(), max(b.buffer.numel() * b.buffer.element_size() for b in ddp._buckets)


def test_ddp_on_pdt_p2p_gloo_inner_large_bucket():
    out = run_ranks(_backend_ddp_worker, 2, use_gpu=True)
    (g0, x0, t0, big), (g1, x1, t1, _) = out
    assert big > 8 << 20, big
    for a, b in zip(g0, g1):
        assert torch.equal(a, b)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(1536, 1536), torch.nn.ReLU(), torch.nn.Linear(1536, 8))
    loss = 0.5 * (torch.nn.functional.mse_loss(model(x0), t0) + torch.nn.functional.mse_loss(model(x1), t1))
    loss.backward()
    for a, p in zip(g0, model.parameters()):
        torch.testing.assert_close(a, p.grad, rtol=1e-4, atol=1e-6)


def test_pdt_p2p_backend_gpu():
    out = run_ranks(_backend_worker, 2, use_gpu=True)
    for t, a, c, calls in out:
        assert torch.equal(t, torch.full((4096,), 3.0)) and torch.equal(a, torch.full((1024,), 1.5))
        assert torch.equal(c, torch.full((16,), 1.0)) and calls == 2


def _overlap_worker(rank, world):
    """Backward/communication overlap, measured: the P2P all-reduce of the FIRST bucket (the last
    layers' gradients) must complete on the GPU before backward's compute ends — i.e. it ran under
    backward, not after it (the reference all-reduces only after backward, train.py:49-50)."""
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    from pytorch_distributed_training_example_amd.parallel.p2p import (P2PAllReduce, P2PHookState,
                                                                        p2p_allreduce_hook)
    torch.manual_seed(0)
    layers = []
    for _ in range(12):
        layers += [torch.nn.Linear(1024, 1024), torch.nn.ReLU()]
    model = torch.nn.Sequential(*layers).cuda()
    ddp = DistributedDataParallel(model, bucket_cap_mb=4, first_bucket_mb=4)
    state = P2PHookState(P2PAllReduce(capacity_bytes=8 << 20))
    done = []

    def hook(st, bucket):
        fut = p2p_allreduce_hook(st, bucket)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(st.stream)  # completion of this bucket's P2P kernel
        done.append(ev)
        return fut
    ddp.register_comm_hook(state, hook)
    ddp.enable_comm_timing(True)
    x = torch.randn(4096, 1024, device="cuda")
    for _ in range(3):
        done.clear()
        ddp.zero_grad(set_to_none=True)
        ddp(x).square().mean().backward()
    torch.cuda.synchronize()
    state.p2p.check()
    end_of_compute = ddp._comm_events[-1][0]  # recorded when backward's compute was all issued
    lead_ms = done[0].elapsed_time(end_of_compute)  # > 0: bucket 0 finished before compute ended
    return len(done), lead_ms, ddp.comm_exposed_ms()


def test_first_bucket_allreduce_overlaps_backward():
    out = run_ranks(_overlap_worker, 2, use_gpu=True)
    for nb, lead_ms, exposed in out:
        assert nb >= 3, nb
        assert lead_ms > 0.0, f"bucket 0's all-reduce ended {-lead_ms:.3f} ms AFTER backward's compute"
        assert exposed is not None and exposed >= 0.0


def _overlap_bf16_worker(rank, world):
    """bf16-mixed ResNet-18 (fp32 BN parameters in their own bucket): with buckets in FILL order
    (parallel/buckets.py) the fp32 norm bucket, which fills last, no longer gates the bf16 buckets —
    each bf16 bucket's all-reduce is issued the moment it fills and completes under backward."""
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    from pytorch_distributed_training_example_amd.parallel.p2p import (P2PAllReduce, P2PHookState,
                                                                        p2p_allreduce_hook)
    torch.manual_seed(0)
    model = to_bf16_mixed(get_model("resnet18", num_classes=16).cuda().to(memory_format=torch.channels_last))
    ddp = DistributedDataParallel(model, bucket_cap_mb=4, first_bucket_mb=1)
    state = P2PHookState(P2PAllReduce(capacity_bytes=8 << 20))
    done = []

    def hook(st, bucket):
        fut = p2p_allreduce_hook(st, bucket)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(st.stream)
        done.append((bucket.index(), str(bucket.buffer().dtype), ev))
        return fut
    ddp.register_comm_hook(state, hook)
    ddp.enable_comm_timing(True)
    g = torch.Generator(device="cuda").manual_seed(1 + rank)
    x = torch.randn(128, 3, 128, 128, device="cuda", generator=g).bfloat16().contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 16, (128,), device="cuda", generator=g)
    for _ in range(3):
        done.clear()
        ddp.zero_grad(set_to_none=True)
        cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    state.p2p.check()
    end_of_compute = ddp._comm_events[-1][0]
    leads = [(i, dt, ev.elapsed_time(end_of_compute)) for i, dt, ev in done]
    return leads, ddp.bucket_ready_lead_ms()


def test_bf16_buckets_allreduce_under_backward():
    """Two ranks share the test box's one GPU, so how fast a bucket's P2P all-reduce finishes depends on
    the other process's progress; what the bucket ORDER decides is when each all-reduce can START. With
    the fp32 norm bucket first in the order (round 4) every launch waited for the end of backward (lead
    ~0 for all buckets); in fill order every bucket but the last is issued under backward's compute, and
    the first bf16 bucket's all-reduce has completed before that compute ends."""
    out = run_ranks(_overlap_bf16_worker, 2, use_gpu=True)
    for leads, ready in out:
        bf16 = [(i, ms) for i, dt, ms in leads if dt == "torch.bfloat16"]
        fp32 = [i for i, dt, _ in leads if dt == "torch.float32"]
        assert len(bf16) >= 3 and fp32, leads
        assert fp32 == [max(i for i, _, _ in leads)], f"the fp32 norm bucket must launch last: {leads}"
        assert bf16[0][1] > 0.0, f"the first bf16 bucket's all-reduce ended after backward's compute: {leads}"
        # launch lead (bench.py's bucket_ready_lead_ms): every bucket but the last issued under backward
        assert ready is not None and len(ready) == len(leads)
        assert all(v > 0.0 for v in ready[:-1]), f"buckets launched only after backward's compute: {ready}"
        assert ready[0] > ready[-1]
