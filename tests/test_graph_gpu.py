"""hipGraph-captured train step == eager train step (same init, same data)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(seed=0):
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    torch.manual_seed(seed)
    return to_bf16_mixed(get_model("resnet18", num_classes=16).cuda().to(memory_format=torch.channels_last))


def _run(base, mode, lr, xs, ys, other=None):
    from pytorch_distributed_training_example_amd.engine.graph import StaticStep
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    from pytorch_distributed_training_example_amd.optim import FusedSGD
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    m = copy.deepcopy(base)
    ddp = DistributedDataParallel(m)
    opt = FusedSGD(m.parameters(), lr=lr, momentum=0.9)

    def step(x, y):
        opt.zero_grad(set_to_none=True)
        loss = cross_entropy(ddp(x), y)
        loss.backward()
        opt.step()
        return loss.detach()

    out = []
    if mode == "eager":
        for _ in range(3):
            step(xs[0], ys[0])
        for x, y in zip(xs[1:], ys[1:]):
            out.append(float(step(x, y)))
    else:
        runner = StaticStep(step, [xs[0], ys[0]], warmup=3)
        runner.capture()
        for x, y in zip(xs[1:], ys[1:]):
            if other is not None:  # another model's eager training forward + backward between replays
                cross_entropy(other(x), y).backward()
            out.append(float(runner(x, y)))
    grads = [p.grad.detach().float().clone() for p in m.parameters()]
    return torch.tensor(out), [p.detach().float().clone() for p in m.parameters()], grads


def _data(n=6):
    g = torch.Generator(device="cuda").manual_seed(3)
    xs = [torch.randn(8, 3, 64, 64, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
          for _ in range(n)]
    ys = [torch.randint(0, 16, (8,), device="cuda", generator=g) for _ in range(n)]
    return xs, ys


@pytest.fixture(autouse=True)
def _solver_mode():
    """Default (non-deterministic) MIOpen solvers in find mode, minus the two capture-unsafe CK
    solvers (engine/graph.py: make_miopen_capture_safe, applied in conftest)."""
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic = False
    torch.backends.cudnn.benchmark = True
    yield
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old


def test_graph_step_lr0_matches_eager():
    """With lr=0 the weights never change: every replayed loss / gradient must equal eager's BIT FOR
    BIT. Every reduction on this path is fixed-order (no MIOpen, no float atomics:
    tests/test_determinism_gpu.py), so any difference is a replay bug (stale buffer, wrong binding)."""
    base = _setup()
    xs, ys = _data()
    le, _, ge = _run(base, "eager", 0.0, xs, ys)
    lg, _, gg = _run(base, "graph", 0.0, xs, ys)
    assert torch.equal(lg, le), (lg, le)
    bad = [i for i, (a, b) in enumerate(zip(gg, ge)) if not torch.equal(a, b)]
    assert not bad, f"{len(bad)} of {len(ge)} gradients differ (first: {bad[:5]})"


def test_graph_step_matches_eager_training():
    """Optimizer / step state across replays (lr > 0, momentum): the step is deterministic, so two
    eager runs are bit-identical and the replayed run must be too — losses and final weights."""
    base = _setup()
    xs, ys = _data()
    le, pe, _ = _run(base, "eager", 0.01, xs, ys)
    le2, pe2, _ = _run(base, "eager", 0.01, xs, ys)
    lg, pg, _ = _run(base, "graph", 0.01, xs, ys)
    assert torch.equal(le2, le), (le2, le)
    assert all(torch.equal(a, b) for a, b in zip(pe2, pe)), "eager is not run-to-run deterministic"
    assert torch.equal(lg, le), (lg, le)
    bad = [i for i, (a, b) in enumerate(zip(pg, pe)) if not torch.equal(a, b)]
    assert not bad, f"{len(bad)} of {len(pe)} weights differ after the replayed steps (first: {bad[:5]})"
    # and the updates really happened
    moved = [(a - p0.float()).norm().item() for a, p0 in zip(pg, base.parameters())]
    assert max(moved) > 0


def test_graph_replay_survives_other_models_training_forward():
    """The captured step holds the addresses of the per-step weight transforms (W^T / flipped 3x3,
    ops/conv.py prepare_weights). Another model's training forward re-runs prepare_weights for ITS
    convs; the captured model's buffers must stay alive and untouched (they are owned by the
    weights, not by the module-global map), so the replay still equals eager bit for bit."""
    base = _setup()
    other = _setup(seed=7)
    xs, ys = _data()
    le, _, ge = _run(base, "eager", 0.0, xs, ys)
    lg, _, gg = _run(base, "graph", 0.0, xs, ys, other=other)
    assert torch.equal(lg, le), (lg, le)
    bad = [i for i, (a, b) in enumerate(zip(gg, ge)) if not torch.equal(a, b)]
    assert not bad, f"{len(bad)} of {len(ge)} gradients differ (first: {bad[:5]})"


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_side_stream_wgrad_matches_in_stream(arch):
    """Weight gradients on the side stream (ops/conv.py _WgradFork, PDT_WGRAD_STREAM_M): the same kernels
    on other streams, joined before the gradient is consumed — eager AND the captured graph (fork / join
    as graph edges) must equal the in-stream eager step bit for bit (lr = 0: gradients compared)."""
    from pytorch_distributed_training_example_amd.config import SW
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    torch.manual_seed(0)
    base = to_bf16_mixed(get_model(arch, num_classes=16).cuda().to(memory_format=torch.channels_last))
    xs, ys = _data()
    old = SW.wgrad_stream_m
    try:
        SW.wgrad_stream_m = 0
        le, _, ge = _run(base, "eager", 0.0, xs, ys)
        SW.wgrad_stream_m = 1 << 30
        ls, _, gs = _run(base, "eager", 0.0, xs, ys)
        lg, _, gg = _run(base, "graph", 0.0, xs, ys)
    finally:
        SW.wgrad_stream_m = old
    for tag, l2, g2 in (("eager", ls, gs), ("graph", lg, gg)):
        assert torch.equal(l2, le), (tag, l2, le)
        bad = [i for i, (a, b) in enumerate(zip(g2, ge)) if not torch.equal(a, b)]
        assert not bad, f"{tag}: {len(bad)} of {len(ge)} gradients differ (first: {bad[:5]})"


def test_linear_bias_grad_replays_after_allocations():
    """The ResNet head (ops/linear.py Linear) at 1024 rows: a captured backward replayed after later
    allocations gives the eager bias gradient. aten's sum(0) there does not (profiles/r6/graph_colsum_bwd.txt),
    which trained the graphed 1024/GPU bench to NaN."""
    from pytorch_distributed_training_example_amd.ops.linear import Linear
    torch.manual_seed(0)
    lin = Linear(2048, 1000).cuda().bfloat16()
    x = torch.randn(1024, 2048, device="cuda").bfloat16()
    t = torch.randn(1024, 1000, device="cuda").bfloat16()

    def fb():
        for p in lin.parameters():
            if p.grad is not None:
                p.grad.zero_()
        (lin(x).float() * t).sum().backward()

    for _ in range(3):
        fb()
    torch.cuda.synchronize()
    ref = lin.bias.grad.float().clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fb()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        fb()
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(lin.bias.grad.float(), ref)
        junk = [torch.randn(1024, 1000, device="cuda") for _ in range(8)]  # reuse of freed non-graph memory
        del junk


def test_resnet50_b1024_captured_backward_replays_bitwise():
    """The bench's shape (ResNet-50, 1024/GPU): a captured forward+backward replayed after unrelated
    allocations gives every gradient bit-identical to eager (tools/diag_graph_model.py, whole model)."""
    from pytorch_distributed_training_example_amd.engine.graph import make_miopen_capture_safe
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    make_miopen_capture_safe()
    torch.manual_seed(0)
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    m = to_bf16_mixed(get_model("resnet50").cuda().to(memory_format=torch.channels_last))
    x = torch.randn(1024, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (1024,), device="cuda")
    params = [p for p in m.parameters() if p.requires_grad]

    def fb():
        for p in params:
            if p.grad is not None:
                p.grad.zero_()
        cross_entropy(m(x), y, label_smoothing=0.1).backward()

    for _ in range(2):
        fb()
    torch.cuda.synchronize()
    ref = [p.grad.clone() for p in params]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fb()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        fb()
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        bad = [i for i, (p, r) in enumerate(zip(params, ref)) if not torch.equal(p.grad, r)]
        assert not bad, f"{len(bad)} gradients differ after replay, first: param {bad[0]}"
        junk = [torch.randn(1 << 20, device="cuda") for _ in range(64)]
        del junk
    del g
