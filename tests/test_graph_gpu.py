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


def _run(base, mode, lr, xs, ys):
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
    """With lr=0 the weights never change: every replayed loss/grad must equal eager's."""
    base = _setup()
    xs, ys = _data()
    le, _, ge = _run(base, "eager", 0.0, xs, ys)
    _, _, ge2 = _run(base, "eager", 0.0, xs, ys)
    lg, _, gg = _run(base, "graph", 0.0, xs, ys)
    torch.testing.assert_close(lg, le, rtol=1e-3, atol=1e-3)
    # per-tensor relative error against the eager-vs-eager noise: MIOpen's non-deterministic
    # (atomic split-K) solvers differ run to run at the bf16-rounding level even without capture,
    # and the side-stream weight gradients change their interleaving; a broken replay is O(1) off
    rel = lambda a, b: ((a - b).norm() / (b.norm() + 1e-12)).item()  # noqa: E731
    for i, (a, b, b2) in enumerate(zip(gg, ge, ge2)):
        assert rel(a, b) < max(5e-2, 3 * rel(b2, b)), (i, rel(a, b), rel(b2, b))


def test_graph_step_matches_eager_training():
    """Optimizer/step state across replays. Two *eager* runs are not bit-identical (MIOpen's
    atomic split-K solvers, and a few bf16 SGD updates amplify any rounding difference), so the
    yardstick is the eager-vs-eager drift: a broken replay (stale optimizer state, wrong input
    binding) is O(1) off, far above it. Runs on the default solver set: MIOpen's deterministic
    mode combined with the capture-safe solver exclusions has no solver for one of these
    backward shapes on a fresh find-db (miopenStatusBadParm, seen on the round-end box)."""
    base = _setup()
    xs, ys = _data()
    le, pe, _ = _run(base, "eager", 0.01, xs, ys)
    le2, _, _ = _run(base, "eager", 0.01, xs, ys)
    lg, pg, _ = _run(base, "graph", 0.01, xs, ys)
    assert torch.isfinite(lg).all()
    eager_drift = (le2 - le).abs().max().item()
    graph_drift = (lg - le).abs().max().item()
    print(f"loss drift eager/eager {eager_drift:.3e} graph/eager {graph_drift:.3e}")
    # the first replay runs on weights one (identical) eager update away: rounding-level agreement.
    # Later steps compound differences chaotically (tiny-batch BatchNorm statistics; the captured
    # step runs its own solver / kernel choices, picked without timing): one box measured 0.14 of
    # loss drift by step 5 against 0.027 eager/eager, so later steps get a training-scale bound —
    # a replay that stopped updating or re-read a stale batch fails the weight-motion check below
    # and the lr=0 test above.
    assert abs(lg[0] - le[0]).item() <= max(3e-2, 4 * abs(le2[0] - le[0]).item()), (lg, le)
    assert graph_drift <= max(0.25, 4 * eager_drift), (graph_drift, eager_drift, lg, le)
    # the replayed updates must actually train: weights moved like eager's did
    base_ps = [p.detach().float() for p in base.parameters()]
    for a, b, p0 in zip(pg, pe, base_ps):
        da, db = (a - p0).norm().item(), (b - p0).norm().item()
        assert db < 1e-8 or (0.5 * db < da < 2 * db), (da, db)
