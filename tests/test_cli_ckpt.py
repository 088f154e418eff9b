"""CLI parity with the reference, checkpoint format/resume, elastic restart after an injected fault."""
import importlib.util
import os
import subprocess
import sys

import pytest
import torch

from dist_utils import run_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_CNN = "/root/reference/cnn.py"
LENET_KEYS = ['ConvNet.1.weight', 'ConvNet.1.bias', 'ConvNet.4.weight', 'ConvNet.4.bias', 'ConvNet.7.weight',
              'ConvNet.7.bias', 'FC.0.weight', 'FC.0.bias', 'FC.2.weight', 'FC.2.bias']
ENV = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")


def _train(args, cwd, timeout=600, torchrun=None, env=None):
    cmd = [sys.executable]
    if torchrun:
        cmd += ["-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(torchrun[0]),
                "--master-addr", "127.0.0.1", "--master-port", str(torchrun[1])] + torchrun[2:]
    cmd += [os.path.join(ROOT, "train.py"), "--no-cuda"] + args
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=str(cwd), env=env or ENV)


def test_lenet_keys_and_size_match_reference_model():
    from pytorch_distributed_training_example_amd.models import LeNet
    m = LeNet()
    assert list(m.state_dict()) == LENET_KEYS
    assert sum(p.numel() for p in m.parameters()) == 61706
    if os.path.exists(REF_CNN):
        spec = importlib.util.spec_from_file_location("ref_cnn", REF_CNN)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        ref = mod.LeNet()
        ref.load_state_dict(m.state_dict())  # checkpoints interchange
        x = torch.randn(4, 1, 28, 28)
        torch.testing.assert_close(ref(x), m(x))  # reference outputs softmax probabilities


def test_cli_reference_flags_two_ranks(tmp_path):
    r = _train(["--world-size", "2", "--epochs", "1", "--dry-run", "--batch-size", "64", "--train-samples", "600",
                "--save-model", "--log-interval", "1"], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    # reference log formats (train.py:52-55, 73-76)
    assert "Train Epoch: 1 [0/300 (0%)]\tLoss: " in r.stdout
    assert "Test set on 0: Average loss: " in r.stdout
    sd = torch.load(tmp_path / "mnist_cnn.pt", weights_only=True)
    assert list(sd) == LENET_KEYS


def test_cli_reference_loss_mode(tmp_path):
    r = _train(["--world-size", "1", "--epochs", "1", "--dry-run", "--loss", "nll_on_probs", "--train-samples", "600",
                "--batch-size", "64", "--sharding", "sampler", "--loader", "reference"], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("Train Epoch")][0]
    assert float(line.split("Loss: ")[1]) < 0  # nll on probabilities is in [-1, 0] like the reference


def _resume_worker(rank, world, path, phase):
    from pytorch_distributed_training_example_amd.engine.checkpoint import load_checkpoint, save_checkpoint
    from pytorch_distributed_training_example_amd.models import LeNet
    from pytorch_distributed_training_example_amd.optim import FusedAdadelta, build_scheduler
    from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
    torch.manual_seed(0)
    model = DistributedDataParallel(LeNet(output="logits"))
    opt = FusedAdadelta(model.parameters(), lr=1.0)
    sch = build_scheduler("step", opt, gamma=0.5)
    g = torch.Generator().manual_seed(rank)
    data = [(torch.randn(8, 1, 28, 28, generator=g), torch.randint(0, 10, (8,), generator=g)) for _ in range(4)]

    def epoch(e):
        for x, y in data:
            opt.zero_grad()
            torch.nn.functional.cross_entropy(model(x), y).backward()
            opt.step()
        sch.step()

    if phase == "straight":
        for e in range(4):
            epoch(e)
    else:
        for e in range(2):
            epoch(e)
        save_checkpoint(path, model, opt, sch, epoch=2)
        torch.manual_seed(123)
        model2 = DistributedDataParallel(LeNet(output="logits"))
        opt2 = FusedAdadelta(model2.parameters(), lr=1.0)
        sch2 = build_scheduler("step", opt2, gamma=0.5)
        ck = load_checkpoint(path, model2, opt2, sch2)
        assert ck["epoch"] == 2
        model, opt, sch = model2, opt2, sch2
        for e in range(2, 4):
            epoch(e)
    return {k: v.clone() for k, v in model.module.state_dict().items()}, opt.param_groups[0]["lr"]


def test_checkpoint_resume_is_exact(tmp_path):
    a = run_ranks(_resume_worker, 2, (str(tmp_path / "ck.pt"), "straight"))
    b = run_ranks(_resume_worker, 2, (str(tmp_path / "ck.pt"), "resume"))
    for k in a[0][0]:
        torch.testing.assert_close(a[0][0][k], b[0][0][k], rtol=0, atol=0)
    assert a[0][1] == b[0][1]


def test_load_torch_ddp_prefixed_checkpoint(tmp_path):
    from pytorch_distributed_training_example_amd.engine.checkpoint import load_model
    from pytorch_distributed_training_example_amd.models import LeNet
    m = LeNet()
    torch.save({"module." + k: v for k, v in m.state_dict().items()}, tmp_path / "ddp.pt")
    m2 = LeNet()
    load_model(m2, str(tmp_path / "ddp.pt"))
    for (k, v), (k2, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(v, v2)


@pytest.mark.slow
def test_elastic_restart_after_injected_fault(tmp_path):
    """rank 1 dies mid-epoch 2; torchrun restarts the group; training resumes from the epoch-1 checkpoint."""
    from pytorch_distributed_training_example_amd.parallel.launcher import find_free_port
    env = dict(ENV, PDT_FAULT="1:14")  # 600 samples/2 ranks/bs 32 -> 10 steps/epoch; die at step 14
    for attempt in range(4):
        ck = tmp_path / f"ck{attempt}.pt"
        r = _train(["--epochs", "3", "--batch-size", "64", "--train-samples", "600", "--log-interval", "100",
                    "--checkpoint", str(ck), "--resume"], tmp_path,
                   torchrun=[2, find_free_port(), "--max-restarts", "1"], env=env, timeout=900)
        # gloo's TCP mesh setup is occasionally refused in this sandbox before training starts;
        # that is an environment flake, not the behaviour under test: retry it
        flake = r.returncode != 0 and "Connection refused" in r.stderr and not os.path.exists(ck)
        if not flake:
            break
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "resumed from" in r.stdout and "at epoch 2" in r.stdout
    assert r.stdout.count("Test set on 0") >= 3  # epoch 1 (first attempt) + epochs 2, 3 (after restart)


def _desync_worker(rank, world):
    from pytorch_distributed_training_example_amd.parallel.debug import check_replicas_in_sync
    ps = [torch.ones(3), torch.zeros(2)]
    check_replicas_in_sync(ps)
    if rank == 1:
        ps[1][0] = 1e-3
    try:
        check_replicas_in_sync(ps)
    except RuntimeError as e:
        return str(e)
    return "no error"


def test_replica_desync_detected():
    res = run_ranks(_desync_worker, 2)
    assert all("[1]" in r and "desync" in r for r in res)
