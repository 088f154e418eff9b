"""End-to-end model steps on one MI355X: HIP-kernel path vs the PyTorch reference path."""
import copy
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _grads(model, x, y, loss_fn):
    model.zero_grad(set_to_none=True)
    loss = loss_fn(model(x), y)
    loss.backward()
    return float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}


def _compare(name, make_input, loss_fn, tol=0.08, **kw):
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops import _native
    torch.manual_seed(0)
    m = get_model(name, **kw).cuda()
    if name.startswith("resnet"):
        m = m.to(memory_format=torch.channels_last)
    m = to_bf16_mixed(m)
    x, y = make_input()
    ref = copy.deepcopy(m)
    l_nat, g_nat = _grads(m, x, y, loss_fn)
    os.environ["PDT_DISABLE_NATIVE"] = "1"
    try:
        l_ref, g_ref = _grads(ref, x, y, loss_fn)
    finally:
        os.environ.pop("PDT_DISABLE_NATIVE")
    assert abs(l_nat - l_ref) < 0.02 * max(1.0, abs(l_ref)), (l_nat, l_ref)
    bad = []
    for n in g_ref:
        err = ((g_nat[n] - g_ref[n]).norm() / (g_ref[n].norm() + 1e-6)).item()
        if err > tol:
            bad.append((n, err))
    assert not bad, bad[:5]


def _ce(out, y):
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    return cross_entropy(out.reshape(-1, out.shape[-1]), y.reshape(-1))


def test_resnet50_native_matches_reference():
    def inp():
        x = torch.randn(16, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        return x, torch.randint(0, 1000, (16,), device="cuda")
    _compare("resnet50", inp, _ce)


def test_vit_native_matches_reference():
    def inp():
        return torch.randn(8, 3, 32, 32, device="cuda").bfloat16(), torch.randint(0, 1000, (8,), device="cuda")
    _compare("vit_tiny", inp, _ce)


def test_gpt2_native_matches_reference():
    def inp():
        return torch.randint(0, 512, (4, 64), device="cuda"), torch.randint(0, 512, (4, 64), device="cuda")
    _compare("gpt2_tiny", inp, _ce)


def test_train_cli_lenet_one_gpu(tmp_path):
    """The reference's CLI on one GPU over RCCL: trains, logs reference lines, saves mnist_cnn.pt."""
    out = tmp_path / "mnist_cnn.pt"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py"), "--epochs", "2", "--world-size", "1",
                        "--train-samples", "20000", "--batch-size", "256", "--log-interval", "20", "--save-model", "--save-path", str(out),
                        "--lr", "1.0"], capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Train Epoch: 1 [0/20000 (0%)]" in r.stdout, r.stdout[-2000:]
    assert "Test set on 0: Average loss:" in r.stdout
    sd = torch.load(out, weights_only=True)
    assert list(sd) == ['ConvNet.1.weight', 'ConvNet.1.bias', 'ConvNet.4.weight', 'ConvNet.4.bias',
                        'ConvNet.7.weight', 'ConvNet.7.bias', 'FC.0.weight', 'FC.0.bias', 'FC.2.weight', 'FC.2.bias']
    acc = [line for line in r.stdout.splitlines() if "Accuracy" in line][-1]
    correct, total = acc.split("Accuracy: ")[1].split(" ")[0].split("/")
    assert int(correct) > 0.3 * int(total), acc  # learned on synthetic MNIST (chance = 10%)
