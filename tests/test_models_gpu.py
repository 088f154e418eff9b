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


def _compare(name, make_input, loss_fn, slack=1.3, **kw):
    """Native bf16 path must be as accurate as the stock bf16 path, both measured against an fp32
    oracle. (A direct native-vs-stock comparison is meaningless for deep random-init nets: two
    bf16 runs differing by 1e-3 in the input already disagree by >100% in early-layer grads.)"""
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    torch.manual_seed(0)
    base = get_model(name, **kw).cuda()
    if name.startswith("resnet"):
        base = base.to(memory_format=torch.channels_last)
    x, y = make_input()
    xb = x.bfloat16() if x.is_floating_point() else x
    from pytorch_distributed_training_example_amd.config import SW
    os.environ["PDT_DISABLE_NATIVE"] = "1"
    SW.reload()
    try:
        l32, g32 = _grads(copy.deepcopy(base), x, y, loss_fn)
        l_ref, g_ref = _grads(to_bf16_mixed(copy.deepcopy(base)), xb, y, loss_fn)
    finally:
        os.environ.pop("PDT_DISABLE_NATIVE")
        SW.reload()
    l_nat, g_nat = _grads(to_bf16_mixed(copy.deepcopy(base)), xb, y, loss_fn)
    assert abs(l_nat - l32) <= slack * abs(l_ref - l32) + 0.02 * max(1.0, abs(l32)), (l_nat, l_ref, l32)
    e = lambda a, b: ((a - b).norm() / (b.norm() + 1e-9)).item()
    e_nat = torch.tensor([e(g_nat[n], g32[n]) for n in g32])
    e_ref = torch.tensor([e(g_ref[n], g32[n]) for n in g32])
    assert e_nat.median() <= slack * e_ref.median() + 0.02, (e_nat.median(), e_ref.median())
    assert e_nat.max() <= slack * e_ref.max() + 0.05, (e_nat.max(), e_ref.max())


def _ce(out, y):
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    return cross_entropy(out.reshape(-1, out.shape[-1]), y.reshape(-1))


def test_resnet50_native_matches_reference():
    def inp():
        x = torch.randn(16, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
        return x, torch.randint(0, 1000, (16,), device="cuda")
    _compare("resnet50", inp, _ce)


def test_vit_native_matches_reference():
    def inp():
        return torch.randn(8, 3, 32, 32, device="cuda"), torch.randint(0, 1000, (8,), device="cuda")
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


@pytest.mark.parametrize("extra", [["--hipgraph"], ["--loss", "nll_on_probs", "--hipgraph"]])
def test_train_cli_lenet_hipgraph(tmp_path, extra):
    """--hipgraph: every train step replays one captured graph (fused LeNet kernels, MIOpen fp32
    convs, fused Adadelta); training must still learn like the eager run."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py"), "--epochs", "2", "--world-size", "1",
                        "--train-samples", "20000", "--batch-size", "256", "--log-interval", "20", "--lr", "1.0"]
                       + extra, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    acc = [line for line in r.stdout.splitlines() if "Accuracy" in line][-1]
    correct, total = acc.split("Accuracy: ")[1].split(" ")[0].split("/")
    assert int(correct) > 0.3 * int(total), acc


def test_global_avgpool_channels_last_grad():
    """ResNet's channels_last global average pool (models/resnet.py _GlobalAvgPoolFn): same values
    and gradient as nn.AdaptiveAvgPool2d + flatten, and a channels_last gradient."""
    from pytorch_distributed_training_example_amd.models.resnet import _GlobalAvgPoolFn
    torch.manual_seed(0)
    x = torch.randn(4, 96, 7, 5, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = _GlobalAvgPoolFn.apply(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    yr = torch.flatten(torch.nn.AdaptiveAvgPool2d((1, 1))(xr), 1)
    yr.backward(gy.float())
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-3)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)


def _r50_grads(dtype, native: bool, corrupt=None):
    """ResNet-50 parameter gradients at 96 x 96, batch 8, in ``dtype`` with our native ops on or off. Each residual
    branch's last BatchNorm starts at gamma = 0.2: a well-conditioned net (the default random init amplifies fp32
    rounding to a 2 % gradient spread even between stock fp32 and fp64: profiles/r6/diag_oracle_fp64.txt)."""
    from pytorch_distributed_training_example_amd.config import SW
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.resnet import Bottleneck
    if not native:
        os.environ["PDT_DISABLE_NATIVE"] = "1"
    SW.reload()
    try:
        torch.manual_seed(0)
        m = get_model("resnet50").cuda().to(memory_format=torch.channels_last).to(dtype)
        for b in m.modules():
            if isinstance(b, Bottleneck):
                torch.nn.init.constant_(b.bn3.weight, 0.2)
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(8, 3, 96, 96, device="cuda", generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (8,), device="cuda", generator=g)
        if corrupt is not None:
            corrupt(m)
        torch.nn.functional.cross_entropy(m(x), y).backward()
        return {k: p.grad.double().clone() for k, p in m.named_parameters()}
    finally:
        os.environ.pop("PDT_DISABLE_NATIVE", None)
        SW.reload()


def _oracle_errors(g, g64):
    big = max(float(v.norm()) for v in g64.values())
    return {k: float((g[k] - v).norm() / v.norm()) for k, v in g64.items() if float(v.norm()) > 1e-6 * big}


def check_fp32_native_against_fp64(corrupt=None):
    """(passed, message): fp32 ResNet-50 with native ops on, against the fp64 gradient of the same model and batch
    (stock PyTorch ops in float64 — no reduced-precision solver anywhere), next to stock fp32's own distance."""
    g64 = _r50_grads(torch.float64, native=False)
    en = _oracle_errors(_r50_grads(torch.float32, native=True, corrupt=corrupt), g64)
    es = _oracle_errors(_r50_grads(torch.float32, native=False), g64)
    worst = sorted(en, key=lambda k: -en[k])[:3]
    msg = "worst native: " + ", ".join(f"{k} {en[k]:.2e} (stock {es[k]:.2e})" for k in worst)
    med = sorted(en.values())[len(en) // 2]
    # fp32 rounding (MIOpen's fp32 convolution solvers included: 1e-6 .. 6e-3 from fp64 on this stack, solver
    # dependent) stays under 1e-2 per tensor; a wrong channel in one BatchNorm's backward or a dropped branch does
    # not (measured: median 2.2e-2, max 5.7e-2 with one of 256 channels dropped — tools/oracle_negative_check.py,
    # profiles/r6/oracle_negative_check.txt). Stock fp32's distance is reported, not bounded against: MIOpen picks
    # its fp32 solver per process, so stock and native land at 5e-6 or at 5e-3 independently of each other.
    ok = max(en.values()) < 1e-2 and med < 5e-3
    return ok, f"median {med:.2e} max {max(en.values()):.2e}; {msg}"


def test_resnet50_fp32_native_matches_fp64_oracle():
    """fp32 ResNet-50 with native ops enabled, against fp64. Round 5 found the bottleneck's residual-gradient link
    taken in fp32 (conv1's branch gradient dropped, the stem gradient 360x too small); the round-5 bound
    (median 5 % / max 50 % against stock fp32) was mostly oracle noise of an ill-conditioned random init."""
    ok, msg = check_fp32_native_against_fp64()
    print(msg)
    assert ok, msg


def test_resnet50_frozen_bn3_keeps_conv1_branch_gradient():
    """A training bottleneck whose bn3 is frozen (eval mode, running statistics) must not take the
    residual-gradient link: the eval BatchNorm returns the shortcut gradient through autograd, so the
    link stays empty and conv1's backward would park its branch gradient for a partner that never
    comes (models/resnet.py). Linked path on vs off: same gradients to bf16 noise."""
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models import resnet as R
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed

    def grads(link):
        R.RESIDUAL_GRAD_LINK[0] = link
        try:
            torch.manual_seed(0)
            m = to_bf16_mixed(get_model("resnet50", num_classes=16).cuda().to(memory_format=torch.channels_last))
            for mod in m.modules():
                if isinstance(mod, R.Bottleneck):
                    mod.bn3.eval()
            g = torch.Generator(device="cuda").manual_seed(2)
            x = torch.randn(4, 3, 96, 96, device="cuda", generator=g).bfloat16().contiguous(
                memory_format=torch.channels_last)
            y = torch.randint(0, 16, (4,), device="cuda", generator=g)
            torch.nn.functional.cross_entropy(m(x).float(), y).backward()
            return {k: p.grad.float().clone() for k, p in m.named_parameters()}
        finally:
            R.RESIDUAL_GRAD_LINK[0] = True

    ga, gb = grads(True), grads(False)
    ratio = float(ga["conv1.weight"].norm() / gb["conv1.weight"].norm())
    assert 0.9 < ratio < 1.1, ratio
    e = torch.tensor([float((ga[k] - gb[k]).norm() / gb[k].norm().clamp_min(1e-12)) for k in gb
                      if gb[k].norm() > 0])
    assert float(e.median()) < 2e-2, float(e.median())
