"""LeNet fused kernels (csrc/kernels/lenet.hip) vs fp32 PyTorch references of the same ops."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _close(a, b, tol=1e-4):
    torch.testing.assert_close(a.float(), b.float(), rtol=tol, atol=tol)


@pytest.mark.parametrize("n", [1, 7, 128])
def test_stem_fwd_bwd(n):
    from pytorch_distributed_training_example_amd.ops.lenet import lenet_stem, stem_reference
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, 1, 28, 28, device="cuda", generator=g)
    w = (torch.randn(6, 1, 5, 5, device="cuda", generator=g) * 0.2).requires_grad_()
    b = (torch.randn(6, device="cuda", generator=g) * 0.1).requires_grad_()
    y = lenet_stem(x, w, b)
    w2, b2 = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = stem_reference(x, w2, b2)
    _close(y, yr)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    _close(w.grad, w2.grad, 2e-3)
    _close(b.grad, b2.grad, 2e-3)


@pytest.mark.parametrize("shape", [(64, 16, 10, 10), (2, 3, 7, 9)])
def test_leaky_pool_fwd_bwd(shape):
    from pytorch_distributed_training_example_amd.ops.lenet import leaky_pool, leaky_pool_reference
    x = torch.randn(*shape, device="cuda", requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    y, yr = leaky_pool(x), leaky_pool_reference(xr)
    _close(y, yr, 0)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    _close(x.grad, xr.grad, 1e-6)


@pytest.mark.parametrize("mode", ["ce", "prob_nll"])
@pytest.mark.parametrize("v,dtype", [(10, torch.float32), (1000, torch.float32), (100, torch.bfloat16)])
def test_softmax_nll(mode, v, dtype):
    from pytorch_distributed_training_example_amd.ops.lenet import softmax_nll, softmax_nll_reference
    g = torch.Generator(device="cuda").manual_seed(v)
    z = (torch.randn(257, v, device="cuda", generator=g) * 3).to(dtype).requires_grad_()
    t = torch.randint(0, v, (257,), device="cuda", generator=g)
    zr = z.detach().float().clone().requires_grad_()
    ls = 0.1 if mode == "ce" else 0.0
    l, lr = softmax_nll(z, t, mode, ls), softmax_nll_reference(zr, t, mode, ls)
    _close(l, lr, 1e-4)
    (l * 3).backward()
    (lr * 3).backward()
    _close(z.grad, zr.grad, 1e-2 if dtype == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("mode", ["ce", "prob_nll"])
def test_eval_metrics(mode):
    from pytorch_distributed_training_example_amd.ops.lenet import eval_metrics_
    z = torch.randn(1000, 10, device="cuda")
    t = torch.randint(0, 10, (1000,), device="cuda")
    acc = torch.zeros(3, dtype=torch.float64, device="cuda")
    eval_metrics_(acc, z[:600], t[:600], mode)
    eval_metrics_(acc, z[600:], t[600:], mode)
    ref = torch.zeros(3, dtype=torch.float64)
    eval_metrics_(ref, z.cpu(), t.cpu(), mode)
    torch.testing.assert_close(acc.cpu(), ref, rtol=1e-5, atol=1e-4)


def test_lenet_fused_matches_module_path():
    from pytorch_distributed_training_example_amd.models import LeNet
    torch.manual_seed(0)
    m = LeNet(output="logits").cuda()
    ref = LeNet(output="logits", fused=False).cuda()
    ref.load_state_dict(m.state_dict())
    x = torch.randn(96, 1, 28, 28, device="cuda")
    t = torch.randint(0, 10, (96,), device="cuda")
    out, outr = m(x), ref(x)
    _close(out, outr, 1e-4)
    torch.nn.functional.cross_entropy(out, t).backward()
    torch.nn.functional.cross_entropy(outr, t).backward()
    for (n, p), pr in zip(m.named_parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, pr.grad, rtol=2e-3, atol=2e-4, msg=n)


def _tail_params(g):
    from pytorch_distributed_training_example_amd.ops.lenet import _TAIL_SHAPES
    ps = []
    for s in _TAIL_SHAPES:
        fan = 1
        for d in s[1:]:
            fan *= d
        ps.append((torch.randn(*s, device="cuda", generator=g) / max(fan, 1) ** 0.5).requires_grad_())
    return ps


@pytest.mark.parametrize("n", [1, 5, 128])
def test_tail_fwd_bwd_matches_fp32(n):
    """conv2 + pool + conv3 + fc1 + fc2 (csrc/kernels/lenet_tail.hip) against the aten ops in fp32:
    logits, every parameter gradient and the gradient of the stem output."""
    from pytorch_distributed_training_example_amd.ops.lenet import lenet_tail, tail_reference
    g = torch.Generator(device="cuda").manual_seed(100 + n)
    p1 = torch.randn(n, 6, 14, 14, device="cuda", generator=g).requires_grad_()
    ps = _tail_params(g)
    p1r = p1.detach().clone().requires_grad_()
    psr = [p.detach().clone().requires_grad_() for p in ps]
    y, yr = lenet_tail(p1, ps), tail_reference(p1r, psr)
    _close(y, yr, 1e-4)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    _close(p1.grad, p1r.grad, 1e-4)
    for a, b in zip(ps, psr):
        _close(a.grad, b.grad, 2e-4 * max(1, n) ** 0.5)


def test_lenet_model_fused_matches_modules():
    """The whole reference model on our kernels (stem + tail) vs the plain nn.Sequential path."""
    import copy
    from pytorch_distributed_training_example_amd.models.lenet import LeNet
    torch.manual_seed(0)
    m = LeNet(output="probs").cuda()
    mr = copy.deepcopy(m)
    mr.fused = False
    x = torch.randn(64, 1, 28, 28, device="cuda")
    t = torch.randint(0, 10, (64,), device="cuda")
    y, yr = m(x), mr(x)
    _close(y, yr, 1e-5)
    torch.nn.functional.nll_loss(y, t).backward()
    torch.nn.functional.nll_loss(yr, t).backward()
    for (na, a), (_, b) in zip(m.named_parameters(), mr.named_parameters()):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-3, atol=1e-5, msg=na)
