"""Fused backward of a bottleneck's conv3 + bn3 (csrc/kernels/conv1x1_bwd_fused.hip) against fp32
PyTorch references of the same math: the BatchNorm backward apply formed on load, the 1x1 conv's data
and weight gradients, and the producing BatchNorm's backward partial sums; plus the coefficient-only
BatchNorm backward (bn_bwd_coef) against the full native backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _native():
    from pytorch_distributed_training_example_amd.ops._native import native
    return native()


def _bits(b: torch.Tensor) -> torch.Tensor:
    """bool [M*C] -> uint8 [M*C/8], bit j of byte k = element 8k + j (the BatchNorm mask layout)."""
    w = (1 << torch.arange(8, device=b.device, dtype=torch.int32))
    return (b.view(-1, 8).int() * w).sum(1).to(torch.uint8)


def _unbits(m: torch.Tensor) -> torch.Tensor:
    return ((m.view(-1, 1).int() >> torch.arange(8, device=m.device)) & 1).view(-1).bool()


def _nhwc(t2d, N, H, W):
    C = t2d.shape[1]
    return t2d.view(N, H, W, C).permute(0, 3, 1, 2)


@pytest.mark.parametrize("N,H,W", [(2, 56, 56), (3, 7, 7), (1, 5, 13), (16, 14, 14)])
@pytest.mark.parametrize("bstats", [True, False])
@pytest.mark.parametrize("C4,CW", [(256, 64), (512, 128)])
def test_fused_matches_fp32(N, H, W, bstats, C4, CW):
    M = N * H * W
    g = torch.Generator(device="cuda").manual_seed(M + bstats + C4)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    dy = r(M, C4).bfloat16()
    z = (r(M, C4) + 0.3).bfloat16()
    m3 = torch.rand(M * C4, device="cuda", generator=g) > 0.4
    mean = r(C4) * 0.1 + 0.3
    coef = torch.stack([r(C4).abs() + 0.5, r(C4) * 0.01, r(C4) * 0.01]).contiguous()
    w = (r(C4, CW) / 16).bfloat16().view(C4, CW, 1, 1)
    xa = r(M, CW).relu().bfloat16()
    xb = r(M, CW).bfloat16()
    mb = torch.rand(M * CW, device="cuda", generator=g) > 0.5
    meanb = r(CW) * 0.1
    args = [_nhwc(dy, N, H, W), _nhwc(z, N, H, W), _bits(m3), mean, coef, w, _nhwc(xa, N, H, W)]
    if bstats:
        out = _native().conv1x1_bwd_fused(*args, _nhwc(xb, N, H, W), _bits(mb), meanb)
    else:
        out = _native().conv1x1_bwd_fused(*args, None, None, None)
    assert len(out) == 3
    dxa, dw, part = out
    # fp32 reference (dz rounded to bf16 as the kernel stages it)
    gm = torch.where(m3.view(M, C4), dy.float(), 0.0)
    dz = (coef[0] * gm + coef[1] * (z.float() - mean) + coef[2]).bfloat16().float()
    ref_dxa = dz @ w.view(C4, CW).float()
    ref_dw = dz.t() @ xa.float()
    d2 = dxa.permute(0, 2, 3, 1).reshape(M, CW).float()
    torch.testing.assert_close(d2, ref_dxa, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(dw.view(C4, CW).float(), ref_dw, rtol=2e-2, atol=2e-2 * max(1.0, M ** 0.5 / 8))
    if bstats:
        gb = torch.where(mb.view(M, CW), d2, 0.0)
        s1, s2 = gb.sum(0), (gb * (xb.float() - meanb)).sum(0)
        assert part.shape[0] == 2 and part.shape[2] == CW
        torch.testing.assert_close(part[0].sum(0), s1, rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(part[1].sum(0), s2, rtol=1e-3, atol=1e-2)
    else:
        assert part is None


@pytest.mark.parametrize("C4,CW", [(256, 64), (512, 128)])
def test_fused_is_deterministic(C4, CW):
    N, H, W = 4, 28, 28
    M = N * H * W
    torch.manual_seed(0)
    dy = torch.randn(M, C4, device="cuda").bfloat16()
    z = torch.randn(M, C4, device="cuda").bfloat16()
    mz = _bits(torch.rand(M * C4, device="cuda") > 0.5)
    mean = torch.randn(C4, device="cuda")
    coef = torch.randn(3, C4, device="cuda")
    w = torch.randn(C4, CW, 1, 1, device="cuda").bfloat16()
    xa = torch.randn(M, CW, device="cuda").bfloat16()
    args = (_nhwc(dy, N, H, W), _nhwc(z, N, H, W), mz, mean, coef, w, _nhwc(xa, N, H, W),
            _nhwc(xa, N, H, W), None, mean[:CW].contiguous())
    a = _native().conv1x1_bwd_fused(*args)
    b = _native().conv1x1_bwd_fused(*args)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_unsupported_shape_returns_empty():
    t = torch.zeros(1, 128, 4, 4, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x = torch.zeros(1, 32, 4, 4, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.zeros(128, 32, 1, 1, device="cuda").bfloat16()
    out = _native().conv1x1_bwd_fused(t, t, torch.zeros(256, dtype=torch.uint8, device="cuda"),
                                      torch.zeros(128, device="cuda"), torch.zeros(3, 128, device="cuda"), w, x,
                                      None, None, None)
    assert out == []


@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("with_part", [False, True])
def test_bn_bwd_coef_matches_full_backward(relu, with_part):
    N, C, H, W = 4, 256, 14, 14
    M = N * H * W
    torch.manual_seed(1)
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(x)
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda")
    y, mask, mean, invstd = _native().bn_fwd_train(x, None, gamma, beta, None, None, 0.1, 1e-5, relu, None, True)
    dx, _, dg, db = _native().bn_bwd_train(dy, x, mask, gamma, mean, invstd, relu, False, True)
    part = None
    if with_part:  # the reduction as a producer epilogue would hand it over: [2, T, C]
        x2, g2 = x.permute(0, 2, 3, 1).reshape(M, C).float(), dy.permute(0, 2, 3, 1).reshape(M, C).float()
        if relu:
            g2 = torch.where(_unbits(mask).view(M, C), g2, 0.0)
        part = torch.stack([g2.view(4, -1, C).sum(1), (g2 * (x2 - mean)).view(4, -1, C).sum(1)]).contiguous()
    coef, dg2, db2 = _native().bn_bwd_coef(dy, x, part, mask, gamma, mean, invstd, relu, True)
    gm = dy.float()
    if relu:
        gm = torch.where(_unbits(mask).view(M, C).view(N, H, W, C).permute(0, 3, 1, 2), gm, 0.0)
    sh = (1, C, 1, 1)
    dx2 = coef[0].view(sh) * gm + coef[1].view(sh) * (x.float() - mean.view(sh)) + coef[2].view(sh)
    torch.testing.assert_close(dx2, dx.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(dg2, dg, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(db2, db, rtol=1e-3, atol=1e-3)


def _grads(seed=0):
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    torch.manual_seed(seed)
    m = to_bf16_mixed(get_model("resnet50").cuda().to(memory_format=torch.channels_last))
    x = torch.randn(8, 3, 96, 96, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (8,), device="cuda")
    loss = torch.nn.functional.cross_entropy(m(x).float(), y)
    loss.backward()
    return {n: p.grad.float().clone() for n, p in m.named_parameters()}


def test_resnet50_grads_fused_vs_unfused(switch):
    """The whole model's gradients with the fused conv3 + bn3 backward (layer 1) against the unfused
    kernel chain: same math, different rounding points (dz is rounded once, in LDS)."""
    from pytorch_distributed_training_example_amd.ops import conv as conv_ops
    calls = []
    orig = conv_ops._bwd_fused

    def spy(*a):
        r = orig(*a)
        calls.append(r is not None)
        return r
    conv_ops._bwd_fused = spy
    try:
        switch("PDT_BWD_FUSED", "1")
        ga = _grads()
    finally:
        conv_ops._bwd_fused = orig
    assert calls == [True] * 7, calls  # the three layer-1 and four layer-2 blocks, all on the fused kernel
    switch("PDT_BWD_FUSED", "0")
    gb = _grads()
    assert ga.keys() == gb.keys()
    for n in ga:
        a, b = ga[n], gb[n]
        rel = (a - b).norm() / b.norm().clamp_min(1e-12)
        assert rel < 2e-2, (n, float(rel))
