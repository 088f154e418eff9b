"""Stride-2 3x3 convolution on our MFMA kernels (csrc/kernels/conv3x3_s2.hip forward / 4-phase data
gradient, csrc/kernels/conv3x3_wgrad.hip at S = 2) against an fp32 PyTorch conv of the same bf16
inputs, plus the fused BatchNorm epilogues (forward statistics, backward reduction)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("N,C_in,C_out,H,W", [(2, 128, 128, 56, 56), (3, 256, 256, 28, 28), (4, 512, 512, 14, 14),
                                              (2, 128, 256, 13, 11), (1, 256, 128, 2, 2), (2, 128, 128, 9, 30),
                                              (3, 64, 128, 24, 24), (2, 64, 64, 17, 20), (2, 128, 64, 30, 30)])
def test_conv3x3s2_ours_matches_fp32(N, C_in, C_out, H, W, switch):
    from pytorch_distributed_training_example_amd.ops._native import native
    from pytorch_distributed_training_example_amd.ops.conv import SplitConv2d, conv3x3s2_eligible
    switch("PDT_CONV3X3_S2", "ours")
    torch.manual_seed(0)
    m = SplitConv2d(C_in, C_out, 3, stride=2, padding=1, bias=False).cuda().bfloat16().to(
        memory_format=torch.channels_last)
    x = torch.randn(N, C_in, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    assert conv3x3s2_eligible(m, x)
    x.requires_grad_(True)
    y = m(x)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    assert y.shape == (N, C_out, Ho, Wo) and y.is_contiguous(memory_format=torch.channels_last)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    wr = m.weight.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=2, padding=1)
    yr.backward(gy.float())
    for name, a, b in (("y", y, yr), ("dx", x.grad, xr.grad), ("dw", m.weight.grad, wr.grad)):
        err = _rel(a, b)
        assert err < 1e-2, (name, err)
    # forward and data gradient came from our kernels, bit for bit
    gyc = gy.contiguous(memory_format=torch.channels_last)
    assert torch.equal(native().conv3x3s2_fwd(x.detach(), m.weight, False)[0], y)
    assert torch.equal(native().conv3x3s2_dgrad(gyc, native().conv3x3_flip(m.weight), H, W)[0], x.grad)
    dw = native().conv3x3s2_wgrad(x.detach(), gyc)
    if (H, W) != (13, 11) and (H, W) != (9, 30):  # shapes the S = 2 weight-gradient kernel is sized for
        assert dw is not None and torch.equal(dw, m.weight.grad), "stride-2 weight gradient not on our kernel"


@pytest.mark.parametrize("co_tile", [64, 128])
def test_conv3x3s2_wgrad_co_tiles(co_tile):
    """Both workgroup shapes of the stride-2 weight gradient (CO_T 128: prefetching 8-wave workgroup;
    CO_T 64: two 4-wave workgroups per CU) on every ResNet-50 stride-2 shape, small batch."""
    from pytorch_distributed_training_example_amd.ops._native import native
    torch.manual_seed(1)
    try:
        native().conv3x3_wgrad_tune(-1, co_tile)
        for C, H in ((128, 56), (256, 28), (512, 14)):
            x = torch.randn(2, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            gy = torch.randn(2, C, H // 2, H // 2, device="cuda").bfloat16().contiguous(
                memory_format=torch.channels_last)
            dw = native().conv3x3s2_wgrad(x, gy)
            assert dw is not None
            xr = x.float().requires_grad_(True)
            wr = torch.zeros(C, C, 3, 3, device="cuda", requires_grad=True)
            F.conv2d(xr, wr, stride=2, padding=1).backward(gy.float())
            assert _rel(dw, wr.grad) < 1e-2, (C, H, co_tile)
    finally:
        native().conv3x3_wgrad_tune(-1, 0)


@pytest.mark.parametrize("C,Co", [(128, 256), (64, 64)])
def test_conv3x3s2_fused_bn_epilogues(C, Co):
    """Forward statistics (per-tile sum, centred sum of squares of the bf16 output) and the 4-phase
    data gradient's BatchNorm backward partials (sum dz, sum dz (x - mean), dz = dx * ReLU mask)
    against direct reductions."""
    from pytorch_distributed_training_example_amd.ops._native import native
    torch.manual_seed(2)
    N, H = 3, 28
    x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, C, 3, 3, device="cuda") / 30).bfloat16().contiguous(memory_format=torch.channels_last)
    y, part = native().conv3x3s2_fwd(x, w, True)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, Co)
    M = yf.shape[0]
    T = (M + 255) // 256
    assert part.shape == (2, T, Co)
    s = part[0].sum(0)
    q = part[1].double().sum(0) + (part[0].double() ** 2 / torch.tensor(
        [min(256, M - 256 * t) for t in range(T)], device="cuda", dtype=torch.float64).view(-1, 1)).sum(0)
    torch.testing.assert_close(s, yf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(q.float(), (yf.double() ** 2).sum(0).float(), rtol=1e-3, atol=1e-1)
    # data gradient with the producing BatchNorm's backward reduction
    gy = torch.randn(N, Co, H // 2, H // 2, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    bn_x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    mean = bn_x.float().mean((0, 2, 3)).contiguous()
    relu_bits = (torch.rand(N * H * H * C, device="cuda") > 0.3)
    mask = (relu_bits.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(
        1).to(torch.uint8)
    wf = native().conv3x3_flip(w)
    dx, bpart = native().conv3x3s2_dgrad(gy, wf, H, H, bn_x=bn_x, bn_mask=mask, bn_mean=mean)
    assert torch.equal(dx, native().conv3x3s2_dgrad(gy, wf, H, H)[0])
    dz = dx.float().permute(0, 2, 3, 1).reshape(-1, C) * relu_bits.view(-1, C).float()
    xc = bn_x.float().permute(0, 2, 3, 1).reshape(-1, C) - mean
    torch.testing.assert_close(bpart[0].sum(0), dz.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(bpart[1].sum(0), (dz * xc).sum(0), rtol=1e-3, atol=1e-2)


def test_resnet50_stride2_blocks_use_our_kernels(switch):
    """A ResNet-50 train step routes the three stride-2 3x3 convs through _Conv3x3S2Fn (no MIOpen
    conv call for them) and matches the MIOpen-routed step's loss."""
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops import conv as C
    losses = {}
    for mode in ("ours", "miopen"):
        switch("PDT_CONV3X3_S2", mode)
        torch.manual_seed(0)
        model = to_bf16_mixed(get_model("resnet50").cuda().to(memory_format=torch.channels_last))
        calls = []
        orig = C._Conv3x3S2Fn.apply

        def spy(*a):
            calls.append(a[0].shape)
            return orig(*a)
        C._Conv3x3S2Fn.apply = spy
        try:
            x = torch.randn(4, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            loss = model(x).float().logsumexp(1).mean()
            loss.backward()
        finally:
            C._Conv3x3S2Fn.apply = orig
        losses[mode] = loss.item()
        assert len(calls) == (3 if mode == "ours" else 0), calls
    assert abs(losses["ours"] - losses["miopen"]) < 2e-2 * abs(losses["miopen"]), losses
