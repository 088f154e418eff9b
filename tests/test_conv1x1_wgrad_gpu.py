"""Our 1x1-conv weight-gradient kernel (csrc/kernels/conv1x1_wgrad.hip) against an fp32 PyTorch
reference dW = dY^T X, on every channel-block configuration (64x64, 256x64, 64x256, 128x256),
multi-block shapes, pixel counts that are not a multiple of the 32-pixel stage, and through the
Conv1x1 module's backward (the ResNet-50 layer-1 path that replaced MIOpen's igemm_wrw)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (M, Ci, Co): layer-1 blocks, multi-block (nblk > 1), ragged M, small split counts
SHAPES = [(4096, 64, 64), (8192, 64, 256), (8192, 256, 64), (4096, 256, 128), (1000, 64, 256),
          (777, 128, 512), (50000, 256, 64), (96, 512, 256), (3000, 192, 320)]


def _native():
    from pytorch_distributed_training_example_amd.ops._native import native
    return native()


@pytest.mark.parametrize("M,Ci,Co", SHAPES)
def test_wgrad_matches_fp32(M, Ci, Co):
    g = torch.Generator(device="cuda").manual_seed(M + Ci + Co)
    x = torch.randn(M, Ci, device="cuda", generator=g).bfloat16()
    dy = torch.randn(M, Co, device="cuda", generator=g).bfloat16()
    dw = _native().conv1x1_wgrad(x, dy)
    assert dw is not None and dw.shape == (Co, Ci) and dw.dtype == torch.bfloat16
    ref = dy.float().t() @ x.float()
    # fp32 accumulation, one bf16 rounding of the result
    tol = 2e-2 * M ** 0.5
    torch.testing.assert_close(dw.float(), ref, rtol=1e-2, atol=tol * 0.05)


def test_wgrad_deterministic():
    x = torch.randn(20000, 64, device="cuda").bfloat16()
    dy = torch.randn(20000, 256, device="cuda").bfloat16()
    a = _native().conv1x1_wgrad(x, dy)
    b = _native().conv1x1_wgrad(x, dy)
    assert torch.equal(a, b)


def test_wgrad_target_wgs_invariant_values():
    """Split count changes only the fp32 summation order: results agree to rounding."""
    x = torch.randn(16384, 64, device="cuda").bfloat16()
    dy = torch.randn(16384, 64, device="cuda").bfloat16()
    n = _native()
    base = n.conv1x1_wgrad(x, dy).float()
    n.conv1x1_wgrad_tune(7, -2, 1)
    try:
        other = n.conv1x1_wgrad(x, dy).float()
    finally:
        n.conv1x1_wgrad_tune(0, -2, -1)
    torch.testing.assert_close(other, base, rtol=1e-2, atol=0.5)


def test_conv1x1_module_weight_grad_on_ours(switch):
    """The Conv1x1 module's backward with the weight gradient forced onto our kernel equals the
    fp32 reference conv's weight gradient (channels_last bf16, ResNet layer-1-like shape)."""
    from pytorch_distributed_training_example_amd.ops.conv import Conv1x1
    switch("PDT_CONV1X1", "ours")
    torch.manual_seed(0)
    conv = Conv1x1(64, 256).cuda().bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(8, 64, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = conv(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    wf = conv.weight.detach().float().requires_grad_(True)
    out = torch.nn.functional.conv2d(x.detach().float(), wf)
    out.backward(gy.float())
    torch.testing.assert_close(conv.weight.grad.float(), wf.grad, rtol=2e-2, atol=0.3)
