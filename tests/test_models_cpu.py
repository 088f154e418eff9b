"""CPU checks of model building blocks whose GPU path is a reformulation (patch embedding as a GEMM)."""


def test_patch_conv_gemm_path_matches_conv2d(monkeypatch):
    """PatchConv2d's patchify + GEMM formulation (the GPU path, forced here on CPU fp32) equals
    nn.Conv2d with kernel == stride: output, weight and bias gradients; the returned [B, D, gh, gw]
    view flattens to a contiguous token sequence."""
    import torch
    from torch import nn
    from pytorch_distributed_training_example_amd.ops.conv import PatchConv2d
    torch.manual_seed(0)
    ref = nn.Conv2d(3, 32, kernel_size=8, stride=8)
    m = PatchConv2d(3, 32, kernel_size=8, stride=8)
    m.load_state_dict(ref.state_dict())
    monkeypatch.setattr(PatchConv2d, "_patch_ok", lambda self, x: True)
    x = torch.randn(2, 3, 35, 40)  # crops to 32 x 40 like the strided conv
    y, yr = m(x), ref(x)
    assert y.shape == yr.shape
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    assert y.flatten(2).transpose(1, 2).is_contiguous()
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(m.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-4)
