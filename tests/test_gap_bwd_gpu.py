"""ResNet head: the global-average-pool gradient on our kernel (batchnorm.hip gap_bwd_kernel) — dy bit-identical
to PyTorch's bf16 (g / HW) broadcast, the pooled BatchNorm's backward partials equal to an fp64 reduction, and a
ResNet-50 step's gradients with the kernel on (PDT_GAP_NATIVE=1, the last bn3 skipping its reduce pass) matching
the PyTorch path."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C,H,W", [(4, 2048, 7, 7), (3, 512, 5, 3), (2, 64, 4, 4), (4, 96, 7, 5)])
def test_gap_bwd_kernel(N, C, H, W):
    from pytorch_distributed_training_example_amd.ops._native import native
    g = torch.Generator(device="cuda").manual_seed(C + H)
    gy = torch.randn(N, C, device="cuda", generator=g).bfloat16()
    x = torch.randn(N, C, H, W, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    mean = x.float().mean((0, 2, 3))
    pos = (torch.rand(N, C, H, W, device="cuda", generator=g) > 0.4)
    bits = pos.permute(0, 2, 3, 1).reshape(-1, 8).to(torch.int32)
    mask = (bits << torch.arange(8, device="cuda", dtype=torch.int32)).sum(1).to(torch.uint8)
    want = (gy * (1.0 / (H * W))).view(N, C, 1, 1).expand(N, C, H, W).contiguous(memory_format=torch.channels_last)
    assert torch.equal(native().gap_bwd(gy, H, W)[0], want)
    r = native().gap_bwd(gy, H, W, x, mask, mean)
    if 256 % (C // 8):  # the reduction needs a fixed channel chunk per thread: dy only
        assert len(r) == 1 and torch.equal(r[0], want)
        return
    # with the BatchNorm reduction, dy is stored masked by that BatchNorm's ReLU bits (tile_stats.h mask8)
    assert torch.equal(r[0], want * pos)
    part = r[1]
    dz = want.double() * pos.double()
    s1 = dz.sum((0, 2, 3))
    s2 = (dz * (x.double() - mean.double().view(1, C, 1, 1))).sum((0, 2, 3))
    torch.testing.assert_close(part[0].double().sum(0), s1, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(part[1].double().sum(0), s2, rtol=1e-4, atol=1e-5)


def test_resnet50_grads_with_native_gap(switch):
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops import batchnorm as B
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    torch.manual_seed(0)
    m = to_bf16_mixed(get_model("resnet50", num_classes=16).cuda().to(memory_format=torch.channels_last))
    x = torch.randn(8, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 16, (8,), device="cuda")
    deposits = []
    orig = B.GradStatsSource.deposit

    def spy(self, part, grad, **kw):
        deposits.append(tuple(grad.shape))
        return orig(self, part, grad, **kw)
    switch("PDT_BWD_ALG", "0")  # the last block's conv3 + bn3 backward the same both ways (ALG needs the masked
    out = {}                    # gradient the kernel stores; tests/test_bwd_alg_gpu.py covers that path)
    for on in ("1", "0"):
        switch("PDT_GAP_NATIVE", on)
        deposits.clear()
        B.GradStatsSource.deposit = spy
        try:
            m.zero_grad(set_to_none=True)
            cross_entropy(m(x), y).backward()
        finally:
            B.GradStatsSource.deposit = orig
        out[on] = ([p.grad.float().clone() for p in m.parameters()], list(deposits))
    # one more [8, 2048, 2, 2] deposit with the kernel on: the pool gradient's (the layer-4 dgrads deposit too)
    assert out["1"][1].count((8, 2048, 2, 2)) == out["0"][1].count((8, 2048, 2, 2)) + 1, (out["1"][1], out["0"][1])
    for a, b in zip(out["1"][0], out["0"][0]):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 1e-2, err
