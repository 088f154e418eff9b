"""A BatchNorm(+residual)+ReLU apply run as the producing 1x1 conv's GEMM again with the apply epilogue
(csrc/kernels/conv1x1.hip APPLY, ops/batchnorm.py ``gemm``): the kernel against an fp32 PyTorch
reference, and whole bottleneck blocks with the path on / off (bit-identical: the GEMM recomputes the
same bf16 conv output and applies the same fp32 operations as the standalone apply pass)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,K,N,rab,atr", [(1000, 64, 256, False, False), (777, 128, 512, True, False),
                                           (513, 64, 64, False, True), (2048, 128, 512, True, True)])
def test_gemm_apply_matches_fp32(M, K, N, rab, atr):
    from pytorch_distributed_training_example_amd.ops._native import native
    g = torch.Generator(device="cuda").manual_seed(M + K)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    a = r(M, K).bfloat16()
    b = (r(N, K) / K ** 0.5).bfloat16()
    res = r(M, N).bfloat16()
    ab = torch.stack([r(N).abs() + 0.5, r(N) * 0.1])
    rabt = torch.stack([r(N).abs() + 0.5, r(N) * 0.1]) if rab else None
    acoef = torch.stack([r(K).abs() + 0.5, r(K) * 0.2]) if atr else None
    y, mask = native().conv1x1_gemm_apply(a, b, res, ab, rabt, acoef)
    af = a.float()
    if atr:
        af = (af * acoef[0] + acoef[1]).clamp_min(0).bfloat16().float()
    z = (af @ b.float().t()).bfloat16().float()  # the conv output as the first GEMM stored it
    rr = res.float() if rabt is None else res.float() * rabt[0] + rabt[1]
    t = z * ab[0] + ab[1] + rr
    want = t.clamp_min(0)
    err = (y.float() - want).norm() / want.norm()
    assert err < 1e-2, float(err)
    bits = (mask.view(-1, 1) >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1
    pos = bits.view(M, N).bool()
    sure = t.abs() > 0.05  # away from the ReLU threshold (z rounding differences)
    assert torch.equal(pos[sure], (t > 0)[sure])
    assert torch.equal(pos, y.float() > 0) or bool(((y.float() > 0) & ~pos).sum() == 0)


@pytest.mark.parametrize("defer", ["0", "1"])
@pytest.mark.parametrize("layer,block", [(1, 1), (1, 0), (2, 2)])
def test_bottleneck_apply_gemm_bit_identical(switch, layer, block, defer):
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops import batchnorm as bn_ops
    torch.manual_seed(0)
    net = to_bf16_mixed(get_model("resnet50").cuda().to(memory_format=torch.channels_last))
    blk = getattr(net, f"layer{layer}")[block]
    cin = blk.conv1.in_channels
    hw = 56 if layer == 1 else 28
    if block == 0 and layer > 1:
        hw *= 2
    g = torch.Generator(device="cuda").manual_seed(layer * 10 + block)
    x0 = torch.randn(4, cin, hw, hw, device="cuda", generator=g).relu().bfloat16()
    x0 = x0.contiguous(memory_format=torch.channels_last)
    calls = []
    orig = bn_ops.native

    def run(k):
        switch("PDT_BN_APPLY_GEMM_K", k)
        switch("PDT_BN2_DEFER", defer)
        blk.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        y = blk(x)
        gy = torch.randn(y.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5)).bfloat16()
        y.backward(gy.contiguous(memory_format=torch.channels_last))
        return [y.detach(), x.grad] + [p.grad.clone() for p in blk.parameters()]

    class Spy:
        def __getattr__(self, n):
            if n == "conv1x1_gemm_apply":
                calls.append(1)
            return getattr(orig(), n)
    bn_ops.native = lambda: Spy()
    try:
        a = run("128")
    finally:
        bn_ops.native = orig
    assert calls, "the GEMM apply path did not run"
    b = run("0")
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), (i, float((u.float() - v.float()).abs().max()))
