"""Our Linear GEMM with fused epilogues (csrc/kernels/gemm.hip) against an fp32 PyTorch reference:
C = A·Bᵀ, + bias (fp32 and bf16 bias), and the MLP's fc1 epilogue H = A·Bᵀ, G = gelu(H + bias) in
the erf (ViT) and tanh (GPT-2) forms; M tails (rows past M clamped, never stored); and the model
path behind PDT_LINEAR_EPILOGUE=1 (forward and every gradient vs the default path)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _C():
    from pytorch_distributed_training_example_amd.ops._native import native
    return native()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,K,N", [(256, 64, 256), (300, 128, 512), (1000, 768, 768), (4096, 1024, 3072),
                                   (25216 // 8, 3072, 768), (8192, 256, 3072), (1000, 128, 384)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_nt_matches_fp32(M, K, N, epi):
    g = torch.Generator(device="cuda").manual_seed(M + K + N + epi)
    a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    b = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) / K ** 0.5).bfloat16()
    bias = (torch.rand(N, device="cuda", generator=g) - 0.5)
    bias = bias.bfloat16() if epi == 1 else bias  # bf16 bias on the Linear path, fp32 on the MLP path
    ref = a.float() @ b.float().t()
    out = _C().gemm_nt(a, b, bias if epi else None, epi, N % 512 == 0)
    if epi == 1:
        ref = ref + bias.float()
    assert out[0].shape == (M, N) and out[0].dtype == torch.bfloat16
    assert _rel(out[0], ref) < 4e-3
    assert torch.isfinite(out[0].float()).all()
    if epi == 2:
        tanh = N % 512 == 0
        gref = F.gelu(out[0].float() + bias, approximate="tanh" if tanh else "none")
        assert _rel(out[1], gref) < 4e-3
        assert (out[1].float() - gref).abs().max().item() < 2e-2


def test_gemm_nt_refuses_unsupported_shape():
    a = torch.zeros(64, 100, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(256, 100, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        _C().gemm_nt(a, b, None, 0, False)


@pytest.mark.parametrize("approximate", ["none", "tanh"])
def test_mlp_on_fused_epilogue_matches_default_path(switch, approximate):
    from pytorch_distributed_training_example_amd.models.transformer import MLP
    torch.manual_seed(0)
    mlp = MLP(256, 1024, approximate).cuda().bfloat16()
    x = torch.randn(4, 100, 256, device="cuda").bfloat16()
    outs = []
    for flag in ("0", "1"):
        switch("PDT_LINEAR_EPILOGUE", flag)
        xi = x.clone().requires_grad_(True)
        mlp.zero_grad(set_to_none=True)
        y = mlp(xi)
        (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        outs.append([y.detach(), xi.grad] + [p.grad for p in mlp.parameters()])
    for a, b in zip(outs[0], outs[1]):
        assert _rel(b, a) < 1e-2, _rel(b, a)



def test_linear_per_shape_dispatch(switch):
    """PDT_LINEAR_EPILOGUE=auto (ops/linear.py _ours): every forward Linear GEMM shape is decided once — table
    or timing — between our MFMA kernel and hipBLASLt; both give the same result to bf16 accuracy, and the
    fused fc1 + bias + GELU kind is decided separately."""
    import torch.nn.functional as F
    from pytorch_distributed_training_example_amd.ops import linear as L
    switch("PDT_LINEAR_EPILOGUE", "auto")
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(4, 197, 768, device="cuda", generator=g).bfloat16()
    w = (torch.randn(2304, 768, device="cuda", generator=g) * 0.03).bfloat16()
    b = torch.randn(2304, device="cuda", generator=g).bfloat16()
    y = L.linear(x, w, b)
    torch.testing.assert_close(y.float(), F.linear(x.float(), w.float(), b.float()), rtol=2e-2, atol=2e-2)
    key = f"bias,{4 * 197},2304,768"
    assert L.linear_choices().get(key) in ("ours", "lib"), L.linear_choices()
    for forced in ("ours", "lib"):
        L._LIN_CHOICE[key] = forced
        torch.testing.assert_close(L.linear(x, w, b).float(), y.float(), rtol=2e-2, atol=2e-2)
    w1 = (torch.randn(3072, 768, device="cuda", generator=g) * 0.03).bfloat16()
    b1 = torch.randn(3072, device="cuda", generator=g)
    gl = L.linear_gelu(x, w1, b1, "tanh")
    ref = F.gelu(F.linear(x.float(), w1.float(), b1), approximate="tanh")
    if gl is not None:
        torch.testing.assert_close(gl.float(), ref, rtol=3e-2, atol=3e-2)
    assert L.linear_choices().get(f"gelu,{4 * 197},3072,768") in ("ours", "lib")
