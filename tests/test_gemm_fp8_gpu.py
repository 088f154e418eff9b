"""Our fp8 MFMA GEMM (csrc/kernels/gemm.hip F8: block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 with unit block
scales, per-tensor dequantisation scales in the epilogue) against a plain PyTorch fp32 product of the
dequantised e4m3 operands, and against torch._scaled_mm (hipBLASLt) on the same operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _q(shape, g, scale):
    x = torch.randn(*shape, device="cuda", generator=g) * scale
    return x.clamp(-440, 440).to(torch.float8_e4m3fn)


@pytest.mark.parametrize("M,N,K", [(256, 128, 128), (300, 256, 256), (1000, 384, 768), (4096, 3072, 1024),
                                   (25216, 768, 768), (2048, 256, 4096),
                                   # weight-gradient shapes (few output tiles, long K): split-K + reduce pass
                                   (2304, 768, 25216), (768, 768, 25216), (1024, 4096, 8192), (200, 128, 2048)])
@pytest.mark.parametrize("bias", [None, "f32", "bf16"])
def test_gemm_nt_fp8_matches_fp32_reference(M, N, K, bias):
    from pytorch_distributed_training_example_amd.ops._native import native
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a, b = _q((M, K), g, 8.0), _q((N, K), g, 4.0)
    sa = torch.tensor([0.03], device="cuda")
    sb = torch.tensor([0.5], device="cuda")
    bv = None
    if bias is not None:
        bv = torch.randn(N, device="cuda", generator=g)
        bv = bv if bias == "f32" else bv.bfloat16()
    out = native().gemm_nt_fp8(a, b, sa, sb, bv)
    assert out.shape == (M, N) and out.dtype == torch.bfloat16
    ref = (a.float() * sa) @ (b.float() * sb).t()
    if bv is not None:
        ref = ref + bv.float()
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err  # bf16 output rounding; the fp32 accumulation itself is exact to ~1e-6
    # and hipBLASLt's fp8 GEMM on the same operands
    if K % 16 == 0 and N % 16 == 0:
        lib = torch._scaled_mm(a, b.t(), scale_a=sa, scale_b=sb, bias=bv if bias == "bf16" else None,
                               out_dtype=torch.bfloat16)
        if bias == "f32":
            lib = (lib.float() + bv).bfloat16()
        err2 = (out.float() - lib.float()).abs().max().item() / ref.abs().max().item()
        assert err2 < 1e-2, err2


def test_gemm_nt_fp8_refuses_unsupported_shape():
    from pytorch_distributed_training_example_amd.ops._native import native
    a = torch.zeros(256, 64, device="cuda").to(torch.float8_e4m3fn)  # K % 128 != 0
    b = torch.zeros(128, 64, device="cuda").to(torch.float8_e4m3fn)
    one = torch.ones(1, device="cuda")
    with pytest.raises(RuntimeError):
        native().gemm_nt_fp8(a, b, one, one)
