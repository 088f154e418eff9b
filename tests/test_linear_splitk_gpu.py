"""Split-K Linear weight gradient (ops/linear.py ``_wgrad``: S bf16 batched GEMM partials + the
fp32-accumulating slice_sum kernel) against one fp32 GEMM, for every slice count the tuner may pick
(S in {1, 2, 4, 8, 16}) on ViT-B/16 / GPT-2-medium-like shapes. Each partial is rounded to bf16
before the fp32 sum, so the bound grows with sqrt(S) (independent rounding errors)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,n_out,n_in", [(4096, 768, 3072), (4096, 3072, 768), (8192, 1024, 1024)])
@pytest.mark.parametrize("S", [1, 2, 4, 8, 16])
def test_linear_wgrad_splitk_matches_fp32(T, n_out, n_in, S, switch):
    from pytorch_distributed_training_example_amd.ops import linear as L
    switch("PDT_LINEAR_SPLITK", "1")
    g = torch.Generator(device="cuda").manual_seed(T + S)
    dy = torch.randn(T, n_out, device="cuda", generator=g).bfloat16()
    x = torch.randn(T, n_in, device="cuda", generator=g).bfloat16()
    key = (T, n_out, n_in, dy.dtype)
    saved = L._WG_CHOICE.get(key)
    L._WG_CHOICE[key] = S  # force the slice count the timing would otherwise choose
    try:
        dw = L._wgrad(dy, x)
    finally:
        if saved is None:
            L._WG_CHOICE.pop(key, None)
        else:
            L._WG_CHOICE[key] = saved
    ref = dy.float().t() @ x.float()
    assert dw.shape == (n_out, n_in) and dw.dtype == torch.bfloat16
    # rigorous bound: each of the S partials is rounded to bf16 (<= 2^-9 of its own magnitude, which
    # can exceed |ref| where partials cancel), then one rounding of the result (rtol)
    pmax = (dy.float().view(S, T // S, n_out).transpose(1, 2) @ x.float().view(S, T // S, n_in)).abs().amax(0)
    atol = (S * 2 ** -9 * pmax).max().item() if S > 1 else 1e-3
    torch.testing.assert_close(dw.float(), ref, rtol=1e-2, atol=atol)
    # and typically far inside it: the mean error stays at the bf16-rounding level
    assert ((dw.float() - ref).abs().mean() / ref.abs().mean()).item() < 4e-3 * math.sqrt(S)
