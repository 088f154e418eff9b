"""The persistent 1x1-conv GEMM (csrc/kernels/conv1x1.hip conv1x1p_kernel) at HEADLINE grid sizes.

The persistent kernel walks ~50 tiles per workgroup and prefetches tile t+1's operands while tile t's
epilogue runs, with hand-counted vmcnt waits; any miscount shows up as a wrong tile. Every epilogue
variant (plain, STATS, ATR, masked accumulate + BSTATS, strided accumulate, APPLY) runs at the ResNet-50
batch-1024 grid sizes — thousands of tiles, so well above the >= 2048-workgroup threshold of the 16-wave
tile (round-4 VERDICT: no test reached it) — and must equal the one-tile-per-workgroup kernel BIT FOR BIT
in its output (same k order, same epilogue arithmetic), match an fp32 oracle, and give the same tile
statistics (to fp32 reduction-order tolerance: the 16- and 8-wave tiles sum their rows in different
orders). Mode 2 (the 16-wave tile persistent too) is checked the same way."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (M, K, N): ResNet-50 at 1024 images — layer-1 conv3 fwd (64->256, M = 3.2M), layer-2 (128->512),
# layer-3 (256->1024), the matching dgrads, a narrow 64-channel output, and a ragged M
SHAPES = [(1024 * 56 * 56, 64, 256), (1024 * 28 * 28, 128, 512), (1024 * 14 * 14, 256, 1024),
          (1024 * 56 * 56, 256, 64), (1024 * 28 * 28 - 37, 512, 128), (300_001, 64, 64)]


def _n():
    from pytorch_distributed_training_example_amd.ops._native import native
    return native()


def _modes(fn):
    """fn() under persistence modes 0 (one tile per workgroup), 1 (default) and 2."""
    n = _n()
    old = n.conv1x1_persist(0)
    try:
        out = {}
        for mode in (0, 1, 2):
            n.conv1x1_persist(mode)
            out[mode] = fn()
            torch.cuda.synchronize()
        return out
    finally:
        n.conv1x1_persist(old)


def _data(M, K, N, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    return a, b, g


def _oracle_rows(a, b, rows):
    return a[rows].float() @ b.float().t()


def _rows(M):
    return torch.cat([torch.arange(0, 4096), torch.randint(4096, M - 4096, (8192,)), torch.arange(M - 4096, M)]).cuda()


@pytest.mark.parametrize("M,K,N", SHAPES)
def test_fwd_stats_persistent_equals_per_tile(M, K, N):
    a, b, _ = _data(M, K, N, 1)
    a = a + 0.25

    def run():
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        part = _n().conv1x1_gemm(a, b, y, False, True)
        return y, part
    r = _modes(run)
    for mode in (1, 2):
        assert torch.equal(r[mode][0], r[0][0]), f"mode {mode}: output differs from the per-tile kernel"
        torch.testing.assert_close(r[mode][1], r[0][1], rtol=1e-4, atol=1e-2)
    rows = _rows(M)
    torch.testing.assert_close(r[1][0][rows].float(), _oracle_rows(a, b, rows), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,K,N", SHAPES[:3])
def test_fwd_atr_persistent_equals_per_tile(M, K, N):
    """ATR: A = relu(a x + b) formed on load (bn2 -> conv3, the deferred BatchNorm apply)."""
    a, b, g = _data(M, K, N, 2)
    coef = torch.stack([torch.rand(K, device="cuda", generator=g) + 0.5, torch.randn(K, device="cuda", generator=g)])

    def run():
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        part = _n().conv1x1_gemm(a, b, y, False, True, a_coef=coef.contiguous())
        return y, part
    r = _modes(run)
    for mode in (1, 2):
        assert torch.equal(r[mode][0], r[0][0])
        torch.testing.assert_close(r[mode][1], r[0][1], rtol=1e-4, atol=1e-2)
    rows = _rows(M)
    ax = torch.relu(a[rows].float() * coef[0] + coef[1]).bfloat16().float()
    torch.testing.assert_close(r[1][0][rows].float(), ax @ b.float().t(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,K,N", [(1024 * 56 * 56, 64, 256), (1024 * 28 * 28, 128, 512),
                                   (1024 * 14 * 14, 256, 1024), (1024 * 56 * 56, 256, 64)])
def test_dgrad_masked_acc_bstats_persistent_equals_per_tile(M, K, N):
    """dX = dY W + dres * mask with the producing BatchNorm's backward reduction (BSTATS) in the epilogue:
    the conv1 data gradient of a ResNet identity block at batch 1024."""
    a, b, g = _data(M, K, N, 3)
    dres = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    cmask = torch.randint(0, 256, (M * N // 8,), device="cuda", generator=g, dtype=torch.int32).to(torch.uint8)
    bx = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    bmask = torch.randint(0, 256, (M * N // 8,), device="cuda", generator=g, dtype=torch.int32).to(torch.uint8)
    bmean = torch.randn(N, device="cuda", generator=g)

    def run():
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        part = _n().conv1x1_gemm(a, b, y, True, False, dres, cmask, bx, bmask, bmean)
        return y, part
    r = _modes(run)
    for mode in (1, 2):
        assert torch.equal(r[mode][0], r[0][0])
        torch.testing.assert_close(r[mode][1], r[0][1], rtol=1e-4, atol=5e-2)
    rows = _rows(M)
    bits = torch.arange(8, device="cuda")
    mexp = ((cmask.view(M, N // 8)[rows].long()[..., None] >> bits) & 1).view(len(rows), N).float()
    bexp = ((bmask.view(M, N // 8)[rows].long()[..., None] >> bits) & 1).view(len(rows), N).float()
    # stored masked by the BatchNorm's ReLU bits (BSTATS, tile_stats.h mask8)
    ref = (_oracle_rows(a, b, rows) + dres[rows].float() * mexp) * bexp
    torch.testing.assert_close(r[1][0][rows].float(), ref, rtol=2e-2, atol=3e-2)


def test_dgrad_strided_acc_bstats_persistent_equals_per_tile():
    """The transition block's dgrad: the stride-2 shortcut's compact gradient added at the sampled
    pixels (STR instantiation) with the BatchNorm backward reduction."""
    Nb, H, W, K, N, s = 1024, 28, 28, 128, 512, 2
    M = Nb * H * W
    a, b, g = _data(M, K, N, 4)
    Hs, Ws = (H - 1) // s + 1, (W - 1) // s + 1
    comp = torch.randn(Nb * Hs * Ws, N, device="cuda", generator=g).bfloat16()
    bx = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    bmean = torch.randn(N, device="cuda", generator=g)

    def run():
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        part = _n().conv1x1_gemm(a, b, y, True, False, comp, None, bx, None, bmean, s, H, W)
        return y, part
    r = _modes(run)
    for mode in (1, 2):
        assert torch.equal(r[mode][0], r[0][0])
        torch.testing.assert_close(r[mode][1], r[0][1], rtol=1e-4, atol=5e-2)
    full = torch.zeros(Nb, H, W, N, device="cuda")
    full[:, ::s, ::s] = comp.float().view(Nb, Hs, Ws, N)
    rows = _rows(M)
    ref = _oracle_rows(a, b, rows) + full.view(M, N)[rows]
    torch.testing.assert_close(r[1][0][rows].float(), ref, rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("deferred_res", [False, True])
@pytest.mark.parametrize("M,K,N", [(1024 * 56 * 56, 64, 256), (1024 * 28 * 28, 128, 512)])
def test_apply_persistent_equals_per_tile(M, K, N, deferred_res):
    """APPLY: relu(a z + b + r) and its ReLU bits written by the recomputed GEMM (bn3 of a bottleneck)."""
    a, b, g = _data(M, K, N, 5)
    res = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    ab = torch.stack([torch.rand(N, device="cuda", generator=g) + 0.5, torch.randn(N, device="cuda", generator=g)])
    rab = torch.stack([torch.rand(N, device="cuda", generator=g), torch.randn(N, device="cuda", generator=g)]) \
        if deferred_res else None

    def run():
        return _n().conv1x1_gemm_apply(a, b, res, ab.contiguous(), rab.contiguous() if rab is not None else None)
    r = _modes(run)
    for mode in (1, 2):
        assert torch.equal(r[mode][0], r[0][0]) and torch.equal(r[mode][1], r[0][1])
    rows = _rows(M)
    z = _oracle_rows(a, b, rows).bfloat16().float()
    rr = res[rows].float()
    if rab is not None:
        rr = rr * rab[0] + rab[1]
    ref = torch.relu(z * ab[0] + ab[1] + rr)
    torch.testing.assert_close(r[1][0][rows].float(), ref, rtol=2e-2, atol=3e-2)
