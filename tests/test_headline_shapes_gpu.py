"""Kernel variants the ResNet-50 bench step runs (1024 images per GPU) at the grid sizes that select them.

Small test shapes pick the small-grid variants (64-channel 3x3 / stride-2 tiles, one-tile-per-workgroup
1x1 kernels), so the 128-channel 3x3 tiles, the 8-wave 1x1 tile with a bare or BN-reduction epilogue,
the persistent 16-wave 1x1 tile without an epilogue and the multi-tensor copies of the DDP reducer were
never launched by a test (tools/kernel_coverage.py against profiles/r5/steady_resnet50_b1024_kernels.csv).
Each case here runs the step's shape (or a grid of the same variant) against an fp32 oracle."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _n():
    from pytorch_distributed_training_example_amd.ops._native import native
    return native()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _bits(M, C, g):
    b = torch.rand(M * C, device="cuda", generator=g) > 0.4
    return b.view(M, C), (b.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)


@pytest.mark.parametrize("N,C,H", [(1024, 256, 14), (256, 128, 28)])
def test_conv3x3_wide_tile_forward_stats(N, C, H):
    """conv3x3h 128-channel tile with the BatchNorm statistics epilogue (layers 2-3 conv2 forward)."""
    g = torch.Generator(device="cuda").manual_seed(C)
    x = _cl(torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16())
    w = _cl((torch.randn(C, C, 3, 3, device="cuda", generator=g) / (9 * C) ** 0.5).bfloat16())
    y, part = _n().conv3x3s1_fwd_stats(x, w)
    ref = torch.nn.functional.conv2d(x[:16].float(), w.float(), padding=1)
    torch.testing.assert_close(y[:16].float(), ref, rtol=2e-2, atol=2e-2)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, C)
    torch.testing.assert_close(part[0].sum(0), yf.sum(0), rtol=1e-3, atol=1e-1)


def test_conv3x3_wide_tile_dgrad_bn_reduction():
    """conv3x3h 128-channel tile, data gradient with the producing BatchNorm's backward reduction."""
    N, C, H = 1024, 256, 14
    g = torch.Generator(device="cuda").manual_seed(7)
    gy = _cl(torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16())
    w = _cl((torch.randn(C, C, 3, 3, device="cuda", generator=g) / (9 * C) ** 0.5).bfloat16())
    bx = _cl(torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16())
    M = N * H * H
    mean = bx.float().permute(0, 2, 3, 1).reshape(M, C).mean(0).contiguous()
    bits, mask = _bits(M, C, g)
    wf = _n().conv3x3_flip(w)
    dx, part = _n().conv3x3s1_fwd_bnbwd(gy, wf, bx, mask, mean)
    assert torch.equal(dx, _n().conv3x3s1_fwd(gy, wf))
    dz = torch.where(bits, dx.float().permute(0, 2, 3, 1).reshape(M, C), 0.0)
    xc = bx.float().permute(0, 2, 3, 1).reshape(M, C) - mean
    torch.testing.assert_close(part[0].sum(0), dz.sum(0), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(part[1].sum(0), (dz * xc).sum(0), rtol=1e-3, atol=1e-1)


def test_conv3x3_stride2_wide_tile():
    """conv3x3g (stride 2) 128-channel tile: forward + statistics and the four-phase data gradient +
    BatchNorm reduction at the layer-3 transition shape (1024 x 256 x 28 x 28 -> 14 x 14)."""
    N, C, H = 1024, 256, 28
    g = torch.Generator(device="cuda").manual_seed(9)
    x = _cl(torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16())
    w = _cl((torch.randn(C, C, 3, 3, device="cuda", generator=g) / (9 * C) ** 0.5).bfloat16())
    y, part = _n().conv3x3s2_fwd(x, w, True)
    ref = torch.nn.functional.conv2d(x[:8].float(), w.float(), stride=2, padding=1)
    torch.testing.assert_close(y[:8].float(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(part[0].sum(0), y.float().sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    gy = _cl(torch.randn(N, C, H // 2, H // 2, device="cuda", generator=g).bfloat16())
    bx = _cl(torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16())
    M = N * H * H
    mean = bx.float().permute(0, 2, 3, 1).reshape(M, C).mean(0).contiguous()
    bits, mask = _bits(M, C, g)
    wf = _n().conv3x3_flip(w)
    dx, bpart = _n().conv3x3s2_dgrad(gy, wf, H, H, bn_x=bx, bn_mask=mask, bn_mean=mean)
    assert torch.equal(dx, _n().conv3x3s2_dgrad(gy, wf, H, H)[0])
    gref = torch.nn.grad.conv2d_input((8, C, H, H), w.float(), gy[:8].float(), stride=2, padding=1)
    torch.testing.assert_close(dx[:8].float(), gref, rtol=2e-2, atol=2e-2)
    dz = torch.where(bits, dx.float().permute(0, 2, 3, 1).reshape(M, C), 0.0)
    torch.testing.assert_close(bpart[0].sum(0), dz.sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("M,K,N,bst", [(1024 * 7 * 7, 2048, 512, True), (1024 * 7 * 7, 2048, 512, False),
                                       (1024 * 28 * 28, 256, 512, False)])
def test_conv1x1_step_tiles_plain_and_bn_reduction(M, K, N, bst):
    """1x1 GEMM: the 8-wave tile (layer 4: 392 tiles) with a bare epilogue or the BatchNorm backward
    reduction, and the persistent 16-wave tile with a bare epilogue (6,272 tiles)."""
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    if bst:
        bx = torch.randn(M, N, device="cuda", generator=g).bfloat16()
        mean = bx.float().mean(0).contiguous()
        part = _n().conv1x1_gemm(a, b, y, False, False, None, None, bx, None, mean)
        T = (M + 255) // 256
        assert part.shape == (2, T, N)
        torch.testing.assert_close(part[0].sum(0), y.float().sum(0), rtol=1e-3, atol=1e-1)
        torch.testing.assert_close(part[1].sum(0), (y.float() * (bx.float() - mean)).sum(0), rtol=1e-3, atol=1e-1)
    else:
        assert _n().conv1x1_gemm(a, b, y, False, False) is None
    rows = torch.cat([torch.arange(0, 1024), torch.randint(1024, M - 1024, (2048,)), torch.arange(M - 1024, M)]).cuda()
    torch.testing.assert_close(y[rows].float(), a[rows].float() @ b.float().t(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("src_dtype,dst_dtype", [(torch.bfloat16, torch.bfloat16), (torch.float32, torch.float32)])
def test_multi_tensor_copy_bucket_pack(src_dtype, dst_dtype):
    """The DDP reducer's bucket packing (ops/multi_tensor.py copy_ -> mt_copy): ResNet-50's gradient
    shapes into a flat bucket, exact."""
    from pytorch_distributed_training_example_amd.ops import multi_tensor
    shapes = [(64, 3, 7, 7), (64,), (256, 64, 1, 1), (512, 128, 3, 3), (2048,), (1000, 2048), (3,), (17, 5)]
    g = torch.Generator(device="cuda").manual_seed(1)
    src = [torch.randn(s, device="cuda", generator=g).to(src_dtype) for s in shapes]
    flat = torch.zeros(sum(t.numel() for t in src) + 64, device="cuda", dtype=dst_dtype)
    dst, off = [], 0
    for t in src:
        dst.append(flat[off:off + t.numel()].view(t.shape))
        off += (t.numel() + 7) // 8 * 8
    multi_tensor.copy_(src, dst)
    for s, d in zip(src, dst):
        assert torch.equal(s.to(dst_dtype), d)


@pytest.mark.parametrize("opt", [41, 41 + 128])
def test_conv3x3_layer1_row_tiles(opt):
    """conv3x3wsr_kernel (layer 1, 64 -> 64 at 56 x 56, whole-row 224-pixel tiles, four-deep halo DMA
    pipeline): forward + statistics against an fp32 oracle, the BN forward finalize from its 224-row
    partials against torch's batch statistics, and the data gradient (same kernel, flipped weights)."""
    C = _n()
    old = C.conv3x3_opt(opt)
    try:
        N, c, H = 24, 64, 56  # 336 tiles: at least one per CU, so the row-tile kernel runs
        g = torch.Generator(device="cuda").manual_seed(3)
        x = _cl(torch.randn(N, c, H, H, device="cuda", generator=g).bfloat16())
        w = _cl((torch.randn(c, c, 3, 3, device="cuda", generator=g) / 24).bfloat16())
        y, part = C.conv3x3s1_fwd_stats(x, w)
        M = N * H * H
        assert part.shape == (2, M // 224, c)
        ref = torch.nn.functional.conv2d(x.float(), w.float(), padding=1)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
        yf = y.float().permute(0, 2, 3, 1).reshape(-1, 224, c)
        torch.testing.assert_close(part[0], yf.sum(1), rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(part[1], ((yf - yf.mean(1, keepdim=True)) ** 2).sum(1), rtol=1e-3, atol=1e-3)
        gamma = torch.rand(c, device="cuda") + 0.5
        beta = torch.randn(c, device="cuda")
        _, _, mean, invstd = C.bn_fwd_train_tiles(y, part, None, gamma, beta, None, None, 0.1, 1e-5, True, None, True)
        yv = y.float().permute(0, 2, 3, 1).reshape(-1, c)
        torch.testing.assert_close(mean, yv.mean(0), rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(invstd, (yv.var(0, unbiased=False) + 1e-5).rsqrt(), rtol=1e-3, atol=1e-3)
        wf = C.conv3x3_flip(w)
        dx = C.conv3x3s1_fwd(y, wf)
        gref = torch.nn.grad.conv2d_input(x.shape, w.float(), y.float(), padding=1)
        torch.testing.assert_close(dx.float(), gref, rtol=2e-2, atol=5e-2)
        if opt & 128:  # the data gradient with the producing BatchNorm's backward reduction (BSTATS)
            bx = _cl(torch.randn(N, c, H, H, device="cuda", generator=g).bfloat16())
            bits, mask = _bits(M, c, g)
            mean = bx.float().permute(0, 2, 3, 1).reshape(M, c).mean(0).contiguous()
            dx2, bpart = C.conv3x3s1_fwd_bnbwd(y, wf, bx, mask, mean)
            assert torch.equal(dx2, dx)
            assert bpart.shape == (2, M // 224, c)
            dz = torch.where(bits, dx.float().permute(0, 2, 3, 1).reshape(M, c), 0.0)
            xc = bx.float().permute(0, 2, 3, 1).reshape(M, c) - mean
            torch.testing.assert_close(bpart[0].sum(0), dz.sum(0), rtol=1e-3, atol=1e-1)
            torch.testing.assert_close(bpart[1].sum(0), (dz * xc).sum(0), rtol=1e-3, atol=1e-1)
            torch.testing.assert_close(bpart[0], dz.view(-1, 224, c).sum(1), rtol=1e-3, atol=1e-2)
            dx3, bpart3 = C.conv3x3s1_fwd_bnbwd(y, wf, bx, None, mean)  # no ReLU mask
            torch.testing.assert_close(bpart3[0].sum(0), dx.float().permute(0, 2, 3, 1).reshape(M, c).sum(0),
                                       rtol=1e-3, atol=1e-1)
        C.conv3x3_opt(9)  # the 256-pixel weight-stationary kernel on the same input: same convolution
        y2 = C.conv3x3s1_fwd(x, w)
        torch.testing.assert_close(y.float(), y2.float(), rtol=1e-2, atol=1e-2)
    finally:
        C.conv3x3_opt(old)
