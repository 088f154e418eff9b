"""Our MFMA 1x1-conv GEMM (csrc/kernels/conv1x1.hip) against fp32 PyTorch references: plain,
in-place accumulate (the shortcut-gradient hand-off) and the fused BatchNorm statistics epilogue,
then the BatchNorm that consumes those statistics against the reduce-pass BatchNorm."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(1000, 64, 256), (512, 256, 64), (4096, 32, 128), (700, 96, 192), (25088 // 8, 2048, 512),
          (256, 512, 2048), (300, 64, 64)]


def _native():
    from pytorch_distributed_training_example_amd.ops._native import native
    return native()


def _ab(M, K, N, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    return a, b


@pytest.mark.parametrize("M,K,N", SHAPES)
def test_gemm_matches_fp32(M, K, N):
    a, b = _ab(M, K, N)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert _native().conv1x1_gemm(a, b, y, False, False) is None
    ref = a.float() @ b.float().t()
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,K,N", SHAPES[:4])
def test_gemm_accumulates_in_place(M, K, N):
    a, b = _ab(M, K, N, 1)
    c = torch.randn(M, N, device="cuda").bfloat16()
    ref = c.float() + a.float() @ b.float().t()
    _native().conv1x1_gemm(a, b, c, True, False)
    torch.testing.assert_close(c.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,K,N", SHAPES)
def test_stats_epilogue(M, K, N):
    a, b = _ab(M, K, N, 2)
    a = a + 0.5  # non-zero channel means
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    part = _native().conv1x1_gemm(a, b, y, False, True)
    T = (M + 255) // 256
    assert part.shape == (2, T, N)
    yf = torch.cat([y.float(), torch.full((T * 256 - M, N), float("nan"), device="cuda")]).view(T, 256, N)
    valid = ~torch.isnan(yf)
    n = valid.sum(1).float()
    s = torch.where(valid, yf, 0).sum(1)
    mu = s / n
    m2 = torch.where(valid, (yf - mu[:, None]) ** 2, 0).sum(1)
    torch.testing.assert_close(part[0], s, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(part[1], m2, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(y.float(), a.float() @ b.float().t(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("relu,res", [(True, False), (False, True), (True, True), (False, False)])
@pytest.mark.parametrize("shape", [(8, 64, 256, 14, 14), (4, 128, 128, 7, 9)])
def test_bn_from_tile_stats_matches_reduce_bn(relu, res, shape):
    N, Ci, Co, H, W = shape
    M = N * H * W
    a, b = _ab(M, Ci, Co, 3)
    y = torch.empty(N, Co, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y2 = y.permute(0, 2, 3, 1).reshape(M, Co)
    part = _native().conv1x1_gemm(a + 1.0, b, y2, False, True)
    r = torch.randn_like(y) if res else None
    w = torch.rand(Co, device="cuda") + 0.5
    bb = torch.randn(Co, device="cuda")
    out = {}
    for kind in ("tiles", "reduce"):
        rm, rv = torch.zeros(Co, device="cuda"), torch.ones(Co, device="cuda")
        if kind == "tiles":
            o = _native().bn_fwd_train_tiles(y, part, r, w, bb, rm, rv, 0.1, 1e-5, relu)
        else:
            o = _native().bn_fwd_train(y, r, w, bb, rm, rv, 0.1, 1e-5, relu)
        out[kind] = (o, rm, rv)
    (ot, rmt, rvt), (orr, rmr, rvr) = out["tiles"], out["reduce"]
    torch.testing.assert_close(ot[2], orr[2], rtol=1e-5, atol=1e-5)  # mean
    torch.testing.assert_close(ot[3], orr[3], rtol=1e-4, atol=1e-5)  # invstd
    torch.testing.assert_close(rmt, rmr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rvt, rvr, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(ot[0].float(), orr[0].float(), rtol=1e-2, atol=1e-2)
    if relu:
        assert (ot[1] != orr[1]).float().mean().item() < 1e-3  # masks (ties at 0 may differ)
    # and both against the fp32 formula
    yf = y.float()
    mu = yf.mean((0, 2, 3))
    var = yf.var((0, 2, 3), unbiased=False)
    torch.testing.assert_close(ot[2], mu, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ot[3], (var + 1e-5).rsqrt(), rtol=1e-3, atol=1e-4)


def test_resnet_bottleneck_uses_fused_stats(monkeypatch, switch):
    """A training Bottleneck on the fused path matches the same block with our GEMM off
    (library GEMMs + reduce-pass BatchNorm): outputs, input and parameter gradients."""
    from pytorch_distributed_training_example_amd.models import resnet as R
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops import conv as C
    torch.manual_seed(0)
    ds = R._Downsample(R.conv1x1(64, 256, 1), R._bn(256))
    blk = to_bf16_mixed(R.Bottleneck(64, 64, 1, ds).cuda().to(memory_format=torch.channels_last))
    x0 = torch.randn(16, 64, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    res = {}
    for ours in ("fwd,dgrad", "none"):
        switch("PDT_CONV1X1_OURS", ours)
        switch("PDT_CONV1X1", "ours" if ours != "none" else "gemm")
        blk.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        h = blk.conv1(x)
        assert (C.bn_stats_of(h) is not None) == (ours != "none")
        y = blk(x)
        y.backward(torch.ones_like(y) * 0.01 + y.detach() * 0.1)
        res[ours] = [y.float()] + [x.grad.float()] + [p.grad.float().clone() for p in blk.parameters()]
    for a, b in zip(res["fwd,dgrad"], res["none"]):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 3e-2, err


@pytest.mark.parametrize("shape", [(4, 128, 128, 28, 28), (8, 256, 256, 14, 14), (2, 64, 128, 9, 11),
                                   (4, 64, 64, 14, 14), (3, 64, 64, 13, 11), (32, 64, 64, 56, 56)])
def test_conv3x3_stats_epilogue(shape):
    """The 3x3 statistics epilogue (halo kernel; 64 -> 64: the weight-stationary kernel, whose waves
    merge four 64-row chunks per tile — ragged last tile; at 32 x 56 x 56 the row-tile kernel with
    224-row tiles, > 1 tile per persistent workgroup): same y as the plain launch, per-tile partials
    match an fp32 recomputation from y."""
    N, Ci, Co, H, W = shape
    torch.manual_seed(0)
    x = torch.randn(N, Ci, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, Ci, 3, 3, device="cuda") / (9 * Ci) ** 0.5 + 0.01).bfloat16()
    r = _native().conv3x3s1_fwd_stats(x, w)
    y0 = _native().conv3x3s1_fwd(x, w)
    torch.testing.assert_close(r[0], y0, rtol=0, atol=0)
    assert len(r) == 2
    part = r[1]
    M = N * H * W
    T = part.shape[1]
    BMt = 224 if (M % 224 == 0 and T == M // 224 and T != (M + 255) // 256) else 256  # row tiles: 224
    assert T == (M + BMt - 1) // BMt
    y2 = r[0].permute(0, 2, 3, 1).reshape(M, Co).float()
    yf = torch.cat([y2, torch.full((T * BMt - M, Co), float("nan"), device="cuda")]).view(T, BMt, Co)
    valid = ~torch.isnan(yf)
    s = torch.where(valid, yf, 0).sum(1)
    mu = s / valid.sum(1).float()
    m2 = torch.where(valid, (yf - mu[:, None]) ** 2, 0).sum(1)
    torch.testing.assert_close(part[0], s, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(part[1], m2, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("shape", [(4, 128, 128, 28, 28), (3, 64, 64, 13, 11), (32, 64, 64, 56, 56),
                                   (1024, 256, 256, 14, 14), (3, 128, 128, 13, 11)])
@pytest.mark.parametrize("with_mask", [True, False])
def test_conv3x3_bn_backward_epilogue(shape, with_mask):
    """The 3x3 data-gradient launch that also takes the BatchNorm backward reduction (halo kernel):
    per 256-row tile, sum(dz) and sum(dz * (x - mean)) with dz = y * ReLU mask, against an fp32
    recomputation from the y it wrote. 64 -> 64 (weight-stationary kernel) returns y alone: the
    caller's reduce pass takes the statistics."""
    N, Ci, Co, H, W = shape
    torch.manual_seed(1)
    x = torch.randn(N, Ci, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, Ci, 3, 3, device="cuda") / (9 * Ci) ** 0.5).bfloat16()
    bx = (torch.randn(N, Co, H, W, device="cuda") + 0.3).bfloat16().contiguous(memory_format=torch.channels_last)
    M = N * H * W
    mean = bx.float().permute(0, 2, 3, 1).reshape(M, Co).mean(0).contiguous()
    bits, mask = _bits_mask(M, Co) if with_mask else (torch.ones(M, Co, dtype=torch.bool, device="cuda"), None)
    r = _native().conv3x3s1_fwd_bnbwd(x, w, bx, mask, mean)
    torch.testing.assert_close(r[0], _native().conv3x3s1_fwd(x, w), rtol=0, atol=0)
    if Ci == 64 and Co == 64:
        assert len(r) == 1
        return
    assert len(r) == 2
    T = (M + 255) // 256
    dz = torch.where(bits, r[0].permute(0, 2, 3, 1).reshape(M, Co).float(), 0)
    xc = bx.permute(0, 2, 3, 1).reshape(M, Co).float() - mean
    pad = T * 256 - M
    dzt = torch.cat([dz, torch.zeros(pad, Co, device="cuda")]).view(T, 256, Co)
    xct = torch.cat([xc, torch.zeros(pad, Co, device="cuda")]).view(T, 256, Co)
    torch.testing.assert_close(r[1][0], dzt.sum(1), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(r[1][1], (dzt * xct).sum(1), rtol=1e-4, atol=1e-3)


def test_gemm_accumulates_masked_source():
    """acc from a separate source masked by a BatchNorm ReLU bit-mask (the shortcut hand-off)."""
    M, K, N = 777, 64, 256
    a, b = _ab(M, K, N, 5)
    dy = torch.randn(M, N, device="cuda").bfloat16()
    bits = torch.rand(M, N, device="cuda") > 0.4
    mask = (bits.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    _native().conv1x1_gemm(a, b, out, True, False, dy, mask)
    ref = torch.where(bits, dy.float(), 0) + a.float() @ b.float().t()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    from pytorch_distributed_training_example_amd.ops.batchnorm import MaskedGrad
    d4 = dy.view(1, 1, M, N).permute(0, 3, 1, 2)  # [1, N, 1, M] channels_last view of [M, N]
    dense = MaskedGrad(d4, mask).dense()
    torch.testing.assert_close(dense.permute(0, 2, 3, 1).reshape(M, N).float(), torch.where(bits, dy.float(), 0))


@pytest.mark.parametrize("masked", ["1", "0"])
def test_identity_block_masked_residual_matches_plain(monkeypatch, masked, switch):
    """Identity Bottleneck: bn3 handing the shortcut gradient over as (dy, mask) gives the same
    gradients as the materialised dres path and as autograd's own add (link off)."""
    from pytorch_distributed_training_example_amd.models import resnet as R
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    torch.manual_seed(0)
    blk = to_bf16_mixed(R.Bottleneck(256, 64, 1, None).cuda().to(memory_format=torch.channels_last))
    x0 = torch.randn(8, 256, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    switch("PDT_RES_MASKED", masked)
    switch("PDT_CONV1X1", "ours")
    out = {}
    for linked in (True, False):
        R.RESIDUAL_GRAD_LINK[0] = linked
        try:
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            y = blk(x)
            y.backward(torch.ones_like(y) * 0.01 + y.detach() * 0.1)
            out[linked] = [x.grad.float()] + [p.grad.float().clone() for p in blk.parameters()]
        finally:
            R.RESIDUAL_GRAD_LINK[0] = True
    for a, b in zip(out[True], out[False]):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 2e-2, err


def _bits_mask(M, N, p=0.4, seed=7):
    g = torch.Generator(device="cuda").manual_seed(seed)
    bits = torch.rand(M, N, device="cuda", generator=g) > p
    mask = (bits.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1)
    return bits, mask.to(torch.uint8)


@pytest.mark.parametrize("acc", [False, True])
@pytest.mark.parametrize("M,K,N", [(1000, 256, 64), (777, 64, 256), (4096, 128, 128), (300, 512, 2048)])
def test_gemm_bn_backward_stats_epilogue(M, K, N, acc):
    """BSTATS: the GEMM writes dy (optionally dy = C*cmask + A B^T) and returns the per-tile sums of
    dz = dy*mask and dz*(x - mean) of the BatchNorm whose output gradient dy is (fp32 reference
    from the bf16 dy actually written)."""
    a, b = _ab(M, K, N, 11)
    xb = (torch.randn(M, N, device="cuda") * 2 + 1).bfloat16()
    mean = xb.float().mean(0)
    bits, mask = _bits_mask(M, N)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    kw = dict(bn_x=xb, bn_mask=mask, bn_mean=mean)
    if acc:
        cin = torch.randn(M, N, device="cuda").bfloat16()
        cbits, cmask = _bits_mask(M, N, 0.5, 3)
        part = _native().conv1x1_gemm(a, b, out, True, False, cin, cmask, **kw)
        ref = torch.where(cbits, cin.float(), 0) + a.float() @ b.float().t()
    else:
        part = _native().conv1x1_gemm(a, b, out, False, False, **kw)
        ref = a.float() @ b.float().t()
    # the gradient at a BatchNorm + ReLU output is stored already masked (tile_stats.h mask8)
    ref = torch.where(bits, ref, 0)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    assert not out[~bits].float().abs().any()
    T = (M + 255) // 256
    assert part.shape == (2, T, N)
    dz = torch.where(bits, out.float(), 0)
    pad = T * 256 - M
    dzt = torch.cat([dz, dz.new_zeros(pad, N)]).view(T, 256, N)
    xt = torch.cat([xb.float() - mean, dz.new_zeros(pad, N)]).view(T, 256, N)
    torch.testing.assert_close(part[0], dzt.sum(1), rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(part[1], (dzt * xt).sum(1), rtol=1e-4, atol=5e-3)
    # no mask: every element counts
    part2 = _native().conv1x1_gemm(a, b, out, False, False, bn_x=xb, bn_mean=mean) if not acc else None
    if part2 is not None:
        o = torch.cat([out.float(), dz.new_zeros(pad, N)]).view(T, 256, N)
        torch.testing.assert_close(part2[0], o.sum(1), rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_backward_from_tiles_matches_reduce(relu, res):
    """bn_bwd_train_tiles with partials from the GEMM epilogue == bn_bwd_train's own reduce."""
    N, C, H, W = 6, 128, 13, 11
    M = N * H * W
    x = (torch.randn(N, C, H, W, device="cuda") + 0.3).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.rand(C, device="cuda") + 0.5
    bb = torch.randn(C, device="cuda")
    y, mask, mean, invstd = _native().bn_fwd_train(x, None, w, bb, None, None, 0.1, 1e-5, relu)
    a, b = _ab(M, 64, C, 13)
    dy = torch.empty_like(x)
    part = _native().conv1x1_gemm(a, b, dy.permute(0, 2, 3, 1).reshape(M, C), False, False,
                                  bn_x=x, bn_mask=mask if relu else None, bn_mean=mean)
    t = _native().bn_bwd_train_tiles(dy, x, part, mask, w, mean, invstd, relu, res, True)
    r = _native().bn_bwd_train(dy, x, mask, w, mean, invstd, relu, res, True)
    torch.testing.assert_close(t[2], r[2], rtol=1e-3, atol=1e-3)  # dgamma
    torch.testing.assert_close(t[3], r[3], rtol=1e-3, atol=1e-3)  # dbeta
    torch.testing.assert_close(t[0].float(), r[0].float(), rtol=1e-2, atol=1e-2)
    if res:
        torch.testing.assert_close(t[1], r[1], rtol=0, atol=0)


def test_bottleneck_chain_takes_bn_backward_stats(monkeypatch, switch):
    """Two Bottlenecks (downsample + identity): with the BN-backward hand-off on, bn2 (conv3's
    dgrad) and the first block's bn3 (the second block's conv1 dgrad, shortcut accumulated) take
    their reduction from the GEMM epilogue (and block 0's conv3 + shortcut run the ALG backward) — and every
    gradient is as close to an fp32 oracle of the same weights and input as the hand-off-off run's, tensor by
    tensor. (The two bf16 runs differ from the oracle by 1-10 % on this random init — forward bf16 rounding, the
    same for both — so a direct on-vs-off bound measures that noise, not the hand-off.)"""
    import copy
    from pytorch_distributed_training_example_amd.models import resnet as R
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops import batchnorm as B
    torch.manual_seed(0)
    ds = R._Downsample(R.conv1x1(64, 256, 1), R._bn(256))
    base = torch.nn.Sequential(R.Bottleneck(64, 64, 1, ds), R.Bottleneck(256, 64, 1, None)).cuda()
    net = to_bf16_mixed(copy.deepcopy(base).to(memory_format=torch.channels_last))
    ref = copy.deepcopy(base).to(memory_format=torch.channels_last)
    x0 = torch.randn(8, 64, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    switch("PDT_CONV1X1", "ours")
    used = []
    orig = B.GradStatsSource.take

    def spy(self, dy):
        p = orig(self, dy)
        used.append(p is not None)
        return p
    monkeypatch.setattr(B.GradStatsSource, "take", spy)

    def grads(m, x_in):
        m.zero_grad(set_to_none=True)
        x = x_in.clone().requires_grad_(True)
        y = m(x)
        y.backward(torch.ones_like(y) * 0.01 + y.detach() * 0.1)
        return [x.grad.double()] + [p.grad.double().clone() for p in m.parameters()]
    out = {}
    for on in ("1", "0"):
        switch("PDT_BN_BWD_STATS", on)
        used.clear()
        out[on] = grads(net, x0)
        if on == "1":
            assert sum(used) >= 3, used  # bn2 of both blocks + block 0's bn3
    switch("PDT_DISABLE_NATIVE", "1")
    want = grads(ref, x0.float())
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-30))  # noqa: E731
    for i, (a, b, w) in enumerate(zip(out["1"], out["0"], want)):
        ea, eb = rel(a, w), rel(b, w)
        assert ea <= 1.25 * eb + 5e-3, (i, ea, eb)


@pytest.mark.parametrize("shape", [(4, 64, 56, 56), (3, 64, 17, 23)])
def test_stem_pool_backward_fused_reduction(monkeypatch, shape, switch):
    """Stem BN+ReLU+MaxPool backward: the pool-gradient kernel taking the BN's backward reduction
    (PDT_STEM_BWD_FUSED=1) gives the same dx / dgamma / dbeta as the separate reduce pass."""
    from pytorch_distributed_training_example_amd.ops.batchnorm import BatchNorm2d
    torch.manual_seed(0)
    bn = BatchNorm2d(shape[1], fused_relu=True).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x0 = torch.randn(*shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    out = {}
    gy = None
    for fused in ("1", "0"):
        switch("PDT_STEM_BWD_FUSED", fused)
        bn.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        y = bn.forward_relu_maxpool(x)
        if gy is None:
            gy = (torch.randn_like(y.float()) * 0.1).to(y.dtype)
        y.backward(gy)
        out[fused] = [x.grad.float(), bn.weight.grad.clone(), bn.bias.grad.clone()]
    for a, b in zip(out["1"], out["0"]):
        torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("ds_masked", [True, False])
def test_downsample_block_masked_shortcut_grad(ds_masked):
    """Downsample Bottleneck: bn3 handing the shortcut gradient to the downsample BN as (dy, mask)
    (no dres written) gives the gradients of the plain autograd path (residual link off)."""
    from pytorch_distributed_training_example_amd.models import resnet as R
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    torch.manual_seed(0)
    ds = R._Downsample(R.conv1x1(128, 256, 1), R._bn(256))
    blk = to_bf16_mixed(R.Bottleneck(128, 64, 1, ds).cuda().to(memory_format=torch.channels_last))
    x0 = torch.randn(8, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    out = {}
    for linked in (True, False):
        R.RESIDUAL_GRAD_LINK[0] = linked
        R.DS_MASKED_GRAD[0] = ds_masked
        try:
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            y = blk(x)
            y.backward(torch.ones_like(y) * 0.01 + y.detach() * 0.1)
            out[linked] = [x.grad.float()] + [p.grad.float().clone() for p in blk.parameters()]
        finally:
            R.RESIDUAL_GRAD_LINK[0] = True
            R.DS_MASKED_GRAD[0] = True
    for a, b in zip(out[True], out[False]):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 2e-2, err


@pytest.mark.parametrize("shape", [(8, 256, 1024, 14), (16, 512, 128, 28)])
def test_conv1x1_wgrad_splitk_matches_miopen(monkeypatch, shape):
    """Weight gradient of a 1x1 conv: the split-K batched-GEMM path (table decision splitk*) equals
    MIOpen's kernel."""
    from pytorch_distributed_training_example_amd.ops import conv as C
    N, Ci, Co, H = shape
    M = N * H * H
    torch.manual_seed(0)
    x0 = torch.randn(N, Ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    conv = C.Conv1x1(Ci, Co).cuda().bfloat16().to(memory_format=torch.channels_last)
    gy = torch.randn(N, Co, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    key = ("bwd_weight", "bf16", M, Ci, Co)
    grads = {}
    for algo in ("splitk16", "miopen"):
        monkeypatch.setitem(C._CHOICE, key, algo)
        conv.weight.grad = None
        conv(x0.clone().requires_grad_(True)).backward(gy)
        grads[algo] = conv.weight.grad.float().clone()
    assert grads["splitk16"].shape == conv.weight.shape
    err = ((grads["splitk16"] - grads["miopen"]).norm() / grads["miopen"].norm()).item()
    assert err < 1e-2, err


def test_gemm_accumulates_strided_compact_source():
    """ACC from a stride-2 shortcut's COMPACT gradient: added only at the sampled pixels."""
    n, H, W, K, N = 3, 9, 14, 64, 128
    M = n * H * W
    a, b = _ab(M, K, N, 21)
    Hs, Ws = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    cmp = torch.randn(n, N, Hs, Ws, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    out = torch.empty(n, N, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    _native().conv1x1_gemm(a, b, out.permute(0, 2, 3, 1).reshape(M, N), True, False, cmp, c_stride=2, c_H=H, c_W=W)
    ref = (a.float() @ b.float().t()).view(n, H, W, N).permute(0, 3, 1, 2).clone()
    ref[:, :, ::2, ::2] += cmp.float()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


def test_downsample_stride2_block_strided_grad(monkeypatch, switch):
    """Stride-2 downsample Bottleneck (gathered shortcut GEMM): the shortcut's compact gradient
    added into conv1's full gradient matches the plain autograd path."""
    from pytorch_distributed_training_example_amd.models import resnet as R
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    torch.manual_seed(0)
    ds = R._Downsample(R.conv1x1(256, 512, 2), R._bn(512))
    blk = to_bf16_mixed(R.Bottleneck(256, 128, 2, ds).cuda().to(memory_format=torch.channels_last))
    x0 = torch.randn(8, 256, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    switch("PDT_CONV1X1", "ours")
    out = {}
    for linked in (True, False):
        R.RESIDUAL_GRAD_LINK[0] = linked
        try:
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            y = blk(x)
            y.backward(torch.ones_like(y) * 0.01 + y.detach() * 0.1)
            out[linked] = [x.grad.float()] + [p.grad.float().clone() for p in blk.parameters()]
        finally:
            R.RESIDUAL_GRAD_LINK[0] = True
    for a, b in zip(out[True], out[False]):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 2e-2, err


def test_strided_shortcut_grad_with_bn_bwd_stats(monkeypatch, switch):
    """A block followed by a stride-2 transition block: the transition conv1's data gradient adds the
    shortcut's compact gradient AND takes the first block's bn3 backward reduction in one GEMM epilogue
    (PDT_STRIDED_BSTATS=1) — gradients match the scatter-add + reduce-pass path (=0), and no
    scatter-add ran."""
    from pytorch_distributed_training_example_amd.models import resnet as R
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops import conv as C
    torch.manual_seed(0)
    ds = R._Downsample(R.conv1x1(256, 512, 2), R._bn(512))
    net = to_bf16_mixed(torch.nn.Sequential(R.Bottleneck(256, 64, 1, None), R.Bottleneck(256, 128, 2, ds))
                        .cuda().to(memory_format=torch.channels_last))
    x0 = torch.randn(8, 256, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, 512, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    switch("PDT_CONV1X1", "ours")
    adds = []
    orig = C.StridedGrad.add_into
    monkeypatch.setattr(C.StridedGrad, "add_into", lambda self, full: adds.append(1) or orig(self, full))
    out = {}
    for on in ("1", "0"):
        switch("PDT_STRIDED_BSTATS", on)
        adds.clear()
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        net(x).backward(gy)
        out[on] = ([x.grad.float()] + [p.grad.float().clone() for p in net.parameters()], len(adds))
    assert out["1"][1] == 0 and out["0"][1] == 1, (out["1"][1], out["0"][1])
    for a, b in zip(out["1"][0], out["0"][0]):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 2e-2, err


def _ds_block_run(blk, x0, defer, bn3_eval=False):
    from pytorch_distributed_training_example_amd.models import resnet as R
    ds = blk.downsample
    old = R.DS_DEFER_APPLY[0]
    R.DS_DEFER_APPLY[0] = defer
    try:
        blk.train()
        if bn3_eval:
            blk.bn3.eval()
        blk.zero_grad(set_to_none=True)
        ds[1].running_mean.zero_()
        ds[1].running_var.fill_(1)
        x = x0.clone().requires_grad_(True)
        y = blk(x)
        y.backward(torch.ones_like(y) * 0.01 + y.detach() * 0.1)
        return ([y.float(), x.grad.float()] + [p.grad.float().clone() for p in blk.parameters()]
                + [ds[1].running_mean.clone(), ds[1].running_var.clone()])
    finally:
        R.DS_DEFER_APPLY[0] = old


def _make_ds_block(stride, cin=128, planes=64):
    from pytorch_distributed_training_example_amd.models import resnet as R
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    torch.manual_seed(0)
    ds = R._Downsample(R.conv1x1(cin, planes * 4, stride), R._bn(planes * 4))
    return to_bf16_mixed(R.Bottleneck(cin, planes, stride, ds).cuda().to(memory_format=torch.channels_last))


@pytest.mark.parametrize("stride", [1, 2])
def test_downsample_bn_deferred_apply(stride):
    """Downsample Bottleneck with the shortcut BN's apply deferred into bn3's (DS_DEFER_APPLY, the
    shortcut BN output never written) == the materialised shortcut: output, input and parameter
    gradients, running statistics."""
    blk = _make_ds_block(stride)
    x0 = torch.randn(8, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    a_all, b_all = _ds_block_run(blk, x0, True), _ds_block_run(blk, x0, False)
    for a, b in zip(a_all, b_all):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 1e-2, err


def test_shortcut_conv_fused_backward(monkeypatch):
    """Layer-1 style downsample block (stride 1, shortcut conv 64 -> 256): the shortcut BN's backward
    apply is deferred into the shortcut conv's fused backward (DS_FUSED_BWD; dx deposited for conv1's
    dgrad) — outputs, input / parameter gradients and running statistics match the unfused run, and
    the fused kernel did run for the linked shortcut conv."""
    from pytorch_distributed_training_example_amd.models import resnet as R
    from pytorch_distributed_training_example_amd.ops import conv as C
    blk = _make_ds_block(1, cin=64, planes=64)
    x0 = torch.randn(8, 64, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    ran = []
    orig = C._bwd_fused
    monkeypatch.setattr(C, "_bwd_fused", lambda ctx, d, x, w: ran.append((ctx.link is not None, tuple(w.shape[:2])))
                        or orig(ctx, d, x, w))
    old = R.DS_FUSED_BWD[0]
    try:
        R.DS_FUSED_BWD[0] = True
        a_all = _ds_block_run(blk, x0, True)
        fused = list(ran)
        R.DS_FUSED_BWD[0] = False
        b_all = _ds_block_run(blk, x0, True)
    finally:
        R.DS_FUSED_BWD[0] = old
    assert (True, (256, 64)) in fused, fused
    for a, b in zip(a_all, b_all):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 1e-2, err


def test_deferred_shortcut_bn3_eval_gradients():
    """The deferred shortcut BN materialised for a non-fused consumer (bn3 frozen in eval while the
    block trains) must pass its gradient through unchanged: x / downsample grads equal the
    non-deferred run (the materialisation used to multiply the gradient by gamma*invstd again)."""
    blk = _make_ds_block(1)
    x0 = torch.randn(8, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    a_all, b_all = _ds_block_run(blk, x0, True, bn3_eval=True), _ds_block_run(blk, x0, False, bn3_eval=True)
    for a, b in zip(a_all, b_all):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 1e-2, err


def test_deferred_shortcut_forward_hook_sees_real_output():
    """A forward hook on downsample.1 sees the real BN output (deferral is skipped for hooked BNs)
    and the block's output is unchanged."""
    blk = _make_ds_block(1)
    x0 = torch.randn(8, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    seen = []
    h = blk.downsample[1].register_forward_hook(lambda m, i, o: seen.append((i[0].detach().clone(), o)))
    try:
        hooked = _ds_block_run(blk, x0, True)
    finally:
        h.remove()
    assert len(seen) == 1 and isinstance(seen[0][1], torch.Tensor)
    xin, out = seen[0]
    ref = torch.nn.functional.batch_norm(xin.float(), None, None, blk.downsample[1].weight.float(),
                                         blk.downsample[1].bias.float(), True, 0.0, 1e-5)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    plain = _ds_block_run(blk, x0, True)
    for a, b in zip(hooked, plain):
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 1e-2, err


def test_deferred_affine_materializes_for_other_readers():
    """A deferred BN output is an internal handle; materialize() gives the BN's value."""
    from pytorch_distributed_training_example_amd.ops.batchnorm import BatchNorm2d, DeferredBNOutput
    torch.manual_seed(0)
    bn = BatchNorm2d(64).cuda()
    x = torch.randn(4, 64, 8, 8, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    h = bn._forward_stats_only(x)
    assert isinstance(h, DeferredBNOutput) and not isinstance(h, torch.Tensor)
    bn2 = BatchNorm2d(64).cuda()
    y_ref = bn2(x)
    torch.testing.assert_close(h.materialize().float(), y_ref.float(), rtol=2e-2, atol=2e-2)
