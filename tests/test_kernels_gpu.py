"""Numerics of every gfx950 HIP kernel vs a plain PyTorch fp32 reference of the same op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _native():
    from pytorch_distributed_training_example_amd.ops._native import native
    return native()


# ----------------------------------------------------------------------------- BatchNorm NHWC
@pytest.mark.parametrize("C", [64, 256, 2048, 4096, 192])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True), (False, True)])
def test_batchnorm_train_fwd_bwd(C, relu, res):
    from pytorch_distributed_training_example_amd.ops.batchnorm import batch_norm_act
    torch.manual_seed(0)
    N, H, W = (4, 7, 9) if C >= 1024 else (8, 14, 13)
    x = (torch.randn(N, C, H, W, device=DEV) * 2 + 0.5).to(torch.bfloat16).to(memory_format=torch.channels_last)
    r = torch.randn_like(x) if res else None
    w = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm2, rv2 = rm.clone(), rv.clone()
    xs = x.detach().requires_grad_(True)
    ws, bs = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rs = r.detach().requires_grad_(True) if res else None
    y = batch_norm_act(xs, rs, ws, bs, rm, rv, True, 0.1, 1e-5, relu)
    # fp32 reference
    xf = x.float().detach().requires_grad_(True)
    wf, bf = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rf = r.float().detach().requires_grad_(True) if res else None
    yf = F.batch_norm(xf, rm2, rv2, wf, bf, True, 0.1, 1e-5)
    if res:
        yf = yf + rf
    if relu:
        yf = F.relu(yf)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), yf, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(rm, rm2, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rv, rv2, rtol=1e-3, atol=1e-3)
    g = torch.randn_like(y)
    y.backward(g)
    yf.backward(g.float())
    torch.testing.assert_close(xs.grad.float(), xf.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(ws.grad, wf.grad, rtol=2e-2, atol=2e-1)
    torch.testing.assert_close(bs.grad, bf.grad, rtol=2e-2, atol=2e-1)
    if res:
        torch.testing.assert_close(rs.grad.float(), rf.grad, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (3, 128, 15, 17)])
def test_bn_relu_maxpool_stem(shape):
    """Fused BN + ReLU + MaxPool2d(3,2,1) (ResNet stem) vs the fp32 unfused reference."""
    from pytorch_distributed_training_example_amd.ops.batchnorm import batch_norm_relu_maxpool
    torch.manual_seed(0)
    N, C, H, W = shape
    x = (torch.randn(N, C, H, W, device=DEV) * 2 + 0.3).to(torch.bfloat16).to(memory_format=torch.channels_last)
    w, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.5
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm2, rv2 = rm.clone(), rv.clone()
    xs = x.detach().requires_grad_(True)
    ws, bs = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = batch_norm_relu_maxpool(xs, ws, bs, rm, rv, True, 0.1, 1e-5)
    xf = x.float().detach().requires_grad_(True)
    wf, bf = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yf = F.max_pool2d(F.relu(F.batch_norm(xf, rm2, rv2, wf, bf, True, 0.1, 1e-5)), 3, 2, 1)
    assert y.shape == yf.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), yf, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(rm, rm2, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    yf.backward(g.float())
    # near-ties inside a window may route a gradient differently than the fp32 oracle: allow a
    # tiny fraction of elements to differ, everything else must match tightly
    bad = ((xs.grad.float() - xf.grad).abs() > 3e-2 + 3e-2 * xf.grad.abs()).float().mean().item()
    assert bad < 1e-4, bad
    torch.testing.assert_close(ws.grad, wf.grad, rtol=2e-2, atol=5e-1)
    torch.testing.assert_close(bs.grad, bf.grad, rtol=2e-2, atol=5e-1)


@pytest.mark.parametrize("C,N,H", [(64, 32, 37), (128, 16, 29), (1024, 12, 15), (2048, 9, 7)])
@pytest.mark.parametrize("variant", [2, 5])
def test_batchnorm_reduce_variants_large_m(C, N, H, variant):
    """The BN reduce implementations (v2: in-kernel two-level finalize; v5 = default: pipelined
    wide-chunk reduce + separate finalize kernel) at row counts that exercise several pipelined
    iterations per workgroup and ragged tails, against the fp32 reference."""
    C_ = _native()
    torch.manual_seed(1)
    try:
        C_.bn_tune(variant, 512, 8, 4)
        x = (torch.randn(N, C, H, H, device=DEV) * 1.5 + 0.7).to(torch.bfloat16).to(memory_format=torch.channels_last)
        w, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        y, mask, mean, invstd = C_.bn_fwd_train(x, None, w, b, rm, rv, 0.1, 1e-5, True)
        xf = x.float()
        mu = xf.mean(dim=(0, 2, 3))
        var = xf.var(dim=(0, 2, 3), unbiased=False)
        torch.testing.assert_close(mean, mu, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(invstd, torch.rsqrt(var + 1e-5), rtol=1e-3, atol=1e-3)
        yf = F.relu((xf - mu.view(1, -1, 1, 1)) * (w * torch.rsqrt(var + 1e-5)).view(1, -1, 1, 1) + b.view(1, -1, 1, 1))
        torch.testing.assert_close(y.float(), yf, rtol=2e-2, atol=3e-2)
        dy = torch.randn_like(x)
        dx, _, dg, db = C_.bn_bwd_train(dy, x, mask, w, mean, invstd, True, False, True)
        dz = dy.float() * (yf > 0)
        xhat = (xf - mu.view(1, -1, 1, 1)) * torch.rsqrt(var + 1e-5).view(1, -1, 1, 1)
        torch.testing.assert_close(db, dz.sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-1)
        torch.testing.assert_close(dg, (dz * xhat).sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-1)
    finally:
        C_.bn_tune(5, 512, 8, 4)


def test_batchnorm_large_mean_stability():
    """Shifted sums must not lose the variance when |mean| >> std."""
    from pytorch_distributed_training_example_amd.ops.batchnorm import batch_norm_act
    C = 64
    x = (torch.randn(32, C, 16, 16, device=DEV) * 0.5 + 40.0).to(torch.bfloat16).to(memory_format=torch.channels_last)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    y = batch_norm_act(x, None, None, None, rm, rv, True, 1.0, 1e-5, False)
    yf = F.batch_norm(x.float(), None, None, None, None, True, 0.0, 1e-5)
    torch.testing.assert_close(y.float(), yf, rtol=3e-2, atol=6e-2)


def test_batchnorm_eval():
    from pytorch_distributed_training_example_amd.ops.batchnorm import BatchNorm2d
    C = 128
    bn = BatchNorm2d(C, fused_relu=True).to(DEV).eval()
    bn.running_mean.uniform_(-1, 1)
    bn.running_var.uniform_(0.5, 2)
    x = torch.randn(4, C, 8, 8, device=DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    y = bn(x)
    yf = F.relu(F.batch_norm(x.float(), bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.1, bn.eps))
    torch.testing.assert_close(y.float(), yf, rtol=2e-2, atol=2e-2)


# ----------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("D", [256, 768, 1024])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm(D, dtype):
    from pytorch_distributed_training_example_amd.ops.layernorm import layer_norm
    torch.manual_seed(0)
    x = (torch.randn(37, 5, D, device=DEV) * 3 + 1).to(dtype).requires_grad_(True)
    w = (torch.rand(D, device=DEV) + 0.5).requires_grad_(True)
    b = torch.randn(D, device=DEV).requires_grad_(True)
    y = layer_norm(x, (D,), w, b, 1e-5)
    xf = x.detach().float().requires_grad_(True)
    wf, bf = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yf = F.layer_norm(xf, (D,), wf, bf, 1e-5)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(y.float(), yf, **tol)
    g = torch.randn_like(yf)
    y.backward(g.to(dtype))
    yf.backward(g.to(dtype).float())
    torch.testing.assert_close(x.grad.float(), xf.grad, **(tol if dtype == torch.float32 else dict(rtol=3e-2, atol=5e-2)))
    torch.testing.assert_close(w.grad, wf.grad, rtol=1e-3 if dtype == torch.float32 else 2e-2, atol=1e-2 if dtype == torch.float32 else 3e-1)
    torch.testing.assert_close(b.grad, bf.grad, rtol=1e-3, atol=1e-2 if dtype == torch.float32 else 3e-1)


@pytest.mark.parametrize("D", [768, 1024])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_add_layernorm_fused(D, dtype):
    """(s, y) = (x + h, LN(x + h)) with both outputs consumed downstream: values and the
    gradients of x, h (ds + LN'(dy), one kernel) against an fp32 PyTorch reference."""
    from pytorch_distributed_training_example_amd.ops.layernorm import LayerNorm, add_layer_norm
    torch.manual_seed(0)
    ln = LayerNorm(D).to(DEV)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.normal_()
    x = (torch.randn(6, 33, D, device=DEV) * 2 + 0.5).to(dtype).requires_grad_(True)
    h = torch.randn(6, 33, D, device=DEV).to(dtype).requires_grad_(True)
    s, y = add_layer_norm(x, h, ln)
    xf, hf = x.detach().float().requires_grad_(True), h.detach().float().requires_grad_(True)
    wf, bf = ln.weight.detach().clone().requires_grad_(True), ln.bias.detach().clone().requires_grad_(True)
    sf = xf + hf
    yf = F.layer_norm(sf, (D,), wf, bf, ln.eps)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(s.float(), sf, **tol)
    torch.testing.assert_close(y.float(), yf, **tol)
    gs, gy = torch.randn_like(sf), torch.randn_like(yf)
    (s.float() * gs.to(dtype).float()).sum().add((y.float() * gy.to(dtype).float()).sum()).backward()
    ((sf * gs.to(dtype).float()).sum() + (yf * gy.to(dtype).float()).sum()).backward()
    gtol = tol if dtype == torch.float32 else dict(rtol=3e-2, atol=5e-2)
    torch.testing.assert_close(x.grad.float(), xf.grad, **gtol)
    torch.testing.assert_close(h.grad.float(), hf.grad, **gtol)
    torch.testing.assert_close(ln.weight.grad, wf.grad, rtol=2e-2, atol=3e-1)
    torch.testing.assert_close(ln.bias.grad, bf.grad, rtol=2e-2, atol=3e-1)


# ----------------------------------------------------------------------------- cross entropy
@pytest.mark.parametrize("V", [10, 1000, 50304, 50257])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_cross_entropy(V, dtype, smoothing):
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    torch.manual_seed(0)
    N = 33
    logits = (torch.randn(N, V, device=DEV) * 3).to(dtype).requires_grad_(True)
    t = torch.randint(0, V, (N,), device=DEV)
    t[3] = -100
    loss = cross_entropy(logits, t, label_smoothing=smoothing)
    lf = logits.detach().float().requires_grad_(True)
    ref = F.cross_entropy(lf, t, label_smoothing=smoothing)
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    loss.backward()
    ref.backward()
    tol = dict(rtol=1e-4, atol=1e-6) if dtype == torch.float32 else dict(rtol=2e-2, atol=1e-4)
    torch.testing.assert_close(logits.grad.float(), lf.grad, **tol)


# ----------------------------------------------------------------------------- bias + gelu
@pytest.mark.parametrize("approx", ["none", "tanh"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,d", [(67, 3072), (4099, 776), (3, 1024)])
def test_bias_gelu(approx, dtype, n, d):
    from pytorch_distributed_training_example_amd.ops.gelu import bias_gelu
    torch.manual_seed(0)
    x = torch.randn(n, d, device=DEV).to(dtype).requires_grad_(True)
    b = torch.randn(d, device=DEV).requires_grad_(True)
    y = bias_gelu(x, b, approx)
    xf = x.detach().float().requires_grad_(True)
    bf = b.detach().clone().requires_grad_(True)
    yf = F.gelu(xf + bf, approximate=approx)
    tol = dict(rtol=1e-4, atol=1e-5) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(y.float(), yf, **tol)
    g = torch.randn_like(yf)
    y.backward(g.to(dtype))
    yf.backward(g.to(dtype).float())
    torch.testing.assert_close(x.grad.float(), xf.grad, **tol)
    torch.testing.assert_close(b.grad, bf.grad, rtol=1e-3 if dtype == torch.float32 else 3e-2, atol=1e-3 if dtype == torch.float32 else 3e-1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8, 1024, 1024), (25216, 768), (5, 3072), (0, 64)])
def test_colsum_bias_grad(dtype, shape):
    from pytorch_distributed_training_example_amd.ops._native import native
    torch.manual_seed(0)
    x = torch.randn(*shape, device=DEV).to(dtype)
    out = native().colsum(x.reshape(-1, shape[-1]), dtype)
    ref = x.reshape(-1, shape[-1]).double().sum(0)
    tol = 1e-3 * max(1.0, (x.numel() / shape[-1]) ** 0.5)
    torch.testing.assert_close(out.double(), ref.to(out.dtype).double(), rtol=1e-2 if dtype == torch.bfloat16 else 1e-5,
                               atol=tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_linear_native_bias_grad(dtype):
    from pytorch_distributed_training_example_amd.ops.linear import linear
    torch.manual_seed(0)
    x = torch.randn(4, 33, 256, device=DEV).to(dtype).requires_grad_(True)
    w = (torch.randn(96, 256, device=DEV) * 0.05).to(dtype).requires_grad_(True)
    b = torch.randn(96, device=DEV).to(dtype).requires_grad_(True)
    y = linear(x, w, b)
    x2, w2, b2 = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    y2 = torch.nn.functional.linear(x2, w2, b2)
    torch.testing.assert_close(y, y2)
    g = torch.randn_like(y)
    y.backward(g)
    y2.backward(g)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=5e-2)
    for a, r in ((x.grad, x2.grad), (w.grad, w2.grad), (b.grad, b2.grad)):
        torch.testing.assert_close(a.float(), r.float(), **tol)


# ----------------------------------------------------------------------------- optimizers
def _params(dtype=torch.float32, channels_last=False):
    torch.manual_seed(0)
    shapes = [(64, 3, 7, 7), (64,), (1000, 2048), (3,), (70001,), (5, 5)]
    ps = []
    for s in shapes:
        p = torch.randn(s, device=DEV)
        if channels_last and len(s) == 4:
            p = p.to(memory_format=torch.channels_last)
        ps.append(torch.nn.Parameter(p.to(dtype)))
    return ps


def _run_opt(make, ps, steps=3, seed=1):
    g = torch.Generator(device=DEV).manual_seed(seed)
    opt = make(ps)
    for _ in range(steps):
        for p in ps:
            p.grad = torch.randn(p.shape, device=DEV, generator=g).to(p.dtype)
            if p.dim() == 4:
                p.grad = p.grad.contiguous(memory_format=torch.channels_last) if p.is_contiguous(memory_format=torch.channels_last) else p.grad
        opt.step()
    return ps, opt


@pytest.mark.parametrize("nesterov,wd,mom", [(False, 0.0, 0.0), (False, 1e-4, 0.9), (True, 5e-5, 0.9)])
def test_fused_sgd_matches_torch(nesterov, wd, mom):
    from pytorch_distributed_training_example_amd.optim import FusedSGD
    a, _ = _run_opt(lambda ps: FusedSGD(ps, lr=0.1, momentum=mom, weight_decay=wd, nesterov=nesterov), _params(channels_last=True))
    b, _ = _run_opt(lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=mom, weight_decay=wd, nesterov=nesterov), _params(channels_last=True))
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("wd,adamw", [(0.0, False), (1e-2, True), (1e-2, False)])
def test_fused_adam_matches_torch(wd, adamw):
    from pytorch_distributed_training_example_amd.optim import FusedAdam
    a, _ = _run_opt(lambda ps: FusedAdam(ps, lr=1e-3, weight_decay=wd, adam_w_mode=adamw), _params())
    cls = torch.optim.AdamW if adamw else torch.optim.Adam
    b, _ = _run_opt(lambda ps: cls(ps, lr=1e-3, weight_decay=wd), _params())
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_fused_adadelta_matches_torch():
    from pytorch_distributed_training_example_amd.optim import FusedAdadelta
    a, oa = _run_opt(lambda ps: FusedAdadelta(ps, lr=0.1), _params())
    b, ob = _run_opt(lambda ps: torch.optim.Adadelta(ps, lr=0.1), _params())
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)
    # state layout identical to torch (checkpoint compatible)
    sa, sb = oa.state_dict()["state"][0], ob.state_dict()["state"][0]
    assert set(sa) == set(sb)


def test_master_weights_bf16():
    from pytorch_distributed_training_example_amd.optim import FusedSGD
    ps = _params(torch.bfloat16)
    ref = [torch.nn.Parameter(p.detach().float()) for p in ps]
    a, oa = _run_opt(lambda q: FusedSGD(q, lr=0.1, momentum=0.9), ps)
    b, _ = _run_opt(lambda q: torch.optim.SGD(q, lr=0.1, momentum=0.9), ref)
    for p, r in zip(a, b):
        m = oa.state[p]["master_param"]
        torch.testing.assert_close(m, r, rtol=2e-2, atol=2e-2)
        assert torch.equal(p.detach(), m.to(torch.bfloat16))


def test_amp_skip_on_inf_and_unscale():
    from pytorch_distributed_training_example_amd.optim import FusedSGD
    from pytorch_distributed_training_example_amd.ops import multi_tensor as mt
    ps = _params()
    before = [p.detach().clone() for p in ps]
    opt = FusedSGD(ps, lr=0.1)
    for p in ps:
        p.grad = torch.ones_like(p) * 4
    ps[2].grad[3, 3] = float("inf")
    inv = torch.full((1,), 0.25, device=DEV)
    found = torch.zeros(1, device=DEV)
    mt.unscale_([p.grad for p in ps], inv, found)
    assert found.item() == 1.0
    assert ps[0].grad[0, 0, 0, 0].item() == 1.0
    opt.step(found_inf=found)
    for p, q in zip(ps, before):
        assert torch.equal(p.detach(), q)


def test_l2norm_and_clip():
    from pytorch_distributed_training_example_amd.ops import multi_tensor as mt
    gs = [torch.randn(s, device=DEV) for s in [(100003,), (7, 9), (64, 64, 3, 3)]] + [torch.randn(1000, device=DEV).bfloat16()]
    ref = torch.sqrt(sum((g.float() ** 2).sum() for g in gs))
    norm = mt.clip_grad_norm_(gs, 1.0)
    torch.testing.assert_close(norm.reshape(()), ref, rtol=1e-4, atol=1e-4)
    after = torch.sqrt(sum((g.float() ** 2).sum() for g in gs))
    assert abs(after.item() - 1.0) < 1e-2


def test_mt_copy_with_scale():
    from pytorch_distributed_training_example_amd.ops import multi_tensor as mt
    src = [torch.randn(s, device=DEV) for s in [(5,), (33333,), (4, 4)]]
    dst = [torch.empty(s.shape, device=DEV, dtype=torch.bfloat16) for s in src]
    mt.copy_(src, dst, factor=0.5)
    for s, d in zip(src, dst):
        torch.testing.assert_close(d.float(), (s * 0.5).bfloat16().float())


# ----------------------------------------------------------------------------- flash attention
@pytest.mark.parametrize("B,T,H,causal", [(2, 197, 3, False), (2, 256, 2, True), (1, 100, 4, True),
                                          (3, 64, 1, False), (1, 1024, 2, True)])
def test_flash_attention_qkv(B, T, H, causal):
    from pytorch_distributed_training_example_amd.ops.attention import _views, attention_qkv, attention_reference
    torch.manual_seed(0)
    Dh = 64
    qkv = (torch.randn(B, T, 3 * H * Dh, device=DEV) * 1.5).bfloat16().requires_grad_(True)
    y = attention_qkv(qkv, H, causal=causal)
    ref_in = qkv.detach().float().requires_grad_(True)
    (q, k, v), _ = _views(ref_in, H)
    yr = attention_reference(q, k, v, causal).transpose(1, 2).reshape(B, T, H * Dh)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g.bfloat16().float())
    err = (qkv.grad.float() - ref_in.grad).norm() / ref_in.grad.norm()
    assert err < 2e-2, err
    # per-slice check (dq / dk / dv)
    for i in range(3):
        a = qkv.grad.float().view(B, T, 3, H, Dh)[:, :, i]
        b = ref_in.grad.view(B, T, 3, H, Dh)[:, :, i]
        assert (a - b).norm() / (b.norm() + 1e-6) < 3e-2, (i, ((a - b).norm() / b.norm()).item())


@pytest.mark.parametrize("S,shape", [(2, (64, 8)), (4, (3072, 1024)), (16, (768, 768)), (64, (128, 512))])
def test_slice_sum_matches_fp32(S, shape):
    """csrc/kernels/slice_sum.hip: sum over the leading slice dimension (split-K weight gradients)."""
    from pytorch_distributed_training_example_amd.ops._native import native
    x = torch.randn(S, *shape, device="cuda").bfloat16()
    out = native().slice_sum(x)
    assert out.shape == shape and out.dtype == torch.bfloat16
    torch.testing.assert_close(out.float(), x.float().sum(0), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("shape,s", [((4, 256, 56, 56), 2), ((3, 64, 9, 14), 2), ((2, 24, 7, 7), 3)])
def test_subsample_gather_and_scatter_add(shape, s):
    """csrc/kernels/subsample.hip: x[:, :, ::s, ::s] and its adjoint full[:, :, ::s, ::s] += t."""
    from pytorch_distributed_training_example_amd.ops._native import native
    x = torch.randn(*shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xs = native().subsample_gather(x, s)
    ref = x[:, :, ::s, ::s]
    assert xs.shape == ref.shape and xs.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(xs, ref, rtol=0, atol=0)
    full = torch.randn(*shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    t = torch.randn_like(xs)
    exp = full.float()
    exp[:, :, ::s, ::s] += t.float()
    native().subsample_scatter_add(t, full, s)
    torch.testing.assert_close(full.float(), exp, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("approx", ["none", "tanh"])
@pytest.mark.parametrize("n,d", [(67, 3072), (4099, 776), (3, 1024)])
def test_bias_gelu_bf16_bias_matches_fp32_bias(approx, n, d):
    """A bf16 bias (a bf16 model's parameter) is read as is: the same y and dx bit for bit as its fp32 copy, and its
    gradient is the fp32 path's bias gradient rounded to bf16 (no aten cast kernels around the MLP)."""
    from pytorch_distributed_training_example_amd.ops.gelu import bias_gelu
    torch.manual_seed(1)
    x = torch.randn(n, d, device=DEV).bfloat16()
    b16 = torch.randn(d, device=DEV).bfloat16()
    g = torch.randn(n, d, device=DEV).bfloat16()
    xa = x.clone().requires_grad_(True)
    ba = b16.clone().requires_grad_(True)
    ya = bias_gelu(xa, ba, approx)
    ya.backward(g)
    xb = x.clone().requires_grad_(True)
    bb = b16.float().requires_grad_(True)
    yb = bias_gelu(xb, bb, approx)
    yb.backward(g)
    assert ba.grad.dtype == torch.bfloat16
    assert torch.equal(ya, yb) and torch.equal(xa.grad, xb.grad)
    assert torch.equal(ba.grad, bb.grad.bfloat16())
