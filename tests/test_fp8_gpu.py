"""FP8 (OCP e4m3fn) casts and Linear layers (csrc/kernels/fp8.hip, ops/fp8.py) vs PyTorch."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,k", [(64, 64), (25216, 768), (48, 2320)])
def test_cast_transpose_exact(m, k):
    from pytorch_distributed_training_example_amd.ops._native import native
    torch.manual_seed(0)
    x = (torch.randn(m, k, device="cuda") * 3).bfloat16()
    x[0, 0] = 1e4  # saturates at 448 after scaling
    st = torch.zeros(3 + 4, device="cuda")
    st[1], st[2] = 0.5, 2.0
    q, qt = native().fp8_cast_transpose(x, st, True)
    ref = (x.float() * 0.5).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(q.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(qt.view(torch.uint8), ref.t().contiguous().view(torch.uint8))
    assert st[0].item() == x.float().abs().max().item()


def test_update_scales_history():
    from pytorch_distributed_training_example_amd.ops.fp8 import Fp8State
    s = Fp8State(2, history=3).cuda()
    for amax in (10.0, 2.0, 1.0, 0.5):
        s.state[:, 0] = amax
        s.update()
    # history now [0.5, 1.0, 2.0] (10 shifted out): scale = 448 / 2
    torch.testing.assert_close(s.state[:, 1].cpu(), torch.full((2,), 224.0))
    torch.testing.assert_close(s.state[:, 2].cpu(), torch.full((2,), 1 / 224.0))
    assert (s.state[:, 0] == 0).all()


def test_fp8_linear_close_to_bf16():
    from pytorch_distributed_training_example_amd.ops.fp8 import Fp8State, fp8_linear
    torch.manual_seed(0)
    st = Fp8State(3, history=4).cuda()
    x = torch.randn(4, 200, 768, device="cuda").bfloat16().requires_grad_(True)
    w = (torch.randn(2304, 768, device="cuda") * 0.02).bfloat16().requires_grad_(True)
    b = torch.randn(2304, device="cuda").bfloat16().requires_grad_(True)
    g = torch.randn(4, 200, 2304, device="cuda").bfloat16()
    for _ in range(2):  # first pass calibrates the delayed scales
        st.update()
        x.grad = w.grad = b.grad = None
        y = fp8_linear(x, w, b, st, 0)
        y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(g.float())

    def rel(a, r):
        return ((a.float() - r).norm() / r.norm()).item()
    assert rel(y, yr) < 0.05
    assert rel(x.grad, xr.grad) < 0.08
    assert rel(w.grad, wr.grad) < 0.08
    assert rel(b.grad, br.grad) < 0.02


def test_vit_tiny_fp8_trains():
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import apply_precision
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    from pytorch_distributed_training_example_amd.optim import FusedAdamW
    torch.manual_seed(0)
    m = apply_precision(get_model("vit_tiny", num_classes=10).cuda(), "fp8")
    assert m.fp8_state.state.shape[0] == 3 * 4 * 2  # 4 linears x 2 blocks
    opt = FusedAdamW(m.parameters(), lr=1e-3)
    x = torch.randn(16, 3, 32, 32, device="cuda").bfloat16()
    y = torch.randint(0, 10, (16,), device="cuda")
    losses = []
    for _ in range(30):
        opt.zero_grad(set_to_none=True)
        loss = cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < 0.5 * losses[0], losses


def _st(scale):
    st = torch.zeros(3 + 4, device="cuda")
    st[1], st[2] = scale, 1.0 / scale
    return st


@pytest.mark.parametrize("m,d,tanh_form", [(25216, 3072, False), (8192, 4096, True), (48, 192, False)])
def test_gelu_cast_fwd_bit_identical_to_unfused(m, d, tanh_form):
    """fp8(gelu(h + b)) and its transpose in one pass == bias+GELU strip kernel then cast-transpose."""
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    torch.manual_seed(1)
    h = (torch.randn(m, d, device="cuda") * 2).bfloat16()
    b = torch.randn(d, device="cuda") * 0.5
    st_ref, st = _st(64.0), _st(64.0)
    g = C.bias_gelu_fwd(h, b, tanh_form)
    q_ref, qt_ref = C.fp8_cast_transpose(g, st_ref, True)
    q, qt, db = C.fp8_gelu_cast(h, None, b, st, tanh_form)
    assert db is None
    assert torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))
    assert torch.equal(qt.view(torch.uint8), qt_ref.view(torch.uint8))
    assert st[0].item() == st_ref[0].item() == g.float().abs().max().item()


@pytest.mark.parametrize("m,d,tanh_form", [(25216, 3072, False), (8192, 4096, True), (48, 192, False)])
def test_gelu_cast_bwd_bit_identical_to_unfused(m, d, tanh_form):
    """fp8(dg * gelu'(h + b)) (+ transpose) == GELU-backward strip kernel then cast-transpose; the
    bias gradient against the strip kernel's and an fp32 reference."""
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    torch.manual_seed(2)
    h = (torch.randn(m, d, device="cuda") * 2).bfloat16()
    dg = torch.randn(m, d, device="cuda").bfloat16()
    b = torch.randn(d, device="cuda") * 0.5
    st_ref, st = _st(32.0), _st(32.0)
    dh, db_ref = C.bias_gelu_bwd(dg, h, b, tanh_form)
    q_ref, qt_ref = C.fp8_cast_transpose(dh, st_ref, True)
    q, qt, db = C.fp8_gelu_cast(h, dg, b, st, tanh_form, torch.float32)
    assert torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))
    assert torch.equal(qt.view(torch.uint8), qt_ref.view(torch.uint8))
    assert st[0].item() == st_ref[0].item()
    torch.testing.assert_close(db, db_ref, rtol=1e-4, atol=1e-3)
    hf = (h.float() + b).requires_grad_(True)
    torch.nn.functional.gelu(hf, approximate="tanh" if tanh_form else "none").backward(dg.float())
    ref = hf.grad.sum(0)
    assert ((db - ref).norm() / ref.norm()).item() < 1e-4


def test_cast_multi_matches_per_tensor():
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    torch.manual_seed(3)
    shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072), (16, 48), (4096, 1024)] * 12  # > 64: two launches
    xs = [(torch.randn(*s, device="cuda") * 0.05).bfloat16() for s in shapes]
    rows = [_st(1024.0 + i) for i in range(len(xs))]
    rows_ref = [_st(1024.0 + i) for i in range(len(xs))]
    out = C.fp8_cast_multi(xs, rows)
    for i, x in enumerate(xs):
        q, qt = C.fp8_cast_transpose(x, rows_ref[i], True)
        assert torch.equal(out[2 * i].view(torch.uint8), q.view(torch.uint8)), i
        assert torch.equal(out[2 * i + 1].view(torch.uint8), qt.view(torch.uint8)), i
        assert rows[i][0].item() == rows_ref[i][0].item(), i


@pytest.mark.parametrize("approximate", ["none", "tanh"])
def test_fp8_mlp_fused_matches_per_linear_path(approximate):
    """The fused fp8 MLP (GELU casts + one-launch weight casts) against the per-Linear fp8 path: the
    same fp8 operands, so every output and gradient is bit-identical except the bias gradients
    (summation order)."""
    from pytorch_distributed_training_example_amd.config import SW
    from pytorch_distributed_training_example_amd.models.transformer import MLP
    from pytorch_distributed_training_example_amd.ops.fp8 import enable_fp8
    torch.manual_seed(4)
    mlp = MLP(768, 3072, approximate).cuda().bfloat16()

    class Wrap(torch.nn.Module):  # enable_fp8 tags Linears inside transformer Blocks; tag all here
        def __init__(self):
            super().__init__()
            self.mlp = mlp

        def forward(self, x):
            return self.mlp(x)
    wrap = Wrap()
    x0 = torch.randn(16, 197, 768, device="cuda").bfloat16()
    g = torch.randn(16, 197, 768, device="cuda").bfloat16()
    res = {}
    saved = (SW.fp8_fused_gelu, SW.fp8_weight_multi, SW.fp8_cast_colsum)
    try:
        for fused in (False, True):
            SW.fp8_fused_gelu = SW.fp8_weight_multi = SW.fp8_cast_colsum = fused
            st = enable_fp8(wrap, history=4, blocks_only=False)
            for _ in range(2):  # calibrate the delayed scales, then measure
                mlp.zero_grad(set_to_none=True)
                x = x0.clone().requires_grad_(True)
                y = wrap(x)
                y.backward(g)
            st.update()  # folds the amax stripes (which workgroup wrote which stripe differs by path)
            res[fused] = [y, x.grad, mlp.c_fc.weight.grad, mlp.c_fc.bias.grad, mlp.c_proj.weight.grad,
                          mlp.c_proj.bias.grad, st.state.clone()]
            wrap._fp8_hook.remove()
    finally:
        SW.fp8_fused_gelu, SW.fp8_weight_multi, SW.fp8_cast_colsum = saved
    a, b = res[False], res[True]
    for i in (0, 1, 2, 4, 6):
        assert torch.equal(a[i], b[i]), i
    for i in (3, 5):  # bias gradients: fused column sums, another summation order
        torch.testing.assert_close(a[i].float(), b[i].float(), rtol=2e-2, atol=1e-2)


@pytest.mark.parametrize("m,d", [(25216, 768), (25216, 2304), (8192, 1024), (48, 192)])
def test_cast_colsum_matches_cast_and_colsum(m, d):
    """dy -> (fp8, transpose) bit-identical to fp8_cast_transpose, and the bias gradient against the
    column-strip kernel and fp32."""
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    torch.manual_seed(5)
    x = torch.randn(m, d, device="cuda").bfloat16()
    st_ref, st = _st(100.0), _st(100.0)
    q_ref, qt_ref = C.fp8_cast_transpose(x, st_ref, True)
    q, qt, db = C.fp8_cast_colsum(x, st, torch.float32)
    assert torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))
    assert torch.equal(qt.view(torch.uint8), qt_ref.view(torch.uint8))
    assert st[0].item() == st_ref[0].item()
    ref = x.double().sum(0)
    assert ((db.double() - ref).norm() / ref.norm()).item() < 1e-5
    torch.testing.assert_close(db, C.colsum(x, torch.float32), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("n,d", [(25216, 768), (8192, 1024), (48, 512)])
def test_ln_fwd_fp8_bit_identical_to_ln_then_cast(n, d):
    """add + LayerNorm emitting e4m3 (+ transpose) == the bf16 add + LayerNorm kernel followed by the
    cast-transpose pass: the same bytes, statistics, residual sum and amax."""
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    torch.manual_seed(6)
    x = torch.randn(n, d, device="cuda").bfloat16()
    h = torch.randn(n, d, device="cuda").bfloat16()
    w = torch.rand(d, device="cuda") + 0.5
    b = torch.randn(d, device="cuda") * 0.1
    st_ref, st = _st(80.0), _st(80.0)
    y, mean_r, rstd_r, s_r = C.ln_fwd(x, w, b, 1e-6, h)
    q_ref, qt_ref = C.fp8_cast_transpose(y, st_ref, True)
    q, qt, mean, rstd, s = C.ln_fwd_fp8(x, w, b, 1e-6, h, st)
    assert torch.equal(s, s_r) and torch.equal(mean, mean_r) and torch.equal(rstd, rstd_r)
    assert torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))
    assert torch.equal(qt.view(torch.uint8), qt_ref.view(torch.uint8))
    assert st[0].item() == st_ref[0].item()


def test_vit_blocks_fp8_ln_matches_cast_path():
    """Two ViT-B/16-width blocks + final LayerNorm, fp8: the add+LayerNorm emitting e4m3 for qkv / fc1
    (PDT_FP8_LN) against the bf16 LayerNorm + cast path — bit-identical outputs and gradients."""
    from pytorch_distributed_training_example_amd.config import SW
    from pytorch_distributed_training_example_amd.models.transformer import Block, run_blocks
    from pytorch_distributed_training_example_amd.ops.fp8 import enable_fp8
    from pytorch_distributed_training_example_amd.ops.layernorm import LayerNorm
    torch.manual_seed(7)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.blocks = torch.nn.ModuleList([Block(768, 12, eps=1e-6) for _ in range(2)])
            self.ln_f = LayerNorm(768, eps=1e-6)

        def forward(self, x):
            return run_blocks(self.blocks, x, self.ln_f)
    net = Net().cuda()
    for m in net.modules():  # bf16 weights, fp32 LayerNorm parameters (models/precision.py)
        if isinstance(m, torch.nn.Linear):
            m.to(torch.bfloat16)
    x0 = torch.randn(16, 197, 768, device="cuda").bfloat16()
    g = torch.randn(16, 197, 768, device="cuda").bfloat16()
    res = {}
    saved = SW.fp8_ln
    try:
        for on in (False, True):
            SW.fp8_ln = on
            st = enable_fp8(net, history=4)
            for _ in range(2):
                net.zero_grad(set_to_none=True)
                x = x0.clone().requires_grad_(True)
                y = net(x)
                y.backward(g)
            st.update()  # folds the amax stripes (which workgroup wrote which stripe differs by path)
            res[on] = [y, x.grad, st.state.clone()] + [p.grad.clone() for p in net.parameters()]
            net._fp8_hook.remove()
    finally:
        SW.fp8_ln = saved
    for i, (a, b) in enumerate(zip(res[False], res[True])):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("kind", ["cast", "colsum", "gelu", "ln"])
def test_striped_amax_rows(kind):
    """Producers writing into a striped state row (Fp8State): after update() the newest history
    entry is the tensor's |x|max, the stripes are cleared, and the bytes equal the unstriped cast."""
    from pytorch_distributed_training_example_amd.ops._native import native
    from pytorch_distributed_training_example_amd.ops.fp8 import Fp8State
    C = native()
    torch.manual_seed(9)
    st = Fp8State(1, history=4).cuda()
    st.state[0, 1], st.state[0, 2] = 8.0, 0.125
    ref = _st(8.0)
    x = torch.randn(25216, 768, device="cuda").bfloat16()
    if kind == "cast":
        q, _ = C.fp8_cast_transpose(x, st.state[0], True)
        q_ref, _ = C.fp8_cast_transpose(x, ref, True)
    elif kind == "colsum":
        q, _, _ = C.fp8_cast_colsum(x, st.state[0], torch.float32)
        q_ref, _, _ = C.fp8_cast_colsum(x, ref, torch.float32)
    elif kind == "gelu":
        b = torch.randn(768, device="cuda")
        q, _, _ = C.fp8_gelu_cast(x, None, b, st.state[0], False)
        q_ref, _, _ = C.fp8_gelu_cast(x, None, b, ref, False)
    else:
        h = torch.randn_like(x)
        w, lb = torch.rand(768, device="cuda") + 0.5, torch.randn(768, device="cuda")
        q = C.ln_fwd_fp8(x, w, lb, 1e-6, h, st.state[0])[0]
        q_ref = C.ln_fwd_fp8(x, w, lb, 1e-6, h, ref)[0]
    assert torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))
    assert st.state[0, 0].item() == 0.0  # the stripes took every workgroup's maximum
    st.update()
    assert st.state[0, Fp8State.STRIPED].item() == ref[0].item() > 0
    assert (st.state[0, 4:Fp8State.STRIPED] == 0).all()


def test_weight_cache_recasts_after_inplace_update():
    """Fp8State.cast_weights caches each weight's fp8 copies for one forward; a weight modified in place after the
    cast (optimizer.step, then a submodule called directly) must not be served from the stale copy."""
    from pytorch_distributed_training_example_amd.ops.fp8 import Fp8State
    torch.manual_seed(5)
    lin = torch.nn.Linear(256, 128, bias=False).cuda().bfloat16()
    st = Fp8State(3).cuda()
    lin._fp8 = (st, st.alloc(3))
    st.cast_weights([lin])
    q0, _ = st.weight_fp8(lin.weight, 0)
    assert st.weight_fp8(lin.weight, 0)[0] is q0  # served from the cache while unchanged
    with torch.no_grad():
        lin.weight.mul_(-1.0)
    q1, _ = st.weight_fp8(lin.weight, 0)
    assert q1 is not q0
    from pytorch_distributed_training_example_amd.ops._native import native
    want, _ = native().fp8_cast_transpose(lin.weight, st.state[1].clone(), True)  # same scale row, fresh cast
    assert torch.equal(q1.view(torch.uint8), want.view(torch.uint8)), "recast of the updated weight"
    assert not torch.equal(q1.view(torch.uint8), q0.view(torch.uint8))
    st.clear_weight_cache()
    assert st.wcache == {}
