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
