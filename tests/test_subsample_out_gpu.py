"""The stride-2 subsample written by a ResNet stage's last BatchNorm apply (ops/batchnorm.py ``sub_stride``,
csrc/kernels/batchnorm.hip SubOut): it equals ``y[:, :, ::2, ::2]`` bit for bit, the next stage's strided shortcut
takes it instead of its gather pass, and the model's outputs and gradients are unchanged. The reference's model has
no strided shortcut (/root/reference/cnn.py:9-23); SURVEY §2.3 asks for the elementwise passes fused."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C,H,W", [(4, 256, 56, 56), (3, 512, 13, 15), (2, 1024, 14, 14)])
def test_apply_writes_subsample(N, C, H, W):
    from pytorch_distributed_training_example_amd.ops._native import native
    torch.manual_seed(N + C)
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x)
    M = N * H * W
    T = (M + 255) // 256
    xf = x.permute(0, 2, 3, 1).reshape(M, C).float()
    pad = torch.cat([xf, xf.new_zeros(T * 256 - M, C)]).view(T, 256, C)
    cnt = torch.tensor([min(256, M - t * 256) for t in range(T)], device="cuda").float().view(T, 1)
    s1 = pad.sum(1)
    mu = s1 / cnt
    q = ((pad - mu.view(T, 1, C)) ** 2 * (torch.arange(256, device="cuda").view(1, 256, 1) <
                                          cnt.view(T, 1, 1)).float()).sum(1)
    part = torch.stack([s1, q]).contiguous()
    w, b = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y, mask, mean, invstd, ys = native().bn_fwd_train_tiles(x, part, res, w, b, rm, rv, 0.1, 1e-5, True, sub=2)
    assert ys.shape == (N, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1)
    assert ys.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(ys, y[:, :, ::2, ::2])
    y2, mask2, _, _ = native().bn_fwd_train_tiles(x, part, res, w, b, rm.clone(), rv.clone(), 0.1, 1e-5, True)
    assert torch.equal(y, y2) and torch.equal(mask, mask2)


def test_resnet50_gather_replaced_and_unchanged():
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops import conv as conv_ops
    torch.manual_seed(0)
    m = to_bf16_mixed(get_model("resnet50", num_classes=10).cuda().to(memory_format=torch.channels_last))
    assert [m.layer1[-1].emit_sub, m.layer2[-1].emit_sub, m.layer3[-1].emit_sub, m.layer4[-1].emit_sub] == [2, 2, 2, 0]
    # (the shape of tests/test_determinism_gpu.py, whose step is bit-reproducible: at 4 x 112 x 112 the stem weight
    # gradient is not, tools/diag_sub_out.py)
    x = torch.randn(8, 3, 96, 96, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    taken = []
    orig = conv_ops.subsample_of

    def spy(t, s):
        r = orig(t, s)
        taken.append(r is not None)
        return r

    def step():
        m.zero_grad(set_to_none=True)
        out = m(x)
        torch.nn.functional.cross_entropy(out.float(), y).backward()
        return [out.detach()] + [p.grad.clone() for p in m.parameters()]
    conv_ops.subsample_of = spy
    try:
        a = step()
        assert taken == [True, True, True], taken
        for blk in (m.layer1[-1], m.layer2[-1], m.layer3[-1]):
            blk.emit_sub = 0
        taken.clear()
        b = step()
        assert taken == [False, False, False], taken
    finally:
        conv_ops.subsample_of = orig
    assert all(torch.equal(u, v) for u, v in zip(a, b))
