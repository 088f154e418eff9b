"""Batched per-step weight transforms (csrc/kernels/weight_prep.hip, ops/conv.py prepare_weights): each
transformed weight equals the per-conv transform it replaces (W^T of a 1x1 weight, conv3x3_flip of a 3x3
weight), and a ResNet-50 step's gradients are bit-identical with the batched prep on and off."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_weight_prep_matches_per_conv_transforms():
    from pytorch_distributed_training_example_amd.ops._native import native
    torch.manual_seed(0)
    shapes = [(256, 64, 1), (64, 256, 1), (2048, 512, 1), (96, 40, 1), (70, 30, 1), (64, 64, 3), (128, 128, 3), (512, 256, 3),
              (192, 64, 3), (24, 13, 3)] * 7  # 70 items: more than one launch
    srcs = []
    for co, ci, k in shapes:
        w = torch.randn(co, ci, k, k, device="cuda").bfloat16()
        srcs.append(w.contiguous(memory_format=torch.channels_last) if k == 3 else w)
    dsts = [torch.empty(ci, co, device="cuda", dtype=torch.bfloat16) if k == 1 else
            torch.empty(ci, co, 3, 3, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
            for co, ci, k in shapes]
    native().weight_prep(srcs, dsts)
    for (co, ci, k), w, d in zip(shapes, srcs, dsts):
        want = w.view(co, ci).t() if k == 1 else native().conv3x3_flip(w)
        assert torch.equal(d, want), (co, ci, k)


def test_resnet50_grads_identical_with_batched_prep():
    from pytorch_distributed_training_example_amd.models import get_model, resnet
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops import conv as conv_ops
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    torch.manual_seed(0)
    m = to_bf16_mixed(get_model("resnet50", num_classes=16).cuda().to(memory_format=torch.channels_last))
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(8, 3, 96, 96, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 16, (8,), device="cuda", generator=g)

    def grads(on):
        resnet.PREP_WEIGHTS[0] = on
        if not on:
            conv_ops._PREP["stamp"] += 1  # invalidate the copies of the previous run
        m.zero_grad(set_to_none=True)
        cross_entropy(m(x), y).backward()
        return [p.grad.clone() for p in m.parameters()]
    calls = []
    orig = conv_ops.prepared

    def spy(w):
        r = orig(w)
        calls.append(r is not None)
        return r
    conv_ops.prepared = spy
    try:
        a = grads(True)
    finally:
        conv_ops.prepared = orig
    b = grads(False)
    resnet.PREP_WEIGHTS[0] = True
    assert calls and all(calls), f"{calls.count(False)} of {len(calls)} backward transforms missed the batched prep"
    bad = [i for i, (u, v) in enumerate(zip(a, b)) if not torch.equal(u, v)]
    assert not bad, bad
