"""CPU checks of the round-6 ResNet plumbing that needs no GPU: which blocks write the next stage's shortcut subsample
(models/resnet.py emit_sub), the subsample hand-off's version check (ops/conv.py subsample_of), and the shortcut
gradient record the ALG shortcut path reads (ops/batchnorm.py MaskedGrad). The reference model has no residual
stages (/root/reference/cnn.py:9-23); SURVEY §2.3 asks for these elementwise passes fused."""
import torch

from pytorch_distributed_training_example_amd.models import get_model
from pytorch_distributed_training_example_amd.ops.batchnorm import MaskedGrad
from pytorch_distributed_training_example_amd.ops.conv import subsample_of


def test_stage_last_blocks_emit_subsample():
    m = get_model("resnet50", num_classes=10)
    assert [m.layer1[-1].emit_sub, m.layer2[-1].emit_sub, m.layer3[-1].emit_sub, m.layer4[-1].emit_sub] == [2, 2, 2, 0]
    assert all(b.emit_sub == 0 for layer in (m.layer1, m.layer2, m.layer3, m.layer4) for b in layer[:-1])
    r18 = get_model("resnet18", num_classes=10)  # BasicBlock stages: no bn3 apply to carry it
    assert not any(getattr(b, "emit_sub", 0) for b in r18.modules())


def test_subsample_handoff_checks_version():
    x = torch.randn(2, 8, 6, 6)
    ys = x[:, :, ::2, ::2].contiguous()
    x._pdt_sub = (2, ys, x._version)
    assert subsample_of(x, 2) is ys
    assert subsample_of(x, 3) is None  # another stride
    x.add_(1.0)  # modified in place after the producer wrote the subsample: stale
    assert subsample_of(x, 2) is None
    assert subsample_of(torch.randn(1, 1, 2, 2), 2) is None


def test_masked_grad_carries_alg_fields():
    dy = torch.randn(2, 8, 3, 3)
    mask = torch.zeros(2 * 8 * 9 // 8, dtype=torch.uint8)
    g = MaskedGrad(dy, mask)
    assert g.masked is False and g.s1 is None  # the identity-block hand-off: unchanged
    s1 = dy.sum((0, 2, 3))
    g2 = MaskedGrad(dy, mask, True, s1)
    assert g2.masked and g2.s1 is s1
