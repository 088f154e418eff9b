"""BatchNorm statistics finalized from producer-epilogue tile partials in ONE launch (batchnorm.hip
bn_tiles_fin_kernel: last-arriver sums of the level-1 entries) against the two-launch path: the running
statistics, outputs and every gradient of a ResNet-50 step are bit-identical (same summation order), at a
batch where the tile columns span several level-1 blocks (P > 1) and where they do not."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch,hw", [(8, 96), (48, 128)])
def test_resnet50_step_identical_with_one_launch_finalize(batch, hw):
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import to_bf16_mixed
    from pytorch_distributed_training_example_amd.ops._native import native
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    import copy
    torch.manual_seed(0)
    base = to_bf16_mixed(get_model("resnet50", num_classes=16).cuda().to(memory_format=torch.channels_last))
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(batch, 3, hw, hw, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 16, (batch,), device="cuda", generator=g)

    def run(on):
        native().bn_tiles_fused(on)
        m = copy.deepcopy(base)
        for _ in range(2):  # the second pass reuses the self-reset arrival counters
            m.zero_grad(set_to_none=True)
            loss = cross_entropy(m(x), y)
            loss.backward()
        torch.cuda.synchronize()
        return [loss.detach()] + [p.grad.clone() for p in m.parameters()] + [b.clone() for b in m.buffers()]
    try:
        a = run(1)
        b = run(0)
    finally:
        native().bn_tiles_fused(1)
    bad = [i for i, (u, v) in enumerate(zip(a, b)) if not torch.equal(u, v)]
    assert not bad, bad
