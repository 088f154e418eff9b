"""Run-to-run reproducibility of the stem weight-gradient kernels on identical inputs (diagnosis)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402

n = native()
for N, H in ((8, 96), (48, 128), (16, 224), (128, 224)):
    g = torch.Generator(device="cuda").manual_seed(N)
    cl = torch.channels_last
    img = torch.randn(N, 3, H, H, device="cuda", generator=g).bfloat16().contiguous(memory_format=cl)
    OH = H // 2
    dz = torch.randn(N, 64, OH, OH, device="cuda", generator=g).bfloat16().contiguous(memory_format=cl)
    xb = torch.randn(N, 64, OH, OH, device="cuda", generator=g).bfloat16().contiguous(memory_format=cl)
    coef = torch.randn(3, 64, device="cuda", generator=g) * 0.1
    mean = torch.randn(64, device="cuda", generator=g) * 0.1
    outs = [n.stem_conv_wgrad_bn(img, dz, xb, coef, mean) for _ in range(6)]
    outs2 = [n.stem_conv_wgrad(img, dz) for _ in range(6)]
    d1 = [float((o.float() - outs[0].float()).abs().max()) for o in outs[1:]]
    d2 = [float((o.float() - outs2[0].float()).abs().max()) for o in outs2[1:]]
    print(f"N={N} H={H}: wgrad_bn max diffs {d1}  wgrad max diffs {d2}")
