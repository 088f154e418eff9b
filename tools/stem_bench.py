"""Time the ResNet stem forward (7x7/s2, 3->64, batch 512, 224x224, bf16 channels_last): our MFMA
kernel (csrc/kernels/conv_stem.hip) vs MIOpen (F.conv2d), plus the max abs difference."""
import sys

import torch
import torch.nn.functional as F

from pytorch_distributed_training_example_amd.ops._native import native


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
x = torch.randn(N, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).bfloat16().contiguous(memory_format=torch.channels_last)
torch.backends.cudnn.benchmark = True
ours = timeit(lambda: native().stem_conv_fwd(x, w))
miop = timeit(lambda: F.conv2d(x, w, stride=2, padding=3))
d = (native().stem_conv_fwd(x, w).float() - F.conv2d(x, w, stride=2, padding=3).float()).abs().max().item()
mb = (x.numel() + N * 64 * 112 * 112) * 2 / 1e6
print(f"stem fwd N={N}: ours {ours:.1f} us ({mb / ours:.2f} TB/s eff)  miopen {miop:.1f} us  max|diff| {d:.3g}")
