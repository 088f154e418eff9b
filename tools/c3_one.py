"""One 3x3 conv launch kind, repeated (for rocprofv3 --pmc passes): layer-1 shape at the bench batch.

    python tools/c3_one.py <opt> [fwd|dgrad] [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402

opt = int(sys.argv[1])
kind = sys.argv[2] if len(sys.argv) > 2 else "dgrad"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
C = native()
N, c, h = 1024, 64, 56
x = torch.randn(N, c, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(c, c, 3, 3, device="cuda") / 24).bfloat16().contiguous(memory_format=torch.channels_last)
C.conv3x3_opt(opt)
for _ in range(reps):
    if kind == "fwd":
        C.conv3x3s1_fwd_stats(x, w)
    else:
        C.conv3x3s1_fwd(x, w)
torch.cuda.synchronize()
print("ok", opt, kind)
