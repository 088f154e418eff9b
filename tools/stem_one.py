"""One stem weight-gradient kernel, a few launches, for rocprofv3 --pmc passes:
    python tools/stem_one.py pool|dz [N] [launches]
pool: stem_conv_wgrad_bn_pool (forms the max-pool gradient from pooled dy + codes), dz: stem_conv_wgrad_bn."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "pool"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
n = native()
cl = torch.channels_last
img = torch.randn(N, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=cl)
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).bfloat16().contiguous(memory_format=cl)
gamma, beta = torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * 0.1
xb = n.stem_conv_fwd(img, w)
y, code, mean, invstd = n.bn_relu_maxpool_fwd(xb, gamma, beta, None, None, 0.1, 1e-5)
dy = torch.randn_like(y)
dz, coef, _, _ = n.maxpool3s2_bwd_bn_coef(dy, code, xb, gamma, mean, invstd, True)
torch.cuda.synchronize()
for _ in range(reps):
    if mode == "pool":
        n.stem_conv_wgrad_bn_pool(img, dy, code, xb, coef, mean)
    else:
        n.stem_conv_wgrad_bn(img, dz, xb, coef, mean)
torch.cuda.synchronize()
print("done", mode, N)
