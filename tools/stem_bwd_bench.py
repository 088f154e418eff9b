"""ResNet stem backward chain at the bench batch (1024 x 224 x 224 default): max-pool gradient with the
BN reduction (maxpool3s2_bwd_bn_coef), then either the separate BN apply + stem weight gradient
(maxpool3s2_bwd_bn + stem_conv_wgrad, the unfused path) or the weight gradient with the apply fused
into its load (stem_conv_wgrad_bn). Prints per-op device times and the fused-vs-unfused difference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402


def timeit(fn, it=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = native()
cl = torch.channels_last
img = torch.randn(N, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=cl)
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).bfloat16().contiguous(memory_format=cl)
gamma, beta = torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * 0.1
rm, rv = torch.zeros(64, device="cuda"), torch.ones(64, device="cuda")
xb = n.stem_conv_fwd(img, w)
y, code, mean, invstd = n.bn_relu_maxpool_fwd(xb, gamma, beta, rm, rv, 0.1, 1e-5)
dy = torch.randn_like(y)

t_pool_coef = timeit(lambda: n.maxpool3s2_bwd_bn_coef(dy, code, xb, gamma, mean, invstd, True))
t_pool_apply = timeit(lambda: n.maxpool3s2_bwd_bn(dy, code, xb, gamma, mean, invstd, True))
dx = n.maxpool3s2_bwd_bn(dy, code, xb, gamma, mean, invstd, True)[0]
dz, coef, _, _ = n.maxpool3s2_bwd_bn_coef(dy, code, xb, gamma, mean, invstd, True)
t_wg = timeit(lambda: n.stem_conv_wgrad(img, dx))
t_wg_bn = timeit(lambda: n.stem_conv_wgrad_bn(img, dz, xb, coef, mean))
ref = n.stem_conv_wgrad(img, dx).float()
got = n.stem_conv_wgrad_bn(img, dz, xb, coef, mean).float()
rel = ((got - ref).abs().max() / ref.abs().max()).item()
print(f"stem bwd N={N}: pool+reduce+apply {t_pool_apply:.1f} us, pool+reduce (coef only) {t_pool_coef:.1f} us, "
      f"wgrad {t_wg:.1f} us, wgrad with fused apply {t_wg_bn:.1f} us")
print(f"unfused chain {t_pool_apply + t_wg:.1f} us vs fused {t_pool_coef + t_wg_bn:.1f} us; "
      f"max |fused - unfused| / max |dw| = {rel:.3g}")
