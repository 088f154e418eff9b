"""Per-shape BN timing (ResNet-50 batch 256 shapes): our kernels (fwd / bwd) vs MIOpen BN, effective GB/s."""
import torch
import torch.nn.functional as F
import sys
sys.path.insert(0, ".")
from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402

C_ = native()


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3  # us


B = 256
shapes = [(64, 112), (64, 56), (256, 56), (128, 56), (128, 28), (512, 28), (256, 14), (1024, 14), (512, 7), (2048, 7)]
print(f"{'C':>5} {'HW':>4} {'MB':>7} | {'fwd us':>7} {'GB/s':>6} | {'bwd us':>7} {'GB/s':>6} | {'miopen f':>8} {'miopen b':>8}")
for C, hw in shapes:
    x = torch.randn(B, C, hw, hw, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x)
    w = torch.ones(C, device="cuda")
    b = torch.zeros(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    nbytes = x.numel() * 2
    tf = t(lambda: C_.bn_fwd_train(x, r, w, b, rm, rv, 0.1, 1e-5, True))
    y, mask, mean, invstd = C_.bn_fwd_train(x, r, w, b, rm, rv, 0.1, 1e-5, True)
    dy = torch.randn_like(x)
    tb = t(lambda: C_.bn_bwd_train(dy, x, mask, w, mean, invstd, True, True, True))
    # traffic: fwd = read x (stats) + read x,res + write y + mask ; bwd = read dy,x,mask (reduce) + read dy,x,mask + write dx,dres
    fb = nbytes * (1 + 3) + nbytes / 16
    bb = nbytes * (2 + 4) + nbytes / 8
    xm = x.detach().clone()
    tm = t(lambda: F.batch_norm(xm, rm, rv, w, b, True, 0.1, 1e-5))
    xg = x.detach().clone().requires_grad_(True)
    wg = w.clone().requires_grad_(True)
    bg = b.clone().requires_grad_(True)
    yy = F.batch_norm(xg, None, None, wg, bg, True, 0.1, 1e-5)
    tmb = t(lambda: torch.autograd.grad(yy, (xg, wg, bg), dy, retain_graph=True))
    print(f"{C:5d} {hw:4d} {nbytes/1e6:7.1f} | {tf:7.1f} {fb/tf/1e3:6.0f} | {tb:7.1f} {bb/tb/1e3:6.0f} | {tm:8.1f} {tmb:8.1f}", flush=True)
