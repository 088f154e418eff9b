"""BatchNorm apply-pass grid cap sweep (batchnorm.hip apply_grid: workgroups per CU before grid-striding),
at ResNet-50 shapes with 1024 images: the forward apply with and without the residual and the backward apply.

    python tools/bn_apply_grid_sweep.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    from pytorch_distributed_training_example_amd.ops._native import native
    n = native()
    cl = torch.channels_last
    for (c, h) in ((512, 28), (64, 56), (1024, 14)):
        x = torch.randn(1024, c, h, h, device="cuda").bfloat16().contiguous(memory_format=cl)
        r = torch.randn_like(x)
        w, b = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda")
        rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
        _, mask, mean, invstd = n.bn_fwd_train(x, None, w, b, rm, rv, 0.1, 1e-5, True)
        dy = torch.randn_like(x)
        row = []
        for cap in (1, 2, 3, 4, 6, 8, 4, 8):
            n.bn_apply_wgs(cap)
            t_res = timeit(lambda: n.bn_fwd_train(x, r, w, b, rm, rv, 0.1, 1e-5, True))
            t_plain = timeit(lambda: n.bn_fwd_train(x, None, w, b, rm, rv, 0.1, 1e-5, True))
            t_bwd = timeit(lambda: n.bn_bwd_train(dy, x, mask, w, mean, invstd, True, False, True))
            row.append(f"cap {cap:2d}: res {t_res:6.1f} plain {t_plain:6.1f} bwd {t_bwd:6.1f}")
        print(f"C={c} H={h} (reduce + apply, us):\n  " + "\n  ".join(row), flush=True)
    n.bn_apply_wgs(0)


if __name__ == "__main__":
    main()
