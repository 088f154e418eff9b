"""Stem max-pool gradient (+ BN backward reduction) kernel time, 2 x 2-block kernel vs per-position kernel
(batchnorm.hip maxpool_bwd2_kernel / maxpool_bwd_kernel), at the ResNet-50 bench shape.

    python tools/pool_bwd_bench.py [--batch 1024]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.ops._native import native
    n = native()
    cl = torch.channels_last
    xb = torch.randn(a.batch, 64, 112, 112, device="cuda").bfloat16().contiguous(memory_format=cl)
    gamma, beta = torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * 0.1
    y, code, mean, invstd = n.bn_relu_maxpool_fwd(xb, gamma, beta, None, None, 0.1, 1e-5)
    dy = torch.randn(y.shape, device="cuda").bfloat16().contiguous(memory_format=cl)
    nbytes = dy.numel() * 2 + code.numel() + 2 * xb.numel() * 2
    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / 10 * 1e3

    fbytes = xb.numel() * 2 + y.numel() * 2 + code.numel()
    for v2, contig, wgs in ((1, 0, 16), (1, 0, 8), (1, 0, 4), (1, 0, 2), (1, 0, 16), (1, 1, 16), (0, 0, 16)):
        n.maxpool_bwd_v2(v2)
        n.pool_fwd_contig(contig)
        n.bn_row_wgs(wgs)
        print(f"row grid cap {wgs:2d} per CU:", end=" ")
        us = timeit(lambda: n.maxpool3s2_bwd_bn_coef(dy, code, xb, gamma, mean, invstd, True))
        fus = timeit(lambda: n.bn_relu_maxpool_fwd(xb, gamma, beta, None, None, 0.1, 1e-5))
        print(f"v2={v2} contig={contig}: backward {us:8.1f} us (pool gradient + BN finalize, {nbytes / us / 1e6:5.2f} TB/s)"
              f"  forward {fus:8.1f} us (BN reduce + apply + pool, {fbytes / fus / 1e6:5.2f} TB/s apply-pass bytes)",
              flush=True)
    n.maxpool_bwd_v2(1)
    n.pool_fwd_contig(0)
    n.bn_row_wgs(0)


if __name__ == "__main__":
    main()
