"""Fused conv3 + bn3 backward (csrc/kernels/conv1x1_bwd_fused.hip) vs the unfused kernel chain it
replaces, at ResNet-50 layer-1 shapes: BN backward apply (bn_bwd_train_tiles) + our dgrad GEMM with the
bn2 reduction epilogue (conv1x1_gemm bn_x) + our 1x1 weight gradient (conv1x1_wgrad). Interleaved rounds
in one process (cdna_hip_programming.md §5.4 rule 24); prints per-call us and the HBM-floor estimate.

usage: python tools/bwd_fused_bench.py [--batch 1024] [--rounds 5] [--grid 0]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--layer", type=int, default=1, choices=[1, 2], help="ResNet-50 layer: 1 (256/64, 56x56), 2 (512/128, 28x28)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--grid", type=int, default=0)
    a = ap.parse_args()
    n = native()
    if a.grid:
        n.conv1x1_bwd_fused_tune(a.grid)
    N = a.batch
    H = W = 56 if a.layer == 1 else 28
    C4, CW = (256, 64) if a.layer == 1 else (512, 128)
    M = N * H * W
    cl = torch.channels_last
    t = lambda c, s=1.0: (torch.randn(N, c, H, W, device="cuda") * s).bfloat16().contiguous(memory_format=cl)  # noqa
    dy, z = t(C4), t(C4)
    mz = torch.randint(0, 256, (M * C4 // 8,), device="cuda", dtype=torch.uint8)
    mean, invstd = torch.randn(C4, device="cuda") * 0.1, torch.rand(C4, device="cuda") + 0.5
    gamma = torch.rand(C4, device="cuda") + 0.5
    coef = torch.randn(3, C4, device="cuda") * 0.01
    w = (torch.randn(C4, CW, 1, 1, device="cuda") / 16).bfloat16()
    xa, xb = t(CW).relu(), t(CW)
    mb = torch.randint(0, 256, (M * CW // 8,), device="cuda", dtype=torch.uint8)
    meanb = torch.randn(CW, device="cuda") * 0.1
    part3 = torch.randn(2, (M + 255) // 256, C4, device="cuda")

    def fused():
        n.conv1x1_bwd_fused(dy, z, mz, mean, coef, w, xa, xb, mb, meanb)

    wt = w.view(C4, CW).t().contiguous()

    def unfused():
        dz = n.bn_bwd_train_tiles(dy, z, part3, mz, gamma, mean, invstd, True, False, True)[0]
        dz2 = dz.permute(0, 2, 3, 1).reshape(M, C4)
        dxa = torch.empty_like(xa)
        n.conv1x1_gemm(dz2, wt, dxa.permute(0, 2, 3, 1).reshape(M, CW), False, False, None, None, xb, mb, meanb, 0, 0, 0)
        n.conv1x1_wgrad(xa.permute(0, 2, 3, 1).reshape(M, CW), dz2)

    def time(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps

    res = {"fused": [], "unfused": []}
    for _ in range(a.rounds):
        res["fused"].append(time(fused))
        res["unfused"].append(time(unfused))
    T = M * CW * 2
    floor_fused = (2 * 4 * T + 2 * 4 * T / 16 + 3 * T + T / 8) / 5.5e12 * 1e6
    for k, v in res.items():
        v.sort()
        print(f"{k:14s} median {v[len(v) // 2]:9.1f} us  min {v[0]:9.1f} us")
    print(f"fused HBM floor at 5.5 TB/s: {floor_fused:.1f} us  (M={M}, T={T / 1e6:.0f} MB)")


if __name__ == "__main__":
    main()
