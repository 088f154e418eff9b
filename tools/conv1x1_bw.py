"""Achieved HBM bandwidth of our 1x1-conv GEMM (conv1x1.hip) per ResNet-50 shape at the bench batch:
forward with the BatchNorm-statistics epilogue, and the data gradient (plain / shortcut-accumulate), against
a same-bytes copy (torch.Tensor.copy_ of the output size + a read of the input size) as the practical floor.

    python tools/conv1x1_bw.py [--batch 1024] [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

# (count in ResNet-50 fwd, Ci, Co, H)
SHAPES = [(1, 64, 64, 56), (3, 64, 256, 56), (2, 256, 64, 56), (4, 128, 512, 28), (3, 512, 128, 28),
          (6, 256, 1024, 14), (5, 1024, 256, 14), (3, 512, 2048, 7), (2, 2048, 512, 7)]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    print(f"{'(n, Ci, Co, H)':<22} | {'fwd us':>7} {'GB':>6} {'TB/s':>5} | {'copy us':>7} {'TB/s':>5} | "
          f"{'dgrad us':>8} {'TB/s':>5} | {'acc us':>7} {'TB/s':>5}")
    tot_f = tot_c = 0.0
    for n, ci, co, h in SHAPES:
        B = a.batch
        M = B * h * h
        x = torch.randn(M, ci, device="cuda").bfloat16()
        w = (torch.randn(co, ci, device="cuda") / ci ** 0.5).bfloat16()
        y = torch.empty(M, co, device="cuda", dtype=torch.bfloat16)
        t_f = timeit(lambda: C.conv1x1_gemm(x, w, y, False, True), a.reps)
        gb_f = (M * ci + M * co) * 2 / 1e9
        src = torch.empty(M, co, device="cuda", dtype=torch.bfloat16)
        t_c = timeit(lambda: y.copy_(src), a.reps)
        gb_c = 2 * M * co * 2 / 1e9
        # data gradient: dX [M, ci] = dY [M, co] W [co, ci]
        gy = torch.randn(M, co, device="cuda").bfloat16()
        wt = w.t().contiguous()
        dx = torch.empty(M, ci, device="cuda", dtype=torch.bfloat16)
        t_d = timeit(lambda: C.conv1x1_gemm(gy, wt, dx, False, False), a.reps)
        gb_d = (M * co + M * ci) * 2 / 1e9
        t_a = timeit(lambda: C.conv1x1_gemm(gy, wt, dx, True, False), a.reps)
        gb_a = (M * co + 2 * M * ci) * 2 / 1e9
        tot_f += n * t_f
        tot_c += n * t_c * gb_f / gb_c
        print(f"({n}, {ci:4d}, {co:4d}, {h:2d})".ljust(22) + f" | {t_f:7.1f} {gb_f:6.2f} {gb_f / t_f * 1e3:5.2f} | "
              f"{t_c:7.1f} {gb_c / t_c * 1e3:5.2f} | {t_d:8.1f} {gb_d / t_d * 1e3:5.2f} | {t_a:7.1f} {gb_a / t_a * 1e3:5.2f}")
    print(f"forward total (x count): {tot_f / 1e3:.2f} ms; at copy bandwidth: {tot_c / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
