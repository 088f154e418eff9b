"""Split-K depth of our weight-gradient kernels (3x3: conv3x3_wgrad.hip, 1x1: conv1x1_wgrad.hip) at a
given batch: every workgroup-count target, time per call including the fixed-order partial
reduction. The default targets one workgroup per CU; at small batches the fp32 partials (nsplit x
9 Co Ci floats for a 3x3) can cost as much as the gradient itself.

    python tools/wgrad_target_sweep.py [--batch 128] [--targets 0,32,64,128,256]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--targets", default="0,32,64,128,256")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    N = a.batch
    targets = [int(t) for t in a.targets.split(",")]
    cases = []
    for w, h in ((64, 56), (128, 28), (256, 14), (512, 7)):  # stride-1 3x3 of each stage
        x = cl(torch.randn(N, w, h, h, device="cuda").bfloat16())
        gy = cl(torch.randn(N, w, h, h, device="cuda").bfloat16())
        cases.append((f"3x3 s1 wgrad {w}@{h}", "3", lambda x=x, gy=gy: C.conv3x3s1_wgrad(x, gy)))
    for ci, co, h in ((256, 64, 56), (64, 256, 56), (512, 128, 28), (128, 512, 28), (1024, 256, 14),
                      (256, 1024, 14), (2048, 512, 7), (512, 2048, 7)):
        M = N * h * h
        x = torch.randn(M, ci, device="cuda").bfloat16()
        dy = torch.randn(M, co, device="cuda").bfloat16()
        cases.append((f"1x1 wgrad {ci}->{co}@{h}", "1", lambda x=x, dy=dy: C.conv1x1_wgrad(x, dy)))
    print(f"batch {N}; us per call (kernel + partial reduction) by workgroup target (0 = default)")
    print(f"{'case':<28}" + "".join(f"{t:>9}" for t in targets), flush=True)
    for name, kind, fn in cases:
        ts = {t: [] for t in targets}
        for _ in range(a.rounds):
            for t in targets:
                if kind == "3":
                    C.conv3x3_wgrad_tune(t, -1)
                else:
                    C.conv1x1_wgrad_tune(t, -1, -1)
                ts[t].append(timeit(fn))
        C.conv3x3_wgrad_tune(0, -1)
        C.conv1x1_wgrad_tune(0, -1, -1)
        print(f"{name:<28}" + "".join(f"{statistics.median(ts[t]):9.1f}" for t in targets), flush=True)


if __name__ == "__main__":
    main()
