"""Every 3x3 conv launch of the ResNet-50 step at the bench batch (1024), timed per kind, with the
3x3 variant bits (csrc/kernels/conv3x3.hip conv3x3_opt) A/B'd in interleaved rounds in one process.

    python tools/conv3x3_bench.py [--batch 1024] [--rounds 5] [--opts 0,1]

Kinds per layer: forward + BN statistics, data gradient (+ the producing BN's backward reduction where
the step takes it in the epilogue), weight gradient; the stride-2 transition convs of layers 2-4 too.
The last column is the step's share (calls per step x median of the first opt).
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--opts", default="0,1")
    ap.add_argument("--only", default="", help="comma list of case-name substrings")
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    opts = [int(o) for o in a.opts.split(",")]
    only = [s for s in a.only.split(",") if s]
    N = a.batch
    print(f"{'case':<34}{'calls':>6}" + "".join(f"{'opt' + str(o):>10}" for o in opts) + "   TF/s(first)  ms/step",
          flush=True)
    total = {o: 0.0 for o in opts}
    # (width, H of the stride-1 convs, identity blocks' stride-1 3x3 count, stride-2 transition or not)
    for w, h, n_s1, s2 in ((64, 56, 3, False), (128, 28, 3, True), (256, 14, 5, True), (512, 7, 2, True)):
        g = torch.Generator(device="cuda").manual_seed(w)
        x = cl(torch.randn(N, w, h, h, device="cuda", generator=g).bfloat16())
        wt = cl((torch.randn(w, w, 3, 3, device="cuda", generator=g) / (9 * w) ** 0.5).bfloat16())
        wf = C.conv3x3_flip(wt)
        gy = cl(torch.randn(N, w, h, h, device="cuda", generator=g).bfloat16())
        bx = cl(torch.randn(N, w, h, h, device="cuda", generator=g).bfloat16())
        M = N * h * h
        mask = torch.randint(0, 256, (M * w // 8,), device="cuda", dtype=torch.int32).to(torch.uint8)
        mean = torch.randn(w, device="cuda")
        fl = 2.0 * M * w * w * 9
        cases = [(f"s1 fwd+stats {w}@{h}", n_s1 + (0 if s2 else 0), lambda: C.conv3x3s1_fwd_stats(x, wt), fl)]
        if w == 64:  # plain, and with the BN reduction where the kernel takes it (opt bit 7)
            cases.append((f"s1 dgrad {w}@{h}", n_s1, lambda: C.conv3x3s1_fwd(gy, wf), fl))
            cases.append((f"s1 dgrad+bnred {w}@{h} (if taken)", 0,
                          lambda: C.conv3x3s1_fwd_bnbwd(gy, wf, bx, mask, mean), fl))
        else:
            cases.append((f"s1 dgrad+bnred {w}@{h}", n_s1, lambda: C.conv3x3s1_fwd_bnbwd(gy, wf, bx, mask, mean), fl))
        cases.append((f"s1 wgrad {w}@{h}", n_s1, lambda: C.conv3x3s1_wgrad(x, gy), fl))
        if s2:
            hi = 2 * h
            xi = cl(torch.randn(N, w, hi, hi, device="cuda", generator=g).bfloat16())
            bxi = cl(torch.randn(N, w, hi, hi, device="cuda", generator=g).bfloat16())
            maski = torch.randint(0, 256, (N * hi * hi * w // 8,), device="cuda", dtype=torch.int32).to(torch.uint8)
            cases += [
                (f"s2 fwd+stats {w}@{hi}->{h}", 1, lambda: C.conv3x3s2_fwd(xi, wt, True), fl),
                (f"s2 dgrad+bnred {w}@{h}->{hi}", 1,
                 lambda: C.conv3x3s2_dgrad(gy, wf, hi, hi, bn_x=bxi, bn_mask=maski, bn_mean=mean), fl),
                (f"s2 wgrad {w}@{hi}->{h}", 1, lambda: C.conv3x3s2_wgrad(xi, gy), fl),
            ]
        for name, calls, fn, flops in cases:
            if only and not any(s in name for s in only):
                continue
            ts = {o: [] for o in opts}
            for _ in range(a.rounds):
                for o in opts:
                    C.conv3x3_opt(o)
                    ts[o].append(timeit(fn))
            C.conv3x3_opt(-1)
            med = {o: statistics.median(v) for o, v in ts.items()}
            for o in opts:
                total[o] += calls * med[o] / 1e3
            print(f"{name:<34}{calls:>6}" + "".join(f"{med[o]:10.1f}" for o in opts) +
                  f"   {flops / med[opts[0]] / 1e6:10.0f}  {calls * med[opts[0]] / 1e3:7.3f}", flush=True)
        torch.cuda.empty_cache()
    print("3x3 total ms/step: " + "  ".join(f"opt{o} {total[o]:.3f}" for o in opts), flush=True)


if __name__ == "__main__":
    main()
