"""Sweep the BN reduce implementation / grid on every ResNet-50 (batch 256) BN shape.

For each tuning (variant, target workgroups, rows in flight fwd/bwd) it times the training
forward (stats reduce + apply) and backward (reduce + apply) of each shape with HIP events,
weights them by how often the shape occurs in one ResNet-50 step, and checks the outputs
against the v1 kernels (same math, different summation tree: tolerance-level equality).

usage: python tools/bn_reduce_sweep.py [--batch 256]
"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402

# (C, H=W, count per step, relu, residual) for torchvision-style ResNet-50 v1.5 (stride on 3x3)
SHAPES = [
    (64, 56, 6, True, False), (256, 56, 3, True, True), (256, 56, 1, False, False),
    (128, 56, 1, True, False), (128, 28, 7, True, False), (512, 28, 4, True, True), (512, 28, 1, False, False),
    (256, 28, 1, True, False), (256, 14, 11, True, False), (1024, 14, 6, True, True), (1024, 14, 1, False, False),
    (512, 14, 1, True, False), (512, 7, 5, True, False), (2048, 7, 3, True, True), (2048, 7, 1, False, False),
]
TUNINGS = [  # (variant, target_blocks, u_fwd, u_bwd)
    (2, 512, 8, 4), (3, 512, 8, 4), (3, 512, 4, 4), (3, 512, 8, 8), (3, 512, 4, 2), (3, 1024, 8, 4),
    (3, 1024, 4, 2), (3, 256, 8, 4), (3, 768, 4, 4), (2, 512, 8, 4),
]


def timed(fn, it=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    C_ = native()
    data = []
    for C, hw, n, relu, res in SHAPES:
        x = torch.randn(a.batch, C, hw, hw, device="cuda").mul_(2).add_(0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        r = torch.randn_like(x) if res else None
        dy = torch.randn_like(x)
        w = torch.rand(C, device="cuda") + 0.5
        b = torch.randn(C, device="cuda")
        data.append((x, r, dy, w, b))
    ref = None
    print(f"{'tuning':>22} | " + " ".join(f"{C}x{hw}".rjust(9) for C, hw, *_ in SHAPES) + " | step ms")
    for tu in TUNINGS:
        C_.bn_tune(*tu)
        outs, cols, total = [], [], 0.0
        for (C, hw, n, relu, res), (x, r, dy, w, b) in zip(SHAPES, data):
            rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
            tf = timed(lambda: C_.bn_fwd_train(x, r, w, b, rm, rv, 0.1, 1e-5, relu))
            y, mask, mean, invstd = C_.bn_fwd_train(x, r, w, b, rm, rv, 0.1, 1e-5, relu)
            tb = timed(lambda: C_.bn_bwd_train(dy, x, mask if relu else None, w, mean, invstd, relu, res, True))
            g = C_.bn_bwd_train(dy, x, mask if relu else None, w, mean, invstd, relu, res, True)
            outs.append([mean, invstd, y] + [t for t in g if t is not None])
            cols.append(f"{tf:4.0f}/{tb:4.0f}")
            total += n * (tf + tb)
        print(f"{str(tu):>22} | " + " ".join(c.rjust(9) for c in cols) + f" | {total / 1e3:6.2f}", flush=True)
        if ref is None:
            ref = outs
        else:
            for o, rf in zip(outs, ref):
                for t, u in zip(o, rf):
                    # different summation trees move mean/invstd in the last bits, which can flip
                    # a handful of ReLU decisions at exactly-zero pre-activations: allow 1e-6
                    tf_, uf = t.float(), u.float()
                    # per-channel sums (dbeta = sum dy) can cancel to ~0: scale atol by the vector's max
                    atol = 2e-2 if uf.numel() > 4096 else 2e-3 * uf.abs().max().item()
                    bad = ((tf_ - uf).abs() > atol + 2e-2 * uf.abs()).sum().item()
                    assert bad <= max(2, t.numel() // 1_000_000), (tu, bad, t.shape)


# measured on MI355X (round 1): (2, 512, 8, 4) = 10.50 ms/step of BN vs v1 11.50 ms; more
# workgroups are slower (2048: 14.45 ms, 4096: 18.1 ms). A v3 with 128/256-channel chunks per
# workgroup (longer contiguous row segments) measured 10.12-10.23 ms vs 10.14: no gain, not kept.
# Interleaving the row groups across workgroups (all blocks streaming one contiguous window, like
# the grid-stride apply kernels) measured 10.68 vs 10.46 ms: not kept either.


if __name__ == "__main__":
    main()
