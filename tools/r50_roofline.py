"""Per-shape roofline of ResNet-50's convolutions and BatchNorms at the bench batch (bf16, NHWC).

For every distinct convolution (forward, data gradient, weight gradient) it times MIOpen and, for
1x1 convs, the GEMM formulation, and prints the HBM-traffic / MFMA floor next to it:
floor = max(bytes / 6.0 TB/s, flops / 1.6 PF/s) (measured-achievable HBM rate, ~65 % of dense bf16
MFMA peak). For BatchNorm it times our forward (stats + apply) and backward (reduce + apply) per
shape and reports effective TB/s. Output: one table per part, totals weighted by the number of
times each shape occurs in one training step.

usage: python tools/r50_roofline.py [--batch 512] [--part conv|bn|all]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM, MFMA = 6.0e12, 1.6e15


def timeit(fn, it=10):
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


def conv_shapes():
    """(Cin, Cout, k, stride, H_in) -> count per step, ResNet-50 v1.5 (stride on the 3x3)."""
    shapes = {}

    def add(ci, co, k, s, h, n=1):
        shapes[(ci, co, k, s, h)] = shapes.get((ci, co, k, s, h), 0) + n
    add(3, 64, 7, 2, 224)
    for (w, blocks, h, ci) in [(64, 3, 56, 64), (128, 4, 56, 256), (256, 6, 28, 512), (512, 3, 14, 1024)]:
        s = 1 if w == 64 else 2
        ho = h // s
        add(ci, w, 1, 1, h)
        add(w, w, 3, s, h)
        add(w, 4 * w, 1, 1, ho)
        add(ci, 4 * w, 1, s, h)
        add(4 * w, w, 1, 1, ho, blocks - 1)
        add(w, w, 3, 1, ho, blocks - 1)
        add(w, 4 * w, 1, 1, ho, blocks - 1)
    return shapes


def conv_part(B):
    torch.backends.cudnn.benchmark = True
    print(f"{'(ci,co,k,s,h)':24s} n | {'fwd':>6} {'floor':>6} | {'dgrad':>6} {'floor':>6} | {'wgrad':>6} {'floor':>6} |"
          f" {'mm_f':>6} {'mm_d':>6} {'mm_w':>6}  (us)")
    tot = {"best": 0.0, "floor": 0.0, "miopen": 0.0}
    for (ci, co, k, s, h), n in sorted(conv_shapes().items()):
        x = torch.randn(B, ci, h, h, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(co, ci, k, k, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        pad = k // 2
        y = F.conv2d(x, w, stride=s, padding=pad)
        gy = torch.randn_like(y)
        args = ([s, s], [pad, pad], [1, 1], False, [0, 0], 1)
        cf = timeit(lambda: F.conv2d(x, w, stride=s, padding=pad))
        cd = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, *args, [True, False, False])) \
            if ci > 3 else 0.0
        cw = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, *args, [False, True, False]))
        flops = 2 * y.numel() * ci * k * k
        xb, yb, wb = x.numel() * 2, y.numel() * 2, w.numel() * 2
        fl = [max((xb + yb + wb) / HBM, flops / MFMA) * 1e6] * 3
        if ci <= 3:
            fl[1] = 0.0
        line = f"{str((ci, co, k, s, h)):24s} {n} | {cf:6.0f} {fl[0]:6.0f} | {cd:6.0f} {fl[1]:6.0f} | {cw:6.0f} {fl[2]:6.0f} |"
        best = [cf, cd, cw]
        if k == 1:
            xs = x[:, :, ::s, ::s] if s > 1 else x
            a = xs.permute(0, 2, 3, 1).reshape(-1, ci)
            wm = w.reshape(co, ci)
            g2 = gy.permute(0, 2, 3, 1).reshape(-1, co)
            mm = [timeit(lambda: a @ wm.t()), timeit(lambda: g2 @ wm), timeit(lambda: g2.t() @ a)]
            line += f" {mm[0]:6.0f} {mm[1]:6.0f} {mm[2]:6.0f}"
            best = [min(p, q) for p, q in zip(best, mm)]
        print(line, flush=True)
        tot["best"] += n * sum(best)
        tot["floor"] += n * sum(fl)
        tot["miopen"] += n * (cf + cd + cw)
        del x, w, y, gy
    print(f"per step (ms): MIOpen {tot['miopen'] / 1e3:.2f}  best-of {tot['best'] / 1e3:.2f}  floor {tot['floor'] / 1e3:.2f}")


def bn_shapes():
    """(C, H) -> count per step (ResNet-50 BN layers after each conv, stem excluded)."""
    sh = {}
    for (w, blocks, h) in [(64, 3, 56), (128, 4, 56), (256, 6, 28), (512, 3, 14)]:
        s = 1 if w == 64 else 2
        ho = h // s
        for key, n in (((w, h), 1), ((w, ho), 1), ((4 * w, ho), 1), ((4 * w, ho), 1),
                       ((w, ho), 2 * (blocks - 1)), ((4 * w, ho), blocks - 1)):
            sh[key] = sh.get(key, 0) + n
    return sh


def bn_part(B):
    from pytorch_distributed_training_example_amd.ops._native import native
    C_ = native()
    print(f"{'C':>5} {'H':>4} n {'MB':>7} | {'fwd us':>7} {'TB/s':>5} | {'fwd+res':>7} {'TB/s':>5} | {'bwd us':>7} {'TB/s':>5}"
          f" | {'bwd+res':>7} {'TB/s':>5}")
    tot = 0.0
    for (C, h), n in sorted(bn_shapes().items()):
        x = torch.randn(B, C, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x)
        w, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nb = x.numel() * 2
        tf = timeit(lambda: C_.bn_fwd_train(x, None, w, b, rm, rv, 0.1, 1e-5, True))
        tfr = timeit(lambda: C_.bn_fwd_train(x, r, w, b, rm, rv, 0.1, 1e-5, True))
        y, mask, mean, invstd = C_.bn_fwd_train(x, r, w, b, rm, rv, 0.1, 1e-5, True)
        dy = torch.randn_like(x)
        tb = timeit(lambda: C_.bn_bwd_train(dy, x, mask, w, mean, invstd, True, False, True))
        tbr = timeit(lambda: C_.bn_bwd_train(dy, x, mask, w, mean, invstd, True, True, True))
        f_b, fr_b = nb * 3 + nb / 16, nb * 4 + nb / 16
        b_b, br_b = nb * 5 + nb / 8, nb * 6 + nb / 8
        print(f"{C:5d} {h:4d} {n} {nb / 1e6:7.1f} | {tf:7.1f} {f_b / tf / 1e6:5.2f} | {tfr:7.1f} {fr_b / tfr / 1e6:5.2f} |"
              f" {tb:7.1f} {b_b / tb / 1e6:5.2f} | {tbr:7.1f} {br_b / tbr / 1e6:5.2f}", flush=True)
        tot += n * (tf + tb)
        del x, r, y, dy, mask
    print(f"per step (ms, no-residual variants): {tot / 1e3:.2f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--part", default="all")
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.engine.miopen_cache import use_repo_miopen_cache
    use_repo_miopen_cache()
    if a.part in ("bn", "all"):
        bn_part(a.batch)
    if a.part in ("conv", "all"):
        conv_part(a.batch)


if __name__ == "__main__":
    main()
