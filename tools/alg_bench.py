"""Microbenchmark of the ALG conv3 + bn3 backward kernels (ops/conv.py _bwd_alg) at ResNet-50's layer 2-4
bottleneck shapes (batch 1024 by default): conv1x1_wgrad_seg, bn_alg_small_gemm + assemble, conv1x1_gemm_seg
(with the BSTATS epilogue), against the HBM floor of the bytes each must move. The A/B knobs
(PDT_SEG_TILE, PDT_WGRAD_SEG_VARIANT) are read once per process: run one process per setting.

    python tools/alg_bench.py [--batch 1024]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402


def timeit(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--ds", action="store_true", help="the downsample shortcuts' shapes (Co = 2 Ci) instead of conv3's")
    a = ap.parse_args()
    C = native()
    tag = f"tile={os.environ.get('PDT_SEG_TILE', '0')} wvar={os.environ.get('PDT_WGRAD_SEG_VARIANT', '-1')}"
    shapes = ((56, 256, 64), (28, 512, 256), (14, 1024, 512)) if a.ds else ((28, 512, 128), (14, 1024, 256), (7, 2048, 512))
    for H, C4, CW in shapes:
        M = a.batch * H * H
        g = torch.randn(M, C4, device="cuda").bfloat16()
        x = torch.randn(M, CW, device="cuda").relu().bfloat16()
        w = (torch.randn(C4, CW, device="cuda") * 0.05).bfloat16()
        coef = torch.randn(3, C4, device="cuda").abs().contiguous()
        mean = torch.randn(C4, device="cuda")
        xb = torch.randn(M, CW, device="cuda").bfloat16()
        bmask = torch.randint(0, 256, (M * CW // 8,), device="cuda", dtype=torch.int32).to(torch.uint8)
        bmean = torch.randn(CW, device="cuda")
        wg = C.conv1x1_wgrad_seg(x, g, x)
        t_wg = timeit(lambda: C.conv1x1_wgrad_seg(x, g, x))
        wt = w.t().contiguous()
        t_sv = timeit(lambda: C.bn_alg_small_gemm(w, coef, wg))  # fp32 VALU
        t_sm = timeit(lambda: C.bn_alg_small_gemm(w, coef, wg, wt))  # matrix cores (hi / lo bf16 pairs)
        G, B = C.bn_alg_small_gemm(w, coef, wg, wt)
        t_as = timeit(lambda: C.bn_alg_assemble(w, coef, mean, G, wg, B))
        bcat, _ = C.bn_alg_assemble(w, coef, mean, G, wg, B)
        out = torch.empty(M, CW, device="cuda", dtype=torch.bfloat16)
        t_gm = timeit(lambda: C.conv1x1_gemm_seg(g, x, 2, bcat, out, bn_x=xb, bn_mask=bmask, bn_mean=bmean))
        f_wg = M * (C4 + CW) * 2 / 5.5e12 * 1e6
        f_gm = M * (C4 + 2 * CW + CW + CW + CW / 8) * 2 / 5.5e12 * 1e6
        tf_wg = 2 * M * (C4 + CW + 128) * CW / (t_wg * 1e-6) / 1e12
        tf_gm = 2 * M * (C4 + 2 * CW + 32) * CW / (t_gm * 1e-6) / 1e12
        print(f"[{tag}] M={M:7d} {C4:4d}/{CW:3d}: wgrad_seg {t_wg:6.1f} us ({tf_wg:4.0f} TF, floor {f_wg:5.1f}) | "
              f"small VALU {t_sv:5.1f} MFMA {t_sm:5.1f} assemble {t_as:5.1f} | gemm_seg {t_gm:6.1f} us ({tf_gm:4.0f} TF, floor {f_gm:5.1f})", flush=True)


if __name__ == "__main__":
    main()
