"""Where the 1x1-conv GEMM's time goes (conv1x1.hip diagnosis probe): each variant timed with parts of the
kernel switched off — 1 = no output stores, 2 = no MFMA, 4 = no operand DMA (results are garbage while a
probe is set). ResNet-50 layer-1 / layer-2 shapes at the bench batch.

    python tools/conv1x1_probe.py [--batch 1024]
"""
from __future__ import annotations

import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    probes = [int(v) for v in os.environ.get("PDT_PROBES", "0,64,0,64,1,65").split(",")]
    print("probe: 1 = no stores, 2 = no MFMA, 4 = no operand DMA, 8 = 64-channel tiles, 16 = no statistics, 32 = no mask stores, 64 = no 256-channel tiles")
    print(f"{'case':<34}" + "".join(f"{p:>9}" for p in probes) + "   GB  TB/s(p0)")
    for h, ci, co in ((56, 64, 256), (28, 128, 512), (14, 256, 1024), (7, 512, 2048)):
        M = a.batch * h * h
        x = torch.randn(M, ci, device="cuda").bfloat16()
        w = (torch.randn(co, ci, device="cuda") / ci ** 0.5).bfloat16()
        y = torch.empty(M, co, device="cuda", dtype=torch.bfloat16)
        res = torch.randn(M, co, device="cuda").bfloat16()
        ab = torch.randn(2, co, device="cuda")
        gy = torch.randn(M, co, device="cuda").bfloat16()
        wt = w.t().contiguous()
        dx = torch.empty(M, ci, device="cuda", dtype=torch.bfloat16)
        dres = torch.randn(M, ci, device="cuda").bfloat16()
        bx = torch.randn(M, ci, device="cuda").bfloat16()
        bmean = torch.randn(ci, device="cuda")
        cases = [
            (f"fwd+stats {ci}->{co} @{h}", lambda: C.conv1x1_gemm(x, w, y, False, True), (M * ci + M * co) * 2),
            (f"apply {ci}->{co} @{h}", lambda: C.conv1x1_gemm_apply(x, w, res, ab), (M * ci + 2 * M * co + M * co // 8) * 2),
            (f"dgrad+acc+bst {co}->{ci} @{h}",
             lambda: C.conv1x1_gemm(gy, wt, dres, True, False, None, None, bx, None, bmean),
             (M * co + 3 * M * ci) * 2),
        ]
        for name, fn, nbytes in cases:
            ts = []
            for p in probes:
                C.conv1x1_probe(p)
                ts.append(timeit(fn))
            C.conv1x1_probe(0)
            print(f"{name:<34}" + "".join(f"{t:9.1f}" for t in ts) + f"  {nbytes / 1e9:5.2f}  {nbytes / ts[0] / 1e6:5.2f}")


if __name__ == "__main__":
    main()
