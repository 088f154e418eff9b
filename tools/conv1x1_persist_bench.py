"""A/B of the 1x1-conv GEMM's persistence modes (csrc/kernels/conv1x1.hip: 0 = one tile per workgroup,
1 = persistent 8- / 4-wave tiles, 2 = persistent 16-wave tile too) on the ResNet-50 shapes at the bench
batch, every epilogue kind the step runs. Interleaved rounds in one process, median per mode.

    python tools/conv1x1_persist_bench.py [--batch 1024] [--rounds 5]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--modes", default="0,1,2",
                    help="persistence modes; 'w' = mode 0 with the 256-channel tile off (probe 64: 128-channel tiles)")
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    modes = [m if m == "w" else int(m) for m in a.modes.split(",")]
    print(f"{'case':<36}" + "".join(f"{'mode' + str(m):>10}" for m in modes) + "     GB" +
          "".join(f"  TB/s m{m}" for m in modes), flush=True)
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
        cmask = torch.randint(0, 256, (M * ci // 8,), device="cuda", dtype=torch.int32).to(torch.uint8)
        cmasko = torch.randint(0, 256, (M * co // 8,), device="cuda", dtype=torch.int32).to(torch.uint8)
        bx = torch.randn(M, ci, device="cuda").bfloat16()
        bxo = torch.randn(M, co, device="cuda").bfloat16()
        bmean = torch.randn(ci, device="cuda")
        bmeano = torch.randn(co, device="cuda")
        coef = torch.rand(2, ci, device="cuda").contiguous()
        cases = [
            (f"fwd+stats {ci}->{co} @{h}", lambda: C.conv1x1_gemm(x, w, y, False, True), (M * ci + M * co) * 2),
            (f"fwd+atr+stats {ci}->{co} @{h}", lambda: C.conv1x1_gemm(x, w, y, False, True, a_coef=coef),
             (M * ci + M * co) * 2),
            (f"apply {ci}->{co} @{h}", lambda: C.conv1x1_gemm_apply(x, w, res, ab), (M * ci + 2 * M * co + M * co // 8) * 2),
            (f"dgrad+macc+bst {co}->{ci} @{h}",
             lambda: C.conv1x1_gemm(gy, wt, dx, True, False, dres, cmask, bx, cmask, bmean),
             (M * co + 3 * M * ci) * 2 + 2 * M * ci // 8),
            (f"dgrad+bst {ci}->{co} @{h}",
             lambda: C.conv1x1_gemm(x, w, y, False, False, None, None, bxo, None, bmeano),
             (M * ci + 2 * M * co) * 2),
            # conv1's data gradient of an identity block: K = width, N = 4 width, the shortcut gradient
            # accumulated (masked) and the previous bn3's backward reduction in the epilogue
            (f"dgrad+macc+bst {ci}->{co} @{h}",
             lambda: C.conv1x1_gemm(x, w, y, True, False, res, cmasko, bxo, cmasko, bmeano),
             (M * ci + 3 * M * co) * 2 + 2 * M * co // 8),
        ]
        for name, fn, nbytes in cases:
            ts = {m: [] for m in modes}
            for _ in range(a.rounds):
                for m in modes:
                    C.conv1x1_persist(0 if m == "w" else m)
                    C.conv1x1_probe(64 if m == "w" else 0)
                    ts[m].append(timeit(fn))
            C.conv1x1_persist(-1)
            C.conv1x1_probe(0)
            med = {m: statistics.median(v) for m, v in ts.items()}
            print(f"{name:<36}" + "".join(f"{med[m]:10.1f}" for m in modes) + f"  {nbytes / 1e9:5.2f}" +
                  "".join(f"  {nbytes / med[m] / 1e6:7.2f}" for m in modes), flush=True)
        del x, w, y, res, gy, wt, dx, dres, cmask, cmasko, bx, bxo
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
