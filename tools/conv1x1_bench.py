"""Per-shape timing of ResNet-50's stride-1 1x1 convs (batch 512): our MFMA GEMM (conv1x1.hip)
against the library kernels, forward with the consuming BatchNorm (fused statistics vs reduce
pass) and data gradient (plain and with the shortcut gradient accumulated in place).

    python tools/conv1x1_bench.py [--batch 512] [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# (count in ResNet-50, Ci, Co, H)
SHAPES = [(1, 64, 64, 56), (4, 64, 256, 56), (2, 256, 64, 56), (1, 256, 128, 56), (4, 128, 512, 28),
          (3, 512, 128, 28), (1, 512, 256, 28), (6, 256, 1024, 14), (5, 1024, 256, 14), (1, 1024, 512, 14),
          (3, 512, 2048, 7), (2, 2048, 512, 7)]


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
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.engine.gemm_tuning import use_repo_gemm_tuning
    from pytorch_distributed_training_example_amd.engine.miopen_cache import use_repo_miopen_cache
    from pytorch_distributed_training_example_amd.ops._native import native
    use_repo_miopen_cache()
    use_repo_gemm_tuning()  # the library GEMMs as the bench runs them (measured solution table)
    C = native()
    table = {}
    dev = "cuda"
    tot = {"lib_f": 0.0, "ours_f": 0.0, "lib_d": 0.0, "ours_d": 0.0}
    print(f"{'(n, Ci, Co, H)':<22} | {'mm':>6} {'conv':>6} {'ours':>6} | {'bn':>6} {'bnT':>6} | "
          f"{'lib+bn':>7} {'ours+bnT':>8} | {'mm_d':>6} {'conv_d':>6} {'ours_d':>6} {'addmm':>6} {'ours_acc':>8}")
    for n, ci, co, h in SHAPES:
        B = a.batch
        M = B * h * h
        x = torch.randn(B, ci, h, h, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 1, 1, device=dev) / ci ** 0.5).bfloat16()
        x2 = x.permute(0, 2, 3, 1).reshape(M, ci)
        w2 = w.reshape(co, ci).contiguous()
        y = torch.empty(B, co, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y2 = y.permute(0, 2, 3, 1).reshape(M, co)
        t_mm = timeit(lambda: torch.mm(x2, w2.t()), a.reps)
        t_cv = timeit(lambda: F.conv2d(x, w), a.reps)
        t_ours = timeit(lambda: C.conv1x1_gemm(x2, w2, y2, False, False), a.reps)
        part = C.conv1x1_gemm(x2, w2, y2, False, True)
        t_ours_s = timeit(lambda: C.conv1x1_gemm(x2, w2, y2, False, True), a.reps)
        g = torch.rand(co, device=dev) + 0.5
        bb = torch.zeros(co, device=dev)
        rm, rv = torch.zeros(co, device=dev), torch.ones(co, device=dev)
        t_bn = timeit(lambda: C.bn_fwd_train(y, None, g, bb, rm, rv, 0.1, 1e-5, True), a.reps)
        t_bnt = timeit(lambda: C.bn_fwd_train_tiles(y, part, None, g, bb, rm, rv, 0.1, 1e-5, True), a.reps)
        # data gradient: dX[M, ci] = dY[M, co] W[co, ci]
        gy2 = y2
        wt = w2.t().contiguous()
        dx = torch.empty(M, ci, device=dev, dtype=torch.bfloat16)
        t_mmd = timeit(lambda: torch.mm(gy2, w2), a.reps)
        t_cvd = timeit(lambda: torch.ops.aten.convolution_backward(y, x, w, None, [1, 1], [0, 0], [1, 1], False,
                                                                  [0, 0], 1, [True, False, False]), a.reps)
        t_oursd = timeit(lambda: C.conv1x1_gemm(gy2, wt, dx, False, False), a.reps)
        t_addmm = timeit(lambda: dx.addmm_(gy2, w2), a.reps)
        t_oursacc = timeit(lambda: C.conv1x1_gemm(gy2, wt, dx, True, False), a.reps)
        lib_f = min(t_mm, t_cv) + t_bn
        ours_f = t_ours_s + t_bnt
        table[f"fwd,bf16,{M},{ci},{co}"] = "ours" if ours_f < lib_f else ("gemm" if t_mm < t_cv else "miopen")
        # data gradient of THIS conv: dX[M, ci]; with the shortcut hand-off (beta = 1) when ci is a block input
        d_lib = min(t_mmd, t_cvd)
        table[f"bwd_data,bf16,{M},{ci},{co}"] = "ours" if t_oursd < d_lib and t_oursacc <= t_addmm * 1.02 else (
            "gemm" if t_mmd < t_cvd else "miopen")
        tot["lib_f"] += n * lib_f
        tot["ours_f"] += n * min(ours_f, lib_f)
        tot["lib_d"] += n * min(t_mmd, t_cvd)
        tot["ours_d"] += n * min(t_oursd, t_mmd, t_cvd)
        print(f"{str((n, ci, co, h)):<22} | {t_mm:6.0f} {t_cv:6.0f} {t_ours:6.0f} | {t_bn:6.0f} {t_bnt:6.0f} | "
              f"{lib_f:7.0f} {ours_f:8.0f} | {t_mmd:6.0f} {t_cvd:6.0f} {t_oursd:6.0f} {t_addmm:6.0f} "
              f"{t_oursacc:8.0f}  (stats epilogue +{t_ours_s - t_ours:.0f})", flush=True)
        del x, y, dx, part
        torch.cuda.empty_cache()
    print("per step (ms, ours_* = best of both): " + "  ".join(f"{k} {v / 1e3:.2f}" for k, v in tot.items()))
    # weight gradient dW[co, ci] = dY^T X (library kernels), against the HBM floor of reading dY and X once
    print(f"{'(n, Ci, Co, H)':<22} | {'miopen_w':>8} {'mm_w':>6} | {'floor':>6} (us at 5.3 TB/s)")
    wsum = fsum = 0.0
    for n, ci, co, h in SHAPES:
        B = a.batch
        M = B * h * h
        x = torch.randn(B, ci, h, h, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 1, 1, device=dev) / ci ** 0.5).bfloat16()
        gy = torch.randn(B, co, h, h, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        x2, g2 = x.permute(0, 2, 3, 1).reshape(M, ci), gy.permute(0, 2, 3, 1).reshape(M, co)
        t_cw = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [0, 0], [1, 1], False,
                                                                 [0, 0], 1, [False, True, False]), a.reps)
        t_mw = timeit(lambda: torch.mm(g2.t(), x2), a.reps)
        floor = M * (ci + co) * 2 / 5.3e12 * 1e6
        wsum += n * min(t_cw, t_mw)
        fsum += n * floor
        print(f"{str((n, ci, co, h)):<22} | {t_cw:8.0f} {t_mw:6.0f} | {floor:6.0f}", flush=True)
        del x, gy
        torch.cuda.empty_cache()
    print(f"wgrad per step: best library {wsum / 1e3:.2f} ms, HBM floor {fsum / 1e3:.2f} ms")
    import json
    print("TABLE " + json.dumps(table, sort_keys=True))


if __name__ == "__main__":
    main()
