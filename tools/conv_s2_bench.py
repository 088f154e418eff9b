"""Per-shape timing of ResNet-50's stride-2 3x3 convs (batch 1024 default): our kernels
(conv3x3_s2.hip forward / 4-phase data gradient, conv3x3_wgrad.hip S = 2 with CO_T 128 and 64)
against MIOpen, with the MFMA rate each reaches.

    python tools/conv_s2_bench.py [--batch 1024] [--reps 10]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = [(128, 56), (256, 28), (512, 14)]  # (C, input H = W), Co = C


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
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.engine.miopen_cache import use_repo_miopen_cache
    from pytorch_distributed_training_example_amd.ops._native import native
    use_repo_miopen_cache()
    C = native()
    print(f"{'(C, H)':<12} | {'mio_f':>6} {'ours_f':>6} {'+stats':>6} | {'mio_d':>6} {'ours_d':>6} | "
          f"{'mio_w':>6} {'w128':>6} {'w64':>6} | PF/s ours f/d/w")
    tot = {"mio": 0.0, "ours": 0.0}
    for c, h in SHAPES:
        B = a.batch
        x = torch.randn(B, c, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(c, c, 3, 3, device="cuda") / (3 * c ** 0.5)).bfloat16().contiguous(
            memory_format=torch.channels_last)
        gy = torch.randn(B, c, h // 2, h // 2, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        flop = 2.0 * B * (h // 2) ** 2 * c * c * 9
        t_mf = timeit(lambda: F.conv2d(x, w, None, 2, 1), a.reps)
        t_of = timeit(lambda: C.conv3x3s2_fwd(x, w, False), a.reps)
        t_os = timeit(lambda: C.conv3x3s2_fwd(x, w, True), a.reps)
        args = (gy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1)
        t_md = timeit(lambda: torch.ops.aten.convolution_backward(*args, [True, False, False]), a.reps)
        wf = C.conv3x3_flip(w)
        t_od = timeit(lambda: C.conv3x3s2_dgrad(gy, wf, h, h), a.reps)
        t_mw = timeit(lambda: torch.ops.aten.convolution_backward(*args, [False, True, False]), a.reps)
        C.conv3x3_wgrad_tune(-1, 0)
        t_w128 = timeit(lambda: C.conv3x3s2_wgrad(x, gy), a.reps)
        C.conv3x3_wgrad_tune(-1, 64)
        t_w64 = timeit(lambda: C.conv3x3s2_wgrad(x, gy), a.reps)
        C.conv3x3_wgrad_tune(-1, 0)
        ours_w = min(t_w128, t_w64)
        tot["mio"] += t_mf + t_md + t_mw
        tot["ours"] += t_os + t_od + ours_w
        print(f"{str((c, h)):<12} | {t_mf:6.0f} {t_of:6.0f} {t_os:6.0f} | {t_md:6.0f} {t_od:6.0f} | "
              f"{t_mw:6.0f} {t_w128:6.0f} {t_w64:6.0f} | {flop / t_of / 1e9:.2f} {flop / t_od / 1e9:.2f} "
              f"{flop / ours_w / 1e9:.2f}", flush=True)
        del x, gy
        torch.cuda.empty_cache()
    print(f"per step (3 convs, fwd+dgrad+wgrad): MIOpen {tot['mio'] / 1e3:.2f} ms, ours {tot['ours'] / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
